"""FD barrier engines (BarrierEngine / DoubleBarrier signatures) on the CPU
oracle: consistency with the closed forms.  Every-step projection is discrete
monitoring, which converges to the continuous closed form at O(sqrt(dt)); the
checks are that convergence and exact in/out parity, not bitwise parity."""
import math

import numpy as np
import pytest

from backends import oracle_engine
from finite_difference_amd.analytic import BarrierEngine, DoubleBarrier
from finite_difference_amd.fd_barrier import FDBarrierEngine, FDDoubleBarrier, price_many

ARGS = dict(s=100.0, b=0.03, r=0.05, t=0.5, x=100.0, sigma=0.25)


@pytest.mark.parametrize("of", "cp")
@pytest.mark.parametrize("df", "ud")
def test_fd_barrier_close_to_closed_form_and_parity(of, df):
    eng = oracle_engine()
    h = 115.0 if df == "u" else 88.0
    engines = [FDBarrierEngine(**ARGS, h=h, optionflag=of, directionflag=df, in_out_flag=io,
                               k=0.0, n_space=512, n_time=1000, engine=eng) for io in "io"]
    fin, fout = price_many(engines)
    assert eng.launches == 1
    ain = BarrierEngine(**ARGS, h=h, optionflag=of, directionflag=df, in_out_flag="i", k=0.0)
    aout = BarrierEngine(**ARGS, h=h, optionflag=of, directionflag=df, in_out_flag="o", k=0.0)
    assert abs(fin - ain.price()) < 0.06
    assert abs(fout - aout.price()) < 0.06
    assert fout > aout.price() - 1e-9          # discrete monitoring knocks out less
    assert math.isclose(fin + fout, ain.vanilla(), rel_tol=1e-12)


def test_fd_barrier_converges_with_steps():
    h = 115.0
    errs = []
    for nt in (250, 1000, 4000):
        e = FDBarrierEngine(**ARGS, h=h, optionflag="c", directionflag="u", in_out_flag="o",
                            k=0.0, n_space=1024, n_time=nt, engine=oracle_engine())
        errs.append(abs(e.price() - BarrierEngine(**ARGS, h=h, optionflag="c",
                                                  directionflag="u", in_out_flag="o",
                                                  k=0.0).price()))
    assert errs[2] < errs[1] < errs[0]


def test_crossed_status_is_closed_form():
    e = FDBarrierEngine(**ARGS, h=115.0, optionflag="c", directionflag="u", in_out_flag="i",
                        k=1.0, barrier_status="crossed", engine=oracle_engine())
    assert e.price() == BarrierEngine(**ARGS, h=115.0, optionflag="c", directionflag="u",
                                      in_out_flag="i", k=1.0, barrier_status="crossed").price()


@pytest.mark.parametrize("cf", "cp")
def test_fd_double_barrier_vs_douady(cf):
    P = (20.786, 21.0, 19.0, 23.0, 0.10994120968)
    b, r, T = 0.049493018, 0.0709454892, 49 / 365
    fd_out = FDDoubleBarrier(*P, cf, "out", n_space=512, n_time=2000,
                             engine=oracle_engine()).price(b, r, T)
    fd_in = FDDoubleBarrier(*P, cf, "in", n_space=512, n_time=2000,
                            engine=oracle_engine()).price(b, r, T)
    an = DoubleBarrier(*P, cf, "out", corrected_put=True).price(b, r, T)
    assert abs(fd_out - an) < 0.01
    assert math.isclose(fd_in + fd_out, DoubleBarrier._bs_price(cf, P[0], P[1], r, b, P[4], T),
                        rel_tol=1e-12)
