"""Knock-out window (finite_difference_amd/ko_window.py) on the CPU oracle:
the windowed march equals the whole-grid march at every node.

The window drops the part of the grid beyond a barrier that is projected on
every step; its influence on the live nodes is below 1e-18 relative (the
decay margin), so the bound written here is 1e-12 of max(1, max|V|) -- the
same rounding-level agreement as two orderings of the same solve -- and the
nodes outside the window must equal the projection value exactly."""
import math

import numpy as np
import pytest

from backends import oracle_engine
from finite_difference_amd.engine import Boundary
from finite_difference_amd.fd_barrier import FDBarrierEngine, FDDoubleBarrier, price_many
from finite_difference_amd.ko_window import decay_rate, ko_window, margin_nodes

TOL = 1e-12
CFG5 = dict(S=20.786, X=21.0, L=19.0, U=23.0, sigma=0.10994120968)
B5, R5, T5 = 0.049493018, 0.0709454892, 49 / 365


def _close(v_win, v_full):
    scale = max(1.0, float(np.max(np.abs(v_full))))
    return float(np.max(np.abs(v_win - v_full))) / scale


def test_config5_window_equals_whole_grid_at_every_node():
    """BASELINE config 5 at its full 4096 x 8192 size: the window keeps about
    a sixth of the grid and reproduces every node."""
    d = FDDoubleBarrier(**CFG5, callflag="c", inflag="out", n_space=4096, n_time=8192)
    sv = d.solve_for(B5, R5, T5)
    w = ko_window(sv, sv.ko_value)
    assert w is not None
    assert w.solve.n_nodes < 0.2 * sv.n_nodes
    K = margin_nodes(sv)
    assert decay_rate(sv) ** (K - 8) <= 1e-18
    assert w.a == sv.ko_lo + 1 - K and w.a + w.solve.n_nodes - 1 == sv.ko_hi - 1 + K
    eng = oracle_engine()
    v_full, v_win = eng.run([sv, w.solve])
    v = w.expand(v_win)
    assert _close(v, v_full) <= TOL
    outside = np.r_[0:w.a, w.a + w.solve.n_nodes:sv.n_nodes]
    assert np.all(v[outside] == 0.0) and np.all(v_full[outside] == 0.0)


@pytest.mark.parametrize("cf", "cp")
@pytest.mark.parametrize("inflag", ["out", "in"])
def test_double_barrier_price_window_on_off(cf, inflag):
    kw = dict(**CFG5, callflag=cf, inflag=inflag, n_space=1024, n_time=2000)
    on = FDDoubleBarrier(**kw, engine=oracle_engine()).price(B5, R5, T5)
    off = FDDoubleBarrier(**kw, engine=oracle_engine(), active_window=False).price(B5, R5, T5)
    assert abs(on - off) <= TOL * max(1.0, abs(off))


ARGS = dict(s=100.0, b=0.03, r=0.05, t=0.5, x=100.0, sigma=0.25)


@pytest.mark.parametrize("of,df,h", [("c", "u", 115.0), ("p", "d", 88.0), ("c", "d", 90.0),
                                     ("p", "u", 112.0)])
@pytest.mark.parametrize("io,k,timing", [("o", 0.0, None), ("o", 2.0, "hit"),
                                         ("o", 2.0, "expiry"), ("i", 1.5, "expiry"),
                                         ("i", 1.5, "hit")])
def test_single_barrier_window_on_off(of, df, h, io, k, timing):
    """Every rebate form (out at hit / at expiry, in-rebates' extra solves):
    the window's Dirichlet value is the projection value as the kernel
    evaluates it from the Boundary, the full march's from mon_rebates."""
    rt = dict(rebate_timing_out=timing) if io == "o" else dict(rebate_timing_in=timing)
    kw = dict(**ARGS, h=h, optionflag=of, directionflag=df, in_out_flag=io, k=k,
              n_space=1024, n_time=1500, **({} if timing is None else rt))
    on = FDBarrierEngine(**kw, engine=oracle_engine())
    off = FDBarrierEngine(**kw, engine=oracle_engine(), active_window=False)
    plan = on.planned()
    assert all(w is not None for _, w in plan)
    p_on, p_off = on.price(), off.price()
    assert abs(p_on - p_off) <= TOL * max(1.0, abs(p_off))


def test_price_many_mixes_windowed_and_whole_grid():
    eng = oracle_engine()
    es = [FDBarrierEngine(**ARGS, h=115.0, optionflag="c", directionflag="u", in_out_flag="o",
                          k=0.0, n_space=512, n_time=800, engine=eng),
          FDBarrierEngine(**ARGS, h=115.0, optionflag="c", directionflag="u", in_out_flag="o",
                          k=0.0, n_space=512, n_time=800, engine=eng,
                          monitor_times=[0.1, 0.2, 0.3, 0.4, 0.5])]
    assert es[0].planned()[0][1] is not None and es[1].planned()[0][1] is None
    got = price_many(es)
    want = [FDBarrierEngine(**ARGS, h=115.0, optionflag="c", directionflag="u", in_out_flag="o",
                            k=0.0, n_space=512, n_time=800, engine=oracle_engine(),
                            monitor_times=mt, active_window=False).price()
            for mt in (None, [0.1, 0.2, 0.3, 0.4, 0.5])]
    assert abs(got[0] - want[0]) <= TOL and got[1] == want[1]


def test_no_window_without_every_step_projection_or_cut():
    d = FDDoubleBarrier(**CFG5, callflag="c", inflag="out", n_space=512, n_time=400,
                        monitor_times=[0.05, 0.1])
    sv = d.solve_for(B5, R5, T5)
    assert ko_window(sv, sv.ko_value) is None               # discrete monitoring
    d = FDDoubleBarrier(**CFG5, callflag="c", inflag="out", n_space=512, n_time=400)
    sv = d.solve_for(B5, R5, T5)
    sv.ko_lo, sv.ko_hi = -1, 1 << 30
    assert ko_window(sv, Boundary()) is None                # nothing knocked out
    sv = d.solve_for(B5, R5, T5)
    sv.ko_lo, sv.ko_hi = 2, sv.n_nodes - 3
    assert ko_window(sv, Boundary()) is None                # too little to cut


def test_margin_covers_the_rannacher_phase():
    """The theta = 1 steps decay slower: the margin is sized by the larger
    of the two phases' factors."""
    d = FDDoubleBarrier(**CFG5, callflag="c", inflag="out", n_space=4096, n_time=8192)
    sv = d.solve_for(B5, R5, T5)
    a, c, bc = sv.coeffs
    rhos = []
    for th in (1.0, 0.5):
        AL, AC, AU = -th * sv.dt * a, 1 - th * sv.dt * bc, -th * sv.dt * c
        r = 0.5 * (AC + math.sqrt(AC * AC - 4 * AL * AU))
        rhos.append(max(abs(AL / r), abs(AU / r)))
    assert decay_rate(sv) == max(rhos) and rhos[0] > rhos[1]
