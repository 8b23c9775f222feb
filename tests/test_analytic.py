"""Analytic engines vs the reference's outputs (tests/golden/analytic_cases.json)."""
import math

import numpy as np
import pytest

from conftest import load_golden
from finite_difference_amd.analytic import BarrierEngine, DoubleBarrier

G = load_golden("analytic_cases.json")


@pytest.mark.parametrize("case", G["barrier_engine"])
def test_barrier_engine(case):
    e = BarrierEngine(**case["args"])
    assert math.isclose(e.price(), case["price"], rel_tol=1e-12, abs_tol=1e-13)
    assert math.isclose(e.vanilla(), case["vanilla"], rel_tol=1e-12, abs_tol=1e-13)


@pytest.mark.parametrize("case", G["double_barrier"])
def test_double_barrier_matches_reference(case):
    a = dict(case["args"])
    b, r, T = a.pop("b"), a.pop("r"), a.pop("T")
    p = DoubleBarrier(**a)
    assert math.isclose(p.price(b=b, r=r, T=T), case["price"], rel_tol=1e-12, abs_tol=1e-13)
    assert math.isclose(DoubleBarrier._bs_price(a["callflag"], a["S"], a["X"], r, b,
                                                a["sigma"], T), case["bs"], rel_tol=1e-12)


def test_double_barrier_corrected_put_is_bounded_by_vanilla():
    # the reference's put branch (lower limit 1 instead of l) can exceed the
    # vanilla; the corrected series is a proper knock-out value.
    args = dict(S=100.0, X=100.0, L=60.0, U=160.0, sigma=0.2, callflag="p", inflag="out")
    fixed = DoubleBarrier(corrected_put=True, **args).price(b=0.03, r=0.05, T=0.5)
    van = DoubleBarrier._bs_price("p", 100.0, 100.0, 0.05, 0.03, 0.2, 0.5)
    assert 0.0 < fixed <= van
