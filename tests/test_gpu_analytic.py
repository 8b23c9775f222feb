"""Batched closed-form engines on the MI355X (fdcn_rr_barrier_batch,
fdcn_double_barrier_batch) against the reference's outputs
(tests/golden/analytic_cases.json) and against the host engines.

Tolerance: the device's erfc/exp/log/pow differ from glibc's in the last
ulps, and the A-F factors subtract nearly equal terms, so agreement is
|gpu - ref| <= 1e-11 |ref| + 1e-12 (the host engines match the reference to
1e-12 relative, test_analytic.py).
"""
import math

import numpy as np
import pytest

from conftest import load_golden
from finite_difference_amd import capi
from finite_difference_amd.analytic import (BarrierEngine, DoubleBarrier, barrier_engine_batch,
                                            double_barrier_batch)

pytestmark = pytest.mark.gpu
G = load_golden("analytic_cases.json")
RTOL, ATOL = 1e-11, 1e-12


def _close(a, b):
    return abs(a - b) <= RTOL * abs(b) + ATOL


def test_rr_barrier_golden():
    price, vanilla = barrier_engine_batch([c["args"] for c in G["barrier_engine"]])
    worst = 0.0
    for c, p, v in zip(G["barrier_engine"], price, vanilla):
        assert _close(p, c["price"]), (c["args"], p, c["price"])
        assert _close(v, c["vanilla"]), (c["args"], v, c["vanilla"])
        worst = max(worst, abs(p - c["price"]) / max(1.0, abs(c["price"])))
    print(f"[rr golden] {len(price)} contracts, worst rel err {worst:.2e}")


def test_rr_barrier_random_batch_vs_host():
    rng = np.random.default_rng(11)
    n = 4000
    contracts = []
    for i in range(n):
        up = bool(rng.integers(2))
        s = float(rng.uniform(50, 150))
        contracts.append(dict(
            s=s, b=float(rng.uniform(-0.02, 0.08)), r=float(rng.uniform(0.0, 0.1)),
            t=float(rng.uniform(0.05, 2.0)), x=float(rng.uniform(0.7, 1.3) * s),
            sigma=float(rng.uniform(0.1, 0.6)),
            h=float(s * (rng.uniform(1.02, 1.4) if up else rng.uniform(0.6, 0.98))),
            optionflag="cp"[i % 2], directionflag="u" if up else "d",
            in_out_flag="io"[(i // 2) % 2], k=float(rng.uniform(0, 3)),
            barrier_status=(None, "crossed", "not_crossed")[i % 3],
            rebate_timing_in=("hit", "expiry")[(i // 3) % 2],
            rebate_timing_out=("hit", "expiry")[(i // 5) % 2]))
    price, vanilla = barrier_engine_batch(contracts)
    worst = 0.0
    for c, p, v in zip(contracts, price, vanilla):
        e = BarrierEngine(**c)
        ref_p, ref_v = e.price(), e.vanilla()
        assert _close(p, ref_p) and _close(v, ref_v), (c, p, ref_p, v, ref_v)
        worst = max(worst, abs(p - ref_p) / max(1.0, abs(ref_p)))
    print(f"[rr random] {n} contracts, worst rel err vs host {worst:.2e}")


def test_double_barrier_golden_and_corrected_put():
    cases = [dict(c["args"]) for c in G["double_barrier"]]
    m = cases[0]["m"]
    price = double_barrier_batch(cases, m=m)
    for c, p in zip(G["double_barrier"], price):
        assert _close(p, c["price"]), (c["args"], p, c["price"])
    fixed = dict(S=100.0, X=100.0, L=60.0, U=160.0, sigma=0.2, callflag="p", inflag="out",
                 b=0.03, r=0.05, T=0.5, corrected_put=True)
    got = double_barrier_batch([fixed])[0]
    ref = DoubleBarrier(100.0, 100.0, 60.0, 160.0, 0.2, "p", "out",
                        corrected_put=True).price(b=0.03, r=0.05, T=0.5)
    assert _close(got, ref)


def test_bad_flags_raise():
    P = np.ones((1, capi.RR_NPARAM))
    F = np.array([[0, 0, 0, 0, 9]], dtype=np.int32)
    with pytest.raises(capi.FdcnError):
        capi.rr_barrier_batch(P, F)
    with pytest.raises(ValueError):
        barrier_engine_batch([dict(s=1, b=0, r=0, t=1, x=1, sigma=0.0, h=1, k=0,
                                   optionflag="c", directionflag="u", in_out_flag="i")])
