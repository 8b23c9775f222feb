"""Pin the CPU oracle to the reference: bit-for-bit on golden vectors.

The vectors in tests/golden/*.json were produced by running the reference
code itself (tests/golden/make_golden.py, build container only).
"""
import math

import numpy as np
import pytest

from conftest import load_golden


def _log_grid(S_min, S_max, n):
    x_min, x_max = math.log(S_min), math.log(S_max)
    dx = (x_max - x_min) / n
    return dx, [math.exp(x_min + i * dx) for i in range(n + 1)]


@pytest.mark.parametrize("case", load_golden("cn_log_cases.json"),
                         ids=lambda c: c["inputs"]["name"])
def test_cnlog_solver_bitwise(oracle_lib, case):
    inp = case["inputs"]
    dx, s = _log_grid(case["S_min"], case["S_max"], case["N_space"])
    kw = dict(n_time=case["N_time"], T=inp["T"], dx=dx, sigma=inp["sigma"], r_disc=inp["r"],
              b_carry=inp["b"], option_type=inp["opt"], K=inp["K"],
              lower_barrier=inp["lo"], upper_barrier=inp["up"], rebate=inp["rebate"],
              monitor_idx=case["monitor_idx"])
    bt = inp["bt"]
    if "V_ko" in case:
        v = oracle_lib.ref_cnlog_solve(s, barrier_type=bt, apply_KO=True, **kw)
        assert np.array_equal(v, np.array(case["V_ko"]))
    v = oracle_lib.ref_cnlog_solve(s, barrier_type=bt, apply_KO=False, **kw)
    assert np.array_equal(v, np.array(case["V_noko"]))


@pytest.mark.parametrize("case", load_golden("barrier_cases.json")["cases"],
                         ids=lambda c: c["name"])
def test_barrier_solver_bitwise(oracle_lib, case):
    inp, at = case["inputs"], case["attrs"]
    bt = inp["barrier_type"].replace("-in", "-out")
    kw = dict(n_time=inp["num_time_steps"], T=at["time_to_expiry"], dx=case["dx"],
              sigma=inp["sigma"], r=at["discount_rate_nacc"], b=at["carry_rate_nacc"],
              q=at["div_yield_nacc"], rannacher_steps=2, option_type=inp["option_type"],
              K=inp["strike"], barrier_type=bt, lower_barrier=inp.get("lower_barrier"),
              upper_barrier=inp.get("upper_barrier"),
              rebate_amount=inp.get("rebate_amount", 0.0),
              rebate_at_hit=inp.get("rebate_at_hit", True), carry=at["carry_rate_nacc"],
              monitor_idx=case["monitor_idx"])
    v = oracle_lib.ref_barrier_solve(case["s_nodes"], apply_KO=True, **kw)
    assert len(v) == case["N_s"]
    assert np.array_equal(v, np.array(case["V_ko"]))
    v = oracle_lib.ref_barrier_solve(case["s_nodes"], apply_KO=False, **kw)
    assert np.array_equal(v, np.array(case["V_noko"]))


@pytest.mark.parametrize("case", [c for c in load_golden("american_cases.json")["cases"]
                                  if not c["inputs"]["divs"]], ids=lambda c: c["name"])
def test_american_segment_bitwise(oracle_lib, case):
    inp, at = case["inputs"], case["attrs"]
    s = case["s_nodes"]
    K = at["strike_snapped"]
    call = inp["option_type"] == "call"
    v0 = [max(x - K, 0.0) if call else max(K - x, 0.0) for x in s]
    v = oracle_lib.ref_american_segment(
        s, at["dx"], v0, 0.0, at["time_to_expiry"], inp["M"], True, 2, inp["sigma"],
        at["discount_rate_nacc"], at["carry_rate_nacc"], inp["option_type"], K)
    assert np.array_equal(v, np.array(case["V"]))
