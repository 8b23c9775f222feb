"""DiscreteBarrierCrankNicolsonLog host logic (auto grid, round() monitor
indexing, KO thresholds, 3-solve vega), driven by the CPU oracle, against the
reference's own outputs (tests/golden/cn_log_cases.json), bit-for-bit."""
import numpy as np
import pytest

from backends import oracle_engine
from conftest import load_golden
from finite_difference_amd.cn_log import DiscreteBarrierCrankNicolsonLog

CASES = load_golden("cn_log_cases.json")


def make(inp, engine):
    return DiscreteBarrierCrankNicolsonLog(
        S0=inp["S0"], K=inp["K"], T=inp["T"], sigma=inp["sigma"], r_disc=inp["r"],
        b_carry=inp["b"], option_type=inp["opt"], barrier_type=inp["bt"],
        lower_barrier=inp["lo"], upper_barrier=inp["up"], rebate=inp["rebate"],
        monitor_times=inp["monitor_times"], N_space=inp["N"], N_time=inp["M"], engine=engine)


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["inputs"]["name"])
def test_cn_log_bitwise(case):
    p = make(case["inputs"], oracle_engine())
    assert p.price() == case["price"]
    p.configure_grid()
    assert (p.N_space, p.N_time) == (case["N_space"], case["N_time"])
    assert (p._S_min, p._S_max) == (case["S_min"], case["S_max"])
    assert sorted(p._monitor_indices_tau(p.T / p.N_time)) == case["monitor_idx"]
    if "greeks" in case:
        assert p.greeks() == case["greeks"]
    else:  # reference raises (missing method); ours returns vanilla - KO
        g = p.greeks()
        assert set(g) == {"price", "delta", "gamma", "theta", "vega"}
        assert np.isfinite(list(g.values())).all()
    if "V_ko" in case:
        assert p._solve_grid(apply_KO=True) == case["V_ko"]
    assert p._solve_grid(apply_KO=False) == case["V_noko"]


def test_three_solves_one_launch():
    eng = oracle_engine()
    p = make(CASES[0]["inputs"], eng)
    p.greeks()
    assert eng.launches == 1 and eng.solves == 3
