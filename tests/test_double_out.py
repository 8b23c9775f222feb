"""The production barrier engine's double knock-out branch
(discrete_barrier_fdm_pricer.py:435-437), pinned to the reference itself:
tests/golden/double_out_cases.json holds _solve_grid(apply_KO=True) value
vectors the reference produced for double-out puts and calls, with and
without a rebate (tests/golden/make_golden.py gen_double_out).

CPU: the oracle's literal restatement and the product facade (driven by the
oracle) reproduce them bit for bit; price_log2 refuses double-* as the
reference does (:946).  GPU: the HIP march reproduces them to
max|V - V_ref| <= 1e-10 max(1, max|V_ref|) (reassociated Thomas, FMA)."""
import numpy as np
import pytest

from backends import oracle_engine
from conftest import load_golden
from finite_difference_amd.engine import Engine
from test_barrier_host import make

CASES = load_golden("double_out_cases.json")["cases"]


def _inputs(case):
    inp = dict(case["inputs"])
    inp.pop("name", None)
    inp["barrier_type"] = "double-out"
    return inp


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_oracle_double_out_bitwise(oracle_lib, case):
    inp, at = case["inputs"], case["attrs"]
    v = oracle_lib.ref_barrier_solve(
        case["s_nodes"], n_time=inp["num_time_steps"], T=at["time_to_expiry"], dx=case["dx"],
        sigma=inp["sigma"], r=at["discount_rate_nacc"], b=at["carry_rate_nacc"],
        q=at["div_yield_nacc"], rannacher_steps=2, option_type=inp["option_type"],
        K=inp["strike"], barrier_type="double-out", lower_barrier=inp["lower_barrier"],
        upper_barrier=inp["upper_barrier"], rebate_amount=inp.get("rebate_amount", 0.0),
        rebate_at_hit=inp.get("rebate_at_hit", True), carry=at["carry_rate_nacc"],
        monitor_idx=case["monitor_idx"], apply_KO=True)
    assert len(v) == case["N_s"]
    assert np.array_equal(v, np.array(case["V_ko"]))


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_facade_double_out_bitwise_through_oracle(case):
    p = make(_inputs(case), oracle_engine())
    V = p._solve_grid(apply_KO=True)
    assert p.s_nodes == case["s_nodes"]
    assert V == case["V_ko"]
    assert case["price_log2_raises"] == "ValueError"
    with pytest.raises(ValueError):
        p.price_log2()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_double_out_on_gpu(case):
    p = make(_inputs(case), Engine())
    V = np.array(p._solve_grid(apply_KO=True))
    ref = np.array(case["V_ko"])
    assert V.shape == ref.shape
    err = float(np.max(np.abs(V - ref))) / max(1.0, float(np.max(np.abs(ref))))
    print(f"[double-out {case['name']}] rel err {err:.2e}")
    assert err <= 1e-10
