"""Pricer façades on the MI355X (HIP engine) against the reference.

Tolerances (fp64; the kernel reassociates the Thomas solve, so agreement is
to rounding, not bitwise):
  price, delta:            |x - ref| <= 1e-10 + 1e-9 |ref|
  gamma, theta, vega:      |x - ref| <= 1e-8 * max(1, |ref|)
  value vectors:           max|V - V_ref| <= 1e-10 * max(1, max|V_ref|)
"""
import datetime as dt
import math
import os

import numpy as np
import pandas as pd
import pytest

from backends import oracle_engine
from conftest import GOLDEN, load_golden
from finite_difference_amd import scenarios
from finite_difference_amd.engine import Engine
from finite_difference_amd.fd_barrier import FDDoubleBarrier

pytestmark = pytest.mark.gpu

TIGHT = {"price": (1e-10, 1e-9), "delta": (1e-10, 1e-9)}


def close(name, x, ref):
    atol, rtol = TIGHT.get(name, (1e-8, 1e-8))
    return abs(x - ref) <= atol + rtol * abs(ref) if name in TIGHT else \
        abs(x - ref) <= 1e-8 * max(1.0, abs(ref))


def check_greeks(g, ref, label):
    worst = {k: abs(g[k] - ref[k]) for k in ref}
    print(f"[{label}] abs err {worst}")
    for k in ref:
        assert close(k, g[k], ref[k]), (label, k, g[k], ref[k])


def test_american_golden_on_gpu():
    import test_american_host as T
    for case in T.CASES:
        p = T.make(case, Engine())
        assert close("price", p.price_log(), case["price_log"])
        assert close("price", p.price_log2(), case["price_log2"])
        check_greeks(p.greeks_log2(), case["greeks_log2"], "american " + case["name"])


def test_black76_golden_on_gpu():
    import test_black76_host as T
    for case in T.CASES:
        p = T.make(case, Engine())
        V = p._solve_grid()
        ref = np.array(case["V"])
        assert np.max(np.abs(np.array(V) - ref)) <= 1e-10 * max(1.0, np.max(np.abs(ref)))
        assert close("price", p.price_log(), case["price_log"])
        assert close("price", p.price_log2(), case["price_log2"])
        check_greeks(p.greeks_log2(), case["greeks_log2"], "black76 " + case["name"])


def test_american_config2_full_grid():
    rec = load_golden("american_cases.json")["config2"]
    from finite_difference_amd.american import AmericanFDMPricer
    from finite_difference_amd import market
    c = market.iso_curve(market.create_rate_df(math.exp(0.07053828272) - 1.0))
    p = AmericanFDMPricer(spot=176.39, strike=170.0, valuation_date=dt.date(2025, 7, 28),
                          maturity_date=dt.date(2025, 8, 28), sigma=0.296783211249,
                          option_type="put", discount_curve=c, forward_curve=c,
                          num_space_nodes=2048, num_time_steps=4096, rannacher_steps=2)
    V = p._solve_grid()
    assert len(V) == rec["V_len"]
    for i, v in rec["V_sample"].items():
        assert abs(V[int(i)] - v) <= 1e-10 * max(1.0, abs(v))
    # every node, against the oracle's march of the same plan (the golden
    # record holds the reference's vector at every 64th node only)
    q = AmericanFDMPricer(spot=176.39, strike=170.0, valuation_date=dt.date(2025, 7, 28),
                          maturity_date=dt.date(2025, 8, 28), sigma=0.296783211249,
                          option_type="put", discount_curve=c, forward_curve=c,
                          num_space_nodes=2048, num_time_steps=4096, rannacher_steps=2,
                          engine=oracle_engine())
    Vo = np.asarray(q._solve_grid())
    err = np.max(np.abs(np.asarray(V) - Vo)) / max(1.0, float(np.max(np.abs(Vo))))
    print(f"[config2] full-vector max rel err vs oracle {err:.2e}")
    assert err <= 1e-10
    print(f"[config2] price {p.price_log()!r} ref {rec['price_log']!r}")
    assert close("price", p.price_log(), rec["price_log"])


def test_barrier_golden_on_gpu():
    import test_barrier_host as T
    for case in T.GOLD["cases"]:
        p = T.make(case["inputs"], Engine())
        assert close("price", p.price_log2(), case["price_log2"])
        check_greeks(p.greeks_log2(), case["greeks_log2"], "barrier " + case["name"])


@pytest.mark.parametrize("cfg,res", [("config_scenarios.csv", "scenario_results.csv"),
                                     ("config_scenarios_space_1.csv", "scenario_results_1.csv")])
def test_runner_committed_results_on_gpu(cfg, res, tmp_path):
    out = tmp_path / "o.csv"
    scenarios.run_all_scenarios(os.path.join(GOLDEN, "ref_csv", cfg), str(out),
                                scenarios.runner_base_params("put", 500), verbose=False)
    got = pd.read_csv(out, float_precision="round_trip")
    ref = pd.read_csv(os.path.join(GOLDEN, "ref_csv", res), float_precision="round_trip")
    for col in ("model_price", "model_delta", "model_gamma", "model_vega"):
        err = float(np.max(np.abs(got[col].to_numpy() - ref[col].to_numpy())))
        print(f"[{res}] {col} max abs err {err:.3e}")
        # price/delta: 1e-10 abs; gamma/vega (finite differences / 0.01): 1e-8
        assert err <= (1e-10 if col in ("model_price", "model_delta") else 1e-8)


def test_cn_log_golden_on_gpu():
    import test_cn_log_host as T
    for case in T.CASES:
        p = T.make(case["inputs"], Engine())
        assert close("price", p.price(), case["price"])
        if "greeks" in case:
            check_greeks(p.greeks(), case["greeks"], "cnlog " + case["inputs"]["name"])


def test_config3_explicit_batch_sample_vs_oracle():
    """BASELINE config 3 shape: 1024 x 2000 explicit grid, mixed barrier types."""
    rng = np.random.default_rng(20250728)
    base = scenarios.runner_base_params("put", 1024)
    base["num_time_steps"] = 2000
    base["grid_mode"] = "explicit"
    rows = []
    kinds = ["up-and-out", "down-and-out", "up-and-in", "down-and-in"]
    for i in range(16):
        bt = kinds[i % 4]
        rows.append(dict(scenario_name=f"s{i}", S0=229.74, K=float(rng.uniform(150, 300)),
                         sigma=float(rng.uniform(0.15, 0.45)), rate=0.073086, barrier_type=bt,
                         upper_barrier=float(rng.uniform(1.02, 1.5) * 229.74) if "up" in bt else None,
                         lower_barrier=float(rng.uniform(0.6, 0.98) * 229.74) if "down" in bt else None))
    gpu = scenarios.run_rows(rows, dict(base, opt_type="call"))
    ref = scenarios.run_rows(rows, dict(base, opt_type="call"), engine=oracle_engine())
    for g, r in zip(gpu, ref):
        for k in ("model_price", "model_delta"):
            assert abs(g[k] - r[k]) <= 1e-10 + 1e-9 * abs(r[k]), (k, g[k], r[k])
        for k in ("model_gamma", "model_vega"):
            assert abs(g[k] - r[k]) <= 1e-8 * max(1.0, abs(r[k])), (k, g[k], r[k])


def test_config5_double_barrier_full_grid_vs_oracle():
    P = (20.786, 21.0, 19.0, 23.0, 0.10994120968)
    b, r, T = 0.049493018, 0.0709454892, 49 / 365
    d_gpu = FDDoubleBarrier(*P, "c", "out", n_space=4096, n_time=8192)
    sv = d_gpu.solve_for(b, r, T)
    Vg = Engine().run([sv])[0]
    Vo = oracle_engine().run([sv])[0]
    err = float(np.max(np.abs(Vg - Vo))) / max(1.0, float(np.max(np.abs(Vo))))
    print(f"[config5] rel err {err:.3e} price {d_gpu.finish(Vg, b, r, T)}")
    assert err <= 1e-10


def test_config5_knockout_window_on_gpu_vs_whole_grid_oracle():
    """The façade's default path (ko_window.py): the windowed march on the GPU
    against the whole-grid oracle march, every node of the configured grid,
    and the price through FDDoubleBarrier.price against the whole-grid
    oracle price.  Single-barrier every-step engine too (one side cut)."""
    from finite_difference_amd.fd_barrier import FDBarrierEngine
    from finite_difference_amd.ko_window import ko_window
    P = (20.786, 21.0, 19.0, 23.0, 0.10994120968)
    b, r, T = 0.049493018, 0.0709454892, 49 / 365
    d = FDDoubleBarrier(*P, "c", "out", n_space=4096, n_time=8192)
    sv = d.solve_for(b, r, T)
    w = ko_window(sv, sv.ko_value)
    assert w is not None and w.solve.n_nodes < 0.2 * sv.n_nodes
    Vg = w.expand(Engine().run([w.solve])[0])
    Vo = oracle_engine().run([sv])[0]
    err = float(np.max(np.abs(Vg - Vo))) / max(1.0, float(np.max(np.abs(Vo))))
    print(f"[config5 window] {w.solve.n_nodes} of {sv.n_nodes} nodes, rel err {err:.3e}")
    assert err <= 1e-10
    p_gpu = FDDoubleBarrier(*P, "c", "out", n_space=4096, n_time=8192).price(b, r, T)
    p_ref = FDDoubleBarrier(*P, "c", "out", n_space=4096, n_time=8192, engine=oracle_engine(),
                            active_window=False).price(b, r, T)
    assert abs(p_gpu - p_ref) <= 1e-10 + 1e-9 * abs(p_ref)
    kw = dict(s=100.0, b=0.03, r=0.05, t=0.5, x=100.0, sigma=0.25, h=88.0, optionflag="p",
              directionflag="d", in_out_flag="i", k=1.5, rebate_timing_in="hit",
              n_space=2048, n_time=4000)
    e_gpu = FDBarrierEngine(**kw)
    assert all(wi is not None for _, wi in e_gpu.planned())
    p_gpu = e_gpu.price()
    p_ref = FDBarrierEngine(**kw, engine=oracle_engine(), active_window=False).price()
    assert abs(p_gpu - p_ref) <= 1e-10 + 1e-9 * abs(p_ref)
