"""Vectorised whole-file American runner (american_batch.py) against the
per-row façade, through the CPU oracle engine.

* fdcn_american_plan's grids, payoffs, coefficients, boundaries and readout
  positions are bit-identical to AmericanFDMPricer's (_build_log_grid,
  snapping, _segment_solve + engine.pack, session.readout);
* price_log2 / greeks_log2 of every row equal the per-row façade's (==),
  puts and calls, two curves, with and without discrete dividends.
"""
import datetime as dt

import numpy as np
import pytest

from backends import oracle_engine
from finite_difference_amd import american_batch, capi, scenarios
from finite_difference_amd.american import prefetch_many
from finite_difference_amd.engine import pack
from finite_difference_amd.session import readout

VAL, MAT = dt.date(2025, 7, 28), dt.date(2025, 8, 28)


def _base(opt, divs=None, n=64, m=40):
    return dict(valuation=VAL, maturity=MAT, opt_type=opt, divs=divs or [],
                num_space_nodes=n, num_time_steps=m)


def _rows(n, seed):
    rng = np.random.default_rng(seed)
    return [dict(scenario_name=f"a{i}", S0=float(176.39 * rng.uniform(0.9, 1.1)),
                 K=float(rng.uniform(150, 200)), sigma=float(rng.uniform(0.15, 0.45)),
                 rate=(0.0705, 0.065)[i % 2], FA_price=(None, 5.0)[i % 2], FA_delta=-0.4,
                 FA_gamma=float("nan"), FA_vega=0.2) for i in range(n)]


def _per_row(rows, base):
    ps = [scenarios.make_american_pricer(r["S0"], r["K"], r["sigma"], r["rate"],
                                         engine=oracle_engine(), **base) for r in rows]
    prefetch_many(ps)
    return [(p.price_log2(), p.greeks_log2()) for p in ps]


@pytest.mark.parametrize("opt", ["put", "call"])
@pytest.mark.parametrize("divs", [None, [(dt.date(2025, 8, 11), 1.5)],
                                  [(dt.date(2025, 8, 4), 0.8), (dt.date(2025, 8, 18), 1.1)]],
                         ids=["nodiv", "div1", "div2"])
def test_vectorized_equals_per_row(opt, divs):
    base = _base(opt, divs)
    rows = _rows(8, 3)
    ref = _per_row(rows, base)
    cols = {k: [r[k] for r in rows] for k in american_batch.ROW_KEYS}
    res = american_batch.price_columns(cols, base, oracle_engine())
    for i, (p2, g) in enumerate(ref):
        assert res["price_log2"][i] == p2, (i, res["price_log2"][i], p2)
        for k in ("price", "delta", "gamma", "vega", "theta"):
            assert res[k][i] == g[k], (i, k, res[k][i], g[k])


def test_result_rows_match_runner_schema(tmp_path):
    import pandas as pd
    base = _base("put")
    rows = _rows(5, 9)
    cfg = tmp_path / "a.csv"
    pd.DataFrame(rows).to_csv(cfg, index=False)
    df = scenarios.run_all_american_scenarios(str(cfg), None, base, oracle_engine(),
                                              verbose=False)
    rows = [dict(r) for _, r in pd.read_csv(cfg).iterrows()]  # the values the CSV holds
    ref = _per_row(rows, base)
    assert list(df.columns)[:5] == ["scenario_name", "S0", "K", "sigma", "rate"]
    for i, (p2, g) in enumerate(ref):
        assert df["model_price"].iloc[i] == p2
        assert df["model_delta"].iloc[i] == g["delta"]
        assert df["model_vega"].iloc[i] == g["vega"]


@pytest.mark.parametrize("with_grids", [True, False], ids=["grids", "lazy_nodes"])
@pytest.mark.parametrize("opt", ["call", "put"])
def test_plan_bitwise_equal_facade(opt, with_grids):
    """fdcn_american_plan against the facade, bit for bit: with the grids
    returned (every node evaluated) and without (nodes evaluated where read,
    the payoff's out-of-the-money side written as zeros without an exp)."""
    base = _base(opt, n=50)
    rows = _rows(6, 5)
    jobs, calls, solves, reads = [], [], [], []
    for q, r in enumerate(rows):
        p = scenarios.make_american_pricer(r["S0"], r["K"], r["sigma"], r["rate"], **base)
        p._build_log_grid()
        sv = p._segment_solve(p._payoff_array(), 0.0, p.time_to_expiry, p.num_time_steps, True)
        solves.append(sv)
        jobs.append((p.spot, p.strike, p.sigma, p.carry_rate_nacc, p.discount_rate_nacc))
        calls.append(1 if opt == "call" else 0)
        s = p.s_nodes
        i = int(np.argmin(np.abs(np.asarray(s) - p.spot_snapped)))
        i = 1 if i < 1 else (len(s) - 3 if i > len(s) - 3 else i)
        reads += [readout(q, s, p.spot_snapped),
                  readout(q, s, p.spot_snapped, p.spot_snapped, dg_mode=2, idx=i)]
        T, smm = p.time_to_expiry, p.s_max_mult
    plan = capi.american_plan(np.array(jobs), np.array(calls), 50, smm, T, with_grids=with_grids)
    g = pack(solves, list(range(len(solves))))
    P = plan["params"].copy()
    P[:, capi.P_DT] = g.params[:, capi.P_DT]
    np.testing.assert_array_equal(P, g.params)
    np.testing.assert_array_equal(plan["iparams"], g.iparams)
    np.testing.assert_array_equal(plan["payoff"], g.v_init)
    np.testing.assert_array_equal(plan["payoff"], g.payoff)
    np.testing.assert_array_equal(plan["rint"],
                                  np.array([(x.slot, x.icase, x.ilo, x.idx, x.dg_mode) for x in reads]))
    np.testing.assert_array_equal(plan["rdbl"], np.array([x.dbl for x in reads]))


def test_rejects_bad_rows():
    base = _base("put")
    rows = _rows(3, 1)
    rows[2]["sigma"] = 0.0
    cols = {k: [r[k] for r in rows] for k in american_batch.ROW_KEYS}
    with pytest.raises(ValueError):
        american_batch.price_columns(cols, base, oracle_engine())
