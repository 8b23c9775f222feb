"""Vectorised whole-file runner (scenario_batch.py) against the per-row
runner, through the CPU oracle engine.

* fdcn_barrier_plan's launch arrays are bit-identical to the per-row facade's
  (_make_solve + engine.pack) and its readouts to session.readout;
* run_rows_vectorized's result rows equal scenarios.run_rows's exactly, for
  every barrier type, puts and calls, two curves, dividends, rebates with
  either timing, already_hit / already_in, parity and explicit grids.
"""
import datetime as dt
import math

import numpy as np
import pytest

from backends import oracle_engine
from finite_difference_amd import capi, scenario_batch, scenarios
from finite_difference_amd.engine import pack


def _rows(n, seed, spot=229.74):
    rng = np.random.default_rng(seed)
    kinds = ["up-and-out", "down-and-out", "up-and-in", "down-and-in", "none"]
    rows = []
    for i in range(n):
        bt = kinds[i % 5]
        rows.append(dict(
            scenario_name=f"r{i}", S0=float(spot * rng.uniform(0.9, 1.1)),
            K=float(rng.uniform(180, 280)), sigma=float(rng.uniform(0.15, 0.45)),
            rate=(0.073086, 0.065, 0.08)[i % 3], barrier_type=bt,
            upper_barrier=float(rng.uniform(1.02, 1.4) * spot) if "up" in bt else None,
            lower_barrier=float(rng.uniform(0.7, 0.98) * spot) if "down" in bt else None,
            FA_price=(None, 1.0, 0.0)[i % 3], FA_delta=0.5, FA_gamma=float("nan"),
            FA_vega=0.2))
    return rows


def _same(a, b):
    if isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b):
        return True
    return a == b


def _check_rows(rows, base):
    a = scenarios.run_rows(rows, base, oracle_engine())
    b = scenario_batch.run_rows_vectorized(rows, base, oracle_engine())
    assert b is not None and len(a) == len(b)
    for ra, rb in zip(a, b):
        assert list(ra.keys()) == list(rb.keys())
        for k in ra:
            assert _same(ra[k], rb[k]), (ra["scenario_name"], ra["barrier_type"], k, ra[k], rb[k])


@pytest.mark.parametrize("mode,n", [("parity", 40), ("explicit", 64)])
@pytest.mark.parametrize("opt", ["put", "call"])
def test_vectorized_equals_per_row(mode, n, opt):
    base = scenarios.runner_base_params(opt, n)
    base.update(num_time_steps=40, grid_mode=mode)
    _check_rows(_rows(15, 3), base)


def test_vectorized_dividends_and_rebates():
    base = scenarios.runner_base_params("call", 48)
    base.update(num_time_steps=36, grid_mode="explicit", rebate_amount=1.5,
                rebate_at_hit=False, divs=[(dt.date(2025, 8, 10), 2.0),
                                           (dt.date(2025, 8, 20), 1.25)])
    _check_rows(_rows(10, 5), base)
    base.update(opt_type="put", rebate_at_hit=True)
    _check_rows(_rows(10, 6), base)


@pytest.mark.parametrize("flag", ["already_hit", "already_in"])
def test_vectorized_status_flags(flag):
    base = scenarios.runner_base_params("put", 40)
    base.update(num_time_steps=40, rebate_amount=2.0, **{flag: True})
    _check_rows(_rows(10, 7), base)


def test_vectorized_rejects_what_the_reference_rejects():
    base = scenarios.runner_base_params("put", 40)
    base.update(num_time_steps=40)
    rows = _rows(3, 1)
    rows[1]["barrier_type"] = "double-out"
    with pytest.raises(ValueError):
        scenarios.run_rows(rows, base, oracle_engine())
    with pytest.raises(ValueError):
        scenario_batch.run_rows_vectorized(rows, base, oracle_engine())
    rows = _rows(3, 1)
    rows[0]["sigma"] = 0.0
    with pytest.raises(ValueError):
        scenario_batch.run_rows_vectorized(rows, base, oracle_engine())


def test_empty_file():
    base = scenarios.runner_base_params("put", 40)
    assert scenario_batch.run_rows_vectorized([], base, oracle_engine()) == []


@pytest.mark.parametrize("opt", ["put", "call"])
@pytest.mark.parametrize("mode", ["parity", "explicit"])
def test_plan_arrays_bitwise_equal_facade(mode, opt):
    """The C plan builder against _make_solve + pack + session.readout (its
    grid nodes evaluated where read, the payoff's out-of-the-money side
    written as zeros without an exp: bit for bit, calls and puts)."""
    from finite_difference_amd.barrier import KI_TO_KO, tail_quantile
    from finite_difference_amd.session import readout
    base = scenarios.runner_base_params(opt, 64)
    base.update(num_time_steps=48, grid_mode=mode, rebate_amount=0.75, rebate_at_hit=False,
                divs=[(dt.date(2025, 8, 12), 1.0)])
    rows = [r for r in _rows(12, 11) if r["barrier_type"] != "none"]
    solves, reads, tpar = [], [], []
    R = len(rows)
    row = np.zeros((R, capi.BP_NROW))
    flag = np.zeros((R, capi.BP_NFLAG), np.int32)
    for j, r in enumerate(rows):
        bt = KI_TO_KO.get(r["barrier_type"], r["barrier_type"])
        p = scenarios.make_barrier_pricer(r["S0"], r["K"], r["sigma"], r["rate"], bt,
                                          r["upper_barrier"], r["lower_barrier"], **base)
        (sb, gb), (su, gu) = p.pde_solves(True, 0.0001)
        solves += [sb, su]
        reads += [readout(2 * j, gb.s_arr, p.spot - p.pv_divs, p.spot, dg_mode=1,
                          n_v=sb.n_nodes),
                  readout(2 * j + 1, gu.s_arr, p.spot - p.pv_divs, n_v=su.n_nodes)]
        tpar.append((p.sigma, p.spot, p.carry_rate_nacc, p.div_yield_nacc,
                     p.discount_rate_nacc, 0.0001, 0.0, 0.0))
        row[j] = (r["S0"], r["K"], r["sigma"], r["lower_barrier"] or 0.0,
                  r["upper_barrier"] or 0.0, p.carry_rate_nacc, p.div_yield_nacc,
                  p.discount_rate_nacc, p.pv_divs, 0.75)
        flag[j] = (1 if opt == "put" else 0, 1 if bt == "down-and-out" else 2,
                   r["lower_barrier"] is not None,
                   r["upper_barrier"] is not None)
        mon = np.asarray(sorted(k for k in p._monitor_indices_tau(p.time_to_expiry / 48)
                                if 1 <= k <= 48), np.int32)
    g = pack(solves, list(range(len(solves))))
    plan = capi.barrier_plan(row, flag, p.time_to_expiry, 64, 48, 1 if mode == "explicit" else 0,
                             tail_quantile(), 0.0001, False, mon)
    assert plan["n_nodes"] == g.n_nodes
    np.testing.assert_array_equal(plan["params"], g.params)
    np.testing.assert_array_equal(plan["iparams"], g.iparams)
    np.testing.assert_array_equal(plan["v_init"], g.v_init)
    np.testing.assert_array_equal(plan["mon_rebate"], g.mon_rebate)
    np.testing.assert_array_equal(np.tile(mon, len(solves)), g.mon_step)
    exp_ri = np.array([(x.slot, x.icase, x.ilo, x.idx, x.dg_mode) for x in reads], np.int32)
    exp_rd = np.array([x.dbl for x in reads], np.float64)
    np.testing.assert_array_equal(plan["rint"], exp_ri)
    np.testing.assert_array_equal(plan["rdbl"], exp_rd)
    np.testing.assert_array_equal(plan["tparams"], np.array(tpar))


def test_plan_rejects_small_capacity_and_bad_args():
    row = np.zeros((1, capi.BP_NROW))
    row[0, :3] = (100.0, 100.0, 0.2)
    flag = np.zeros((1, capi.BP_NFLAG), np.int32)
    flag[0, 1] = 1
    L = capi.lib()
    out = [np.zeros(64) for _ in range(7)]
    nn = np.zeros(1, np.int32)
    ptrs = [o.ctypes.data for o in out]
    rc = L.fdcn_barrier_plan(1, row.ctypes.data, flag.ctypes.data, 0.1, 100, 40, 1, 50, 3.0,
                             1e-4, 1, 0, None, *ptrs, nn.ctypes.data)
    assert rc != 0 and "n_nodes_cap" in capi.lib().fdcn_last_error().decode()
    rc = L.fdcn_barrier_plan(1, row.ctypes.data, flag.ctypes.data, 0.1, 100, 0, 1, 200, 3.0,
                             1e-4, 1, 0, None, *ptrs, nn.ctypes.data)
    assert rc != 0


def test_vmath_matches_python_math():
    rng = np.random.default_rng(0)
    x = rng.uniform(-30, 30, 20000)
    y = np.abs(x) + 1e-3
    assert all(a == math.exp(b) for a, b in zip(capi.vmath(capi.VM_EXP, x), x))
    assert all(a == math.log(b) for a, b in zip(capi.vmath(capi.VM_LOG, y), y))
    assert all(a == math.sqrt(b) for a, b in zip(capi.vmath(capi.VM_SQRT, y), y))
    assert all(a == b ** 2 for a, b in zip(capi.vmath(capi.VM_SQUARE, x), x))


def test_grids_that_differ_fall_back_to_the_per_row_path(monkeypatch):
    """A plan whose rows' grids differ in size (the plan builder's "differ"
    error) makes price_columns decline (None), so run_all_scenarios takes the
    per-row facades; other plan errors propagate."""
    base = scenarios.runner_base_params("put", 40)
    base.update(num_time_steps=40, grid_mode="parity")
    rows = _rows(6, 5)
    cols = scenario_batch.rows_to_columns(rows)

    def differ(*a, **k):
        raise capi.FdcnError("fdcn_barrier_plan: grid sizes differ across rows")
    monkeypatch.setattr(scenario_batch.capi, "barrier_plan", differ)
    assert scenario_batch.price_columns(cols, base, oracle_engine()) is None
    assert scenario_batch.run_rows_vectorized(rows, base, oracle_engine()) is None

    def broken(*a, **k):
        raise capi.FdcnError("fdcn_barrier_plan: NULL argument")
    monkeypatch.setattr(scenario_batch.capi, "barrier_plan", broken)
    with pytest.raises(capi.FdcnError):
        scenario_batch.price_columns(cols, base, oracle_engine())
