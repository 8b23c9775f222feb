"""Scenario batch runners: drop-ins for run_config_scenarios.py and
run_american_scenarios.py.

``run_scenario`` / ``run_american_scenario`` keep the reference signatures and
result dictionaries (run_config_scenarios.py:9-132,
run_american_scenarios.py:46-206).  ``run_all_scenarios`` /
``run_all_american_scenarios`` read the same configuration CSVs and write the
same result schema, but instead of pricing rows one after another
(run_config_scenarios.py:158) they build every trade first and march all of
their grids together: one kernel launch per grid shape for the whole file.

With ``world_size > 1`` (torch.distributed initialised) the rows are split
into contiguous blocks, one per rank, and rank 0 gathers the result rows --
the only collective in the path (see distributed.py).
"""
from __future__ import annotations

import datetime as dt
import math
from typing import Any, Dict, List, Optional

import numpy as np

from . import market
from .american import AmericanFDMPricer, prefetch_many
from .barrier import DiscreteBarrierFDMPricer, price_many
from .engine import Engine

_CURVES: Dict[float, Any] = {}


def _flat_curve(rate: float):
    """ISO-dated flat NACA curve (utils.create_rate_df + the runners' date
    conversion), cached per rate."""
    c = _CURVES.get(rate)
    if c is None:
        c = market.iso_curve(market.create_rate_df(rate))
        _CURVES[rate] = c
    return c


def _pct_diff(model_val: float, fa_val: Optional[float]) -> float:
    if fa_val is None or np.isnan(fa_val) or fa_val == 0.0:
        return np.nan
    return abs(model_val - fa_val) / abs(fa_val) * 100.0


def _result_row(scenario_name, S0, K, sigma, rate, extra: Dict[str, Any], model_price, greeks,
                FA_price, FA_delta, FA_gamma, FA_vega) -> Dict[str, Any]:
    row = {"scenario_name": scenario_name, "S0": S0, "K": K, "sigma": sigma, "rate": rate}
    row.update(extra)

    def pair(name, model, fa):
        row[f"model_{name}"] = model
        row[f"FA_{name}"] = fa if fa is not None else np.nan
        row[f"{name}_diff"] = abs(model - fa) if fa is not None else np.nan
        row[f"{name}_pct_diff"] = _pct_diff(model, fa)

    pair("price", model_price, FA_price)
    pair("delta", greeks["delta"], FA_delta)
    pair("gamma", greeks["gamma"], FA_gamma)
    pair("vega", greeks["vega"], FA_vega)
    return row


# ---------------------------------------------------------------------------
# discrete barrier
# ---------------------------------------------------------------------------
def make_barrier_pricer(S0, K, sigma, rate, barrier_type, upper_barrier, lower_barrier,
                        valuation: dt.date, maturity: dt.date, monitor_dates: list,
                        opt_type: str = "call", trade_number: int = 201871103,
                        quantity: int = 1000, contract_size: int = 1, position: str = "long",
                        divs: list = None, rebate_amount: float = 0,
                        rebate_at_hit: bool = True,
                        use_one_sided_greeks_near_barrier: bool = False,
                        already_hit: bool = False, already_in: bool = False,
                        underlying_spot_days: int = 0, option_days: int = 0,
                        option_settlement_days: int = 0, day_count: str = "ACT/365",
                        grid_type: str = "uniform", num_space_nodes: int = 500,
                        num_time_steps: int = 500, grid_mode: str = "parity",
                        engine: Optional[Engine] = None) -> DiscreteBarrierFDMPricer:
    """The pricer run_scenario builds (run_config_scenarios.py:60-94)."""
    curve = _flat_curve(rate)
    return DiscreteBarrierFDMPricer(
        spot=S0, strike=K, valuation_date=valuation, maturity_date=maturity, sigma=sigma,
        option_type=opt_type, barrier_type=barrier_type, lower_barrier=lower_barrier,
        upper_barrier=upper_barrier, already_in=already_in, already_hit=already_hit,
        monitor_dates=monitor_dates, discount_curve=curve, forward_curve=curve,
        dividend_schedule=divs or [], trade_id=trade_number, direction=position,
        quantity=quantity, underlying_spot_days=underlying_spot_days, option_days=option_days,
        option_settlement_days=option_settlement_days, rebate_amount=rebate_amount,
        rebate_at_hit=rebate_at_hit, contract_multiplier=contract_size,
        use_one_sided_greeks_near_barrier=use_one_sided_greeks_near_barrier,
        num_space_nodes=num_space_nodes, num_time_steps=num_time_steps, grid_type=grid_type,
        rannacher_steps=2, restart_on_monitoring=False, mollify_final=False,
        mollify_band_nodes=2, day_count=day_count, engine=engine, grid_mode=grid_mode)


def run_scenario(scenario_name: str, S0: float, K: float, sigma: float, rate: float,
                 barrier_type: str, upper_barrier: Optional[float],
                 lower_barrier: Optional[float], FA_price: Optional[float],
                 FA_delta: Optional[float], FA_gamma: Optional[float],
                 FA_vega: Optional[float], valuation: dt.date, maturity: dt.date,
                 monitor_dates: list, engine: Optional[Engine] = None,
                 **base) -> Dict[str, Any]:
    """One barrier scenario -> headline results (run_config_scenarios.py:9-132)."""
    p = make_barrier_pricer(S0, K, sigma, rate, barrier_type, upper_barrier, lower_barrier,
                            valuation, maturity, monitor_dates, engine=engine, **base)
    return _barrier_row(scenario_name, S0, K, sigma, rate, barrier_type, upper_barrier,
                        lower_barrier, p, FA_price, FA_delta, FA_gamma, FA_vega)


def _barrier_row(name, S0, K, sigma, rate, barrier_type, upper_barrier, lower_barrier, p,
                 FA_price, FA_delta, FA_gamma, FA_vega):
    model_price = p.price_log2()
    greeks = p.greeks_log2()
    extra = {"barrier_type": barrier_type,
             "upper_barrier": upper_barrier if upper_barrier is not None else np.nan,
             "lower_barrier": lower_barrier if lower_barrier is not None else np.nan}
    return _result_row(name, S0, K, sigma, rate, extra, model_price, greeks, FA_price,
                       FA_delta, FA_gamma, FA_vega)


def _opt(row, key):
    import pandas as pd
    v = row[key] if key in row else None
    return None if v is None or pd.isna(v) else v


def run_rows(rows: List[dict], base_params: Dict[str, Any],
             engine: Optional[Engine] = None) -> List[Dict[str, Any]]:
    """Price a list of scenario rows with all their grids in shared launches."""
    pricers = []
    for row in rows:
        pricers.append(make_barrier_pricer(row["S0"], row["K"], row["sigma"], row["rate"],
                                           row["barrier_type"], _opt(row, "upper_barrier"),
                                           _opt(row, "lower_barrier"), engine=engine,
                                           **base_params))
    price_many(pricers)
    out = []
    for row, p in zip(rows, pricers):
        out.append(_barrier_row(row["scenario_name"], row["S0"], row["K"], row["sigma"],
                                row["rate"], row["barrier_type"], _opt(row, "upper_barrier"),
                                _opt(row, "lower_barrier"), p, _opt(row, "FA_price"),
                                _opt(row, "FA_delta"), _opt(row, "FA_gamma"),
                                _opt(row, "FA_vega")))
    return out


def run_rows_batched(rows: List[dict], base_params: Dict[str, Any],
                     engine: Optional[Engine] = None,
                     dv_sigma: float = 0.0001) -> List[Dict[str, Any]]:
    """run_rows with one pricer per curve instead of one per row.

    Every row of a scenario file shares the dates, monitoring calendar, lags
    and numerics; only spot, strike, vol, rate and the barrier differ.  One
    pricer per distinct rate is re-pointed at each row
    (DiscreteBarrierFDMPricer._reset_trade) and the same methods as the
    per-row path build the solves, finish the Greeks and price the
    knock-in legs, so the results are identical to run_rows (tested); all
    rows' solves go into one engine.run."""
    from .barrier import KI_TO_KO, price_many  # noqa: F401  (same KO mapping)
    calcs: Dict[float, DiscreteBarrierFDMPricer] = {}

    def pricer_for(row) -> DiscreteBarrierFDMPricer:
        rate = row["rate"]
        p = calcs.get(rate)
        if p is None:
            p = make_barrier_pricer(row["S0"], row["K"], row["sigma"], rate, row["barrier_type"],
                                    _opt(row, "upper_barrier"), _opt(row, "lower_barrier"),
                                    engine=engine, **base_params)
            calcs[rate] = p
        p._reset_trade(row["S0"], row["K"], row["sigma"], row["barrier_type"],
                       _opt(row, "lower_barrier"), _opt(row, "upper_barrier"))
        return p

    plan, solves, specs = [], [], []
    for row in rows:
        p = pricer_for(row)
        bt = p.barrier_type.lower()
        kbt = None
        if bt in ("down-and-out", "up-and-out") and not p.already_hit:
            kbt = bt
        elif bt in ("down-and-in", "up-and-in") and not p.already_in:
            kbt = KI_TO_KO[bt]
        if kbt is None:
            plan.append((row, None, None, None, 0))
            continue
        p.barrier_type = kbt
        (sb, gb), (su, gu) = p.pde_solves(True, dv_sigma)
        specs.append(p._device_spec(sb, gb, su, gu, dv_sigma))
        plan.append((row, kbt, gb, gu, len(solves)))
        solves.extend([sb, su])
    eng = engine if engine is not None else (
        next(iter(calcs.values()))._engine() if calcs else None)
    dev = None
    if solves and eng.on_device:  # value vectors stay in HBM; 6 numbers per trade come back
        from .barrier import finish_on_device
        dev = iter(finish_on_device(eng, specs))
    res = eng.run(solves) if solves and dev is None else []
    out = []
    for row, kbt, gb, gu, i in plan:
        p = pricer_for(row)
        if kbt is not None:
            keep = p.barrier_type
            p.barrier_type = kbt
            p._pde_cache[p._pde_key(True, dv_sigma)] = (
                next(dev) if dev is not None else
                p._pde_finish(res[i], gb, res[i + 1], gu, dv_sigma))
            p.barrier_type = keep
        out.append(_barrier_row(row["scenario_name"], row["S0"], row["K"], row["sigma"],
                                row["rate"], row["barrier_type"], _opt(row, "upper_barrier"),
                                _opt(row, "lower_barrier"), p, _opt(row, "FA_price"),
                                _opt(row, "FA_delta"), _opt(row, "FA_gamma"),
                                _opt(row, "FA_vega")))
    return out


def run_all_scenarios(config_csv_path: str, output_csv_path: Optional[str],
                      base_params: Dict[str, Any], engine: Optional[Engine] = None,
                      verbose: bool = True):
    """Read the configuration CSV, price every row, write the results CSV
    (run_config_scenarios.py:137-195).

    One path at every world size: this rank's contiguous block of rows
    (all of them without torch.distributed) goes through one native plan
    build, one launch and the device epilogue (scenario_batch.price_columns);
    with torch.distributed initialised -- world size 1 included -- rank 0
    then gathers the result columns (the only collective)."""
    import pandas as pd
    from . import distributed
    from . import scenario_batch
    cfg = pd.read_csv(config_csv_path)
    sharded = distributed.is_initialized()
    if sharded:
        distributed.bind_device()  # this rank's GPU, before any launch
    mine = distributed.shard_range(len(cfg))
    part = cfg.iloc[mine.start:mine.stop]
    # the columns as NumPy arrays: the whole-file path converts nothing per row
    cols = {k: part[k].to_numpy() for k in scenario_batch.ROW_KEYS if k in part.columns}
    priced = scenario_batch.price_columns(cols, base_params, engine)
    if priced is not None:
        out = scenario_batch.result_columns(cols, priced)
    else:  # shapes the whole-file plan declines: the per-row facades, batched
        rows = run_rows_batched([dict(r) for _, r in part.iterrows()], base_params, engine)
        out = scenario_batch.rows_as_result_columns(rows)
    if sharded:
        out = distributed.gather_columns(out)
        if out is None:  # non-zero rank
            return None
    df = pd.DataFrame(out)
    res = df.to_dict("records") if verbose else None
    return _finish_scenarios(df, res, output_csv_path, verbose)


def _finish_scenarios(df, res, output_csv_path, verbose):
    if verbose:
        for r in res:
            print(f"{r['scenario_name']}: Price %Diff: {r['price_pct_diff']:.4f}%, "
                  f"Delta %Diff: {r['delta_pct_diff']:.4f}%, "
                  f"Gamma %Diff: {r['gamma_pct_diff']:.4f}%, "
                  f"Vega %Diff: {r['vega_pct_diff']:.4f}%")
    if output_csv_path:
        df.to_csv(output_csv_path, index=False)
    return df


# ---------------------------------------------------------------------------
# American
# ---------------------------------------------------------------------------
def make_american_pricer(S0, K, sigma, rate, valuation: dt.date, maturity: dt.date,
                         opt_type: str = "call", trade_number: int = 201871103,
                         quantity: int = 1000, contract_size: int = 1, position: str = "long",
                         divs: Optional[list] = None, underlying_spot_days: int = 0,
                         option_days: int = 0, option_settlement_days: int = 0,
                         day_count: str = "ACT/365", grid_type: str = "uniform",
                         num_space_nodes: int = 500, num_time_steps: int = 500,
                         rannacher_steps: int = 2,
                         engine: Optional[Engine] = None) -> AmericanFDMPricer:
    """The pricer run_american_scenario builds (run_american_scenarios.py:145-167).

    The reference parses the forward curve's dates with "%Y/%m/%m"
    (run_american_scenarios.py:141), which raises in pandas; the intended
    "%Y/%m/%d" is used here."""
    curve = _flat_curve(rate)
    return AmericanFDMPricer(spot=S0, strike=K, valuation_date=valuation, maturity_date=maturity,
                             sigma=sigma, option_type=opt_type, discount_curve=curve,
                             forward_curve=curve, dividend_schedule=divs or [],
                             trade_id=trade_number, direction=position, quantity=quantity,
                             contract_multiplier=contract_size,
                             underlying_spot_days=underlying_spot_days, option_days=option_days,
                             option_settlement_days=option_settlement_days,
                             day_count=day_count, grid_type=grid_type,
                             num_space_nodes=num_space_nodes, num_time_steps=num_time_steps,
                             rannacher_steps=rannacher_steps, engine=engine)


def run_american_scenario(scenario_name: str, S0: float, K: float, sigma: float, rate: float,
                          FA_price: Optional[float], FA_delta: Optional[float],
                          FA_gamma: Optional[float], FA_vega: Optional[float],
                          valuation: dt.date, maturity: dt.date,
                          engine: Optional[Engine] = None, **base) -> Dict[str, Any]:
    """One American scenario (run_american_scenarios.py:46-206)."""
    p = make_american_pricer(S0, K, sigma, rate, valuation, maturity, engine=engine, **base)
    prefetch_many([p])
    return _result_row(scenario_name, S0, K, sigma, rate, {}, p.price_log2(), p.greeks_log2(),
                       FA_price, FA_delta, FA_gamma, FA_vega)


def run_all_american_scenarios(config_csv_path: str, output_csv_path: Optional[str],
                               base_params: Dict[str, Any], engine: Optional[Engine] = None,
                               verbose: bool = True):
    """run_american_scenarios.py:209-277 with every grid of the file batched."""
    import pandas as pd
    from . import distributed
    from . import american_batch
    cfg = pd.read_csv(config_csv_path)
    if distributed.is_initialized():
        distributed.bind_device()
    rows = distributed.shard([dict(r) for _, r in cfg.iterrows()])
    # the whole shard in one plan build, lock-step launches and one epilogue
    # (american_batch.py); the per-row façades when it declines
    res = american_batch.run_rows_vectorized(rows, base_params, engine)
    if res is None:
        pricers = [make_american_pricer(r["S0"], r["K"], r["sigma"], r["rate"], engine=engine,
                                        **base_params) for r in rows]
        prefetch_many(pricers)
        res = [_result_row(r["scenario_name"], r["S0"], r["K"], r["sigma"], r["rate"], {},
                           p.price_log2(), p.greeks_log2(), _opt(r, "FA_price"),
                           _opt(r, "FA_delta"), _opt(r, "FA_gamma"), _opt(r, "FA_vega"))
               for r, p in zip(rows, pricers)]
    res = distributed.gather_rows(res)
    if res is None:
        return None
    df = pd.DataFrame(res)
    if verbose:
        for r in res:
            print(f"{r['scenario_name']}: Price %Diff: {r['price_pct_diff']:.4f}%")
    if output_csv_path:
        df.to_csv(output_csv_path, index=False)
    return df


# the monitoring calendar of run_config_scenarios.py:204-229
RUNNER_MONITOR_DATES = [dt.date(2025, 7, 28), dt.date(2025, 7, 29), dt.date(2025, 7, 30),
                        dt.date(2025, 7, 31), dt.date(2025, 8, 1), dt.date(2025, 8, 4),
                        dt.date(2025, 8, 5), dt.date(2025, 8, 6), dt.date(2025, 8, 7),
                        dt.date(2025, 8, 8), dt.date(2025, 8, 11), dt.date(2025, 8, 12),
                        dt.date(2025, 8, 13), dt.date(2025, 8, 14), dt.date(2025, 8, 15),
                        dt.date(2025, 8, 18), dt.date(2025, 8, 19), dt.date(2025, 8, 20),
                        dt.date(2025, 8, 21), dt.date(2025, 8, 22), dt.date(2025, 8, 25),
                        dt.date(2025, 8, 26), dt.date(2025, 8, 27), dt.date(2025, 8, 28)]


def runner_base_params(opt_type: str = "put", n: int = 500) -> Dict[str, Any]:
    """base_params of run_config_scenarios.py:235-257."""
    return {"valuation": dt.date(2025, 7, 28), "maturity": dt.date(2025, 8, 28),
            "monitor_dates": RUNNER_MONITOR_DATES, "opt_type": opt_type,
            "trade_number": 201871100, "quantity": 1000, "contract_size": 1,
            "position": "long", "divs": [], "rebate_amount": 0, "rebate_at_hit": True,
            "use_one_sided_greeks_near_barrier": False, "already_hit": False,
            "already_in": False, "underlying_spot_days": 0, "option_days": 0,
            "option_settlement_days": 0, "day_count": "ACT/365", "grid_type": "uniform",
            "num_space_nodes": n, "num_time_steps": n}
