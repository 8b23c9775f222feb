"""Generate golden vectors for the CN hot path from the reference code.

THIS SCRIPT RUNS ONLY IN THE BUILD CONTAINER, where the reference is mounted
read-only at /root/reference.  Nothing on the GPU box (tests, smoke(),
bench.py) runs it or reads /root/reference; they read the JSON fixtures it
wrote next to itself.

How the reference is loaded (see DESIGN.md "Oracle pinning"):

* ``discrete_barrier_fdm_pricer_cn.py``: the file does not import as shipped
  (NameError at line 639, IndentationError at 795).  Its longest executable
  prefix, lines 1-637, defines ``DiscreteBarrierCrankNicolsonLog`` and only
  needs the standard library.
* ``discrete_barrier_fdm_pricer.py``: does not import as shipped
  (IndentationError at line 749; the constructor calls the missing
  ``_build_stock_price_grid`` at line 167).  Lines 1-745 + 883-1084 are
  executed, and ``_build_stock_price_grid`` is given a stand-in returning
  ``[0.0, 1.0]``: its value only feeds the unused ``grid_spacing``.  This
  rebuild reproduces the committed ``scenario_results*.csv`` (checked in
  ``tests/test_oracle_golden.py`` through the oracle).
* ``fd_american_equity.py`` and ``discrete_barrier_fdm_pricer.py`` import
  ``workalendar.africa.SouthAfrica``, which is not installed.  A stub whose
  ``add_working_days(d, n)`` returns ``d`` for ``n == 0`` and raises otherwise
  is injected; every fixture below uses zero business-day lags, as the
  reference runners do (run_config_scenarios.py:250-252).

Usage:  python tests/golden/make_golden.py   (writes tests/golden/*.json)
"""
from __future__ import annotations

import datetime as dt
import json
import math
import os
import shutil
import sys
import time
import types

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# reference loaders
# --------------------------------------------------------------------------
def _install_workalendar_stub() -> None:
    class SouthAfrica:  # noqa: D401 - stub
        def add_working_days(self, d, n):
            if n != 0:
                raise NotImplementedError("stub only supports zero-day lags")
            return d

    pkg = types.ModuleType("workalendar")
    sub = types.ModuleType("workalendar.africa")
    sub.SouthAfrica = SouthAfrica
    pkg.africa = sub
    sys.modules["workalendar"] = pkg
    sys.modules["workalendar.africa"] = sub


def _exec_lines(fname: str, ranges, modname: str):
    lines = open(os.path.join(REF, fname)).read().splitlines()
    chunks = []
    for lo, hi in ranges:  # 1-based inclusive
        chunks.extend(lines[lo - 1:hi])
    mod = types.ModuleType(modname)
    mod.__file__ = os.path.join(REF, fname)
    sys.modules[modname] = mod  # dataclasses resolves the module during exec
    exec(compile("\n".join(chunks) + "\n", fname, "exec"), mod.__dict__)
    return mod


def load_cn_log():
    return _exec_lines("discrete_barrier_fdm_pricer_cn.py", [(1, 637)], "ref_cn_log")


def load_barrier():
    _install_workalendar_stub()
    mod = _exec_lines("discrete_barrier_fdm_pricer.py", [(1, 745), (883, 1084)],
                      "discrete_barrier_fdm_pricer")
    mod.DiscreteBarrierFDMPricer._build_stock_price_grid = lambda self: [0.0, 1.0]
    return mod


def load_american():
    _install_workalendar_stub()
    sys.path.insert(0, REF)
    import fd_american_equity  # type: ignore
    return fd_american_equity


def load_utils():
    sys.path.insert(0, REF)
    import utils  # type: ignore
    return utils


def load_barrier_engine():
    sys.path.insert(0, REF)
    import barrier_engine  # type: ignore
    return barrier_engine


def load_double_barrier():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_double_barrier",
                                                  os.path.join(REF, "double _barrier.py"))
    mod = importlib.util.module_from_spec(spec)
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        spec.loader.exec_module(mod)  # the module prints its own example
    return mod


# --------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------
VAL = dt.date(2025, 7, 28)
MAT = dt.date(2025, 8, 28)
DAILY = [dt.date(2025, 7, 28) + dt.timedelta(days=i) for i in range(32)]
DAILY = [d for d in DAILY if d.weekday() < 5 or d == MAT]
# the exact list used by run_config_scenarios.py:204-229
RUNNER_MONITORS = [dt.date(2025, 7, 28), dt.date(2025, 7, 29), dt.date(2025, 7, 30),
                   dt.date(2025, 7, 31), dt.date(2025, 8, 1), dt.date(2025, 8, 4),
                   dt.date(2025, 8, 5), dt.date(2025, 8, 6), dt.date(2025, 8, 7),
                   dt.date(2025, 8, 8), dt.date(2025, 8, 11), dt.date(2025, 8, 12),
                   dt.date(2025, 8, 13), dt.date(2025, 8, 14), dt.date(2025, 8, 15),
                   dt.date(2025, 8, 18), dt.date(2025, 8, 19), dt.date(2025, 8, 20),
                   dt.date(2025, 8, 21), dt.date(2025, 8, 22), dt.date(2025, 8, 25),
                   dt.date(2025, 8, 26), dt.date(2025, 8, 27), dt.date(2025, 8, 28)]


def iso(d):
    return d.isoformat()


def curve(rate):
    utils = load_utils()
    import pandas as pd
    c = utils.create_rate_df(rate)
    c["Date"] = pd.to_datetime(c["Date"], format="%Y/%m/%d").dt.strftime("%Y-%m-%d")
    return c


def dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    print("wrote", path)


# --------------------------------------------------------------------------
# 1. CN-log class (config 1 and variants)
# --------------------------------------------------------------------------
def gen_cn_log():
    m = load_cn_log()
    C = m.DiscreteBarrierCrankNicolsonLog
    T = 31 / 365
    mon_days = [7, 10, 15, 21, 25, 30, 31]  # Aug 4,7,12,18,22,27,28 from Jul 28
    cases = []
    specs = [
        dict(name="config1_call_uo", S0=229.74, K=220.0, sigma=0.261319016, r=0.070538822,
             b=0.070538822, opt="call", bt="up-and-out", lo=None, up=270.0, rebate=0.0,
             N=512, M=1000),
        dict(name="put_do_rebate", S0=229.74, K=240.0, sigma=0.30, r=0.07, b=0.05,
             opt="put", bt="down-and-out", lo=205.0, up=None, rebate=1.25, N=128, M=200),
        dict(name="call_do", S0=100.0, K=95.0, sigma=0.22, r=0.05, b=0.03,
             opt="call", bt="down-and-out", lo=90.0, up=None, rebate=0.0, N=96, M=150),
        dict(name="put_ui", S0=229.74, K=230.0, sigma=0.25, r=0.07, b=0.07,
             opt="put", bt="up-and-in", lo=None, up=250.0, rebate=0.0, N=128, M=128),
        dict(name="call_auto_grid", S0=229.74, K=225.0, sigma=0.28, r=0.07, b=0.065,
             opt="call", bt="up-and-out", lo=None, up=260.0, rebate=0.0, N=None, M=None),
    ]
    for s in specs:
        mon = [d / 365 for d in mon_days]
        p = C(S0=s["S0"], K=s["K"], T=T, sigma=s["sigma"], r_disc=s["r"], b_carry=s["b"],
              option_type=s["opt"], barrier_type=s["bt"], lower_barrier=s["lo"],
              upper_barrier=s["up"], rebate=s["rebate"], monitor_times=mon,
              N_space=s["N"], N_time=s["M"])
        rec = dict(inputs=dict(s, T=T, monitor_times=mon))
        t0 = time.time()
        rec["price"] = p.price()
        rec["price_seconds"] = time.time() - t0
        p.configure_grid()
        rec["N_space"], rec["N_time"] = p.N_space, p.N_time
        rec["S_min"], rec["S_max"] = p._S_min, p._S_max
        dt_ = T / p.N_time
        rec["monitor_idx"] = sorted(p._monitor_indices_tau(dt_))
        try:
            rec["greeks"] = p.greeks()
        except Exception as e:  # the shipped greeks() needs a method the prefix lacks
            rec["greeks_error"] = type(e).__name__
        if s["bt"].endswith("out"):
            rec["V_ko"] = p._solve_grid(apply_KO=True)
        rec["V_noko"] = p._solve_grid(apply_KO=False)
        cases.append(rec)
    dump("cn_log_cases.json", cases)


# --------------------------------------------------------------------------
# 2. production barrier engine
# --------------------------------------------------------------------------
def make_barrier(m, **kw):
    base = dict(valuation_date=VAL, maturity_date=MAT, monitor_dates=RUNNER_MONITORS,
                rebate_amount=0.0, rebate_at_hit=True, already_hit=False, already_in=False,
                underlying_spot_days=0, option_days=0, option_settlement_days=0,
                dividend_schedule=[], rannacher_steps=2, restart_on_monitoring=False,
                mollify_final=False, mollify_band_nodes=2, day_count="ACT/365",
                grid_type="uniform", use_one_sided_greeks_near_barrier=False,
                num_space_nodes=500)
    rate = kw.pop("rate")
    base["discount_curve"] = curve(rate)
    base["forward_curve"] = curve(rate)
    base.update(kw)
    return m.DiscreteBarrierFDMPricer(**base)


def gen_barrier():
    m = load_barrier()
    out = dict(ns_for_nt={}, cases=[])
    # H1: N_s override for several N_t (depends only on N_t, checked on one trade)
    for nt in (8, 40, 50, 100, 500, 1000, 2000, 4096, 8192):
        p = make_barrier(m, spot=229.74, strike=190.0, sigma=0.287899982, option_type="put",
                         barrier_type="up-and-out", upper_barrier=260.0, rate=0.073086,
                         num_time_steps=nt)
        p._build_log_grid()
        out["ns_for_nt"][str(nt)] = dict(N_s=p.num_space_nodes, S_min=p._S_min,
                                         S_max=p._S_max,
                                         monitor_idx=sorted(p._monitor_indices_tau(
                                             p.time_to_expiry / nt)))
    specs = [
        dict(name="put_uo", spot=229.74, strike=190.0, sigma=0.287899982, option_type="put",
             barrier_type="up-and-out", upper_barrier=260.0, rate=0.073086, num_time_steps=40),
        dict(name="put_do", spot=229.74, strike=190.0, sigma=0.287899982, option_type="put",
             barrier_type="down-and-out", lower_barrier=200.0, rate=0.073086, num_time_steps=40),
        dict(name="call_uo_rebate_expiry", spot=229.74, strike=220.0, sigma=0.25,
             option_type="call", barrier_type="up-and-out", upper_barrier=250.0, rate=0.07,
             rebate_amount=2.0, rebate_at_hit=False, num_time_steps=40),
        dict(name="call_do_rebate_hit", spot=229.74, strike=220.0, sigma=0.25,
             option_type="call", barrier_type="down-and-out", lower_barrier=215.0, rate=0.07,
             rebate_amount=1.5, rebate_at_hit=True, num_time_steps=60),
        dict(name="call_ui", spot=229.74, strike=240.0, sigma=0.3, option_type="call",
             barrier_type="up-and-in", upper_barrier=245.0, rate=0.07, num_time_steps=50),
        dict(name="put_di", spot=229.74, strike=250.0, sigma=0.24, option_type="put",
             barrier_type="down-and-in", lower_barrier=210.0, rate=0.073086, num_time_steps=50),
        dict(name="call_do_divs", spot=229.74, strike=225.0, sigma=0.27, option_type="call",
             barrier_type="down-and-out", lower_barrier=205.0, rate=0.072,
             dividend_schedule=[(dt.date(2025, 8, 12), 2.5)], num_time_steps=45),
        dict(name="put_uo_n500", spot=229.74, strike=260.0, sigma=0.234882165755,
             option_type="put", barrier_type="up-and-out", upper_barrier=280.0,
             rate=0.073085649282, num_time_steps=500),
    ]
    for s in specs:
        kw = dict(s)
        name = kw.pop("name")
        p = make_barrier(m, **kw)
        rec = dict(name=name, inputs={k: (v if not isinstance(v, list) else
                                         [[iso(a), b] for a, b in v]) for k, v in s.items()})
        t0 = time.time()
        rec["price_log2"] = p.price_log2()
        rec["greeks_log2"] = p.greeks_log2()
        rec["seconds"] = time.time() - t0
        rec["attrs"] = dict(time_to_expiry=p.time_to_expiry, time_to_carry=p.time_to_carry,
                            time_to_discount=p.time_to_discount,
                            discount_rate_nacc=p.discount_rate_nacc,
                            carry_rate_nacc=p.carry_rate_nacc, div_yield_nacc=p.div_yield_nacc,
                            pv_divs=p.pv_divs, b=p.b, monitor_times=p.monitor_times)
        bt = p.barrier_type
        if bt.endswith("-in"):
            p.barrier_type = bt.replace("-in", "-out")
        rec["V_ko"] = p._solve_grid(apply_KO=True)
        rec["V_noko"] = p._solve_grid(apply_KO=False)
        rec["N_s"] = p.num_space_nodes
        rec["S_min"], rec["S_max"] = p._S_min, p._S_max
        rec["dx"] = p._build_log_grid()
        rec["s_nodes"] = p.s_nodes
        rec["monitor_idx"] = sorted(p._monitor_indices_tau(p.time_to_expiry /
                                                           p.num_time_steps))
        p.barrier_type = bt
        rec["vanilla_price"] = p._vanilla_black76_price()
        rec["vanilla_greeks"] = p._vanilla_black76_greeks_fd()
        out["cases"].append(rec)
    dump("barrier_cases.json", out)

    # the committed golden CSVs are reference data files: copy them verbatim
    dst = os.path.join(HERE, "ref_csv")
    os.makedirs(dst, exist_ok=True)
    for f in ("config_scenarios.csv", "config_scenarios 1.csv", "scenario_results.csv",
              "scenario_results_1.csv"):
        shutil.copy(os.path.join(REF, f), os.path.join(dst, f.replace(" ", "_space_")))


def gen_double_out():
    """The production engine's "double-out" branch (discrete_barrier_fdm_pricer.py
    :435-437).  price_log2 raises for double-* (:946), so the fixtures pin the
    march itself: _solve_grid(apply_KO=True) with both barriers, put and call,
    with and without a rebate (paid at hit / discounted), parity-mode grids."""
    m = load_barrier()
    specs = [
        dict(name="dko_call", spot=229.74, strike=220.0, sigma=0.25, option_type="call",
             lower_barrier=205.0, upper_barrier=250.0, rate=0.07, num_time_steps=40),
        dict(name="dko_put", spot=229.74, strike=235.0, sigma=0.30, option_type="put",
             lower_barrier=210.0, upper_barrier=255.0, rate=0.073086, num_time_steps=50),
        dict(name="dko_call_rebate_hit", spot=229.74, strike=225.0, sigma=0.28,
             option_type="call", lower_barrier=200.0, upper_barrier=260.0, rate=0.07,
             rebate_amount=1.5, rebate_at_hit=True, num_time_steps=45),
        dict(name="dko_put_rebate_expiry", spot=229.74, strike=240.0, sigma=0.22,
             option_type="put", lower_barrier=215.0, upper_barrier=245.0, rate=0.072,
             rebate_amount=2.0, rebate_at_hit=False, num_time_steps=60),
    ]
    cases = []
    for sp in specs:
        kw = dict(sp)
        name = kw.pop("name")
        p = make_barrier(m, barrier_type="double-out", **kw)
        rec = dict(name=name, inputs=dict(sp))
        rec["V_ko"] = p._solve_grid(apply_KO=True)
        rec["N_s"] = p.num_space_nodes
        rec["S_min"], rec["S_max"] = p._S_min, p._S_max
        rec["dx"] = p._build_log_grid()
        rec["s_nodes"] = p.s_nodes
        rec["monitor_idx"] = sorted(p._monitor_indices_tau(p.time_to_expiry /
                                                           p.num_time_steps))
        rec["attrs"] = dict(time_to_expiry=p.time_to_expiry,
                            discount_rate_nacc=p.discount_rate_nacc,
                            carry_rate_nacc=p.carry_rate_nacc, div_yield_nacc=p.div_yield_nacc)
        try:
            p.price_log2()
            rec["price_log2_raises"] = None
        except Exception as e:  # the reference refuses double-* here (:946)
            rec["price_log2_raises"] = type(e).__name__
        cases.append(rec)
    dump("double_out_cases.json", dict(cases=cases))


def gen_spot():
    """DiscreteBarrierFDMPricer2 (discrete_barrier_fdm_pricer_2.py): the
    spot-space CN with per-row coefficients, the FIS barrier rows and the BGK
    window.  Its explicit off-diagonals have the wrong sign (:383-385), so the
    prices grow without bound with M; at the small step counts below they are
    still finite, and the value vectors pin the march to the reference."""
    sys.path.insert(0, REF)
    import discrete_barrier_fdm_pricer_2 as m  # type: ignore
    v0, v1 = dt.date(2025, 7, 28), dt.date(2026, 1, 28)
    daily = [v0 + dt.timedelta(days=i) for i in range(1, 40)]
    weekly = [v0 + dt.timedelta(days=7 * i) for i in range(1, 27)]
    specs = [
        dict(name="vanilla_call", spot=100.0, strike=100.0, volatility=0.25, option_type="call",
             barrier_type="none", flat_rate_nacc=0.05, num_space_nodes=200, num_time_steps=6),
        dict(name="put_do_weekly", spot=100.0, strike=105.0, volatility=0.3, option_type="put",
             barrier_type="down-and-out", lower_barrier=85.0, monitoring_dates=weekly,
             flat_rate_nacc=0.04, num_space_nodes=220, num_time_steps=8),
        dict(name="call_uo_weekly", spot=100.0, strike=95.0, volatility=0.22, option_type="call",
             barrier_type="up-and-out", upper_barrier=125.0, monitoring_dates=weekly,
             flat_rate_nacc=0.05, num_space_nodes=200, num_time_steps=5),
        dict(name="dko_bgk_window", spot=100.0, strike=100.0, volatility=0.2, option_type="call",
             barrier_type="double-out", lower_barrier=80.0, upper_barrier=130.0,
             monitoring_dates=daily, flat_rate_nacc=0.05, num_space_nodes=200, num_time_steps=3),
        dict(name="put_di_divs", spot=100.0, strike=100.0, volatility=0.25, option_type="put",
             barrier_type="down-and-in", lower_barrier=90.0, monitoring_dates=weekly,
             flat_rate_nacc=0.05, dividends=[(dt.date(2025, 10, 15), 1.5)],
             num_space_nodes=200, num_time_steps=4),
    ]
    cases = []
    for sp in specs:
        kw = dict(sp)
        name = kw.pop("name")
        p = m.DiscreteBarrierFDMPricer2(valuation_date=v0, maturity_date=v1, **kw)
        Sg, Vg, S_eff = p._solve_grid_once()
        rec = dict(name=name, inputs={k: ([[iso(a), b] for a, b in v] if k == "dividends" else
                                         ([iso(d) for d in v] if k == "monitoring_dates" else v))
                                     for k, v in sp.items()},
                   S_shifted=Sg, V=Vg, S_eff=S_eff, price=p.price(), greeks=p.greeks(),
                   use_bgk=p.use_bgk_correction, bgk=[p.bgk_lower, p.bgk_upper],
                   window=[p.k_first_cont, p.k_last_cont],
                   monitor_map=sorted(p._monitoring_step_map()), S_nodes=p.S_nodes)
        cases.append(rec)
    dump("spot_cases.json", dict(valuation=iso(v0), maturity=iso(v1), cases=cases))


# --------------------------------------------------------------------------
# 3. American engine
# --------------------------------------------------------------------------
def gen_american(with_config2: bool):
    m = load_american()
    cases = []
    specs = [
        dict(name="put_200", spot=176.39, strike=170.0, sigma=0.296783211249, option_type="put",
             naca=math.exp(0.07053828272) - 1.0, N=200, M=200, divs=[]),
        dict(name="call_200", spot=176.39, strike=170.0, sigma=0.296783211249,
             option_type="call", naca=math.exp(0.07053828272) - 1.0, N=200, M=200, divs=[]),
        dict(name="put_1div", spot=176.39, strike=180.0, sigma=0.3, option_type="put",
             naca=0.073, N=120, M=100, divs=[(dt.date(2025, 8, 10), 1.5)]),
        dict(name="call_2div", spot=176.39, strike=172.0, sigma=0.28, option_type="call",
             naca=0.073, N=120, M=90, divs=[(dt.date(2025, 8, 5), 1.0),
                                            (dt.date(2025, 8, 19), 2.0)]),
        dict(name="put_small_grid", spot=100.0, strike=105.0, sigma=0.35, option_type="put",
             naca=0.06, N=64, M=50, divs=[]),
    ]
    for s in specs:
        c = curve(s["naca"])
        p = m.AmericanFDMPricer(spot=s["spot"], strike=s["strike"], valuation_date=VAL,
                                maturity_date=MAT, sigma=s["sigma"],
                                option_type=s["option_type"], discount_curve=c,
                                forward_curve=c, dividend_schedule=s["divs"],
                                num_space_nodes=s["N"], num_time_steps=s["M"],
                                rannacher_steps=2)
        rec = dict(name=s["name"], inputs={k: (v if k != "divs" else
                                              [[iso(a), b] for a, b in v])
                                          for k, v in s.items()})
        t0 = time.time()
        rec["price_log"] = p.price_log()
        rec["V"] = p._solve_grid()
        rec["s_nodes"] = p.s_nodes
        rec["price_log2"] = p.price_log2()
        rec["greeks_log2"] = p.greeks_log2()
        rec["seconds"] = time.time() - t0
        rec["attrs"] = dict(time_to_expiry=p.time_to_expiry,
                            discount_rate_nacc=p.discount_rate_nacc,
                            carry_rate_nacc=p.carry_rate_nacc, S_min=p._S_min, S_max=p._S_max,
                            spot_snapped=p.spot_snapped, strike_snapped=p.strike_snapped,
                            dx=p._dx,
                            div_times_tau=p._div_times_tau())
        cases.append(rec)
    out = dict(cases=cases)
    if with_config2:
        c = curve(math.exp(0.07053828272) - 1.0)
        p = m.AmericanFDMPricer(spot=176.39, strike=170.0, valuation_date=VAL,
                                maturity_date=MAT, sigma=0.296783211249, option_type="put",
                                discount_curve=c, forward_curve=c, dividend_schedule=[],
                                num_space_nodes=2048, num_time_steps=4096, rannacher_steps=2)
        t0 = time.time()
        V = p._solve_grid()
        secs = time.time() - t0
        out["config2"] = dict(price_log=p._interp_price(V), seconds=secs,
                              V_sample={str(i): V[i] for i in range(0, len(V), 64)},
                              V_len=len(V))
    dump("american_cases.json", out)


def gen_black76():
    """fd_american_black76.py (AmericanFwdFDMPricer): same march, Black-76
    coefficients (mu_x = -sigma^2/2) and discounted boundaries."""
    _install_workalendar_stub()
    sys.path.insert(0, REF)
    import fd_american_black76 as m  # type: ignore
    specs = [
        dict(name="fwd_put_200", spot=176.39, strike=170.0, sigma=0.296783211249,
             option_type="put", naca=math.exp(0.07053828272) - 1.0, N=200, M=200),
        dict(name="fwd_call_160", spot=176.39, strike=170.0, sigma=0.296783211249,
             option_type="call", naca=math.exp(0.07053828272) - 1.0, N=160, M=120),
        dict(name="fwd_put_itm", spot=95.0, strike=110.0, sigma=0.4, option_type="put",
             naca=0.09, N=128, M=100),
    ]
    cases = []
    for s in specs:
        c = curve(s["naca"])
        p = m.AmericanFwdFDMPricer(spot=s["spot"], strike=s["strike"], valuation_date=VAL,
                                   maturity_date=MAT, sigma=s["sigma"],
                                   option_type=s["option_type"], discount_curve=c,
                                   forward_curve=c, num_space_nodes=s["N"],
                                   num_time_steps=s["M"], rannacher_steps=2)
        rec = dict(name=s["name"], inputs=s)
        rec["price_log"] = p.price_log()
        rec["V"] = p._solve_grid()
        rec["s_nodes"] = p.s_nodes
        rec["price_log2"] = p.price_log2()
        rec["greeks_log2"] = p.greeks_log2()
        rec["attrs"] = dict(time_to_expiry=p.time_to_expiry,
                            discount_rate_nacc=p.discount_rate_nacc, S_min=p._S_min,
                            S_max=p._S_max, spot_snapped=p.spot_snapped,
                            strike_snapped=p.strike_snapped, dx=p._dx)
        cases.append(rec)
    dump("black76_cases.json", dict(cases=cases))


# --------------------------------------------------------------------------
# 4. analytic engines
# --------------------------------------------------------------------------
def gen_analytic():
    be = load_barrier_engine()
    db = load_double_barrier()
    rows = []
    for of in ("c", "p"):
        for df in ("u", "d"):
            for io in ("i", "o"):
                for x in (90.0, 100.0, 110.0):
                    h = 115.0 if df == "u" else 88.0
                    for status in (None, "crossed"):
                        for rti, rto in ((None, None), ("hit", "expiry")):
                            e = be.BarrierEngine(s=100.0, b=0.03, r=0.05, t=0.5, x=x,
                                                 sigma=0.25, h=h, optionflag=of,
                                                 directionflag=df, in_out_flag=io, k=1.5,
                                                 barrier_status=status,
                                                 rebate_timing_in=rti, rebate_timing_out=rto)
                            rows.append(dict(args=dict(s=100.0, b=0.03, r=0.05, t=0.5, x=x,
                                                       sigma=0.25, h=h, optionflag=of,
                                                       directionflag=df, in_out_flag=io,
                                                       k=1.5, barrier_status=status,
                                                       rebate_timing_in=rti,
                                                       rebate_timing_out=rto),
                                             price=float(e.price()),
                                             vanilla=float(e.vanilla())))
    dbl = []
    for (S, X, L, U, r, b, T, sig, cf) in (
            (20.786, 21.0, 19.0, 23.0, 0.0709454892, 0.049493018, 49 / 365, 0.10994120968, "c"),
            (17.862, 19.0, 15.0, 21.0, 0.0709454892, 0.02526685, 49 / 365, 0.143176220424, "p"),
            (100.0, 100.0, 80.0, 125.0, 0.05, 0.03, 0.5, 0.2, "c"),
            (100.0, 100.0, 80.0, 125.0, 0.05, 0.03, 0.5, 0.2, "p")):
        for inout in ("in", "out"):
            p = db.DoubleBarrier(S, X, L, U, sig, cf, inout, 4)
            dbl.append(dict(args=dict(S=S, X=X, L=L, U=U, sigma=sig, callflag=cf,
                                      inflag=inout, m=4, b=b, r=r, T=T),
                            price=float(p.price(b=b, r=r, T=T)),
                            bs=float(db.DoubleBarrier._bs_price(cf, S, X, r, b, sig, T))))
    dump("analytic_cases.json", dict(barrier_engine=rows, double_barrier=dbl))


def gen_spot_analytic():
    """DiscreteBarrierFDMPricerAnalytic (discrete_barrier_analytic_pricer.py):
    the FIS n_lim decision, the BGK-shifted analytic engines on the continuous
    window (barrier_engine.BarrierEngine; DoubleBarrier), the CN overlay with
    knock-out on discrete monitoring steps or on every step of the window,
    knock-ins as CN vanilla minus the knock-out leg, bump-and-reprice Greeks.

    The module imports ``from double_barrier import DoubleBarrier``; the
    reference's file is "double _barrier.py" (a space in the name), so as
    shipped DoubleBarrier is None and the double-barrier continuous branch
    falls back to the CN overlay.  Cases marked ``douady`` bind the module's
    DoubleBarrier to "double _barrier.py" (what the import intends); the
    others run the module as shipped."""
    import pandas as pd
    sys.path.insert(0, REF)
    import discrete_barrier_analytic_pricer as m  # type: ignore
    shipped_db = m.DoubleBarrier
    assert shipped_db is None, "expected the shipped import of double_barrier to fail"
    v0, v1 = pd.Timestamp("2025-07-28"), pd.Timestamp("2026-01-28")
    daily = [v0 + pd.Timedelta(days=i) for i in range(1, 185)]
    weekly = [v0 + pd.Timedelta(days=7 * i) for i in range(1, 27)]
    monthly = [v0 + pd.Timedelta(days=30 * i) for i in range(1, 7)]
    base = dict(trade_id="T1", direction="long", quantity=1, contract_multiplier=1.0,
                valuation_date=v0, maturity_date=v1)
    specs = [
        dict(name="put_do_weekly_cn", option_type="put", barrier_type="down-and-out",
             strike=105.0, lower_barrier=85.0, upper_barrier=None, spot=100.0, volatility=0.3,
             monitoring_dates=weekly, rate=0.06, time_steps=8, space_nodes=150),
        dict(name="call_uo_monthly_cn_short", option_type="call", barrier_type="up-and-out",
             strike=95.0, lower_barrier=None, upper_barrier=125.0, spot=100.0, volatility=0.22,
             monitoring_dates=monthly, rate=0.05, time_steps=6, space_nodes=160,
             direction="short", quantity=10, contract_multiplier=2.0),
        dict(name="call_uo_daily_rr", option_type="call", barrier_type="up-and-out",
             strike=100.0, lower_barrier=None, upper_barrier=130.0, spot=100.0,
             volatility=0.25, monitoring_dates=daily, rate=0.05, time_steps=10,
             space_nodes=150, n_desired_for_decision=20, rebate_amount=1.5,
             rebate_timing_out="expiry"),
        dict(name="put_di_daily_rr", option_type="put", barrier_type="down-and-in",
             strike=100.0, lower_barrier=85.0, upper_barrier=None, spot=100.0, volatility=0.3,
             monitoring_dates=daily, rate=0.05, time_steps=8, space_nodes=140,
             n_desired_for_decision=20, divs=[("2025-10-15", 1.5)]),
        dict(name="call_ui_weekly_cn_divs", option_type="call", barrier_type="up-and-in",
             strike=98.0, lower_barrier=None, upper_barrier=120.0, spot=100.0, volatility=0.2,
             monitoring_dates=weekly, rate=0.07, time_steps=6, space_nodes=150,
             divs=[("2025-09-01", 1.0), ("2025-12-01", 1.25)]),
        dict(name="call_uo_daily_crossed_cn", option_type="call", barrier_type="up-and-out",
             strike=100.0, lower_barrier=None, upper_barrier=130.0, spot=100.0,
             volatility=0.25, monitoring_dates=daily, rate=0.05, time_steps=8, space_nodes=150,
             n_desired_for_decision=20, barrier_status="not_crossed"),
        dict(name="dko_daily_cn", option_type="call", barrier_type="double-out", strike=100.0,
             lower_barrier=80.0, upper_barrier=125.0, spot=100.0, volatility=0.2,
             monitoring_dates=daily, rate=0.05, time_steps=6, space_nodes=150,
             n_desired_for_decision=20),
        dict(name="dko_daily_douady", douady=True, option_type="call", barrier_type="double-out",
             strike=100.0, lower_barrier=80.0, upper_barrier=125.0, spot=100.0, volatility=0.2,
             monitoring_dates=daily, rate=0.05, time_steps=6, space_nodes=150,
             n_desired_for_decision=20),
        dict(name="put_dki_daily_douady", douady=True, option_type="put",
             barrier_type="double-in", strike=100.0, lower_barrier=82.0, upper_barrier=120.0,
             spot=100.0, volatility=0.2, monitoring_dates=daily, rate=0.05, time_steps=6,
             space_nodes=150, n_desired_for_decision=20),
        # greeks() with abs_vol_bump > volatility: the sigma-down repricing's
        # BarrierEngine raises and the reference falls back to the CN overlay
        # (:486-519); the Douady case likewise if DoubleBarrier raises
        dict(name="call_uo_daily_rr_vol_bump_past_zero", option_type="call",
             barrier_type="up-and-out", strike=100.0, lower_barrier=None, upper_barrier=130.0,
             spot=100.0, volatility=0.25, monitoring_dates=daily, rate=0.05, time_steps=10,
             space_nodes=150, n_desired_for_decision=20, greeks_kw=dict(abs_vol_bump=0.3)),
        dict(name="dko_daily_douady_vol_bump_past_zero", douady=True, option_type="call",
             barrier_type="double-out", strike=100.0, lower_barrier=80.0, upper_barrier=125.0,
             spot=100.0, volatility=0.2, monitoring_dates=daily, rate=0.05, time_steps=6,
             space_nodes=150, n_desired_for_decision=20, greeks_kw=dict(abs_vol_bump=0.25)),
        dict(name="vanilla_put", option_type="put", barrier_type="none", strike=100.0,
             lower_barrier=None, upper_barrier=None, spot=100.0, volatility=0.25,
             monitoring_dates=[], rate=0.05, time_steps=6, space_nodes=150,
             snap_strike_and_barrier=False),
    ]
    cases = []
    for sp in specs:
        kw = dict(base)
        kw.update({k: v for k, v in sp.items()
                   if k not in ("name", "rate", "divs", "douady", "greeks_kw")})
        c = curve(sp["rate"])
        kw["discount_curve"] = c
        kw["forward_curve"] = c
        kw["dividend_schedule"] = [(pd.Timestamp(d), a) for d, a in sp.get("divs", [])]
        m.DoubleBarrier = load_double_barrier().DoubleBarrier if sp.get("douady") else shipped_db
        try:
            p = m.DiscreteBarrierFDMPricerAnalytic(**kw)
            rec = dict(name=sp["name"],
                       inputs={k: ([str(d.date()) for d in v] if k == "monitoring_dates" else v)
                               for k, v in sp.items()},
                       spot_grid=list(p.spot_grid), flat_rate_r=p.flat_rate_r,
                       flat_dividend_q=p.flat_dividend_q,
                       use_continuous_window=p.use_continuous_window,
                       window=[p.window_k0, p.window_k1],
                       bgk=[p.bgk_lower_barrier, p.bgk_upper_barrier],
                       monitor_discrete=sorted(p.monitor_steps_discrete),
                       monitor_continuous=sorted(p.monitor_steps_continuous))
            # the value vectors price() marches (escrowed grid)
            S_eff = p._escrowed_spot()
            grid0 = p.spot_grid[:]
            p.spot_grid = [max(0.0, s - (p.spot - S_eff)) for s in grid0]
            p.grid_step_dS = p.spot_grid[1] - p.spot_grid[0]
            rec["S_eff"] = S_eff
            rec["grid_escrowed"] = list(p.spot_grid)
            rec["V_discrete"] = p._cn_stepper(p.lower_barrier, p.upper_barrier,
                                              p.monitor_steps_discrete)
            rec["V_vanilla"] = p._cn_stepper(None, None, {})
            if p.monitor_steps_continuous:
                rec["V_continuous"] = p._cn_stepper(p.bgk_lower_barrier, p.bgk_upper_barrier,
                                                    p.monitor_steps_continuous)
            p.spot_grid = grid0
            p.grid_step_dS = p.spot_grid[1] - p.spot_grid[0]
            rec["price"] = p.price()
            rec["greeks"] = p.greeks(**sp.get("greeks_kw", {}))
        finally:
            m.DoubleBarrier = shipped_db
        cases.append(rec)
    dump("spot_analytic_cases.json", dict(curve_rates={c["name"]: c["rate"] for c in specs},
                                          cases=cases))


if __name__ == "__main__":
    which = sys.argv[1:] or ["cn", "barrier", "double", "spot", "american", "analytic",
                             "black76", "spot_analytic"]
    if "black76" in which:
        gen_black76()
    if "cn" in which:
        gen_cn_log()
    if "barrier" in which:
        gen_barrier()
    if "double" in which:
        gen_double_out()
    if "spot" in which:
        gen_spot()
    if "american" in which:
        gen_american(with_config2="config2" in which or not sys.argv[1:])
    if "analytic" in which:
        gen_analytic()
    if "spot_analytic" in which:
        gen_spot_analytic()
