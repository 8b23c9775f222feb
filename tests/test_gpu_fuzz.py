"""Seeded random launches, HIP vs the CPU oracle, on the planner's own choice.

The other kernel tests pin shapes and variants; these draw everything at
once, per launch: CN or IT, grid size (6 to ~6000 nodes), step count,
Rannacher steps (including n_ranna >= n_time), batch size (which moves the
planner between the single-trade, throughput and paired flavours), and per
scenario the boundary form, knock-out sides, monitoring schedule (sparse,
or every step), rebates, accumulated tau and tau0.  Work per launch is
bounded so the oracle finishes in well under a second.

Bound: the kernel tests' 1e-10 of max(1, max|V|) per scenario, scaled by
n/2048 above 2048 nodes (test_gpu_kernels.py explains the scaling).
"""
import numpy as np
import pytest

from finite_difference_amd import capi
from finite_difference_amd.engine import Engine
from plan_factory import random_solve
from test_gpu_kernels import OracleBackend

pytestmark = pytest.mark.gpu

TOL = 1e-10
WORK_CAP = 1.5e8  # node-steps per launch


def _draw(seed: int):
    rng = np.random.default_rng(9100 + seed)
    it = bool(rng.integers(0, 2))
    n_nodes = int(np.exp(rng.uniform(np.log(6), np.log(6000))))
    n_time = int(rng.integers(1, 160))
    n_ranna = int(rng.choice([0, 1, 2, 2, 3, 5]))
    B = int(rng.choice([1, 2, 7, 33, 300, 1500]))
    B = max(1, min(B, int(WORK_CAP // max(1, n_nodes * n_time))))
    solves = []
    for i in range(B):
        s = random_solve(rng, n_nodes, n_time, n_ranna, it=it, drop_top=bool(rng.integers(0, 2)))
        s.tau_accumulate = bool(rng.integers(0, 2))
        s.tau0 = float(rng.choice([0.0, 0.0, 0.021]))
        if not it and rng.integers(0, 4) == 0:  # every-step projection (config 5)
            s.mon_steps = list(range(1, n_time + 1))
            s.mon_rebates = [float(s.mon_rebates[0]) if len(s.mon_rebates) else 0.0] * n_time
        solves.append(s)
    return it, n_nodes, n_time, n_ranna, solves


@pytest.mark.parametrize("seed", range(32))
def test_random_launch_vs_oracle(seed):
    it, n_nodes, n_time, n_ranna, solves = _draw(seed)
    B = len(solves)
    gpu = Engine().run(solves)
    ref = Engine(OracleBackend()).run(solves)
    tol = TOL * max(1.0, n_nodes / 2048)
    worst = 0.0
    for g, r in zip(gpu, ref):
        assert np.all(np.isfinite(g))
        worst = max(worst, float(np.max(np.abs(g - r))) / max(1.0, float(np.max(np.abs(r)))))
    print(f"[fuzz {seed}] {'it' if it else 'cn'} n={n_nodes} m={n_time} r={n_ranna} B={B} "
          f"{capi.variant_name(n_nodes, it, B=B)} worst={worst:.2e}")
    assert worst <= tol


def test_paired_flavour_random_batch_vs_oracle():
    """A batch large enough for two scenarios per wave (B >= 4096, grids of
    at most 2 * 64 * 4 nodes), mixed monitoring and odd B."""
    rng = np.random.default_rng(9999)
    n_nodes, n_time, B = 200, 40, 4097
    solves = [random_solve(rng, n_nodes, n_time, 2, it=False, drop_top=bool(i % 2))
              for i in range(B)]
    for i, s in enumerate(solves):
        s.tau_accumulate = i % 3 == 0
    name = capi.variant_name(n_nodes, False, B=B)
    assert name.endswith(",4>"), name  # the paired flavour (ZG bit 2)
    gpu = Engine().run(solves)
    ref = Engine(OracleBackend()).run(solves)
    worst = max(float(np.max(np.abs(g - r))) / max(1.0, float(np.max(np.abs(r))))
                for g, r in zip(gpu, ref))
    print(f"[fuzz paired] {name} worst={worst:.2e}")
    assert worst <= TOL


@pytest.mark.parametrize("form", ["auto", "stencil"])
@pytest.mark.parametrize("seed", range(16))
def test_random_spot_space_pricer_vs_oracle(seed, form):
    """fdcn_vc (the spot-space per-row CN of DiscreteBarrierFDMPricer2) on
    seeded random trades: grid 6-3000 nodes, 5-200 steps, every barrier
    type, weekly or no monitoring, the corrected explicit sign (the
    reference's sign diverges, see test_spot_barrier.py).  "auto": the
    pointwise form these trades classify into; "stencil": every scenario
    forced onto the stencil form (include/fdcn_diag.h)."""
    from finite_difference_amd import capi
    capi.vc_force_variant(0, 0, form == "stencil")
    try:
        _spot_space_trade(seed, form)
    finally:
        capi.vc_force_variant(0, 0, False)


def _spot_space_trade(seed, form):
    import datetime as dt
    from backends import oracle_engine
    from finite_difference_amd.spot_barrier import DiscreteBarrierFDMPricer2
    rng = np.random.default_rng(7300 + seed)
    v0, v1 = dt.date(2025, 1, 6), dt.date(2025, 7, 7)
    n = int(np.exp(rng.uniform(np.log(6), np.log(3000))))
    m = int(rng.integers(5, 200))
    bt = str(rng.choice(["none", "up-and-out", "down-and-out", "double-out", "up-and-in",
                         "down-and-in"]))
    S0 = 100.0
    lo = float(rng.uniform(60.0, 95.0)) if ("down" in bt or "double" in bt) else None
    hi = float(rng.uniform(105.0, 150.0)) if ("up" in bt or "double" in bt) else None
    weekly = [v0 + dt.timedelta(days=7 * i) for i in range(1, 26)] if rng.integers(0, 2) else None
    p = DiscreteBarrierFDMPricer2(
        spot=S0, strike=float(rng.uniform(80.0, 120.0)), valuation_date=v0, maturity_date=v1,
        volatility=float(rng.uniform(0.12, 0.45)), option_type=str(rng.choice(["call", "put"])),
        barrier_type=bt, lower_barrier=lo, upper_barrier=hi, monitoring_dates=weekly,
        flat_rate_nacc=float(rng.uniform(0.0, 0.08)), num_space_nodes=n, num_time_steps=m,
        engine=Engine(), explicit_sign="corrected")
    _, _, solves = p._grid_solves()
    from finite_difference_amd import capi
    from finite_difference_amd.engine import pack_vc
    g = pack_vc(solves, list(range(len(solves))))
    forms = capi.vc_forms(g.n_nodes, g.n_time, g.n_ranna, g.diag)
    assert np.all(forms == (1 if form == "auto" else 0)), forms
    gpu = Engine().run_vc(solves)
    ref = oracle_engine().run_vc(solves)
    worst = max(float(np.max(np.abs(g - r))) / max(1.0, float(np.max(np.abs(r))))
                for g, r in zip(gpu, ref))
    print(f"[fuzz vc {seed} {form}] n={n} m={m} {bt} monitored={weekly is not None} "
          f"solves={len(solves)} worst={worst:.2e}")
    assert worst <= TOL * max(1.0, n / 2048)


@pytest.mark.parametrize("seed", range(12))
def test_random_american_trade_device_vs_oracle(seed):
    """The whole American stack on seeded random trades: the device path
    (session marches per dividend segment, spline jumps and the Richardson /
    cubic Greeks epilogue on the GPU) against the host path on the CPU oracle
    (oracle march, host jumps, host epilogue).  Put or call, 0-2 cash
    dividends, 40-400 space nodes and steps.  Bounds: price and vega 1e-9,
    delta / gamma / theta 1e-7 relative to max(1, |x|) (the device epilogue
    solves the 4x4 cubic with its own LU, not LAPACK's)."""
    import datetime as dt
    from backends import oracle_engine
    from finite_difference_amd import market
    from finite_difference_amd.american import AmericanFDMPricer
    rng = np.random.default_rng(8800 + seed)
    val, mat = dt.date(2025, 7, 28), dt.date(2025, 7, 28) + dt.timedelta(days=int(rng.integers(20, 300)))
    n_div = int(rng.integers(0, 3))
    span = (mat - val).days
    divs = sorted((val + dt.timedelta(days=int(d)), float(rng.uniform(0.2, 2.5)))
                  for d in rng.choice(np.arange(1, span), size=n_div, replace=False))
    naca = float(rng.uniform(0.0, 0.09))
    kw = dict(spot=float(rng.uniform(60.0, 140.0)), strike=100.0, valuation_date=val,
              maturity_date=mat, sigma=float(rng.uniform(0.12, 0.5)),
              option_type=str(rng.choice(["put", "call"])), dividend_schedule=divs,
              num_space_nodes=int(rng.integers(40, 400)), num_time_steps=int(rng.integers(40, 400)),
              rannacher_steps=int(rng.choice([0, 2])))

    def make(engine):
        curve = market.iso_curve(market.create_rate_df(naca))
        return AmericanFDMPricer(discount_curve=curve, forward_curve=curve, engine=engine, **kw)

    dev, host = make(Engine()), make(oracle_engine())
    pd_, ph = dev.price_log2(), host.price_log2()
    gd, gh = dev.greeks_log2(), host.greeks_log2()
    print(f"[fuzz american {seed}] {kw['option_type']} N={kw['num_space_nodes']} "
          f"M={kw['num_time_steps']} divs={n_div} price {pd_:.6f} vs {ph:.6f}")
    assert abs(pd_ - ph) <= 1e-9 * max(1.0, abs(ph))
    for k, tol in (("price", 1e-9), ("vega", 1e-9), ("delta", 1e-7), ("gamma", 1e-7),
                   ("theta", 1e-7)):
        assert abs(gd[k] - gh[k]) <= tol * max(1.0, abs(gh[k])), (k, gd[k], gh[k])


@pytest.mark.parametrize("seed", range(12))
def test_random_barrier_trade_device_vs_oracle(seed):
    """DiscreteBarrierFDMPricer (the runner's pricer) on seeded random trades:
    every barrier type, call/put, parity-mode or explicit grids, rebates at
    hit or at expiry, one-sided Greeks near the barrier, dividends; the
    device path (one launch, Greeks epilogue on the GPU) against the host
    path on the CPU oracle.  price_log2 and every greeks_log2 key to 1e-9 of
    max(1, |x|) (the march differs by rounding; the epilogue is the same
    arithmetic)."""
    import datetime as dt
    from backends import oracle_engine
    from finite_difference_amd import scenarios
    rng = np.random.default_rng(6600 + seed)
    val = dt.date(2025, 7, 28)
    mat = val + dt.timedelta(days=int(rng.integers(10, 200)))
    S0 = 100.0
    bt = str(rng.choice(["up-and-out", "down-and-out", "up-and-in", "down-and-in"]))
    up = float(rng.uniform(103.0, 150.0)) if "up" in bt else None
    lo = float(rng.uniform(60.0, 97.0)) if "down" in bt else None
    mon = sorted({val + dt.timedelta(days=int(d)) for d in rng.integers(1, (mat - val).days + 1,
                                                                         int(rng.integers(1, 30)))})
    divs = ([(val + dt.timedelta(days=int(rng.integers(1, (mat - val).days))), 0.8)]
            if rng.integers(0, 3) == 0 else [])
    kw = dict(opt_type=str(rng.choice(["call", "put"])), divs=divs,
              rebate_amount=float(rng.choice([0.0, 0.0, 1.25])),
              rebate_at_hit=bool(rng.integers(0, 2)),
              use_one_sided_greeks_near_barrier=bool(rng.integers(0, 2)),
              num_space_nodes=int(rng.integers(60, 600)), num_time_steps=int(rng.integers(50, 500)),
              grid_mode=str(rng.choice(["parity", "explicit"])))
    args = (S0, float(rng.uniform(80.0, 120.0)), float(rng.uniform(0.12, 0.45)),
            float(rng.uniform(0.0, 0.09)), bt, up, lo, val, mat, mon)
    dev = scenarios.make_barrier_pricer(*args, engine=Engine(), **kw)
    host = scenarios.make_barrier_pricer(*args, engine=oracle_engine(), **kw)
    pd_, ph = dev.price_log2(), host.price_log2()
    gd, gh = dev.greeks_log2(), host.greeks_log2()
    print(f"[fuzz barrier {seed}] {bt} {kw['opt_type']} {kw['grid_mode']} "
          f"N={kw['num_space_nodes']} M={kw['num_time_steps']} price {pd_:.6f} vs {ph:.6f}")
    assert abs(pd_ - ph) <= 1e-9 * max(1.0, abs(ph))
    for k in gh:
        assert abs(gd[k] - gh[k]) <= 1e-9 * max(1.0, abs(gh[k])), (k, gd[k], gh[k])


@pytest.mark.parametrize("seed", range(10))
def test_random_cn_log_trade_device_vs_oracle(seed):
    """DiscreteBarrierCrankNicolsonLog (config 1's class) on seeded random
    trades: barrier side and in/out, rebate, a random monitoring set, auto
    grids; device (three sigma solves in one launch, device epilogue) against
    the host path on the oracle, price and every Greek to 1e-9 of max(1, |x|)."""
    from backends import oracle_engine
    from finite_difference_amd.cn_log import DiscreteBarrierCrankNicolsonLog
    rng = np.random.default_rng(5500 + seed)
    T = float(rng.uniform(0.05, 0.8))
    bt = str(rng.choice(["up-and-out", "down-and-out", "up-and-in", "down-and-in"]))
    kw = dict(S0=100.0, K=float(rng.uniform(80.0, 120.0)), T=T, sigma=float(rng.uniform(0.12, 0.45)),
              r_disc=float(rng.uniform(0.0, 0.08)), b_carry=float(rng.uniform(-0.02, 0.08)),
              option_type=str(rng.choice(["call", "put"])), barrier_type=bt,
              lower_barrier=float(rng.uniform(60.0, 95.0)) if "down" in bt else None,
              upper_barrier=float(rng.uniform(105.0, 150.0)) if "up" in bt else None,
              rebate=float(rng.choice([0.0, 0.0, 1.0])),
              monitor_times=sorted(float(x) for x in rng.uniform(0.0, T, int(rng.integers(1, 20)))),
              N_space=int(rng.integers(64, 700)), N_time=int(rng.integers(50, 900)))
    dev = DiscreteBarrierCrankNicolsonLog(**kw, engine=Engine())
    host = DiscreteBarrierCrankNicolsonLog(**kw, engine=oracle_engine())
    pd_, ph = dev.price(), host.price()
    print(f"[fuzz cn_log {seed}] {bt} {kw['option_type']} N={kw['N_space']} M={kw['N_time']} "
          f"price {pd_:.6f} vs {ph:.6f}")
    assert abs(pd_ - ph) <= 1e-9 * max(1.0, abs(ph))
    gd, gh = dev.greeks(), host.greeks()
    for k in gh:
        assert abs(gd[k] - gh[k]) <= 1e-9 * max(1.0, abs(gh[k])), (k, gd[k], gh[k])


@pytest.mark.parametrize("seed", range(8))
def test_random_black76_american_device_vs_oracle(seed):
    """AmericanFwdFDMPricer (Black-76 on the forward, the IT kernel with the
    forward's coefficients) on seeded random trades, device vs the host path
    on the oracle: price_log2 and greeks_log2 (Δ/Γ/θ 1e-7, the rest 1e-9)."""
    import datetime as dt
    from backends import oracle_engine
    from finite_difference_amd import market
    from finite_difference_amd.american_black76 import AmericanFwdFDMPricer
    rng = np.random.default_rng(4400 + seed)
    val = dt.date(2025, 7, 28)
    kw = dict(spot=float(rng.uniform(60.0, 140.0)), strike=100.0, valuation_date=val,
              maturity_date=val + dt.timedelta(days=int(rng.integers(20, 300))),
              sigma=float(rng.uniform(0.12, 0.5)), option_type=str(rng.choice(["put", "call"])),
              num_space_nodes=int(rng.integers(40, 400)), num_time_steps=int(rng.integers(40, 400)),
              rannacher_steps=2)
    naca = float(rng.uniform(0.0, 0.09))

    def make(engine):
        curve = market.iso_curve(market.create_rate_df(naca))
        return AmericanFwdFDMPricer(discount_curve=curve, forward_curve=curve, engine=engine, **kw)

    dev, host = make(Engine()), make(oracle_engine())
    pd_, ph = dev.price_log2(), host.price_log2()
    gd, gh = dev.greeks_log2(), host.greeks_log2()
    print(f"[fuzz black76 {seed}] {kw['option_type']} price {pd_:.6f} vs {ph:.6f}")
    assert abs(pd_ - ph) <= 1e-9 * max(1.0, abs(ph))
    for k in gh:
        tol = 1e-7 if k in ("delta", "gamma", "theta") else 1e-9
        assert abs(gd[k] - gh[k]) <= tol * max(1.0, abs(gh[k])), (k, gd[k], gh[k])


@pytest.mark.parametrize("seed", range(10))
def test_random_analytic_pricer_device_vs_oracle(seed):
    """DiscreteBarrierFDMPricerAnalytic on seeded random trades (corrected
    explicit sign): every barrier type, monthly / weekly / daily monitoring
    (daily takes the FIS continuous-window decision: BGK closed forms through
    the batched GPU engines, or the every-step CN overlay), rebates and their
    timing, the Douady double-barrier engine on or off; the device path
    against the host path on the oracle, price to 1e-9 and Greeks to 1e-7 of
    max(1, |x|)."""
    import pandas as pd
    from backends import oracle_engine
    from finite_difference_amd import market
    from finite_difference_amd.spot_barrier_analytic import DiscreteBarrierFDMPricerAnalytic
    rng = np.random.default_rng(3300 + seed)
    val, mat = pd.Timestamp("2025-07-28"), pd.Timestamp("2026-01-28")
    step = int(rng.choice([1, 7, 30]))
    mon = [val + pd.Timedelta(days=d) for d in range(step, (mat - val).days + 1, step)]
    bt = str(rng.choice(["up-and-out", "down-and-out", "up-and-in", "down-and-in", "double-out",
                         "double-in", "none"]))
    c = market.create_rate_df(float(rng.uniform(0.0, 0.08)))
    c["Date"] = pd.to_datetime(c["Date"], format="%Y/%m/%d").dt.strftime("%Y-%m-%d")
    kw = dict(trade_id="T1", direction=str(rng.choice(["long", "short"])), quantity=1,
              contract_multiplier=1.0, valuation_date=val, maturity_date=mat, discount_curve=c,
              forward_curve=c, dividend_schedule=[], monitoring_dates=mon,
              double_barrier_analytic=bool(rng.integers(0, 2)), spot=100.0,
              strike=float(rng.uniform(85.0, 115.0)), volatility=float(rng.uniform(0.15, 0.4)),
              option_type=str(rng.choice(["call", "put"])), barrier_type=bt,
              lower_barrier=float(rng.uniform(65.0, 92.0)) if ("down" in bt or "double" in bt) else None,
              upper_barrier=float(rng.uniform(108.0, 140.0)) if ("up" in bt or "double" in bt) else None,
              rebate_amount=float(rng.choice([0.0, 0.0, 1.0])),
              space_nodes=int(rng.integers(120, 500)), time_steps=int(rng.integers(20, 300)),
              explicit_sign="corrected")
    dev = DiscreteBarrierFDMPricerAnalytic(**kw, engine=Engine())
    host = DiscreteBarrierFDMPricerAnalytic(**kw, engine=oracle_engine())
    pg, ph = dev.price(), host.price()
    print(f"[fuzz analytic {seed}] {bt} every {step}d {kw['option_type']} price {pg:.6f} vs {ph:.6f}")
    assert abs(pg - ph) <= 1e-9 * max(1.0, abs(ph))
    gg, gh = dev.greeks(), host.greeks()
    for k in gh:
        assert abs(gg[k] - gh[k]) <= 1e-7 * max(1.0, abs(gh[k])), (k, gg[k], gh[k])
