"""Whole-file discrete-barrier runner: every row of a scenario file priced by
one native plan build, one launch and one device epilogue.

``run_config_scenarios.run_all_scenarios`` (run_config_scenarios.py:137-195)
prices rows one after another: per row a DiscreteBarrierFDMPricer, a base and
a sigma-bumped ``_solve_grid`` (discrete_barrier_fdm_pricer.py:442-547,
:883-904) and a host epilogue.  ``price_columns`` does that work for all rows
at once:

* per distinct rate, one pricer supplies the curve-derived scalars (dates,
  NACC rates, PV of dividends) -- the per-row facade's own code;
* ``fdcn_barrier_plan`` (csrc/fdcn_plan.hip) builds both grids of every
  knock-out / knock-in row on the host threads, bit-identical to the
  facade's plans (tests/test_scenario_batch.py);
* the 2R solves march as one launch; with the HIP engine the value vectors
  stay in HBM and ``fdcn_session_greeks`` returns price, Delta, Gamma, vega
  and theta of each row (6 doubles per row cross PCIe);
* the Black-76 legs (vanilla rows, knock-in parity; :648-745) run in bulk
  with libm's exp / log (``capi.vmath``) and scipy's ndtr, in the
  reference's operation order.

The result columns equal ``scenarios.run_rows`` (tested through the CPU
oracle engine).  Anything the vectorised path does not cover (option types
other than call / put, grids whose N_s differ across rows) returns None and
the caller takes the per-row path.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import capi
from .barrier import tail_quantile
from .engine import Engine, Group, default_engine

GREEKS = ("price", "delta", "gamma", "vega", "theta")
# the knock-out twins price_log2 / greeks_log2 accept (…pricer.py:907-1026)
KO_KIND = {"down-and-out": 1, "up-and-out": 2}
KI_KIND = {"down-and-in": 1, "up-and-in": 2}


def _missing(v) -> bool:
    """scenarios._opt's test: None or NaN (pandas.isna on a scalar)."""
    if v is None:
        return True
    try:
        return bool(v != v)
    except Exception:  # pragma: no cover - exotic cell values
        import pandas as pd
        return bool(pd.isna(v))


def _opt_col(cols: Dict[str, Sequence], key: str, R: int) -> List[Any]:
    c = cols.get(key)
    if c is None:
        return [None] * R
    return [None if _missing(v) else v for v in c]


def _num_col(cols: Dict[str, Sequence], key: str, R: int) -> np.ndarray:
    """A numeric optional column as float64 with NaN for missing cells (None
    or NaN, as _missing); numpy's own conversion when every cell is a number
    or None, the per-cell test otherwise."""
    c = cols.get(key)
    if c is None:
        return np.full(R, np.nan)
    try:
        return np.asarray(c, dtype=np.float64).reshape(R)
    except (TypeError, ValueError):
        return np.array([np.nan if _missing(v) else float(v) for v in c], np.float64)


def _factorize(col) -> tuple:
    """(distinct values, index of each row's value) of a column; pandas'
    hash factorisation when every cell is a value, else the sorted unique
    strings (str() of every cell, NaN included, as the facade's str(b))."""
    try:
        import pandas as pd
        codes, uniq = pd.factorize(np.asarray(col, dtype=object))
        if len(codes) and codes.min() >= 0:
            return list(uniq), np.asarray(codes, np.int64)
    except ImportError:  # pragma: no cover - pandas ships with the runner
        pass
    u, inv = np.unique(np.asarray([str(b) for b in col]), return_inverse=True)
    return u.tolist(), inv


def _black76(S, K, sigma, t_exp, carry, t_carry, r, t_disc, pv, call, shared=None):
    """_vanilla_black76_price (:648-692) elementwise, same operation order;
    math.exp / math.log through libm (capi.vmath), math.sqrt = np.sqrt
    (both correctly rounded), norm.cdf = scipy.special.ndtr.  ``shared``
    (a dict, optional) caches the subexpressions that repeat across the
    Greeks' repricings -- exp(carry t_carry), exp(-r t_disc), sqrt(t_exp)
    and log(F / K) per distinct input -- each computed by the same
    expression on the same operands, so the values are unchanged."""
    from scipy.special import ndtr
    if shared is None:
        shared = {}
    S = S - pv
    with np.errstate(all="ignore"):
        if ("sqrtT", t_exp) not in shared:
            shared[("sqrtT", t_exp)] = np.sqrt(t_exp)
        sqrtT = shared[("sqrtT", t_exp)]
        if "ec" not in shared:
            shared["ec"] = capi.vmath(capi.VM_EXP, carry * t_carry)
            shared["disc"] = capi.vmath(capi.VM_EXP, -r * t_disc)
        F = S * shared["ec"]
        key = ("lfk", S.tobytes()) if isinstance(S, np.ndarray) else ("lfk", S)
        if key not in shared:
            shared[key] = capi.vmath(capi.VM_LOG, F / K)
        d1 = (shared[key] + (0.5 * sigma * sigma) * t_exp) / (sigma * sqrtT)
        d2 = d1 - sigma * sqrtT
        Nd1, Nd2 = ndtr(d1), ndtr(d2)
        disc = shared["disc"]
        val = (disc * (F * Nd1 - K * Nd2) if call
               else disc * (K * (1.0 - Nd2) - F * (1.0 - Nd1)))
    intr = (t_disc <= 0) | (sigma <= 0)
    if np.any(intr):
        e = S - K if call else K - S
        val = np.where(intr, np.where(e >= 0.0, e, 0.0), val)  # Python max(e, 0.0)
    return val


def _black76_greeks(S0, K, sig0, T0: float, carry, t_carry: float, r, t_disc: float, pv, call,
                    dS=0.0001, dSigma=0.0001, dT=0.0001) -> Dict[str, np.ndarray]:
    """_vanilla_black76_greeks_fd (:694-745) elementwise; the six repricings
    share exp(carry t_carry), the discount factor, sqrt(T) and log(F / K)
    where their inputs agree (_black76's ``shared``)."""
    shared: Dict[Any, np.ndarray] = {}

    def price(S=S0, sigma=sig0, T=T0):
        return _black76(S, K, sigma, T, carry, t_carry, r, t_disc, pv, call, shared)
    h = S0 * dS
    p0 = price()
    pu = price(S=S0 + h)
    pd_ = price(S=S0 - h)
    delta = (pu - pd_) / (2.0 * h)
    gamma = (pu - 2.0 * p0 + pd_) / capi.vmath(capi.VM_SQUARE, h)
    vega = (price(sigma=sig0 + dSigma) - p0) / (100 * dSigma)
    if T0 > 2.0 * dT:
        theta = -((price(T=T0 + dT) - price(T=T0 - dT)) / (2.0 * dT))
    else:
        theta = -((p0 - price(T=max(T0 - dT, 1e-8))) / dT)
    return {"price": p0, "delta": delta, "gamma": gamma, "theta": theta, "vega": vega}


def _greeks_host(V: np.ndarray, rint: np.ndarray, rdbl: np.ndarray, tpar: np.ndarray) -> np.ndarray:
    """FDCN_GK_BARRIER on the host, for a non-device engine (the CPU-oracle
    test path): _pde_finish's arithmetic (:629-646, :949-978, :883-904) on
    the readout positions, in Python floats."""
    R = tpar.shape[0]
    out = np.zeros((R, 6))
    for t in range(R):
        res = []
        for k in (2 * t, 2 * t + 1):
            v = V[int(rint[k, 0])]
            icase, ilo, idx, mode = (int(x) for x in rint[k, 1:5])
            d = [float(x) for x in rdbl[k]]
            if icase == 1:
                pr = float(v[0])
            elif icase == 2:
                pr = float(v[ilo])
            else:
                w = (d[0] - d[1]) / (d[2] - d[1])
                pr = float((1.0 - w) * v[ilo] + w * v[ilo + 1])
            de = ga = 0.0
            if mode == 1:
                h1, h2 = d[5] - d[4], d[6] - d[5]
                Vm, V0, Vp = v[idx - 1], v[idx], v[idx + 1]
                de = float(-h2 / (h1 * (h1 + h2)) * Vm + (h2 - h1) / (h1 * h2) * V0
                           + h1 / (h2 * (h1 + h2)) * Vp)
                ga = float(2.0 * (Vm / (h1 * (h1 + h2)) - V0 / (h1 * h2) + Vp / (h2 * (h1 + h2))))
            res.append((pr, de, ga))
        (pb, de, ga), (pu, _, _) = res
        sig, spot, carry, divy, r, dv = (float(x) for x in tpar[t, :6])
        vega = (pu - pb) / (dv * 100)
        theta = -(0.5 * sig * sig * spot * spot * ga + (carry - divy) * spot * de - r * pb)
        out[t, :5] = (pb, de, ga, vega, theta)
    return out


def _device_session():
    from .session import Session
    return Session()


def _march_and_finish(eng: Engine, plan: dict, n_time: int, n_ranna: int,
                      mon: np.ndarray, overlap=None) -> np.ndarray:
    """A host engine's march of the plan's 2R solves (one run_group) and the
    Greeks epilogue on the host (the CPU-oracle test path; device engines
    take _plan_march_device).  ``overlap`` (optional): host work run first."""
    Q = plan["params"].shape[0]
    g = Group(False, plan["n_nodes"], n_time, min(n_ranna, n_time), plan["params"],
              plan["iparams"], plan["v_init"], None, np.tile(mon, Q), plan["mon_rebate"],
              list(range(Q)))
    RI = plan["rint"]
    if overlap is not None:
        overlap()
    V = eng.backend.run_group(g)
    eng.launches += 1
    eng.solves += Q
    return _greeks_host(V, RI, plan["rdbl"], plan["tparams"])


# the device path plans and marches the rows in chunks: the plan of chunk
# i+1 is built on the host while chunk i's initial vectors cross PCIe and it
# marches.  Two chunks from 4096 PDE rows on: a 10 000-row file 16.4 -> 13.0
# ms, three 13.2, four 14.9, eight 14.8 (tools/chunk_sweep.py; more chunks
# slow the plan builder, whose writes then share host memory with the DMA)
CHUNK_ROWS = 2048
MAX_CHUNKS = 2


def _plan_march_device(eng: Engine, S, row: np.ndarray, flag: np.ndarray, plan_args: tuple,
                       n_time: int, n_ranna: int, mon: np.ndarray, overlap,
                       timing: Optional[Dict[str, float]]) -> Optional[np.ndarray]:
    """The device path of price_columns, pipelined: the rows in up to
    MAX_CHUNKS chunks of at least CHUNK_ROWS, each planned straight into the session's pinned memory
    and marched as one asynchronous launch (H2D + kernel) while the host
    plans the next; one Greeks epilogue over all rows at the end.  The
    solves are the same as one launch's (each scenario is its own
    wavefront), so the results are too.  None when the chunks' grids differ
    (the per-row path groups them)."""
    import time
    from .session import GK_BARRIER
    Rp = row.shape[0]
    n_chunks = max(1, min(MAX_CHUNKS, Rp // CHUNK_ROWS))
    bounds = [Rp * i // n_chunks for i in range(n_chunks + 1)]
    t_plan = 0.0
    n_nodes = None
    RIs, rdbls, tps = [], [], []
    for a, b in zip(bounds[:-1], bounds[1:]):
        t0 = time.perf_counter()
        try:
            plan = capi.barrier_plan(row[a:b], flag[a:b], *plan_args, v_init_out=S.host_buffer)
        except capi.FdcnError as e:
            if "differ" in str(e):
                return None  # two launch shapes: the per-row path groups them
            raise
        t_plan += time.perf_counter() - t0
        if n_nodes is None:
            n_nodes = plan["n_nodes"]
        elif plan["n_nodes"] != n_nodes:
            return None
        Q = plan["params"].shape[0]
        g = Group(False, plan["n_nodes"], n_time, min(n_ranna, n_time), plan["params"],
                  plan["iparams"], plan["v_init"], None, np.tile(mon, Q), plan["mon_rebate"],
                  list(range(Q)))
        slots = S.march(g)
        eng.launches += 1
        eng.solves += Q
        RI = plan["rint"].copy()
        RI[:, 0] = slots[RI[:, 0]]
        RIs.append(RI)
        rdbls.append(plan["rdbl"])
        tps.append(plan["tparams"])
        del plan, g  # the pinned view (the session keeps the memory until it closes)
    t1 = time.perf_counter()
    if overlap is not None:
        overlap()
    res = S.greeks_raw(np.full(Rp, GK_BARRIER, np.int32), np.arange(0, 2 * Rp, 2, dtype=np.int32),
                       np.concatenate(tps), np.concatenate(RIs), np.concatenate(rdbls))
    if timing is not None:
        timing["plan"] = t_plan
        timing["march"] = time.perf_counter() - t1
    return res


def price_columns(cols: Dict[str, Sequence], base_params: Dict[str, Any],
                  engine: Optional[Engine] = None, dv_sigma: float = 0.0001,
                  timing: Optional[Dict[str, float]] = None) -> Optional[Dict[str, np.ndarray]]:
    """Model price and Greeks of every row (the columns of a scenario file:
    S0, K, sigma, rate, barrier_type, upper_barrier, lower_barrier).  Returns
    {"price", "delta", "gamma", "vega", "theta"} arrays, or None when the
    per-row path must be used.  ``timing`` (optional) receives the seconds
    spent in the plan builder ("plan") and in the march + epilogue ("march")."""
    import time
    from . import scenarios
    t_start = time.perf_counter()
    eng = engine if engine is not None else default_engine()
    bp = dict(base_params)
    R = len(cols["S0"])
    if R == 0:
        return {k: np.zeros(0) for k in GREEKS}
    opt = bp.get("opt_type", "call")
    if opt not in ("call", "put"):
        return None
    S0 = np.asarray(cols["S0"], np.float64)
    K = np.asarray(cols["K"], np.float64)
    sig = np.asarray(cols["sigma"], np.float64)
    rate = np.asarray(cols["rate"], np.float64).reshape(R)
    # barrier kinds through the distinct values of the column (a hash
    # factorisation; str() / lower() per distinct value, as the facade does
    # per row)
    ub, binv = _factorize(cols["barrier_type"])
    bts_u = [str(b).lower() for b in ub]
    ups = _num_col(cols, "upper_barrier", R)
    los = _num_col(cols, "lower_barrier", R)
    if np.any(~(S0 > 0)) or np.any(~(K > 0)) or np.any(~(sig > 0)):
        raise ValueError("spot, strike, sigma must be positive.")
    for b in bts_u:
        if b != "none" and b not in KO_KIND and b not in KI_KIND:
            raise ValueError(f"Unsupported barrier_type: {b}")
    # per-rate scalars (one facade per rate, in order of first appearance, as
    # run_rows_batched)
    ur, first_ix, rinv = np.unique(rate, return_index=True, return_inverse=True)
    order = np.argsort(first_ix, kind="stable")
    pos = np.empty(len(order), np.int64)
    pos[order] = np.arange(len(order))
    rix = pos[rinv.reshape(R)]
    per_rate = [scenarios.make_barrier_pricer(float(S0[i]), float(K[i]), float(sig[i]),
                                              float(rate[i]), "none", None, None, **bp)
                for i in first_ix[order].tolist()]
    p0 = per_rate[0]
    T, t_carry, t_disc = p0.time_to_expiry, p0.time_to_carry, p0.time_to_discount
    carry = np.array([p.carry_rate_nacc for p in per_rate])[rix]
    disc = np.array([p.discount_rate_nacc for p in per_rate])[rix]
    pv = np.array([p.pv_divs for p in per_rate])[rix]
    # dividend_yield_nacc (:244-255) per row
    divy = np.zeros(R)
    m = pv > 0.0
    if np.any(m):
        if np.any(pv[m] >= S0[m]):
            raise ValueError("PV(dividend_schedule) >= spot.")
        divy[m] = -capi.vmath(capi.VM_LOG, (S0[m] - pv[m]) / S0[m]) / max(1e-12, t_carry)
    call = opt == "call"
    already_hit = bool(bp.get("already_hit", False))
    already_in = bool(bp.get("already_in", False))

    out = {k: np.zeros(R) for k in GREEKS}
    binv = binv.reshape(R)
    van = None  # Black-76 legs (vanilla rows, knock-in parity), see below
    gv: Dict[str, np.ndarray] = {}

    def black76_legs():
        if van is not None and np.any(van):
            vi = np.nonzero(van)[0]
            gv.update(_black76_greeks(S0[vi], K[vi], sig[vi], T, carry[vi], t_carry, disc[vi],
                                      t_disc, pv[vi], call))
    is_ko = np.array([b in KO_KIND for b in bts_u], bool)[binv]
    kind_u = [KO_KIND[b] if b in KO_KIND and not already_hit else
              KI_KIND[b] if b in KI_KIND and not already_in else 0 for b in bts_u]
    kind = np.asarray(kind_u, np.int32)[binv]
    van = ~is_ko
    pde = np.nonzero(kind)[0]
    if len(pde):
        Rp = len(pde)
        row = np.zeros((Rp, capi.BP_NROW))
        flag = np.zeros((Rp, capi.BP_NFLAG), np.int32)
        row[:, 0], row[:, 1], row[:, 2] = S0[pde], K[pde], sig[pde]
        has_lo, has_up = ~np.isnan(los[pde]), ~np.isnan(ups[pde])
        row[:, 3] = np.where(has_lo, los[pde], 0.0)
        row[:, 4] = np.where(has_up, ups[pde], 0.0)
        flag[:, 2], flag[:, 3] = has_lo, has_up
        row[:, 5], row[:, 6], row[:, 7], row[:, 8] = carry[pde], divy[pde], disc[pde], pv[pde]
        row[:, 9] = float(bp.get("rebate_amount", 0.0))
        flag[:, 0] = 0 if call else 1
        flag[:, 1] = kind[pde]
        n_time = int(p0.num_time_steps)
        dt = T / n_time
        mon = np.asarray(sorted(k for k in p0._monitor_indices_tau(dt) if 1 <= k <= n_time),
                         np.int32)
        plan_args = (T, int(p0._requested_space_nodes), n_time,
                     1 if p0.grid_mode == "explicit" else 0, tail_quantile(), dv_sigma,
                     bool(p0.rebate_at_hit), mon)
        n_ranna = int(p0.rannacher_steps)
        t0 = time.perf_counter()
        if eng.on_device:
            # the Black-76 legs run on the host while the device marches
            with _device_session() as S:
                res = _plan_march_device(eng, S, row, flag, plan_args, n_time, n_ranna, mon,
                                         black76_legs, timing)
                t2 = time.perf_counter()
            if res is None:
                return None
            if timing is not None:
                timing["prep"] = t0 - t_start
                timing["free"] = time.perf_counter() - t2
        else:
            try:
                plan = capi.barrier_plan(row, flag, *plan_args)
            except capi.FdcnError as e:
                if "differ" in str(e):
                    return None  # two launch shapes: the per-row path groups them
                raise
            t1 = time.perf_counter()
            res = _march_and_finish(eng, plan, n_time, n_ranna, mon, overlap=black76_legs)
            if timing is not None:
                timing["prep"] = t0 - t_start
                timing["plan"] = t1 - t0
                timing["march"] = time.perf_counter() - t1
        for j, k in enumerate(GREEKS):
            out[k][pde] = res[:, j]
    # knocked-out rows (already_hit, :907-946): the rebate discounted from the
    # discount end date, zero Greeks
    if already_hit and np.any(is_ko):
        reb = np.array([bp.get("rebate_amount", 0.0) * p.get_discount_factor(p.discount_end_date)
                        for p in per_rate])
        out["price"][is_ko] = reb[rix[is_ko]]
    # Black-76 legs: vanilla rows, knocked-in rows, and knock-in parity
    if np.any(van):
        vi = np.nonzero(van)[0]
        if not gv:  # no PDE rows: nothing to overlap with
            black76_legs()
        ki = kind[vi] != 0  # knock-in with a PDE leg: vanilla - knock-out
        for k in GREEKS:
            out[k][vi] = np.where(ki, gv[k] - out[k][vi], gv[k])
    return out


def _pct_diff(model: np.ndarray, fa: np.ndarray) -> np.ndarray:
    with np.errstate(all="ignore"):
        v = np.abs(model - fa) / np.abs(fa) * 100.0
    return np.where(np.isnan(fa) | (fa == 0.0), np.nan, v)


def result_columns(cols: Dict[str, Sequence], res: Dict[str, np.ndarray]) -> Dict[str, Any]:
    """The result schema of run_config_scenarios.py:101-132 (scenarios._result_row)
    as columns, in the same key order."""
    R = len(cols["S0"])
    out: Dict[str, Any] = {}
    for k in ("scenario_name", "S0", "K", "sigma", "rate", "barrier_type"):
        c = cols[k]
        out[k] = c if isinstance(c, np.ndarray) else list(c)  # arrays stay arrays
    for k in ("upper_barrier", "lower_barrier"):
        out[k] = _num_col(cols, k, R)
    for name in ("price", "delta", "gamma", "vega"):
        model = np.asarray(res[name], np.float64)
        fa = _num_col(cols, f"FA_{name}", R)
        out[f"model_{name}"] = model
        out[f"FA_{name}"] = fa
        out[f"{name}_diff"] = np.abs(model - fa)
        out[f"{name}_pct_diff"] = _pct_diff(model, fa)
    return out


_LIST_KEYS = ("scenario_name", "S0", "K", "sigma", "rate", "barrier_type")


def rows_as_result_columns(rows: List[Dict[str, Any]]) -> Dict[str, Any]:
    """Per-row results (scenarios._result_row) as the columns result_columns
    builds: same keys in the same order, lists for the six input keys and
    float64 arrays for the rest -- so a shard priced by the per-row fallback
    merges with shards priced here (distributed.gather_columns)."""
    if not rows:
        return {}
    out: Dict[str, Any] = {}
    for k in rows[0]:
        vals = [r[k] for r in rows]
        out[k] = vals if k in _LIST_KEYS else np.asarray(vals, np.float64)
    return out


ROW_KEYS = ("scenario_name", "S0", "K", "sigma", "rate", "barrier_type", "upper_barrier",
            "lower_barrier", "FA_price", "FA_delta", "FA_gamma", "FA_vega")


def rows_to_columns(rows: List[dict]) -> Dict[str, List[Any]]:
    return {k: [r.get(k) for r in rows] for k in ROW_KEYS}


def columns_to_rows(out: Dict[str, Any]) -> List[Dict[str, Any]]:
    keys = list(out)
    n = len(out[keys[0]]) if keys else 0
    cols = [out[k].tolist() if isinstance(out[k], np.ndarray) else out[k] for k in keys]
    return [dict(zip(keys, vals)) for vals in zip(*cols)] if n else []


def run_rows_vectorized(rows: List[dict], base_params: Dict[str, Any],
                        engine: Optional[Engine] = None) -> Optional[List[Dict[str, Any]]]:
    """scenarios.run_rows on the vectorised path (None: use run_rows)."""
    cols = rows_to_columns(rows)
    res = price_columns(cols, base_params, engine)
    if res is None:
        return None
    return columns_to_rows(result_columns(cols, res))
