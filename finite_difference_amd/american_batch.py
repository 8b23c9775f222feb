"""Whole-file American runner: every row of a scenario file priced by one
native plan build, lock-step segment launches and one device epilogue.

``run_american_scenarios.run_all_american_scenarios``
(run_american_scenarios.py:209-277) prices rows one after another: per row an
AmericanFDMPricer, ``price_log2`` and ``greeks_log2`` (fd_american_equity.py:
925-1068), i.e. up to seven (sigma, n_time) grids -- N, 2N, sigma +-h,
sigma +-2h and price_log2's 2 * num_space_nodes grid -- each a chain of
``_solve_segment`` calls with dividend jumps in between.  Done per row in
Python that is ~8 ms of host work per row against ~25 us of GPU time.
``price_columns`` does the same work for all rows at once:

* per distinct rate, one pricer supplies the curve-derived scalars (dates,
  NACC rates, dividend times) -- the façade's own code;
* ``fdcn_american_plan`` (csrc/fdcn_plan.hip) builds every (row, sigma) grid
  on the host threads: band, log nodes, snapped spot and strike, payoff,
  coefficients, boundaries, readout positions -- bit-identical to the
  façade's (tests/test_american_batch.py);
* segment i of every job of one step count marches in one launch (a device
  session keeps the vectors in HBM), the dividend jumps run on the device,
  and ``FDCN_GK_AMERICAN`` returns price_log2, price, Delta, Gamma, vega and
  theta per row.

With a non-device engine (the CPU oracle in tests) the same plan is marched
through ``engine.backend`` and finished on the host with the façade's
arithmetic (NumPy's LAPACK for the cubic fit), so the columns equal the
per-row runner's exactly.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import capi
from .engine import Engine, Group, default_engine

GREEKS = ("price", "delta", "gamma", "vega", "theta")


def _jobs(sig: np.ndarray, N: int, nsn: int, h: float):
    """Per row the seven requests of price_log2 + greeks_log2
    (AmericanFDMPricer._device_requests) and their unique (sigma, n_time)
    jobs, in first-use order (the façade's _device_jobs), vectorised over the
    rows: request j of a row reuses the first request j' <= j with the same
    (sigma, n_time) -- the façade's dict of keys, as a 7 x 7 comparison."""
    s0 = np.asarray(sig, np.float64).reshape(-1)
    R = s0.shape[0]
    S = np.stack([s0, s0, s0 + h, s0 - h, s0 + 2.0 * h, s0 - 2.0 * h, s0], axis=1)
    NT = np.array([N, 2 * N, N, N, N, N, 2 * nsn], np.int64)
    eq = (S[:, :, None] == S[:, None, :]) & (NT[:, None] == NT[None, :])[None, :, :]
    first = np.argmax(eq, axis=2)  # the first j' with the same key (j itself at worst)
    new = first == np.arange(7)[None, :]
    n_new = new.sum(axis=1)
    base = np.concatenate(([0], np.cumsum(n_new)[:-1]))
    rank = np.cumsum(new, axis=1) - 1  # a new request's index among its row's new ones
    job_of = base[:, None] + rank      # valid where new
    req = np.take_along_axis(job_of, first, axis=1)
    job_row = np.repeat(np.arange(R, dtype=np.int64), n_new)
    job_sig = S[new]
    job_nt = np.broadcast_to(NT, (R, 7))[new]
    return job_row, job_sig, job_nt.astype(np.int64), req.astype(np.int64)


def _interp(s: np.ndarray, v: np.ndarray, s0: float) -> float:
    """AmericanFDMPricer._interp_price (fd_american_equity.py:855-874)."""
    if s0 <= s[0]:
        return float(v[0])
    if s0 >= s[-1]:
        return float(v[-1])
    hi = int(np.searchsorted(s, s0, side="right"))
    lo = hi - 1
    w = (s0 - s[lo]) / (s[hi] - s[lo])
    return float((1.0 - w) * v[lo] + w * v[hi])


def _cubic(s: np.ndarray, v: np.ndarray, s0: float):
    """AmericanFDMPricer._local_cubic_delta_gamma (:876-907)."""
    n = len(s) - 1
    i = int(np.argmin(np.abs(s - s0)))
    i = 1 if i < 1 else (n - 2 if i > n - 2 else i)
    idx = [i - 1, i, i + 1, i + 2]
    xv = np.array([s[j] for j in idx], dtype=float)
    yv = np.array([v[j] for j in idx], dtype=float)
    z = xv - s0
    design = np.vstack([z ** 3, z ** 2, z, np.ones_like(z)]).T
    _, b_coef, c_coef, _ = np.linalg.solve(design, yv)
    return float(c_coef), float(2.0 * b_coef)


def _finish_host(V, S, snapped, req, spot, sig, carry, disc, h) -> Dict[str, np.ndarray]:
    """price_log2 and greeks_log2 (:925-1068) of every row from the job
    vectors, in the façade's operation order."""
    R = req.shape[0]
    out = {k: np.zeros(R) for k in GREEKS + ("price_log2",)}
    for i in range(R):
        j = req[i]
        pr = lambda k: _interp(S[k], V[k], snapped[k])  # noqa: E731
        p_n, p_2 = pr(j[0]), pr(j[6])
        out["price_log2"][i] = (4.0 * p_2 - p_n) / 3.0
        price_n = pr(j[0])
        delta_n, gamma_n = _cubic(S[j[0]], V[j[0]], snapped[j[0]])
        price_2n = pr(j[1])
        delta_2n, gamma_2n = _cubic(S[j[1]], V[j[1]], snapped[j[1]])
        price = (4.0 * price_2n - price_n) / 3.0
        delta = (4.0 * delta_2n - delta_n) / 3.0
        gamma = (4.0 * gamma_2n - gamma_n) / 3.0
        s0 = float(sig[i])
        first_h = (pr(j[2]) - pr(j[3])) / (2.0 * h)
        first_2h = (pr(j[4]) - pr(j[5])) / (4.0 * h)
        dvds = (4.0 * first_h - first_2h) / 3.0
        vega = dvds / 100.0
        r, b, q, sp = float(disc[i]), float(carry[i]), 0.0, float(spot[i])
        theta = -(0.5 * s0 * s0 * sp * sp * gamma + (b - q) * sp * delta - r * price)
        for k, x in zip(GREEKS, (price, delta, gamma, vega, theta)):
            out[k][i] = float(x)
    return out


def price_columns(cols: Dict[str, Sequence], base_params: Dict[str, Any],
                  engine: Optional[Engine] = None, dv_sigma: float = 0.01,
                  timing: Optional[Dict[str, float]] = None) -> Optional[Dict[str, np.ndarray]]:
    """price_log2 and greeks_log2 of every row (columns S0, K, sigma, rate).
    Returns {"price_log2", "price", "delta", "gamma", "vega", "theta"}
    arrays, or None when the per-row path must be used."""
    import time
    from . import scenarios
    from .american import AmericanFDMPricer
    t_start = time.perf_counter()
    eng = engine if engine is not None else default_engine()
    R = len(cols["S0"])
    if R == 0:
        return {k: np.zeros(0) for k in GREEKS + ("price_log2",)}
    spot = np.asarray(cols["S0"], np.float64)
    K = np.asarray(cols["K"], np.float64)
    sig = np.asarray(cols["sigma"], np.float64)
    rate = [float(x) for x in cols["rate"]]
    if np.any(~(spot > 0)) or np.any(~(K > 0)) or np.any(~(sig > 0)):
        raise ValueError("spot, strike and sigma must be positive.")
    first: Dict[float, int] = {}
    for i, rt in enumerate(rate):
        first.setdefault(rt, i)
    per_rate = [scenarios.make_american_pricer(float(spot[i]), float(K[i]), float(sig[i]), rt,
                                               **base_params) for rt, i in first.items()]
    p0 = per_rate[0]
    if type(p0) is not AmericanFDMPricer or p0.grid_type != "uniform":
        return None
    pos = {rt: j for j, rt in enumerate(first)}
    rix = np.fromiter((pos[x] for x in rate), np.int64, R)
    carry = np.array([p.carry_rate_nacc for p in per_rate])[rix]
    disc = np.array([p.discount_rate_nacc for p in per_rate])[rix]
    N, nsn = int(p0.num_time_steps), int(p0.num_space_nodes)
    call = p0.option_type == "call"
    t0 = time.perf_counter()
    if eng.on_device:
        from .session import Session
        with Session() as S:
            res = _device_chunks(eng, S, p0, spot, K, sig, carry, disc, dv_sigma, call, N, nsn,
                                 timing)
            t2 = time.perf_counter()
        if timing is not None:
            timing["prep"] = t0 - t_start
            timing["free"] = time.perf_counter() - t2
        return res
    job_row, job_sig, job_nt, req = _sorted_jobs(sig, N, nsn, dv_sigma)
    J = len(job_row)
    job = np.stack([spot[job_row], K[job_row], job_sig, carry[job_row], disc[job_row]], axis=1)
    plan = capi.american_plan(job, np.full(J, 1 if call else 0, np.int32), nsn, p0.s_max_mult,
                              p0.time_to_expiry, with_grids=True)
    res = _march_plan(eng, plan, p0, job_nt, req, spot, sig, carry, disc, dv_sigma, call, nsn,
                      timing, t0)
    t2 = time.perf_counter()
    if timing is not None:
        timing["prep"] = t0 - t_start
        timing["march"] = t2 - timing.pop("_t1")
    return res


def _sorted_jobs(sig: np.ndarray, N: int, nsn: int, h: float):
    """_jobs, reordered by step count (stable): each launch's rows are then
    one contiguous block of the plan arrays, handed over as views; req
    follows the new order."""
    job_row, job_sig, job_nt, req = _jobs(sig, N, nsn, h)
    J = len(job_row)
    perm = np.argsort(job_nt, kind="stable")
    inv = np.empty(J, np.int64)
    inv[perm] = np.arange(J)
    return job_row[perm], job_sig[perm], job_nt[perm], inv[req]


# the device path plans and marches the rows in chunks (the next chunk's plan
# on the host while the previous one's launches run), up to four of at least
# 500 rows: a 2 000-row file 49.8 -> 45.7 ms (two 47.4, three 47.6;
# tools/chunk_sweep.py american)
CHUNK_ROWS = 500
MAX_CHUNKS = 4


def _segment_tables(p0, nts, job_nt):
    """Per step count its segments (p0._segments); per job its grid's
    dividend count and each dividend's cash amount."""
    segs = {nt: p0._segments(nt) for nt in nts}
    nt_ix = np.searchsorted(np.asarray(nts, np.int64), job_nt)
    n_div = np.array([len(segs[nt][0]) for nt in nts], np.int64)[nt_ix]
    cash_tab = np.zeros((len(nts), max(1, int(n_div.max(initial=0)))))
    for a, nt in enumerate(nts):
        for d, (_, amt) in enumerate(segs[nt][0]):
            cash_tab[a, d] = amt
    return segs, nt_ix, n_div, cash_tab


def _group(plan: dict, segs, p0, call: bool, n1: int, m: slice, nt: int, seg: int, v_init) -> Group:
    """One launch: the jobs in m (one step count), segment seg.  v_init None:
    the first segment, which starts from the payoff (one array for both, so
    a session copies it once)."""
    _, pts, steps = segs[nt]
    P = plan["params"][m].copy()
    P[:, capi.P_DT] = (pts[seg + 1] - pts[seg]) / float(steps[seg])
    P[:, capi.P_TAU0] = pts[seg]
    restart = seg == 0 or call
    pay = plan["payoff"][m]
    return Group(True, n1, int(steps[seg]), p0.rannacher_steps if restart else 0, P,
                 plan["iparams"][m], pay if v_init is None else v_init, pay,
                 np.zeros(0, np.int32), np.zeros(0), list(range(m.start, m.stop)))


def _members(job_nt: np.ndarray, nts):
    J = len(job_nt)
    bounds = np.searchsorted(job_nt, np.asarray(nts, np.int64), side="left").tolist() + [J]
    return {nt: slice(bounds[a], bounds[a + 1]) for a, nt in enumerate(nts)}


def _device_chunks(eng: Engine, S, p0, spot, K, sig, carry, disc, dv_sigma: float, call: bool,
                   N: int, nsn: int, timing):
    """The device path: rows in up to MAX_CHUNKS chunks, each planned
    (payoffs straight into the session's pinned memory) and launched --
    segment by segment per step count, device dividend jumps between --
    while the host plans the next chunk; one Greeks epilogue over all rows.
    Every job is its own wavefront, so chunking changes no result."""
    import time
    from .session import GK_AMERICAN
    R = len(spot)
    n1 = nsn + 1
    divs = p0._div_times_tau()
    n_chunks = max(1, min(MAX_CHUNKS, R // CHUNK_ROWS))
    bounds = [R * i // n_chunks for i in range(n_chunks + 1)]
    cub = np.array([1, 1, 0, 0, 0, 0, 0], np.int64)  # cubic readouts: the N and 2N grids
    RIs, RDs = [], []
    t_plan = 0.0
    for a, b in zip(bounds[:-1], bounds[1:]):
        t0 = time.perf_counter()
        job_row, job_sig, job_nt, req = _sorted_jobs(sig[a:b], N, nsn, dv_sigma)
        job_row = job_row + a
        J = len(job_row)
        job = np.stack([spot[job_row], K[job_row], job_sig, carry[job_row], disc[job_row]], axis=1)
        plan = capi.american_plan(job, np.full(J, 1 if call else 0, np.int32), nsn,
                                  p0.s_max_mult, p0.time_to_expiry, with_grids=bool(divs),
                                  payoff_out=S.host_buffer)
        nts = sorted(set(job_nt.tolist()))
        segs, nt_ix, n_div, cash_tab = _segment_tables(p0, nts, job_nt)
        members = _members(job_nt, nts)
        t_plan += time.perf_counter() - t0
        slot = np.full(J, -1, np.int32)
        g = None
        for seg in range(max(len(segs[nt][2]) for nt in nts)):
            for nt in nts:
                steps = segs[nt][2]
                if seg >= len(steps) or steps[seg] < 1:
                    continue
                m = members[nt]
                # later segments start from the slots (no host vector)
                g = _group(plan, segs, p0, call, n1, m, nt, seg,
                           None if seg == 0 else np.empty((m.stop - m.start, 0)))
                slot[m] = S.march(g, None if seg == 0 else slot[m])
                eng.launches += 1
                eng.solves += m.stop - m.start
            jump = np.nonzero(seg < n_div)[0]
            if len(jump):
                cash = cash_tab[nt_ix[jump], seg]
                kc = plan["gout"][jump, 1] if call else np.full(len(jump), -1.0)
                slot[jump] = S.dividend_jump(slot[jump], plan["s_nodes"][jump], cash, kc)
        # seven readouts per row
        rows = (2 * req + cub[None, :]).reshape(-1)
        RI = plan["rint"][rows].copy()
        RI[:, 0] = slot[RI[:, 0]]
        RIs.append(RI)
        RDs.append(plan["rdbl"][rows])
        del plan, g  # the pinned views go before the session closes
    t1 = time.perf_counter()
    tp = np.zeros((R, capi.GK_NPARAM))
    tp[:, 0], tp[:, 1], tp[:, 2], tp[:, 3], tp[:, 4] = sig, spot, carry, disc, dv_sigma
    out = S.greeks_raw(np.full(R, GK_AMERICAN, np.int32), np.arange(0, 7 * R, 7, dtype=np.int32),
                       tp, np.concatenate(RIs), np.concatenate(RDs))
    if timing is not None:
        timing["plan"] = t_plan
        timing["march"] = time.perf_counter() - t1
    res = {k: out[:, j] for j, k in enumerate(GREEKS)}
    res["price_log2"] = out[:, 5]
    return res


def _march_plan(eng: Engine, plan: dict, p0, job_nt, req, spot, sig, carry, disc,
                dv_sigma: float, call: bool, nsn: int, timing, t0: float):
    """A host engine's marches (the CPU-oracle test path): every job's
    segments through engine.backend, the dividend jumps and the readouts on
    the host, in the facade's arithmetic."""
    import time
    J = len(job_nt)
    n1 = nsn + 1
    nts = sorted(set(job_nt.tolist()))
    segs, _, _, _ = _segment_tables(p0, nts, job_nt)
    members = _members(job_nt, nts)
    t1 = time.perf_counter()
    if timing is not None:
        timing["plan"] = t1 - t0
        timing["_t1"] = t1
    V = [None] * J
    for seg in range(max(len(segs[nt][2]) for nt in nts)):
        for nt in nts:
            steps = segs[nt][2]
            if seg >= len(steps) or steps[seg] < 1:
                continue
            m = members[nt]
            v0 = None if seg == 0 else np.stack([V[j] for j in range(m.start, m.stop)])
            out = eng.backend.run_group(_group(plan, segs, p0, call, n1, m, nt, seg, v0))
            eng.launches += 1
            eng.solves += m.stop - m.start
            for r_, j in enumerate(range(m.start, m.stop)):
                V[j] = out[r_]
        for j in range(J):
            dv = segs[int(job_nt[j])][0]
            if seg < len(dv):
                kc = float(plan["gout"][j, 1]) if call else -1.0
                V[j] = capi.dividend_jump(plan["s_nodes"][j], V[j], dv[seg][1], kc)
    return _finish_host(V, plan["s_nodes"], plan["gout"][:, 0], req, spot, sig, carry, disc,
                        dv_sigma)


ROW_KEYS = ("scenario_name", "S0", "K", "sigma", "rate", "FA_price", "FA_delta", "FA_gamma",
            "FA_vega")


def result_columns(cols: Dict[str, Sequence], res: Dict[str, np.ndarray]) -> Dict[str, Any]:
    """run_american_scenarios.py's result schema (scenarios._result_row with
    model_price = price_log2, Greeks from greeks_log2) as columns."""
    from .scenario_batch import _num_col, _pct_diff
    R = len(cols["S0"])
    out: Dict[str, Any] = {}
    for k in ("scenario_name", "S0", "K", "sigma", "rate"):
        out[k] = list(cols[k])
    for name, key in (("price", "price_log2"), ("delta", "delta"), ("gamma", "gamma"),
                      ("vega", "vega")):
        model = np.asarray(res[key], np.float64)
        fa = _num_col(cols, f"FA_{name}", R)
        out[f"model_{name}"] = model
        out[f"FA_{name}"] = fa
        out[f"{name}_diff"] = np.abs(model - fa)
        out[f"{name}_pct_diff"] = _pct_diff(model, fa)
    return out


def run_rows_vectorized(rows: List[dict], base_params: Dict[str, Any],
                        engine: Optional[Engine] = None) -> Optional[List[Dict[str, Any]]]:
    from .scenario_batch import columns_to_rows
    cols = {k: [r.get(k) for r in rows] for k in ROW_KEYS}
    res = price_columns(cols, base_params, engine)
    if res is None:
        return None
    return columns_to_rows(result_columns(cols, res))
