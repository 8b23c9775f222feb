"""NumPy restatement of the reference march, batched over scenarios.

TEST INFRASTRUCTURE ONLY (like oracle.py): the second CPU baseline variant of
SURVEY.md §8(d) -- "(ii) NumPy batched-over-scenarios Thomas" -- timed by
bench.py's cpu_baseline leg and checked against the C oracle in
tests/test_oracle_numpy.py.  The product package never imports it.

Same plan arrays as the C ABI (include/fdcn.h) and the same algorithm as the
C oracle's plan_solve_one (fdcn_oracle.c), i.e. the reference's loops
  rhs  discrete_barrier_fdm_pricer.py:531-537 / fd_american_equity.py:681-695
  Thomas (constant diagonals)  :487-509 / fd_american_equity.py:625-653
  IT   fd_american_equity.py:704-717,  KO  discrete_barrier_fdm_pricer.py:413-440
with every per-node operation vectorised over the B scenarios (layout
[node][scenario], so the sequential Thomas sweeps touch contiguous rows).
Operation order matches the C oracle; the boundary values use np.exp, which
can differ from libm's exp in the last ulp, so agreement is to rounding.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

# include/fdcn.h enums
P_DT, P_A, P_C, P_BC, P_TAU0 = 0, 1, 2, 3, 4
P_LO, P_HI = 5, 9
I_LO_FORM, I_HI_FORM, I_KO_LO, I_KO_HI, I_MON_START, I_MON_COUNT, I_TAU_MODE = range(7)


def _bnd(form, c, tau):
    e0 = c[:, 0] * np.exp(c[:, 1] * tau)
    prod = e0 * c[:, 2] * np.exp(c[:, 3] * tau)
    summ = e0 + c[:, 2] * np.exp(c[:, 3] * tau)
    return np.where(form == 1, prod, summ)


def march(it: bool, n_nodes: int, n_time: int, n_ranna: int, params, iparams, v_init,
          payoff=None, mon_step=None, mon_rebate=None,
          max_steps: Optional[int] = None) -> np.ndarray:
    """March B scenarios; returns V [B, n_nodes].  ``max_steps`` stops after
    that many steps (the timed sample of bench.py's CPU baseline)."""
    P = np.asarray(params, dtype=np.float64)
    I = np.asarray(iparams, dtype=np.int32)
    B = P.shape[0]
    n = n_nodes - 2
    V = np.ascontiguousarray(np.asarray(v_init, dtype=np.float64).T)  # [n_nodes, B]
    phi = (np.ascontiguousarray(np.asarray(payoff, dtype=np.float64).T[1:-1])
           if it else None)
    lam = np.zeros((n, B)) if it else None
    dt, a, c, bc = P[:, P_DT], P[:, P_A], P[:, P_C], P[:, P_BC]
    tau0 = P[:, P_TAU0].copy()
    acc = I[:, I_TAU_MODE] == 1
    lof, hif = I[:, I_LO_FORM], I[:, I_HI_FORM]
    clo, chi = P[:, P_LO:P_LO + 4], P[:, P_HI:P_HI + 4]
    ko_lo, ko_hi = I[:, I_KO_LO], I[:, I_KO_HI]
    mpos = I[:, I_MON_START].copy()
    mend = mpos + I[:, I_MON_COUNT]
    ms = np.asarray(mon_step if mon_step is not None and len(mon_step) else [0], np.int64)
    mr = np.asarray(mon_rebate if mon_rebate is not None and len(mon_rebate) else [0.0])
    node = np.arange(n_nodes)[:, None]
    rhs = np.empty((n, B))
    cp = np.empty((n, B))
    dp = np.empty((n, B))
    x = np.empty((n, B))
    tau = tau0.copy()
    steps = n_time if max_steps is None else min(n_time, max_steps)
    for m in range(steps):
        theta = 1.0 if m < n_ranna else 0.5
        AL = -theta * dt * a
        AC = 1.0 - theta * dt * bc
        AU = -theta * dt * c
        BL = (1.0 - theta) * dt * a
        BC = 1.0 + (1.0 - theta) * dt * bc
        BU = (1.0 - theta) * dt * c
        tau = np.where(acc, tau + dt, tau0 + (m + 1) * dt)
        lo, hi = _bnd(lof, clo, tau), _bnd(hif, chi, tau)
        np.multiply(BL, V[:-2], out=rhs)
        rhs += BC * V[1:-1]
        rhs += BU * V[2:]
        if it:
            rhs += dt * lam
        rhs[0] -= AL * lo
        rhs[-1] -= AU * hi
        denom = AC
        cp[0] = AU / denom
        dp[0] = rhs[0] / denom
        for i in range(1, n):
            denom = AC - AL * cp[i - 1]
            cp[i] = AU / denom
            dp[i] = (rhs[i] - AL * dp[i - 1]) / denom
        x[-1] = dp[-1]
        for i in range(n - 2, -1, -1):
            x[i] = dp[i] - cp[i] * x[i + 1]
        if it:
            cand = x - dt * lam
            ln = lam + (phi - x) / dt
            lam = np.where(ln < 0.0, 0.0, ln)
            x = np.where(phi > cand, phi, cand)
        V[0], V[-1] = lo, hi
        V[1:-1] = x
        if not it:
            live = mpos < mend
            hit = live & (ms[np.minimum(mpos, len(ms) - 1)] == m + 1)
            if hit.any():
                reb = mr[np.minimum(mpos, len(mr) - 1)]
                out = hit & ((node <= ko_lo) | (node >= ko_hi))
                V = np.where(out, reb, V)
                mpos = mpos + hit
            while True:  # skip entries at or before this step
                live = mpos < mend
                stale = live & (ms[np.minimum(mpos, len(ms) - 1)] <= m + 1)
                if not stale.any():
                    break
                mpos = mpos + stale
    return np.ascontiguousarray(V.T)
