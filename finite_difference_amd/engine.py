"""Batched solve planner: the seam between the pricer façades and libfdcn.

A ``Solve`` is one time march on one log-spot grid -- the work the reference
does in one call of ``_solve_grid`` (discrete_barrier_fdm_pricer.py:442,
discrete_barrier_fdm_pricer_cn.py:219) or ``_solve_segment``
(fd_american_equity.py:559).  ``Engine.run`` groups solves that share
(mode, n_nodes, n_time, n_ranna) into one kernel launch each and returns the
value vectors in request order.

The engine is the product path: it calls the HIP library and nothing else.
A different backend object with the same ``run_group`` method can be passed
to the pricers (tests use this to drive the CPU oracle as a checker).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import capi

NPARAM, NIPARAM = capi.NPARAM, capi.NIPARAM


def operator_coefficients(sigma: float, b: float, q: float, r: float,
                          dx: float) -> Tuple[float, float, float]:
    """(a, c, bcoef) of the log-spot Black-Scholes operator.

    Same expressions, same operand order as the reference
    (discrete_barrier_fdm_pricer.py:463-472, _cn.py:230-239,
    fd_american_equity.py:600-612) so the plan carries bit-identical inputs.
    """
    sig2 = sigma * sigma
    mu_x = (b - q) - 0.5 * sig2
    alpha = 0.5 * sig2 / (dx * dx)
    beta_adv = mu_x / (2.0 * dx)
    return alpha - beta_adv, alpha + beta_adv, -2.0 * alpha - r


# boundary forms (include/fdcn.h FDCN_I_*_FORM)
FORM_SUM, FORM_PROD = 0, 1


@dataclass
class Boundary:
    """Dirichlet value as a function of tau.

    FORM_SUM:  c0*exp(e0*tau) + c1*exp(e1*tau)
    FORM_PROD: ((c0*exp(e0*tau))*c1)*exp(e1*tau)
    """
    form: int = FORM_SUM
    c0: float = 0.0
    e0: float = 0.0
    c1: float = 0.0
    e1: float = 0.0

    def value(self, tau: float) -> float:
        import math
        if self.form == FORM_PROD:
            return self.c0 * math.exp(self.e0 * tau) * self.c1 * math.exp(self.e1 * tau)
        return self.c0 * math.exp(self.e0 * tau) + self.c1 * math.exp(self.e1 * tau)


@dataclass
class Solve:
    """One independent time march (one scenario of a launch)."""
    it: bool                       # Ikonen-Toivanen (American) vs knock-out mode
    n_time: int
    n_ranna: int
    dt: float
    coeffs: Tuple[float, float, float]   # (a, c, bcoef)
    v_init: np.ndarray                   # [n_nodes]
    lower: Boundary
    upper: Boundary
    tau0: float = 0.0
    tau_accumulate: bool = False         # FDCN_I_TAU_MODE = 1: tau += dt per step (American loop)
    payoff: Optional[np.ndarray] = None  # IT only, [n_nodes]
    ko_lo: int = -1                      # nodes j <= ko_lo knocked out on monitor steps
    ko_hi: int = 1 << 30                 # nodes j >= ko_hi knocked out
    mon_steps: Sequence[int] = ()
    mon_rebates: Sequence[float] = ()

    @property
    def n_nodes(self) -> int:
        return int(self.v_init.shape[0])

    def key(self) -> Tuple[bool, int, int, int]:
        return (self.it, self.n_nodes, int(self.n_time), int(self.n_ranna))


@dataclass
class Group:
    """Flat arrays for one launch (layout of include/fdcn.h)."""
    it: bool
    n_nodes: int
    n_time: int
    n_ranna: int
    params: np.ndarray
    iparams: np.ndarray
    v_init: np.ndarray
    payoff: Optional[np.ndarray]
    mon_step: np.ndarray
    mon_rebate: np.ndarray
    index: List[int] = field(default_factory=list)  # positions in the request list

    @property
    def B(self) -> int:
        return int(self.v_init.shape[0])


def pack(solves: Sequence[Solve], index: Sequence[int]) -> Group:
    s0 = solves[0]
    B = len(solves)
    n = s0.n_nodes
    P = np.zeros((B, NPARAM), dtype=np.float64)
    I = np.zeros((B, NIPARAM), dtype=np.int32)
    V = np.empty((B, n), dtype=np.float64)
    F = np.empty((B, n), dtype=np.float64) if s0.it else None
    mstep: List[int] = []
    mreb: List[float] = []
    for i, s in enumerate(solves):
        if s.key() != s0.key():
            raise ValueError("solves in one group must share (mode, n_nodes, n_time, n_ranna)")
        a, c, bc = s.coeffs
        P[i, capi.P_DT] = s.dt
        P[i, capi.P_A] = a
        P[i, capi.P_C] = c
        P[i, capi.P_BC] = bc
        P[i, capi.P_TAU0] = s.tau0
        P[i, capi.P_LO_C0:capi.P_LO_E1 + 1] = (s.lower.c0, s.lower.e0, s.lower.c1, s.lower.e1)
        P[i, capi.P_HI_C0:capi.P_HI_E1 + 1] = (s.upper.c0, s.upper.e0, s.upper.c1, s.upper.e1)
        I[i, capi.I_LO_FORM] = s.lower.form
        I[i, capi.I_HI_FORM] = s.upper.form
        I[i, capi.I_KO_LO] = max(-1, min(int(s.ko_lo), n))
        I[i, capi.I_KO_HI] = max(-1, min(int(s.ko_hi), n + 1))
        I[i, capi.I_TAU_MODE] = 1 if s.tau_accumulate else 0
        V[i] = s.v_init
        if F is not None:
            if s.payoff is None:
                raise ValueError("IT solve without payoff")
            F[i] = s.payoff
        if not s.it and len(s.mon_steps):
            I[i, capi.I_MON_START] = len(mstep)
            I[i, capi.I_MON_COUNT] = len(s.mon_steps)
            mstep.extend(int(k) for k in s.mon_steps)
            mreb.extend(float(x) for x in s.mon_rebates)
    return Group(s0.it, n, int(s0.n_time), int(s0.n_ranna), P, I, V, F,
                 np.asarray(mstep, dtype=np.int32), np.asarray(mreb, dtype=np.float64),
                 list(index))


def group_solves(solves: Sequence[Solve]) -> List[Group]:
    buckets: Dict[Tuple, List[int]] = {}
    for i, s in enumerate(solves):
        buckets.setdefault(s.key(), []).append(i)
    return [pack([solves[i] for i in idx], idx) for idx in buckets.values()]


@dataclass
class VcSolve:
    """One spot-space march with per-row coefficients (fdcn_vc_batch):
    diag [2, 6, n] = sub, main, sup, a, b, c of the implicit / explicit
    matrices for the Rannacher phase and the Crank-Nicolson phase; bnd
    [n_time, 2] = the Dirichlet values of rows 0 and n-1 per step."""
    n_time: int
    n_ranna: int
    diag: np.ndarray
    bnd: np.ndarray
    v_init: np.ndarray
    ko_lo: int = -1
    ko_hi: int = 1 << 30
    mon_steps: Sequence[int] = ()
    mon_rebates: Sequence[float] = ()

    @property
    def n_nodes(self) -> int:
        return int(self.v_init.shape[0])

    def key(self) -> Tuple[int, int, int]:
        return (self.n_nodes, int(self.n_time), int(self.n_ranna))


@dataclass
class VcGroup:
    n_nodes: int
    n_time: int
    n_ranna: int
    diag: np.ndarray      # [B, 2, 6, n]
    bnd: np.ndarray       # [B, n_time, 2]
    v_init: np.ndarray
    iparams: np.ndarray
    mon_step: np.ndarray
    mon_rebate: np.ndarray
    index: List[int] = field(default_factory=list)

    @property
    def B(self) -> int:
        return int(self.v_init.shape[0])


def pack_vc(solves: Sequence[VcSolve], index: Sequence[int]) -> VcGroup:
    s0 = solves[0]
    B, n = len(solves), s0.n_nodes
    I = np.zeros((B, NIPARAM), dtype=np.int32)
    mstep: List[int] = []
    mreb: List[float] = []
    for i, s in enumerate(solves):
        if s.key() != s0.key():
            raise ValueError("solves in one group must share (n_nodes, n_time, n_ranna)")
        I[i, capi.I_KO_LO] = max(-1, min(int(s.ko_lo), n))
        I[i, capi.I_KO_HI] = max(-1, min(int(s.ko_hi), n + 1))
        if len(s.mon_steps):
            I[i, capi.I_MON_START] = len(mstep)
            I[i, capi.I_MON_COUNT] = len(s.mon_steps)
            mstep.extend(int(k) for k in s.mon_steps)
            mreb.extend(float(x) for x in s.mon_rebates)
    return VcGroup(n, int(s0.n_time), int(s0.n_ranna),
                   np.ascontiguousarray(np.stack([s.diag for s in solves]), dtype=np.float64),
                   np.ascontiguousarray(np.stack([np.asarray(s.bnd, np.float64).reshape(-1, 2)
                                                  for s in solves])),
                   np.ascontiguousarray(np.stack([s.v_init for s in solves]), dtype=np.float64),
                   I, np.asarray(mstep, np.int32), np.asarray(mreb, np.float64), list(index))


class HipBackend:
    """Runs a packed group on the MI355X through libfdcn (host-pointer ABI)."""

    name = "hip"

    def run_vc_group(self, g: VcGroup) -> np.ndarray:
        return capi.vc_batch(g.n_nodes, g.n_time, g.n_ranna, g.diag, g.bnd, g.v_init,
                             g.iparams, g.mon_step, g.mon_rebate)

    def run_rr(self, contracts) -> np.ndarray:
        """BarrierEngine(**c).price() of every contract (fdcn_rr_barrier_batch)."""
        from .analytic import barrier_engine_batch
        return barrier_engine_batch(contracts)[0]

    def run_double(self, contracts, m: int) -> np.ndarray:
        """DoubleBarrier(..., m).price(b, r, T) of every contract
        (fdcn_double_barrier_batch)."""
        from .analytic import double_barrier_batch
        return double_barrier_batch(contracts, m)

    def run_group(self, g: Group) -> np.ndarray:
        if g.it:
            return capi.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                 g.v_init, g.payoff)
        return capi.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                             g.mon_step, g.mon_rebate)


_pool = None
_pool_lock = threading.Lock()


def _launch_pool():
    """The process-wide launch threads.  libfdcn keeps one HIP stream per
    calling thread and device for the thread's lifetime, so the threads that
    issue concurrent launches are kept rather than created per call: a pool
    per call would leave a stream behind with every thread it retired."""
    global _pool
    with _pool_lock:
        if _pool is None:
            from concurrent.futures import ThreadPoolExecutor
            _pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix="fdcn-launch")
        return _pool


class Engine:
    """Batches solves into launches on a backend (default: the HIP library).

    Groups of different shapes are independent launches: with the HIP backend
    they are issued from one host thread each, so they run concurrently on
    the GPU (libfdcn gives every calling thread its own stream; ctypes drops
    the GIL for the call).  A trade whose solves need two step counts -- the
    American Richardson pair N / 2N -- then costs the longer march, not the
    sum of both."""

    def __init__(self, backend=None, concurrent: bool = True):
        self.backend = backend if backend is not None else HipBackend()
        self.concurrent = concurrent
        self.launches = 0
        self.solves = 0

    def _run_groups(self, groups: List[Group]) -> List[np.ndarray]:
        if len(groups) < 2 or not self.concurrent or not isinstance(self.backend, HipBackend):
            return [self.backend.run_group(g) for g in groups]
        dev = capi.current_device()  # the HIP device is per thread: carry it over

        def one(g: Group) -> np.ndarray:
            capi.select_device(dev)
            return self.backend.run_group(g)
        return list(_launch_pool().map(one, groups))

    @property
    def on_device(self) -> bool:
        """True for the HIP engine: the facades then keep value vectors in HBM
        (session.Session) and run the Greeks epilogue there."""
        return isinstance(self.backend, HipBackend)

    def march_slots(self, sess, solves: Sequence[Solve],
                    v_init_slots: Optional[Sequence[int]] = None) -> np.ndarray:
        """Launch `solves` in `sess` (one launch per shape, overlapping on the
        session's streams) and return the output slot of each solve.  With
        v_init_slots, solve i starts from slot v_init_slots[i]."""
        out = np.empty(len(solves), dtype=np.int32)
        for g in group_solves(solves):
            vs = None if v_init_slots is None else np.asarray(
                [v_init_slots[i] for i in g.index], dtype=np.int32)
            out[g.index] = sess.march(g, vs)
            self.launches += 1
            self.solves += g.B
        return out

    def run_vc(self, solves: Sequence[VcSolve]) -> List[np.ndarray]:
        """Spot-space per-row-coefficient marches, one launch per shape."""
        buckets: Dict[Tuple, List[int]] = {}
        for i, s in enumerate(solves):
            buckets.setdefault(s.key(), []).append(i)
        out: List[Optional[np.ndarray]] = [None] * len(solves)
        for idx in buckets.values():
            g = pack_vc([solves[i] for i in idx], idx)
            res = self.backend.run_vc_group(g)
            self.launches += 1
            self.solves += g.B
            for row, i in enumerate(g.index):
                out[i] = res[row]
        return out  # type: ignore[return-value]

    def run_rr(self, contracts) -> np.ndarray:
        """Closed-form single-barrier prices (one batched launch)."""
        self.launches += 1
        return np.asarray(self.backend.run_rr(list(contracts)), np.float64)

    def run_double(self, contracts, m: int) -> np.ndarray:
        """Closed-form double-barrier prices, series n = -m..m (one launch)."""
        self.launches += 1
        return np.asarray(self.backend.run_double(list(contracts), int(m)), np.float64)

    def run(self, solves: Sequence[Solve]) -> List[np.ndarray]:
        out: List[Optional[np.ndarray]] = [None] * len(solves)
        groups = group_solves(solves)
        for g, res in zip(groups, self._run_groups(groups)):
            self.launches += 1
            self.solves += g.B
            for row, i in enumerate(g.index):
                out[i] = res[row]
        return out  # type: ignore[return-value]


_default: Optional[Engine] = None


def default_engine() -> Engine:
    global _default
    if _default is None:
        _default = Engine()
    return _default
