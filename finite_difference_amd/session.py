"""Device-resident sessions: marches, dividend jumps and the Greeks epilogue
chained on the MI355X (libfdcn ``fdcn_session_*``, csrc/fdcn_session.hip).

The reference reads 3-4 nodes of each solved grid (``_interp_price``,
``_delta_gamma_from_grid``, ``_local_cubic_delta_gamma``) and combines the
solves of a trade into vega, theta and Richardson extrapolations
(discrete_barrier_fdm_pricer.py:629-646, :883-904, :949-978;
discrete_barrier_fdm_pricer_cn.py:429-466; fd_american_equity.py:855-1068).
With a session the value vectors stay in HBM: the host builds the launch
plans and the node positions of every readout (bisection on its own grids,
as the pricers do), and only six scalars per trade come back.  American
solves with discrete dividends march segment by segment with the spline
remap (fd_american_equity.py:479-553, :732-772) on the device in between.
"""
from __future__ import annotations

import bisect
import ctypes
import threading
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import capi

GK_BARRIER, GK_CNLOG, GK_AMERICAN, GK_READOUT = 0, 1, 2, 3
GK_NPARAM, GK_NRINT, GK_NRDBL, GK_NOUT = 8, 5, 8, 6
READOUTS = {GK_BARRIER: 2, GK_CNLOG: 3, GK_AMERICAN: 7, GK_READOUT: 1}

_PI = ctypes.POINTER(ctypes.c_int32)
_PD = ctypes.POINTER(ctypes.c_double)
_V = ctypes.c_void_p
_I = ctypes.c_int32


def _bind(L: ctypes.CDLL) -> None:
    if getattr(L, "_fdcn_session_bound", False):
        return
    L.fdcn_session_create.restype = _I
    L.fdcn_session_create.argtypes = [ctypes.POINTER(_V)]
    L.fdcn_session_destroy.restype = _I
    L.fdcn_session_destroy.argtypes = [_V]
    L.fdcn_session_slots.restype = _I
    L.fdcn_session_slots.argtypes = [_V]
    L.fdcn_session_host_buffer.restype = _I
    L.fdcn_session_host_buffer.argtypes = [_V, ctypes.c_int64, ctypes.POINTER(_V)]
    L.fdcn_session_march.restype = _I
    L.fdcn_session_march.argtypes = [_V, _I, _I, _I, _I, _I, _V, _V, _V, _V, _V, _I, _V, _V, _V]
    L.fdcn_session_dividend_jump.restype = _I
    L.fdcn_session_dividend_jump.argtypes = [_V, _I, _I, _V, _V, _V, _V, _V]
    L.fdcn_session_greeks.restype = _I
    L.fdcn_session_greeks.argtypes = [_V, _I, _V, _V, _V, _I, _V, _V, _V]
    L.fdcn_session_fetch.restype = _I
    L.fdcn_session_fetch.argtypes = [_V, _I, _V, _I, _V]
    L._fdcn_session_bound = True


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


@dataclass
class Readout:
    """Node positions of one grid readout (see include/fdcn.h)."""
    slot: int
    icase: int        # 0: between ilo and ilo+1, 1: V[0], 2: V[ilo]
    ilo: int
    idx: int          # centre (3-point) or base (cubic) node
    dg_mode: int      # 0: price only, 1: 3-point Delta/Gamma, 2: cubic
    dbl: tuple        # S_interp, s[ilo], s[ilo+1], S_dg, s[idx-1..idx+2]


def interp_positions(s: Sequence[float], S: float):
    """The branches of _interp_price (discrete_barrier_fdm_pricer.py:629-646,
    fd_american_equity.py:855-874): (icase, ilo, s_lo, s_hi)."""
    n = len(s)
    if S <= s[0]:
        return 1, 0, 0.0, 0.0
    if S >= s[n - 1]:
        return 2, n - 1, 0.0, 0.0
    hi = bisect.bisect_right(s, S)
    return 0, hi - 1, float(s[hi - 1]), float(s[hi])


def nearest_interior(s: Sequence[float], x: float) -> int:
    """1 + argmin_{1 <= i <= len(s)-2} |s_i - x| (first index on ties)."""
    lo, hi = 1, len(s) - 2
    j = bisect.bisect_left(s, x, lo, hi + 1)
    if j <= lo:
        return lo
    if j > hi:
        return hi
    return j - 1 if abs(s[j - 1] - x) <= abs(s[j] - x) else j


def readout(slot: int, s: Sequence[float], S_interp: float, S_dg: Optional[float] = None,
            dg_mode: int = 0, idx: Optional[int] = None, n_v: Optional[int] = None) -> Readout:
    """Readout of the vector in `slot` on grid `s`.  ``n_v`` is the vector's
    length when it is shorter than the grid (the production barrier march
    drops the top node, …pricer.py:449/:543): V[-1] is then V[n_v - 1]."""
    icase, ilo, slo, shi = interp_positions(s, S_interp)
    if icase == 2 and n_v is not None:
        ilo = n_v - 1
    if dg_mode == 1:
        idx = nearest_interior(s, S_dg) if idx is None else idx
        nb = (float(s[idx - 1]), float(s[idx]), float(s[idx + 1]), 0.0)
    elif dg_mode == 2:
        nb = tuple(float(s[idx + k]) for k in (-1, 0, 1, 2))
    else:
        idx, nb = 0, (0.0, 0.0, 0.0, 0.0)
    return Readout(slot, icase, ilo, int(idx), dg_mode,
                   (float(S_interp), slo, shi, float(S_dg or 0.0)) + nb)


class _PinnedView:
    """Owner of one host_buffer array (its ``.base``): keeps the Session
    alive, so the pinned memory cannot be recycled while any view of it
    exists (a traceback holding a plan array past ``with
    Session()`` kept a view of freed or reused pinned memory)."""
    __slots__ = ("session", "__array_interface__", "__weakref__")

    def __init__(self, session: "Session", addr: int, n: int):
        self.session = session
        self.__array_interface__ = {"shape": (n,), "typestr": "<f8", "data": (addr, False),
                                    "version": 3}


class Session:
    """One device session (libfdcn fdcn_session); use as a context manager.

    ``close()`` (and leaving the ``with`` block) destroys the session, unless
    arrays from ``host_buffer`` are still alive: the destroy then waits until
    the last of them is dropped (``close_pending``), so a view never outlives
    the pinned memory it points into.

    Threads: the session's device context (streams, events, pinned arena)
    goes back to the idle pool of the thread that destroys it
    (fdcn_session.hip), so the destroy runs on the thread that created the
    session.  A deferred destroy whose last view is dropped on another thread
    stays pending (``close_pending``) until the creating thread calls
    ``close()`` again -- or, as a last resort, until the garbage collector
    collects the session.  View finalizers do not run at interpreter exit
    (atexit=False): a pending session is then left to process teardown."""

    def __init__(self):
        self._L = capi.lib()
        _bind(self._L)
        capi.require_device()
        h = _V()
        capi._check(self._L.fdcn_session_create(ctypes.byref(h)))
        self._h = h
        self._live_views = 0
        self._close_pending = False
        self._owner = threading.get_ident()

    @property
    def closed(self) -> bool:
        return getattr(self, "_h", None) is None

    @property
    def close_pending(self) -> bool:
        """close() was called while host_buffer views were alive."""
        return getattr(self, "_close_pending", False) and not self.closed

    def _destroy(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            h, self._h = self._h, None
            self._close_pending = False
            capi._check(self._L.fdcn_session_destroy(h))

    def close(self) -> None:
        if getattr(self, "_live_views", 0) > 0:
            self._close_pending = True  # the last view's finaliser destroys
            return
        self._destroy()

    def _view_dropped(self) -> None:
        self._live_views -= 1
        # a deferred destroy runs on the creating thread only (class notes);
        # dropped elsewhere, it stays pending for close() on that thread
        if (self._live_views == 0 and self._close_pending and
                threading.get_ident() == getattr(self, "_owner", None)):
            self._destroy()

    def __enter__(self) -> "Session":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self._destroy()
        except Exception:
            pass

    def host_buffer(self, n: int) -> np.ndarray:
        """n float64 of the session's pinned host memory (fdcn_session_host_buffer).
        A march whose payoff / v_init lies in it copies it to the device
        without staging, asynchronously: leave it unchanged until the next
        greeks_raw / fetch.  The array (and every view of it) keeps the
        session alive: a close() before the last one is dropped defers the
        destroy to that moment (the memory is the session's, recycled after
        the destroy)."""
        if self.closed or self.close_pending:
            raise capi.FdcnError("host_buffer on a closed session")
        p = _V()
        m = max(int(n), 1)
        capi._check(self._L.fdcn_session_host_buffer(self._h, 8 * m, ctypes.byref(p)))
        owner = _PinnedView(self, int(p.value), m)
        self._live_views += 1
        weakref.finalize(owner, self._view_dropped).atexit = False
        return np.asarray(owner)[:int(n)]

    # -- steps ---------------------------------------------------------------
    def march(self, g, v_init_slots: Optional[np.ndarray] = None) -> np.ndarray:
        """One batched launch of an engine.Group; returns its B output slots.
        With v_init_slots the initial vectors are those slots (g.v_init unused)."""
        out = np.empty(g.B, dtype=np.int32)
        vs = None if v_init_slots is None else np.ascontiguousarray(v_init_slots, np.int32)
        vi = None if vs is not None else np.ascontiguousarray(g.v_init, np.float64)
        P = np.ascontiguousarray(g.params, np.float64)
        I = np.ascontiguousarray(g.iparams, np.int32)
        F = np.ascontiguousarray(g.payoff, np.float64) if g.it else None
        ms = np.ascontiguousarray(g.mon_step if len(g.mon_step) else [0], np.int32)
        mr = np.ascontiguousarray(g.mon_rebate if len(g.mon_rebate) else [0.0], np.float64)
        capi._check(self._L.fdcn_session_march(
            self._h, 1 if g.it else 0, g.B, g.n_nodes, g.n_time, g.n_ranna, _ptr(P), _ptr(I),
            _ptr(vi), _ptr(vs), _ptr(F), len(g.mon_step), _ptr(ms), _ptr(mr), _ptr(out)))
        return out

    def dividend_jump(self, slots, s_nodes: np.ndarray, cash, strike_call) -> np.ndarray:
        sl = np.ascontiguousarray(slots, np.int32)
        S = np.ascontiguousarray(s_nodes, np.float64)
        B, n = S.shape
        c = np.ascontiguousarray(cash, np.float64)
        k = np.ascontiguousarray(strike_call, np.float64)
        out = np.empty(B, dtype=np.int32)
        capi._check(self._L.fdcn_session_dividend_jump(self._h, B, n, _ptr(sl), _ptr(S), _ptr(c),
                                                       _ptr(k), _ptr(out)))
        return out

    def greeks(self, trades: Sequence[tuple]) -> np.ndarray:
        """trades: (kind, [Readout, ...], params) -> [T, 6] = price, delta,
        gamma, vega, theta, aux."""
        T = len(trades)
        kind = np.empty(T, np.int32)
        first = np.empty(T, np.int32)
        tp = np.zeros((T, GK_NPARAM))
        rint: List[tuple] = []
        rdbl: List[tuple] = []
        for t, (k, rds, par) in enumerate(trades):
            if len(rds) != READOUTS[k]:
                raise ValueError(f"kind {k} takes {READOUTS[k]} readouts, got {len(rds)}")
            kind[t], first[t] = k, len(rint)
            tp[t, :len(par)] = par
            for r in rds:
                rint.append((r.slot, r.icase, r.ilo, r.idx, r.dg_mode))
                rdbl.append(r.dbl)
        return self.greeks_raw(kind, first, tp, np.array(rint, np.int32).reshape(-1, GK_NRINT),
                               np.array(rdbl, np.float64).reshape(-1, GK_NRDBL))

    def greeks_raw(self, kind, first, tparams, rint, rdbl) -> np.ndarray:
        """The epilogue on flat arrays (include/fdcn.h layout): kind [T],
        first readout [T], tparams [T, GK_NPARAM], rint [n, GK_NRINT] (slot
        first), rdbl [n, GK_NRDBL] -> [T, 6]."""
        kind = np.ascontiguousarray(kind, np.int32)
        first = np.ascontiguousarray(first, np.int32)
        T = kind.shape[0]
        tp = np.ascontiguousarray(tparams, np.float64)
        RI = np.ascontiguousarray(rint, np.int32)
        RD = np.ascontiguousarray(rdbl, np.float64)
        if (first.shape != (T,) or tp.shape != (T, GK_NPARAM) or RI.ndim != 2
                or RI.shape[1] != GK_NRINT or RD.shape != (RI.shape[0], GK_NRDBL)):
            raise ValueError("greeks_raw: array shapes do not match the fdcn.h layout")
        out = np.empty((T, GK_NOUT))
        capi._check(self._L.fdcn_session_greeks(self._h, T, _ptr(kind), _ptr(first), _ptr(tp),
                                                RI.shape[0], _ptr(RI), _ptr(RD), _ptr(out)))
        return out

    def fetch(self, slots, n_nodes: int) -> np.ndarray:
        sl = np.ascontiguousarray(slots, np.int32)
        out = np.empty((len(sl), n_nodes))
        capi._check(self._L.fdcn_session_fetch(self._h, len(sl), _ptr(sl), n_nodes, _ptr(out)))
        return out

    def slots(self) -> int:
        return int(self._L.fdcn_session_slots(self._h))
