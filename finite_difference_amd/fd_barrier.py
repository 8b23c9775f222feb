"""Finite-difference barrier engines with the analytic engines' signatures.

The north star asks for a drop-in for barrier_engine.py that keeps its
arguments and adds grid sizes.  ``FDBarrierEngine`` takes BarrierEngine's
constructor (barrier_engine.py:38-44) plus ``n_space`` / ``n_time`` and
prices the barrier option with the CN kernel, projecting the knock-out at
every time step (the continuous-monitoring limit of the reference's discrete
projection, discrete_barrier_fdm_pricer.py:413-440) -- or only at
``monitor_times`` if given.  ``FDDoubleBarrier`` does the same for
DoubleBarrier.price(b, r, T) (double _barrier.py:33), with both thresholds
(the reference's "double-out" branch, :435-437), BASELINE config 5.

With projection on every step (the default) the façades march only the
live range between the barriers plus a decay margin (ko_window.py: the same
values to 1e-18 relative, every node outside the window holding the
projection value); ``active_window=False`` marches the whole grid.
``solves()`` / ``solve_for()`` always return the whole-grid marches.

Knock-ins use in/out parity with the closed-form vanilla, as the reference's
pricers do (discrete_barrier_fdm_pricer.py:930-944).  Rebates follow
BarrierEngine: out-rebates at hit (projection value K) or at expiry
(K e^{-r tau}); in-rebates are one extra solve ("K at expiry if never hit"
or "K at first hit") in the same launch.

Grid: uniform in log S on [min(e^{x_c - w/2}, s_low/2), max(e^{x_c + w/2},
2 s_high)] with w = 2 * norm.ppf(0.99999) * sigma sqrt(T) around the
geometric centre of spot / strike / barriers -- the production pricer's
domain (discrete_barrier_fdm_pricer.py:270-320) with an explicit n_space.
"""
from __future__ import annotations

import bisect
import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import capi

from .analytic import BarrierEngine, DoubleBarrier, _norm_rebate_timing, black_scholes
from .barrier import tail_quantile
from .engine import FORM_SUM, Boundary, Engine, Solve, default_engine, operator_coefficients
from .ko_window import KoWindow, ko_window


def _domain(cands: Sequence[float], sigma: float, T: float):
    s_low, s_high = min(cands), max(cands)
    w = 2.0 * tail_quantile() * sigma * math.sqrt(T)
    x_c = math.log(math.sqrt(s_low * s_high))
    return (min(math.exp(x_c - 0.5 * w), 0.5 * s_low),
            max(math.exp(x_c + 0.5 * w), 2.0 * s_high))


def _grid(S_min: float, S_max: float, n_space: int):
    x0, x1 = math.log(S_min), math.log(S_max)
    dx = (x1 - x0) / n_space
    return dx, capi.log_grid(x0, dx, n_space)[1].tolist()  # math.exp(x0 + i dx)


def _steps(n_time: int, T: float, monitor_times: Optional[Sequence[float]]) -> List[int]:
    if monitor_times is None:
        return list(range(1, n_time + 1))
    dt = T / n_time
    ks = set()
    for t in monitor_times:
        if 0.0 < t <= T:
            ks.add(max(1, min(n_time, int(math.floor((T - t) / dt + 1e-9)))))
    return sorted(ks)


class FDBarrierEngine:
    """Single barrier on the CN kernel; BarrierEngine's arguments + grid."""

    def __init__(self, s: float, b: float, r: float, t: float, x: float, sigma: float, h: float,
                 optionflag: str, directionflag: str, in_out_flag: str, k: float,
                 barrier_status: Optional[str] = None, rebate_timing_in: Optional[str] = None,
                 rebate_timing_out: Optional[str] = None, n_space: int = 1024,
                 n_time: int = 2000, rannacher_steps: int = 2,
                 monitor_times: Optional[Sequence[float]] = None,
                 engine: Optional[Engine] = None, active_window: bool = True):
        # the analytic engine validates the flags and supplies the vanilla
        self.analytic = BarrierEngine(s, b, r, t, x, sigma, h, optionflag, directionflag,
                                      in_out_flag, k, barrier_status, rebate_timing_in,
                                      rebate_timing_out)
        self.s, self.b, self.r, self.t = float(s), float(b), float(r), float(t)
        self.x, self.sigma, self.h, self.k = float(x), float(sigma), float(h), float(k)
        self.optionflag, self.directionflag = optionflag.lower(), directionflag.lower()
        self.in_out_flag, self.barrier_status = in_out_flag.lower(), barrier_status
        self.rebate_timing_in = _norm_rebate_timing(rebate_timing_in, "expiry")
        self.rebate_timing_out = _norm_rebate_timing(rebate_timing_out, "hit")
        self.n_space, self.n_time, self.rannacher_steps = int(n_space), int(n_time), rannacher_steps
        self.monitor_times = monitor_times
        self.engine = engine
        self.active_window = active_window
        self._value: Optional[float] = None
        self.s_nodes: List[float] = []

    def _engine(self) -> Engine:
        return self.engine if self.engine is not None else default_engine()

    # -- solves --------------------------------------------------------------
    def _base(self, v_init: np.ndarray, lower: Boundary, upper: Boundary, dx: float) -> Solve:
        dt = self.t / self.n_time
        return Solve(it=False, n_time=self.n_time, n_ranna=min(self.rannacher_steps, self.n_time),
                     dt=dt, coeffs=operator_coefficients(self.sigma, self.b, 0.0, self.r, dx),
                     v_init=v_init, lower=lower, upper=upper)

    def solves(self) -> List[Solve]:
        """The launches' scenarios for this trade (empty when closed-form)."""
        if self.barrier_status == "crossed":
            return []
        S_min, S_max = _domain([self.s, self.x, self.h], self.sigma, self.t)
        dx, s = _grid(S_min, S_max, self.n_space)
        self.s_nodes = s
        n = len(s)
        up = self.directionflag == "u"
        ko_lo, ko_hi = (-1, bisect.bisect_left(s, self.h)) if up else \
            (bisect.bisect_right(s, self.h) - 1, n)
        steps = _steps(self.n_time, self.t, self.monitor_times)
        dt = self.t / self.n_time
        X, r, b = self.x, self.r, self.b
        call = self.optionflag == "c"
        pay = np.maximum(np.asarray(s) - X, 0.0) if call else np.maximum(X - np.asarray(s), 0.0)
        if call:
            lo, hi = Boundary(), Boundary(FORM_SUM, s[-1], b - r, -X, -r)
        else:
            lo, hi = Boundary(FORM_SUM, X, -r, 0.0, 0.0), Boundary()
        # the side of the grid beyond the barrier is knocked out: its far
        # Dirichlet value is the projection value (rebate) there.
        out_reb = self.k if self.in_out_flag == "o" else 0.0
        hit_now = self.in_out_flag == "o" and self.rebate_timing_out == "hit"

        def reb(tau):
            return out_reb if hit_now else out_reb * math.exp(-r * tau)

        def ko(sv: Solve, value_fn, value_bnd: Boundary) -> Solve:
            sv.ko_lo, sv.ko_hi = ko_lo, ko_hi
            sv.mon_steps = steps
            sv.mon_rebates = [value_fn(k * dt) for k in steps]
            sv.ko_value = value_bnd  # the projection value as a function of tau (ko_window)
            return sv

        far = Boundary(FORM_SUM, out_reb, 0.0 if hit_now else -r, 0.0, 0.0)
        main = self._base(pay, lo if up else far, far if up else hi, dx)
        out = [ko(main, reb, far)]
        if self.in_out_flag == "i" and self.k != 0.0:
            K = self.k
            if self.rebate_timing_in == "expiry":   # K at expiry if never hit
                v = np.full(n, K)
                alive = Boundary(FORM_SUM, K, -r, 0.0, 0.0)
                sv = self._base(v, alive if up else Boundary(), Boundary() if up else alive, dx)
                out.append(ko(sv, lambda tau: 0.0, Boundary()))
            else:                                    # K at the first hit
                v = np.zeros(n)
                hitb = Boundary(FORM_SUM, K, 0.0, 0.0, 0.0)
                sv = self._base(v, Boundary() if up else hitb, hitb if up else Boundary(), dx)
                out.append(ko(sv, lambda tau: K, hitb))
        return out

    def planned(self) -> List[Tuple[Solve, Optional[KoWindow]]]:
        """The marches to launch: each of solves(), or its knock-out window."""
        out = []
        for sv in self.solves():
            w = ko_window(sv, sv.ko_value) if self.active_window else None
            out.append((w.solve if w else sv, w))
        return out

    def _interp(self, V: np.ndarray) -> float:
        s = self.s_nodes
        hi = bisect.bisect_right(s, self.s)
        lo = hi - 1
        w = (self.s - s[lo]) / (s[hi] - s[lo])
        return float((1.0 - w) * V[lo] + w * V[hi])

    def finish(self, results: Sequence[np.ndarray]) -> float:
        if self.barrier_status == "crossed":
            self._value = float(self.analytic.price())
            return self._value
        ko_val = self._interp(results[0])
        if self.in_out_flag == "o":
            self._value = ko_val
        else:
            reb = self._interp(results[1]) if len(results) > 1 else 0.0
            self._value = float(self.analytic.vanilla()) - ko_val + reb
        return self._value

    def price(self) -> float:
        if self._value is None:
            plan = self.planned()
            res = self._engine().run([p[0] for p in plan]) if plan else []
            self.finish([w.expand(v) if w else v for (_, w), v in zip(plan, res)])
        return self._value

    def vanilla(self) -> float:
        return float(self.analytic.vanilla())


class FDDoubleBarrier:
    """Double knock-out / knock-in on the CN kernel; DoubleBarrier's API."""

    def __init__(self, S, X, L, U, sigma, callflag: str, inflag: str, m: int = 4,
                 n_space: int = 4096, n_time: int = 8192, rannacher_steps: int = 2,
                 monitor_times: Optional[Sequence[float]] = None,
                 engine: Optional[Engine] = None, active_window: bool = True):
        self.S, self.X, self.L, self.U = float(S), float(X), float(L), float(U)
        self.sigma = float(sigma)
        self.callflag, self.inflag = callflag.lower(), inflag.lower()
        if self.callflag not in ("c", "p"):
            raise ValueError("Incorrect callflag (use 'c' or 'p')")
        if self.inflag not in ("in", "out"):
            raise ValueError("Incorrect inflag")
        self.m = m
        self.n_space, self.n_time, self.rannacher_steps = int(n_space), int(n_time), rannacher_steps
        self.monitor_times = monitor_times
        self.engine = engine
        self.active_window = active_window
        self.s_nodes: List[float] = []

    def solve_for(self, b: float, r: float, T: float) -> Solve:
        S_min, S_max = _domain([self.S, self.X, self.L, self.U], self.sigma, T)
        dx, s = _grid(S_min, S_max, self.n_space)
        self.s_nodes = s
        call = self.callflag == "c"
        sa = np.asarray(s)
        pay = np.maximum(sa - self.X, 0.0) if call else np.maximum(self.X - sa, 0.0)
        # the grid extends beyond both barriers: the projection keeps the
        # knocked-out nodes at 0, so both Dirichlet values are 0 as well.
        dt = T / self.n_time
        sv = Solve(it=False, n_time=self.n_time,
                   n_ranna=min(self.rannacher_steps, self.n_time), dt=dt,
                   coeffs=operator_coefficients(self.sigma, b, 0.0, r, dx), v_init=pay,
                   lower=Boundary(), upper=Boundary())
        sv.ko_lo = bisect.bisect_right(s, self.L) - 1
        sv.ko_hi = bisect.bisect_left(s, self.U)
        sv.mon_steps = _steps(self.n_time, T, self.monitor_times)
        sv.mon_rebates = [0.0] * len(sv.mon_steps)
        sv.ko_value = Boundary()
        return sv

    def finish(self, V: np.ndarray, b: float, r: float, T: float) -> float:
        s = self.s_nodes
        hi = bisect.bisect_right(s, self.S)
        lo = hi - 1
        w = (self.S - s[lo]) / (s[hi] - s[lo])
        out = float((1.0 - w) * V[lo] + w * V[hi])
        if self.inflag == "out":
            return out
        return float(black_scholes(self.callflag, self.S, self.X, r, b, self.sigma, T)) - out

    def price(self, b: float, r: float, T: float) -> float:
        if (self.callflag == "c" and self.X >= self.U) or (self.callflag == "p" and self.X <= self.L):
            out = 0.0
            if self.inflag == "out":
                return out
            return float(black_scholes(self.callflag, self.S, self.X, r, b, self.sigma, T))
        eng = self.engine if self.engine is not None else default_engine()
        sv = self.solve_for(b, r, T)
        w = ko_window(sv, sv.ko_value) if self.active_window else None
        V = eng.run([w.solve if w else sv])[0]
        return self.finish(w.expand(V) if w else V, b, r, T)


def price_many(engines: Sequence[FDBarrierEngine]) -> List[float]:
    """Price many FDBarrierEngine trades with their solves in shared launches."""
    plans, spans, all_solves = [], [], []
    for e in engines:
        plan = e.planned()
        spans.append((len(all_solves), len(plan)))
        plans.extend(plan)
        all_solves.extend(p[0] for p in plan)
    res = engines[0]._engine().run(all_solves) if all_solves else []
    res = [w.expand(v) if w else v for (_, w), v in zip(plans, res)]
    return [e.finish(res[a:a + n]) for e, (a, n) in zip(engines, spans)]
