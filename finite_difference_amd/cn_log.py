"""Crank-Nicolson discrete-barrier engine in log-spot, flat-rate variant.

Drop-in for ``DiscreteBarrierCrankNicolsonLog``
(discrete_barrier_fdm_pricer_cn.py:25-637, the file's executable prefix; the
north-star file and BASELINE config 1).  Same dataclass fields, same methods
(``price``, ``greeks``, ``configure_grid`` ...), same numerics: pure CN (no
Rannacher), put lower boundary K e^{-r tau}, monitoring index
round((T - t)/dt) kept when 0 < k < N_time, undiscounted rebate.

The three solves of ``_pde_price_and_greeks`` (base, sigma +- dv) share the
grid and run as one three-scenario launch on the MI355X.

Deviation, documented: the reference's second ``greeks`` definition (:595)
calls ``self._vanilla_black76_price``, which the class never defines, so
``greeks()`` raises AttributeError for "none" and knock-in trades.  Here that
method is the class's own Black-Scholes-with-carry closed form, so those
Greeks are returned instead of raising.
"""
from __future__ import annotations

import bisect
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import capi

from .engine import FORM_SUM, Boundary, Engine, Solve, default_engine, operator_coefficients
from .session import GK_CNLOG, Session, readout

SQRT_2PI = math.sqrt(2.0 * math.pi)


def norm_pdf(x: float) -> float:
    return math.exp(-0.5 * x * x) / SQRT_2PI


def norm_cdf(x: float) -> float:
    return 0.5 * (1.0 + math.erf(x / math.sqrt(2.0)))


@dataclass
class DiscreteBarrierCrankNicolsonLog:
    S0: float
    K: float
    T: float
    sigma: float
    r_disc: float
    b_carry: float
    option_type: str
    barrier_type: str
    lower_barrier: Optional[float] = None
    upper_barrier: Optional[float] = None
    rebate: float = 0.0
    monitor_times: Optional[List[float]] = None
    N_space: Optional[int] = None
    N_time: Optional[int] = None
    engine: Optional[Engine] = field(default=None, repr=False, compare=False)

    _S_min: float = field(init=False, default=0.0)
    _S_max: float = field(init=False, default=0.0)
    s_nodes: List[float] = field(init=False, default_factory=list)

    # ------------------------------------------------------------------ grid
    def configure_grid(self) -> None:
        """Domain [s_low/4, 4 s_high]; auto N_space (12 points per sigma sqrt T)
        and N_time (lambda ~ 0.4, >= N_space, >= 10 per monitoring interval)
        when unset (:59-118)."""
        if self.T <= 0.0:
            raise ValueError("T must be positive")
        if self.sigma <= 0.0:
            raise ValueError("sigma must be positive")
        if self.S0 <= 0.0:
            raise ValueError("S0 must be positive")
        cands = [self.S0, self.K]
        if self.lower_barrier is not None and self.lower_barrier > 0:
            cands.append(self.lower_barrier)
        if self.upper_barrier is not None and self.upper_barrier > 0:
            cands.append(self.upper_barrier)
        s_low, s_high = min(cands), max(cands)
        S_min = max(1e-8, s_low / 4.0)
        S_max = s_high * 4.0
        if S_min >= S_max:
            S_min, S_max = self.S0 / 5.0, self.S0 * 5.0
        self._S_min, self._S_max = S_min, S_max
        x_range = math.log(S_max) - math.log(S_min)
        dx_target = self.sigma * math.sqrt(self.T) / 12
        if dx_target <= 0.0:
            dx_target = x_range / 300.0
        if self.N_space is None:
            self.N_space = max(int(math.ceil(x_range / dx_target)), 300)
        if self.N_time is None:
            dx = x_range / self.N_space
            opt = int(math.ceil(0.5 * self.sigma * self.sigma * self.T / (0.4 * dx * dx)))
            n_mon = len([t for t in (self.monitor_times or []) if 0.0 < t < self.T])
            self.N_time = max(opt, self.N_space, 10 * (n_mon + 1))

    def _build_log_grid(self) -> float:
        if self._S_min <= 0.0 or self._S_max <= 0.0 or self.N_space is None:
            self.configure_grid()
        x_min, x_max = math.log(self._S_min), math.log(self._S_max)
        N = self.N_space
        dx = (x_max - x_min) / N
        self.s_nodes = capi.log_grid(x_min, dx, N)[1].tolist()  # math.exp(x_min + i dx)
        return dx

    def _terminal_payoff(self) -> List[float]:
        return self._payoff(self.s_nodes).tolist()

    def _payoff(self, s_nodes) -> np.ndarray:
        s = np.asarray(s_nodes, dtype=np.float64)
        e = s - self.K if self.option_type.lower() == "call" else self.K - s
        return np.where(0.0 > e, 0.0, e)

    def _boundaries(self) -> Tuple[Boundary, Boundary]:
        """Dirichlet values of :153-171 in kernel form."""
        r, b = self.r_disc, self.b_carry
        if self.option_type.lower() == "call":
            return Boundary(), Boundary(FORM_SUM, self.s_nodes[-1], b - r, -self.K, -r)
        return Boundary(FORM_SUM, self.K, -r, 0.0, 0.0), Boundary()

    def _boundary_values(self, tau: float) -> Tuple[float, float]:
        lo, hi = self._boundaries()
        return lo.value(tau), hi.value(tau)

    def _monitor_indices_tau(self, dt: float) -> set:
        idx = set()
        for t_mon in self.monitor_times or []:
            if t_mon <= 0.0 or t_mon >= self.T:
                continue
            k = int(round((self.T - t_mon) / dt))
            if 0 < k < self.N_time:
                idx.add(k)
        return idx

    def _ko_thresholds(self) -> Tuple[int, int]:
        n = len(self.s_nodes)
        bt = self.barrier_type.lower()
        if bt == "down-and-out" and self.lower_barrier is not None:
            return bisect.bisect_right(self.s_nodes, self.lower_barrier) - 1, n
        if bt == "up-and-out" and self.upper_barrier is not None:
            return -1, bisect.bisect_left(self.s_nodes, self.upper_barrier)
        return -1, n

    def _apply_KO_projection(self, V: List[float]) -> None:
        lo, hi = self._ko_thresholds()
        for i in range(len(self.s_nodes)):
            if i <= lo or i >= hi:
                V[i] = self.rebate

    # ----------------------------------------------------------------- solve
    def _engine(self) -> Engine:
        return self.engine if self.engine is not None else default_engine()

    def _make_solve(self, apply_KO: bool, sigma: float) -> Solve:
        self.configure_grid()
        dx = self._build_log_grid()
        dt = self.T / self.N_time
        coeffs = operator_coefficients(sigma, self.b_carry, 0.0, self.r_disc, dx)
        lower, upper = self._boundaries()
        s = Solve(it=False, n_time=int(self.N_time), n_ranna=0, dt=dt, coeffs=coeffs,
                  v_init=self._payoff(self.s_nodes), lower=lower, upper=upper)
        if apply_KO:
            s.ko_lo, s.ko_hi = self._ko_thresholds()
            s.mon_steps = sorted(self._monitor_indices_tau(dt))
            s.mon_rebates = [self.rebate] * len(s.mon_steps)
        return s

    def _solve_grid(self, apply_KO: bool) -> List[float]:
        """March tau 0 -> T (:219-302) as a one-scenario launch."""
        return self._engine().run([self._make_solve(apply_KO, self.sigma)])[0].tolist()

    # -------------------------------------------------------------- epilogue
    def _interp_price_from_grid(self, V) -> float:
        s = self.s_nodes
        S0 = self.S0
        if S0 <= s[0]:
            return V[0]
        if S0 >= s[-1]:
            return V[-1]
        hi = bisect.bisect_right(s, S0)
        lo = hi - 1
        w = (S0 - s[lo]) / (s[hi] - s[lo])
        return (1.0 - w) * V[lo] + w * V[hi]

    def _delta_gamma_from_grid(self, V) -> Tuple[float, float]:
        s = self.s_nodes
        idx = 1 + int(np.argmin(np.abs(np.asarray(s[1:len(s) - 1]) - self.S0)))
        h1 = s[idx] - s[idx - 1]
        h2 = s[idx + 1] - s[idx]
        Vm, V0, Vp = V[idx - 1], V[idx], V[idx + 1]
        delta = (-h2 / (h1 * (h1 + h2)) * Vm + (h2 - h1) / (h1 * h2) * V0
                 + h1 / (h2 * (h1 + h2)) * Vp)
        gamma = 2.0 * (Vm / (h1 * (h1 + h2)) - V0 / (h1 * h2) + Vp / (h2 * (h1 + h2)))
        return delta, gamma

    # ------------------------------------------------------------- closed form
    def _vanilla_bs_price_and_greeks(self) -> Dict[str, float]:
        """Black-Scholes with carry b and discount r, Greeks in S0 (:359-423)."""
        S0, K, T, sigma, r, b = self.S0, self.K, self.T, self.sigma, self.r_disc, self.b_carry
        if T <= 0.0 or sigma <= 0.0:
            price = max(S0 - K, 0.0) if self.option_type.lower() == "call" else max(K - S0, 0.0)
            return {"price": price, "delta": 0.0, "gamma": 0.0, "theta": 0.0, "vega": 0.0}
        q = r - b
        sqrtT = math.sqrt(T)
        d1 = (math.log(S0 / K) + (b + 0.5 * sigma * sigma) * T) / (sigma * sqrtT)
        d2 = d1 - sigma * sqrtT
        Nd1, Nd2, nd1 = norm_cdf(d1), norm_cdf(d2), norm_pdf(d1)
        disc_q, disc_r = math.exp(-q * T), math.exp(-r * T)
        if self.option_type.lower() == "call":
            price = S0 * disc_q * Nd1 - K * disc_r * Nd2
            delta = disc_q * Nd1
        else:
            price = K * disc_r * norm_cdf(-d2) - S0 * disc_q * norm_cdf(-d1)
            delta = disc_q * (Nd1 - 1.0)
        gamma = disc_q * nd1 / (S0 * sigma * sqrtT)
        vega = S0 * disc_q * nd1 * sqrtT
        theta = -(0.5 * sigma * sigma * S0 * S0 * gamma + b * S0 * delta - r * price)
        return {"price": price, "delta": delta, "gamma": gamma, "theta": theta, "vega": vega}

    def _vanilla_black76_price(self, S: Optional[float] = None, sigma: Optional[float] = None,
                               T: Optional[float] = None) -> float:
        """Closed-form vanilla at (S, sigma, T) (see module docstring)."""
        S0 = self.S0 if S is None else S
        sig = self.sigma if sigma is None else sigma
        T_ = self.T if T is None else T
        r, b, K = self.r_disc, self.b_carry, self.K
        if T_ <= 0.0 or sig <= 0.0:
            return max(S0 - K, 0.0) if self.option_type.lower() == "call" else max(K - S0, 0.0)
        sq = math.sqrt(T_)
        d1 = (math.log(S0 / K) + (b + 0.5 * sig * sig) * T_) / (sig * sq)
        d2 = d1 - sig * sq
        dq, dr = math.exp((b - r) * T_), math.exp(-r * T_)
        if self.option_type.lower() == "call":
            return S0 * dq * norm_cdf(d1) - K * dr * norm_cdf(d2)
        return K * dr * norm_cdf(-d2) - S0 * dq * norm_cdf(-d1)

    def _vanilla_black76_greeks_fd(self, dS: float = 1e-4, dSigma: float = 1e-3,
                                   dT: float = 1e-4) -> Dict[str, float]:
        """Bump Greeks of the closed form (:539-593)."""
        S0, s0, T0 = self.S0, self.sigma, self.T
        p0 = self._vanilla_black76_price(S=S0, sigma=s0, T=T0)
        pu = self._vanilla_black76_price(S=S0 + dS, sigma=s0, T=T0)
        pd_ = self._vanilla_black76_price(S=S0 - dS, sigma=s0, T=T0)
        delta = (pu - pd_) / (2.0 * dS)
        gamma = (pu - 2.0 * p0 + pd_) / (dS * dS)
        vega = (self._vanilla_black76_price(S=S0, sigma=s0 + dSigma, T=T0)
                - self._vanilla_black76_price(S=S0, sigma=s0 - dSigma, T=T0)) / (2.0 * dSigma)
        if T0 > 2.0 * dT:
            theta = -((self._vanilla_black76_price(S=S0, sigma=s0, T=T0 + dT)
                       - self._vanilla_black76_price(S=S0, sigma=s0, T=T0 - dT)) / (2.0 * dT))
        else:
            theta = -((p0 - self._vanilla_black76_price(S=S0, sigma=s0,
                                                         T=max(T0 - dT, 1e-8))) / dT)
        return {"price": p0, "delta": delta, "gamma": gamma, "theta": theta, "vega": vega}

    # -------------------------------------------------------------- PDE greeks
    def _pde_price_and_greeks(self, apply_KO: bool, dv_sigma: float) -> Dict[str, float]:
        """Base, sigma+dv and sigma-dv solves in one launch (:429-466)."""
        s0 = self.sigma
        solves = [self._make_solve(apply_KO, s0), self._make_solve(apply_KO, s0 + dv_sigma),
                  self._make_solve(apply_KO, s0 - dv_sigma)]
        eng = self._engine()
        if eng.on_device:
            # the three grids are one grid (configure_grid does not depend on
            # sigma once N is set): read it on the device, 6 numbers come back
            s = self.s_nodes
            with Session() as S:
                sl = eng.march_slots(S, solves)
                rb = readout(int(sl[0]), s, self.S0, self.S0, dg_mode=1)
                ru, rd = readout(int(sl[1]), s, self.S0), readout(int(sl[2]), s, self.S0)
                o = S.greeks([(GK_CNLOG, [rb, ru, rd],
                               (s0, self.S0, self.b_carry, self.r_disc, dv_sigma))])[0]
            return {"price": float(o[0]), "delta": float(o[1]), "gamma": float(o[2]),
                    "theta": float(o[4]), "vega": float(o[3])}
        V, Vu, Vd = eng.run(solves)
        price = self._interp_price_from_grid(V)
        delta, gamma = self._delta_gamma_from_grid(V)
        theta = -(0.5 * s0 * s0 * self.S0 * self.S0 * gamma + self.b_carry * self.S0 * delta
                  - self.r_disc * price)
        vega = (self._interp_price_from_grid(Vu) - self._interp_price_from_grid(Vd)) / (
            2.0 * dv_sigma)
        return {"price": price, "delta": delta, "gamma": gamma, "theta": theta, "vega": vega}

    # ----------------------------------------------------------------- public
    def price(self) -> float:
        bt = self.barrier_type.lower()
        if bt == "none":
            return self._vanilla_bs_price_and_greeks()["price"]
        if bt in ("down-and-out", "up-and-out"):
            return self._pde_price_and_greeks(True, 1e-3)["price"]
        if bt in ("down-and-in", "up-and-in"):
            g_van = self._vanilla_bs_price_and_greeks()
            self.barrier_type = "down-and-out" if bt == "down-and-in" else "up-and-out"
            try:
                g_ko = self._pde_price_and_greeks(True, 1e-3)
            finally:
                self.barrier_type = bt
            return g_van["price"] - g_ko["price"]
        raise ValueError(f"Unsupported barrier_type: {self.barrier_type}")

    def greeks(self, dv_sigma: float = 1e-3) -> Dict[str, float]:
        bt = self.barrier_type.lower()
        fd = dict(dS=max(1e-4, 1e-4 * self.S0), dSigma=dv_sigma, dT=min(1e-4, 0.5 * self.T))
        if bt == "none":
            return self._vanilla_black76_greeks_fd(**fd)
        if bt in ("down-and-out", "up-and-out"):
            return self._pde_price_and_greeks(True, dv_sigma)
        if bt in ("down-and-in", "up-and-in"):
            self.barrier_type = "none"
            g_van = self._vanilla_black76_greeks_fd(**fd)
            self.barrier_type = "down-and-out" if bt == "down-and-in" else "up-and-out"
            try:
                g_ko = self._pde_price_and_greeks(True, dv_sigma)
            finally:
                self.barrier_type = bt
            return {k: g_van[k] - g_ko[k] for k in g_van}
        raise ValueError(f"Unsupported barrier_type: {self.barrier_type}")
