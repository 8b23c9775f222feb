"""Discrete barrier on a uniform spot grid with the FIS barrier treatment.

Drop-in for ``DiscreteBarrierFDMPricer2`` (discrete_barrier_fdm_pricer_2.py:
16-591): same constructor keywords, same ``price`` / ``greeks`` /
``print_details``, same numerics -- uniform S grid with strike and barriers
snapped to nodes (:146-167), the FIS n_lim decision and BGK-shifted
continuous window (:172-226), the smoothed payoff (:231-249), the
non-symmetric rows next to the barrier (:307-331, :387-412), PV-escrowed
dividends, knock-ins as vanilla minus knock-out (:467-481), the FIS Greeks
stencils (:488-564).

What changes is the march (:336-428).  Every row of the theta-scheme
matrices differs (sigma^2 S_i^2 terms), so the rows of both phases
(Rannacher, Crank-Nicolson) are built here, on the host, with the
reference's expressions and order, and the time loop runs in
``fdcn_vc_batch`` (csrc/fdcn_vc.hip): LU factors once per phase, the
stencil and both sweeps in registers.

Deviation switch, ``explicit_sign``: the reference builds the explicit
off-diagonals with the wrong sign (``a_expl = -0.5 dt (1-theta)(...)`` where
``B = I + (1-theta) dt L`` needs ``+``, :383-385), so its Crank-Nicolson
steps amplify instead of smoothing and prices blow up (3e168 for a 300 x 300
vanilla).  "reference" (the default) keeps that for drop-in parity;
"corrected" uses ``+`` and prices converge to Black-Scholes (tests).
"""
from __future__ import annotations

import math
from datetime import date
from typing import Dict, List, Literal, Optional, Tuple

import numpy as np

from . import capi
from .engine import Engine, VcSolve, default_engine

# ---------------------------------------------------------------------------
# vectorised spot-grid helpers, shared with spot_barrier_analytic.py.  Every
# elementwise expression keeps the reference's operand order, and Python's
# float ** 2 / math.exp become libm pow / exp (capi.vmath), so the arrays are
# bit-identical to the reference's list comprehensions (tests).
# ---------------------------------------------------------------------------
def _sq(x) -> np.ndarray:
    """x ** 2 as CPython evaluates it (libm pow, not x * x)."""
    x = np.asarray(x, np.float64)
    return capi.vmath(capi.VM_SQUARE, x).reshape(x.shape)


def nearest_node(nodes: np.ndarray, x: float) -> int:
    """min(range(len(nodes)), key=lambda i: abs(nodes[i] - x)): first minimiser."""
    return int(np.argmin(np.abs(nodes - x)))


def uniform_spot_grid(s_max: float, n: int, snap=()) -> np.ndarray:
    """s_min = 0 + i dS, i = 0..n, then each anchor in `snap` (None skipped)
    written over its nearest node, in order."""
    dS = (s_max - 0.0) / n
    nodes = 0.0 + np.arange(n + 1, dtype=np.float64) * dS
    for x in snap:
        if x is not None:
            nodes[nearest_node(nodes, x)] = float(x)
    return nodes


def smoothed_payoff(s: np.ndarray, strike: float, call: bool, half_width: int,
                    keep_if_flat: bool) -> np.ndarray:
    """Terminal payoff max(S - K, 0) / max(K - S, 0) with the quadratic
    mollifier over the 2 half_width + 1 nodes around the strike node.  A
    degenerate window (S1 == S0) leaves the payoff when keep_if_flat,
    flattens it to V0 otherwise (the two reference pricers differ there)."""
    e = s - strike if call else strike - s
    V = np.where(0.0 > e, 0.0, e)  # Python max(e, 0.0)
    if half_width <= 0:
        return V
    k = nearest_node(s, strike)
    i0, i1 = max(0, k - half_width), min(len(s) - 1, k + half_width)
    S0, V0, S1, V1 = float(s[i0]), float(V[i0]), float(s[i1]), float(V[i1])
    if S1 != S0:
        a = (V1 - V0) / float(_sq(S1 - S0))
    elif keep_if_flat:
        return V
    else:
        a = 0.0
    V[i0:i1 + 1] = a * _sq(s[i0:i1 + 1] - S0) + V0
    return V


def theta_rows(s: np.ndarray, sig2S2: np.ndarray, dt: float, theta: float, r: float,
               drift: float, explicit_sign: float) -> np.ndarray:
    """[6, N+1] = sub, main, sup of A = I - theta dt L and a, b, c of the
    explicit operator for interior rows 1..N-1 (rows 0 and N: the Dirichlet
    identity), L the spot-space Black-Scholes operator with drift `drift`:
      a = +-0.5 dt (1-theta) (sig2S2/dS^2 - drift S/dS), b = 1 - dt (1-theta) (sig2S2/dS^2 + r)
    (discrete_barrier_fdm_pricer_2.py:354-417, discrete_barrier_analytic_pricer.py
    :408-423); explicit_sign -1 is the reference's sign."""
    N = len(s) - 1
    dS = float(s[1] - s[0])
    S = s[1:N]
    x = sig2S2 / (dS ** 2)
    y = drift * S / dS
    D = np.zeros((6, N + 1))
    D[1, 0] = D[1, N] = 1.0
    D[0, 1:N] = -(0.5 * dt * theta * (x - y))
    D[1, 1:N] = 1.0 + dt * theta * (x + r)
    D[2, 1:N] = -(0.5 * dt * theta * (x + y))
    D[3, 1:N] = explicit_sign * 0.5 * dt * (1 - theta) * (x - y)
    D[4, 1:N] = 1.0 - dt * (1 - theta) * (x + r)
    D[5, 1:N] = explicit_sign * 0.5 * dt * (1 - theta) * (x + y)
    return D


def interp_linear(x: float, xs: np.ndarray, ys) -> float:
    """Clamped linear interpolation on a non-decreasing grid (the reference's
    bisection: the bracket is [j, j+1] with j the last node <= x)."""
    if x <= xs[0]:
        return float(ys[0])
    if x >= xs[-1]:
        return float(ys[-1])
    lo = int(np.searchsorted(xs, x, side="right")) - 1
    x0, x1 = float(xs[lo]), float(xs[lo + 1])
    y0, y1 = float(ys[lo]), float(ys[lo + 1])
    w = (x - x0) / (x1 - x0)
    return float((1 - w) * y0 + w * y1)


def ko_thresholds(s: np.ndarray, barrier_type: str, lo_bar, up_bar) -> Tuple[int, int]:
    """Integer thresholds (KO_LO, KO_HI) of the knock-out projection's
    compares S <= lo_bar / S >= up_bar on the grid s (a non-decreasing
    grid: every knocked-out node lies at or below KO_LO / at or above KO_HI;
    checked)."""
    n = len(s)
    ko_lo, ko_hi = -1, n
    if barrier_type in ("down-and-out", "double-out") and lo_bar is not None:
        hit = s <= lo_bar
        ko_lo = int(np.nonzero(hit)[0][-1]) if hit.any() else -1
        if not hit[:ko_lo + 1].all():
            raise ValueError("knock-out nodes are not a prefix of the grid")
    if barrier_type in ("up-and-out", "double-out") and up_bar is not None:
        hit = s >= up_bar
        ko_hi = int(np.nonzero(hit)[0][0]) if hit.any() else n
        if not hit[ko_hi:].all():
            raise ValueError("knock-out nodes are not a suffix of the grid")
    return ko_lo, ko_hi



BarrierType = Literal["none", "down-and-out", "up-and-out", "double-out", "down-and-in",
                      "up-and-in", "double-in"]
OptionType = Literal["call", "put"]


class DiscreteBarrierFDMPricer2:
    """European discrete barrier, CN + Rannacher on a uniform S grid (FIS)."""

    BGK_BETA = 0.5826
    N_LIM = 5
    MIN_INTERVAL_STEPS = 1
    DEFAULT_DAYCOUNT = "ACT/365"

    def __init__(
        self,
        spot: float,
        strike: float,
        valuation_date: date,
        maturity_date: date,
        volatility: float,
        option_type: OptionType,
        barrier_type: BarrierType = "none",
        lower_barrier: Optional[float] = None,
        upper_barrier: Optional[float] = None,
        monitoring_dates: Optional[List[date]] = None,
        flat_rate_nacc: float = 0.0,
        dividends: Optional[List[Tuple[date, float]]] = None,
        num_space_nodes: int = 600,
        num_time_steps: int = 600,
        rannacher_steps: int = 2,
        day_count: str = DEFAULT_DAYCOUNT,
        smooth_payoff_around_strike: bool = True,
        payoff_smoothing_half_width_nodes: int = 2,
        explicit_sign: Literal["reference", "corrected"] = "reference",
        engine: Optional[Engine] = None,
    ):
        self.spot_price = float(spot)
        self.strike_price = float(strike)
        self.valuation_date = valuation_date
        self.maturity_date = maturity_date
        self.option_type = option_type
        self.barrier_type = barrier_type
        self.barrier_lower = lower_barrier
        self.barrier_upper = upper_barrier
        self.monitoring_dates = sorted(monitoring_dates or [])
        self.volatility = float(volatility)
        self.r_flat = float(flat_rate_nacc)
        self.day_count = day_count.upper()
        self.dividends = [(d, float(a)) for (d, a) in (dividends or [])]
        self.num_space_nodes = int(num_space_nodes)
        self.num_time_steps = int(num_time_steps)
        self.rannacher_steps = int(rannacher_steps)
        self.smooth_payoff_around_strike = bool(smooth_payoff_around_strike)
        self.payoff_smoothing_half_width_nodes = int(payoff_smoothing_half_width_nodes)
        if explicit_sign not in ("reference", "corrected"):
            raise ValueError("explicit_sign must be 'reference' or 'corrected'")
        self.explicit_sign = explicit_sign
        self.engine = engine

        self.year_fraction = self._year_fraction
        self.tenor_years = self.year_fraction(self.valuation_date, self.maturity_date)
        self.dt = self.tenor_years / max(1, self.num_time_steps)
        self.S_nodes = self._build_space_grid()
        self.dS = self.S_nodes[1] - self.S_nodes[0]
        (self.use_bgk_correction, self.bgk_lower, self.bgk_upper, self.k_first_cont,
         self.k_last_cont) = self._decide_and_adjust_for_continuous_window()

    # ------------------------------------------------------------ utilities
    def _year_fraction(self, d0: date, d1: date) -> float:
        if self.day_count in ("ACT/365", "ACT/365F", "ACT/365 FIXED"):
            return max(0, (d1 - d0).days) / 365.0
        if self.day_count in ("ACT/360",):
            return max(0, (d1 - d0).days) / 360.0
        if self.day_count in ("30/360", "30E/360"):
            y0, m0, dd0 = d0.year, d0.month, min(d0.day, 30)
            y1, m1, dd1 = d1.year, d1.month, min(d1.day, 30)
            return ((y1 - y0) * 360 + (m1 - m0) * 30 + (dd1 - dd0)) / 360.0
        return max(0, (d1 - d0).days) / 365.0

    def _pv_dividends_escrow(self) -> float:
        if not self.dividends:
            return 0.0
        pv = 0.0
        for (pay_date, amount) in self.dividends:
            tau = self.year_fraction(self.valuation_date, pay_date)
            if tau > 0:
                pv += amount * math.exp(-self.r_flat * tau)
        return pv

    def _build_space_grid(self) -> List[float]:
        """[0, 4 s_ref e^{sigma sqrt T}], N = max(200, num_space_nodes), K and
        the barriers snapped to their nearest nodes (:146-167)."""
        anchors = [self.spot_price, self.strike_price]
        anchors += [b for b in (self.barrier_lower, self.barrier_upper) if b]
        s_max = 4.0 * max(anchors) * math.exp(self.volatility *
                                              math.sqrt(max(self.tenor_years, 1e-12)))
        return uniform_spot_grid(s_max, max(200, int(self.num_space_nodes)),
                                 (self.strike_price, self.barrier_lower,
                                  self.barrier_upper)).tolist()

    def _decide_and_adjust_for_continuous_window(self):
        """FIS n_lim decision and BGK shift (:172-226)."""
        if self.barrier_type == "none" or len(self.monitoring_dates) == 0:
            return (False, self.barrier_lower, self.barrier_upper, None, None)
        first_mon = min(self.monitoring_dates)
        last_mon = max(self.monitoring_dates)
        if last_mon <= first_mon:
            return (False, self.barrier_lower, self.barrier_upper, None, None)
        sorted_mons = [d for d in self.monitoring_dates
                       if self.valuation_date < d <= self.maturity_date]
        if len(sorted_mons) == 0:
            return (False, self.barrier_lower, self.barrier_upper, None, None)
        dt_uniform = self.tenor_years / max(1, self.num_time_steps)
        intervals = [self.year_fraction(sorted_mons[i - 1], sorted_mons[i])
                     for i in range(1, len(sorted_mons))]
        N_hat = sum(max(self.MIN_INTERVAL_STEPS, int(round(ti / dt_uniform))) for ti in intervals)
        frequent_enough = (N_hat > self.N_LIM * self.num_time_steps)
        num_mon = len(sorted_mons)
        t_b = self.year_fraction(first_mon, last_mon)
        a_b = (t_b / max(1, num_mon))
        phi = self.BGK_BETA * self.volatility * a_b
        adj = math.exp(phi)
        lo_adj = self.barrier_lower
        up_adj = self.barrier_upper
        if self.barrier_lower is not None:
            lo_adj = self.barrier_lower / adj
        if self.barrier_upper is not None:
            up_adj = self.barrier_upper * adj
        k0 = int(round(self.year_fraction(self.valuation_date, first_mon) / self.dt))
        k1 = int(round(self.year_fraction(self.valuation_date, last_mon) / self.dt))
        k0 = max(0, min(self.num_time_steps, k0))
        k1 = max(0, min(self.num_time_steps, k1))
        return (frequent_enough, lo_adj, up_adj, min(k0, k1), max(k0, k1))

    def _terminal_payoff_array(self, s_nodes) -> np.ndarray:
        """Payoff with the strike mollifier (:231-249)."""
        m = self.payoff_smoothing_half_width_nodes if self.smooth_payoff_around_strike else 0
        return smoothed_payoff(np.asarray(s_nodes, np.float64), self.strike_price,
                               self.option_type == "call", m, keep_if_flat=False)

    def _effective_barriers_for_pricing(self) -> Tuple[Optional[float], Optional[float]]:
        if self.use_bgk_correction:
            return self.bgk_lower, self.bgk_upper
        return self.barrier_lower, self.barrier_upper

    def _locate_barrier_interval(self, s_nodes, lo_bar: Optional[float],
                                 up_bar: Optional[float]):
        """(side, j, h_minus, h_plus) of the active knock-out barrier (:307-331)."""
        s = np.asarray(s_nodes, np.float64)
        N = len(s) - 1
        for side, kinds, H in (("down", ("down-and-out", "double-out"), lo_bar),
                               ("up", ("up-and-out", "double-out"), up_bar)):
            if self.barrier_type in kinds and H is not None:
                if H <= s[0]:
                    return (side, 0, 1e-12, float(s[1] - s[0]))
                if H >= s[-1]:
                    return (side, N - 1, float(s[N - 1] - s[N - 2]), 1e-12)
                j = int(np.argmax((s[:-1] <= H) & (H <= s[1:])))  # first bracketing interval
                return (side, j, max(1e-12, H - float(s[j])), max(1e-12, float(s[j + 1]) - H))
        return (None, None, None, None)

    def _ko_nodes(self, s_nodes, lo_bar, up_bar) -> Tuple[int, int]:
        """Integer thresholds equivalent to _apply_knockout_projection's
        compares (:254-268)."""
        return ko_thresholds(np.asarray(s_nodes, np.float64), self.barrier_type, lo_bar, up_bar)

    def _apply_knockout_projection(self, values: List[float], lo_bar: Optional[float],
                                   up_bar: Optional[float], s_nodes: List[float]) -> None:
        """Host form of the projection (the kernel applies it in the march)."""
        lo, hi = self._ko_nodes(s_nodes, lo_bar, up_bar)
        for i in list(range(lo + 1)) + list(range(hi, len(s_nodes))):
            values[i] = 0.0

    # ------------------------------------------------------------------ rows
    def _rows(self, theta: float, s_nodes, side, j_bar, h_minus, h_plus) -> np.ndarray:
        """sub, main, sup, a_expl, b_expl, c_expl of every row for one theta
        (:354-417): the uniform rows vectorised (theta_rows), then the two
        non-symmetric rows beside the barrier from its one-sided
        three-point stencil."""
        s = np.asarray(s_nodes, np.float64)
        N = len(s) - 1
        dt, r, sig = self.dt, self.r_flat, self.volatility
        sgn = 1.0 if self.explicit_sign == "corrected" else -1.0
        D = theta_rows(s, _sq(sig * s[1:N]), dt, theta, r, r, sgn)
        if side is not None:
            hm, hp = float(h_minus), float(h_plus)
            a1 = hp / (hm * (hm + hp))
            b1 = (hp - hm) / (hm * hp)
            c1 = -hm / (hp * (hm + hp))
            d2 = 2.0 / (hm * (hm + hp))
            e2 = -2.0 / (hm * hp)
            f2 = 2.0 / (hp * (hm + hp))
            for i in (j_bar, j_bar + 1):
                if not 1 <= i <= N - 1:
                    continue
                S = float(s[i])
                sig2S2 = float(_sq(sig * S))
                L_left = 0.5 * sig2S2 * f2 + r * S * c1
                L_center = 0.5 * sig2S2 * e2 + r * S * b1 - r
                L_right = 0.5 * sig2S2 * d2 + r * S * a1
                D[:, i] = (theta * dt * L_left, 1.0 - theta * dt * L_center,
                           theta * dt * L_right, (1 - theta) * dt * L_left,
                           1.0 + (1 - theta) * dt * L_center, (1 - theta) * dt * L_right)
        return D

    def _monitoring_step_map(self) -> Dict[int, bool]:
        mp: Dict[int, bool] = {}
        if self.use_bgk_correction:
            for k in range(self.k_first_cont, self.k_last_cont + 1):
                mp[k] = True
        else:
            for d in self.monitoring_dates:
                if self.valuation_date < d <= self.maturity_date:
                    k = int(round(self.year_fraction(self.valuation_date, d) / self.dt))
                    mp[k] = True
        return mp

    def _solve(self, lo_bar, up_bar, monitor_step_index: Dict[int, bool],
               s_nodes: List[float]) -> VcSolve:
        """The work of one _solve_pde_backward call (:336-428) as a kernel
        scenario.  The reference marches m = M..1 with theta = 1 while
        M - m < rannacher_steps; march step k = M - m.  Its Dirichlet rows
        take tau_left = T - (m-1) dt; the projection after step m happens when
        m - 1 is in the monitoring map, i.e. after march step M - (m-1)."""
        M = self.num_time_steps
        side, j_bar, h_minus, h_plus = self._locate_barrier_interval(s_nodes, lo_bar, up_bar)
        r_steps = min(self.rannacher_steps, M)
        diag = np.stack([self._rows(1.0, s_nodes, side, j_bar, h_minus, h_plus),
                         self._rows(0.5, s_nodes, side, j_bar, h_minus, h_plus)])
        # Dirichlet rows at tau_left = T - (m - 1) dt, m = M - k
        tau_left = self.tenor_years - (M - np.arange(M) - 1).astype(np.float64) * self.dt
        disc_K = self.strike_price * capi.vmath(capi.VM_EXP, -self.r_flat * tau_left)
        bnd = np.zeros((M, 2))
        if self.option_type == "call":
            bnd[:, 1] = s_nodes[-1] - disc_K
        else:
            bnd[:, 0] = disc_K
        sv = VcSolve(n_time=M, n_ranna=r_steps, diag=diag, bnd=bnd,
                     v_init=self._terminal_payoff_array(s_nodes))
        if monitor_step_index:
            steps = sorted(M - q for q in monitor_step_index if 0 <= q <= M - 1)
            if steps:
                sv.ko_lo, sv.ko_hi = self._ko_nodes(s_nodes, lo_bar, up_bar)
                sv.mon_steps = steps
                sv.mon_rebates = [0.0] * len(steps)
        return sv

    def _engine(self) -> Engine:
        return self.engine if self.engine is not None else default_engine()

    def _solve_pde_backward(self, lo_bar, up_bar, monitor_step_index, s_nodes) -> List[float]:
        return self._engine().run_vc([self._solve(lo_bar, up_bar, monitor_step_index,
                                                  s_nodes)])[0].tolist()

    @staticmethod
    def _interp_linear(x: float, xs, ys) -> float:
        return interp_linear(x, np.asarray(xs, np.float64), ys)

    # ----------------------------------------------------------- public API
    def _grid_solves(self) -> Tuple[List[float], float, List[VcSolve]]:
        pv_divs = self._pv_dividends_escrow()
        S_eff = self.spot_price - pv_divs
        e = np.asarray(self.S_nodes, np.float64) - pv_divs
        S_shifted = np.where(0.0 > e, 0.0, e).tolist()  # max(s - pv, 0.0)
        lo_eff, up_eff = self._effective_barriers_for_pricing()
        mp = self._monitoring_step_map()
        solves = [self._solve(lo_eff, up_eff, mp, S_shifted)]
        if self.barrier_type in ("down-and-in", "up-and-in", "double-in"):
            solves.append(self._solve(None, None, {}, S_shifted))
        return S_shifted, S_eff, solves

    @staticmethod
    def _combine(barrier_type: str, res: List[np.ndarray]) -> List[float]:
        if barrier_type in ("down-and-in", "up-and-in", "double-in"):
            return (res[1] - res[0]).tolist()  # vanilla - knock-out
        return res[0].tolist()

    def _solve_grid_once(self) -> Tuple[List[float], List[float], float]:
        """(S_grid_shifted, V_grid, effective spot) (:467-481)."""
        Sg, S_eff, solves = self._grid_solves()
        return Sg, self._combine(self.barrier_type, self._engine().run_vc(solves)), S_eff

    def price(self) -> float:
        Sg, Vg, S_eff = self._solve_grid_once()
        return self._interp_linear(S_eff, Sg, Vg)

    def _delta_gamma_from_grid(self, s_nodes: List[float], V: List[float], S_eff: float,
                               lo_bar: Optional[float], up_bar: Optional[float]):
        """FIS Greeks stencils (:488-550)."""
        N = len(s_nodes) - 1
        dS = s_nodes[1] - s_nodes[0]
        iS = max(1, min(N - 1, nearest_node(np.asarray(s_nodes[:N], np.float64), S_eff)))
        delta_c = (V[iS + 1] - V[iS - 1]) / (2.0 * dS)
        gamma_c = (V[iS + 1] - 2.0 * V[iS] + V[iS - 1]) / (dS * dS)
        side, j_bar, h_minus, h_plus = self._locate_barrier_interval(s_nodes, lo_bar, up_bar)
        if side is None or j_bar is None:
            return float(delta_c), float(gamma_c)
        in_first = (iS == j_bar or iS == j_bar + 1)
        in_second = (iS == j_bar - 1 or iS == j_bar + 2)
        if in_first:
            if side == "down":
                i = j_bar + 1
                delta_os = (1.5 * V[i] - 2.0 * V[i - 1] + 0.5 * V[min(N, i + 1)]) / dS
            else:
                i = j_bar
                delta_os = (2.0 * V[i + 1] - 1.5 * V[i] - 0.5 * V[max(0, i - 1)]) / dS
            S_bar = s_nodes[i]
            sig = self.volatility
            r = self.r_flat
            g = 0.0
            gamma_ns = (V[i + 1] - 2.0 * V[i] + V[i - 1]) / (dS * dS)
            denom = max(1e-14, (sig * sig) * S_bar * S_bar)
            gamma_lim = 2.0 * (r * V[i] - g * S_bar * delta_os) / denom
            q = 0.5
            gamma = q * gamma_ns + (1.0 - q) * gamma_lim
            return float(delta_os), float(gamma)
        if in_second:
            if side == "down":
                delta_os = (1.5 * V[iS] - 2.0 * V[iS - 1] + 0.5 * V[min(N, iS + 1)]) / dS
            else:
                delta_os = (2.0 * V[iS + 1] - 1.5 * V[iS] - 0.5 * V[max(0, iS - 1)]) / dS
            gamma_os = (V[iS + 1] - 2.0 * V[iS] + V[iS - 1]) / (dS * dS)
            alpha = 0.5
            return float(alpha * delta_os + (1 - alpha) * delta_c), \
                float(alpha * gamma_os + (1 - alpha) * gamma_c)
        return float(delta_c), float(gamma_c)

    def greeks(self, vega_bump: float = 0.01) -> Dict[str, float]:
        """Delta/Gamma from the grid, vega by +-vega_bump repricing (:552-564);
        the base and both bumped grids march in one launch."""
        lo_eff, up_eff = self._effective_barriers_for_pricing()
        sig0 = self.volatility
        batches = []
        try:
            for sig in (sig0, sig0 + vega_bump, sig0 - vega_bump):
                self.volatility = sig
                batches.append(self._grid_solves())
        finally:
            self.volatility = sig0
        flat = [sv for _, _, sv in batches for sv in sv]
        res = self._engine().run_vc(flat)
        out, pos = [], 0
        for Sg, S_eff, sv in batches:
            out.append((Sg, S_eff, self._combine(self.barrier_type, res[pos:pos + len(sv)])))
            pos += len(sv)
        (Sg, S_eff, Vg), (Su, Su_eff, Vu), (Sd, Sd_eff, Vd) = out
        delta, gamma = self._delta_gamma_from_grid(Sg, Vg, S_eff, lo_eff, up_eff)
        upv = self._interp_linear(Su_eff, Su, Vu)
        dnv = self._interp_linear(Sd_eff, Sd, Vd)
        vega = (upv - dnv) / (2.0 * vega_bump)
        return {"delta": float(delta), "gamma": float(gamma), "vega": float(vega)}

    def print_details(self) -> None:
        lo_eff, up_eff = self._effective_barriers_for_pricing()
        price = self.price()
        greeks = self.greeks()
        print("==== Discrete Barrier Option (FD + CN, Rannacher) ====")
        print(f"Maturity Date           : {self.maturity_date.isoformat()}")
        print(f"T (years)               : {self.tenor_years:.9f}   [{self.day_count}]")
        print(f"Volatility (sigma)      : {self.volatility:.9f}")
        print(f"Flat r (NACC)           : {self.r_flat:.9f}")
        print(f"PV(dividends, escrow)   : {self._pv_dividends_escrow():.9f}")
        print("")
        print(f"Barrier type            : {self.barrier_type}")
        print(f"KO lower / upper        : {self.barrier_lower} / {self.barrier_upper}")
        print(f"BGK lower / upper       : {self.bgk_lower} / {self.bgk_upper}")
        print(f"BGK window steps        : {self.k_first_cont} .. {self.k_last_cont} "
              f"(use_bgk={self.use_bgk_correction})")
        print("")
        print(f"Grid (space,time)       : {self.num_space_nodes}, {self.num_time_steps} "
              f"(Rannacher {self.rannacher_steps})")
        print(f"Spot / Strike           : {self.spot_price:.6f} / {self.strike_price:.6f}")
        print(f"Effective barriers      : {lo_eff} / {up_eff}")
        print("")
        print(f"Price                   : {price:.9f}")
        print(f"Greeks                  : delta={greeks['delta']:.9f}, "
              f"gamma={greeks['gamma']:.9f}, vega={greeks['vega']:.9f}")
