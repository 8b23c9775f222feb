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

from .engine import Engine, VcSolve, default_engine

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
        if self.barrier_lower:
            anchors.append(self.barrier_lower)
        if self.barrier_upper:
            anchors.append(self.barrier_upper)
        s_ref = max(anchors)
        s_max = 4.0 * s_ref * math.exp(self.volatility * math.sqrt(max(self.tenor_years, 1e-12)))
        s_min = 0.0
        N = max(200, int(self.num_space_nodes))
        dS = (s_max - s_min) / N
        nodes = [s_min + i * dS for i in range(N + 1)]

        def snap(x: Optional[float]):
            if x is None:
                return
            j = min(range(len(nodes)), key=lambda i: abs(nodes[i] - x))
            nodes[j] = float(x)

        snap(self.strike_price)
        snap(self.barrier_lower)
        snap(self.barrier_upper)
        return nodes

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

    def _terminal_payoff_scalar(self, S: float) -> float:
        if self.option_type == "call":
            return max(S - self.strike_price, 0.0)
        return max(self.strike_price - S, 0.0)

    def _terminal_payoff_array(self, s_nodes: List[float]) -> List[float]:
        V = [self._terminal_payoff_scalar(S) for S in s_nodes]
        if not self.smooth_payoff_around_strike or self.payoff_smoothing_half_width_nodes <= 0:
            return V
        m = self.payoff_smoothing_half_width_nodes
        k_star = min(range(len(s_nodes)), key=lambda i: abs(s_nodes[i] - self.strike_price))
        i0, i1 = max(0, k_star - m), min(len(s_nodes) - 1, k_star + m)
        S0, V0 = s_nodes[i0], V[i0]
        S1, V1 = s_nodes[i1], V[i1]
        a = (V1 - V0) / ((S1 - S0) ** 2) if S1 != S0 else 0.0
        for i in range(i0, i1 + 1):
            V[i] = a * (s_nodes[i] - S0) ** 2 + V0
        return V

    def _effective_barriers_for_pricing(self) -> Tuple[Optional[float], Optional[float]]:
        if self.use_bgk_correction:
            return self.bgk_lower, self.bgk_upper
        return self.barrier_lower, self.barrier_upper

    def _locate_barrier_interval(self, s_nodes: List[float], lo_bar: Optional[float],
                                 up_bar: Optional[float]):
        """(side, j, h_minus, h_plus) of the active knock-out barrier (:307-331)."""
        N = len(s_nodes) - 1
        for side, kinds, H in (("down", ("down-and-out", "double-out"), lo_bar),
                               ("up", ("up-and-out", "double-out"), up_bar)):
            if self.barrier_type in kinds and H is not None:
                if H <= s_nodes[0]:
                    return (side, 0, 1e-12, s_nodes[1] - s_nodes[0])
                if H >= s_nodes[-1]:
                    return (side, N - 1, s_nodes[N - 1] - s_nodes[N - 2], 1e-12)
                j = max(0, min(N - 1, next(k for k in range(N)
                                           if s_nodes[k] <= H <= s_nodes[k + 1])))
                return (side, j, max(1e-12, H - s_nodes[j]), max(1e-12, s_nodes[j + 1] - H))
        return (None, None, None, None)

    def _ko_nodes(self, s_nodes: List[float], lo_bar, up_bar) -> Tuple[int, int]:
        """Integer thresholds equivalent to _apply_knockout_projection's
        compares (:254-268) on the non-decreasing escrowed grid."""
        s = np.asarray(s_nodes, dtype=np.float64)
        ko_lo, ko_hi = -1, len(s_nodes)
        if self.barrier_type in ("down-and-out", "double-out") and lo_bar is not None:
            ko_lo = int(np.searchsorted(s, lo_bar, side="right")) - 1
        if self.barrier_type in ("up-and-out", "double-out") and up_bar is not None:
            ko_hi = int(np.searchsorted(s, up_bar, side="left"))
        return ko_lo, ko_hi

    def _apply_knockout_projection(self, values: List[float], lo_bar: Optional[float],
                                   up_bar: Optional[float], s_nodes: List[float]) -> None:
        """Host form of the projection (the kernel applies it in the march)."""
        lo, hi = self._ko_nodes(s_nodes, lo_bar, up_bar)
        for i in range(len(s_nodes)):
            if i <= lo or i >= hi:
                values[i] = 0.0

    # ------------------------------------------------------------------ rows
    def _rows(self, theta: float, s_nodes: List[float], side, j_bar, h_minus, h_plus) -> np.ndarray:
        """sub, main, sup, a_expl, b_expl, c_expl of every row for one theta,
        with the reference's expressions and operation order (:354-417)."""
        N = len(s_nodes) - 1
        dt, r, sig = self.dt, self.r_flat, self.volatility
        dS = s_nodes[1] - s_nodes[0]
        sgn = 1.0 if self.explicit_sign == "corrected" else -1.0
        D = np.zeros((6, N + 1))
        D[1, 0] = 1.0
        D[1, N] = 1.0
        for i in range(1, N):
            S = s_nodes[i]
            sig2S2 = (sig * S) ** 2
            if side is None or i not in (j_bar, j_bar + 1):
                a_impl = 0.5 * dt * theta * (sig2S2 / (dS ** 2) - r * S / dS)
                b_impl = 1.0 + dt * theta * (sig2S2 / (dS ** 2) + r)
                c_impl = 0.5 * dt * theta * (sig2S2 / (dS ** 2) + r * S / dS)
                a_expl = sgn * 0.5 * dt * (1 - theta) * (sig2S2 / (dS ** 2) - r * S / dS)
                b_expl = 1.0 - dt * (1 - theta) * (sig2S2 / (dS ** 2) + r)
                c_expl = sgn * 0.5 * dt * (1 - theta) * (sig2S2 / (dS ** 2) + r * S / dS)
            else:
                hm = float(h_minus)
                hp = float(h_plus)
                a1 = hp / (hm * (hm + hp))
                b1 = (hp - hm) / (hm * hp)
                c1 = -hm / (hp * (hm + hp))
                d2 = 2.0 / (hm * (hm + hp))
                e2 = -2.0 / (hm * hp)
                f2 = 2.0 / (hp * (hm + hp))
                L_left = 0.5 * sig2S2 * f2 + r * S * c1
                L_center = 0.5 * sig2S2 * e2 + r * S * b1 - r
                L_right = 0.5 * sig2S2 * d2 + r * S * a1
                a_impl = -theta * dt * L_left
                b_impl = 1.0 - theta * dt * L_center
                c_impl = -theta * dt * L_right
                a_expl = (1 - theta) * dt * L_left
                b_expl = 1.0 + (1 - theta) * dt * L_center
                c_expl = (1 - theta) * dt * L_right
            D[0, i], D[1, i], D[2, i] = -a_impl, b_impl, -c_impl
            D[3, i], D[4, i], D[5, i] = a_expl, b_expl, c_expl
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
        bnd = np.zeros((M, 2))
        for k in range(M):
            m = M - k
            tau_left = self.tenor_years - (m - 1) * self.dt
            if self.option_type == "call":
                bnd[k] = (0.0, s_nodes[-1] - self.strike_price * math.exp(-self.r_flat * tau_left))
            else:
                bnd[k] = (self.strike_price * math.exp(-self.r_flat * tau_left), 0.0)
        sv = VcSolve(n_time=M, n_ranna=r_steps, diag=diag, bnd=bnd,
                     v_init=np.asarray(self._terminal_payoff_array(s_nodes), dtype=np.float64))
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
    def _interp_linear(x: float, xs: List[float], ys: List[float]) -> float:
        if x <= xs[0]:
            return float(ys[0])
        if x >= xs[-1]:
            return float(ys[-1])
        lo, hi = 0, len(xs) - 1
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if x < xs[mid]:
                hi = mid
            else:
                lo = mid
        x0, x1 = xs[lo], xs[hi]
        y0, y1 = ys[lo], ys[hi]
        w = (x - x0) / (x1 - x0)
        return float((1 - w) * y0 + w * y1)

    # ----------------------------------------------------------- public API
    def _grid_solves(self) -> Tuple[List[float], float, List[VcSolve]]:
        pv_divs = self._pv_dividends_escrow()
        S_eff = self.spot_price - pv_divs
        S_shifted = [max(s - pv_divs, 0.0) for s in self.S_nodes]
        lo_eff, up_eff = self._effective_barriers_for_pricing()
        mp = self._monitoring_step_map()
        solves = [self._solve(lo_eff, up_eff, mp, S_shifted)]
        if self.barrier_type in ("down-and-in", "up-and-in", "double-in"):
            solves.append(self._solve(None, None, {}, S_shifted))
        return S_shifted, S_eff, solves

    @staticmethod
    def _combine(barrier_type: str, res: List[np.ndarray]) -> List[float]:
        V = res[0].tolist()
        if barrier_type in ("down-and-in", "up-and-in", "double-in"):
            Vv = res[1].tolist()
            V = [Vv[i] - V[i] for i in range(len(V))]
        return V

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
        iS = max(1, min(N - 1, min(range(N), key=lambda k: abs(S_eff - s_nodes[k]))))
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
