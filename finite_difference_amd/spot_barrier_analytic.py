"""Hybrid analytic / Crank-Nicolson discrete barrier pricer (FIS n_lim rule).

Drop-in for ``DiscreteBarrierFDMPricerAnalytic``
(discrete_barrier_analytic_pricer.py:52-660): same constructor keywords,
``price`` / ``greeks`` / ``print_details``, same numerics:

* flat continuous r from the NACA discount curve at maturity, flat q backed
  out of the PV of the cash dividends (:199-224), spot escrowed by that PV and
  the grid shifted with it (:538-566);
* the FIS decision (:278-342): equidistant dt = T / n, steps per monitoring
  interval max(n_min, round(t_m / dt)), continuous when their sum exceeds
  n_lim n; the continuous window is every step between the first and the last
  monitoring date, with BGK-shifted barriers H exp(+-beta sigma sqrt(avg dt));
* continuous window: the closed-form engines at the shifted barriers
  (:473-519) -- Reiner-Rubinstein for single barriers, the Douady series for
  double barriers -- through the batched GPU engines (fdcn_rr_barrier_batch /
  fdcn_double_barrier_batch); where the reference falls back to its CN overlay
  (barrier status set, a missing shifted barrier, no double-barrier engine),
  the overlay with the projection on EVERY step of the window (:521-529);
* discrete monitoring: the CN overlay with the projection on monitoring steps
  only (:531-536);
* knock-ins: CN vanilla minus the knock-out leg (:547-556).  Two reference
  behaviours are kept for parity: a discrete knock-in's "knock-out leg" gets
  no projection (_apply_knockout_projection only matches the *-out types,
  :347-360, so it prices 0), and a continuous one subtracts the analytic
  KNOCK-IN price (the engine is called with in_out_flag 'i', :500-517);
* Greeks by bump and reprice (:573-616): one-sided Delta near a shifted
  barrier in the continuous window.

The CN overlay (:384-432) is the spot-space theta scheme with per-row
coefficients (sigma^2 S^2 and the carry r - q), so it runs on
``fdcn_vc_batch`` (csrc/fdcn_vc.hip) like ``DiscreteBarrierFDMPricer2``:
rows built vectorised on the host in the reference's operand order, the
march on the GPU.  Every solve of a ``price()`` -- and all of ``greeks()``:
the spot bumps only move the interpolation point, so the five repricings need
at most three distinct grids per leg -- goes out in one launch.

Two switches (not in the reference):
* ``explicit_sign``: the reference's explicit off-diagonals have the wrong
  sign (A_ = -0.5 dt (1-theta)(...), :416-418, as in
  discrete_barrier_fdm_pricer_2.py), so its CN steps amplify; "reference"
  (default) keeps that, "corrected" converges to Black-Scholes.
* ``double_barrier_analytic``: the reference imports ``from double_barrier
  import DoubleBarrier`` (:37-41), but its file is "double _barrier.py", so
  as shipped DoubleBarrier is None and double barriers take the CN overlay.
  False (default) reproduces that; True uses the Douady engine (m = 6) as the
  import intends.
"""
from __future__ import annotations

import math
from typing import Dict, List, Literal, Optional, Tuple

import numpy as np

from . import capi
from .engine import Engine, VcSolve, default_engine
from .spot_barrier import (_sq, interp_linear, ko_thresholds, smoothed_payoff, theta_rows,
                           uniform_spot_grid)

BarrierType = Literal["none", "down-and-out", "up-and-out", "double-out", "down-and-in",
                      "up-and-in", "double-in"]
OptionType = Literal["call", "put"]
KNOCK_INS = ("down-and-in", "up-and-in", "double-in")


def _ts(d):
    import pandas as pd
    return pd.Timestamp(d).normalize()


def _default_valuation():
    import pandas as pd
    return pd.Timestamp.today().normalize()


class DiscreteBarrierFDMPricerAnalytic:
    """See the module docstring."""

    BGK_BETA = 0.5826

    def __init__(
        self,
        trade_id: str,
        direction: Literal["long", "short"],
        quantity: int,
        contract_multiplier: float,
        option_type: OptionType,
        barrier_type: BarrierType,
        strike: float,
        lower_barrier: Optional[float],
        upper_barrier: Optional[float],
        rebate_amount: float = 0.0,
        rebate_timing_in: Optional[str] = None,
        rebate_timing_out: Optional[str] = None,
        barrier_status: Optional[str] = None,
        spot: float = 100.0,
        volatility: float = 0.20,
        valuation_date=None,
        maturity_date=None,
        monitoring_dates: Optional[list] = None,
        discount_curve=None,
        forward_curve=None,
        dividend_schedule: Optional[list] = None,
        day_count: str = "ACT/365",
        time_steps: int = 600,
        space_nodes: int = 600,
        rannacher_steps: int = 2,
        snap_strike_and_barrier: bool = True,
        n_desired_for_decision: int = 400,
        n_min_steps_per_interval: int = 1,
        n_lim_multiplier: int = 5,
        explicit_sign: Literal["reference", "corrected"] = "reference",
        double_barrier_analytic: bool = False,
        engine: Optional[Engine] = None,
    ) -> None:
        import pandas as pd
        if valuation_date is None:
            valuation_date = _default_valuation()
        if maturity_date is None:
            maturity_date = _default_valuation() + pd.Timedelta(days=365)
        if spot <= 0 or strike <= 0 or volatility <= 0:
            raise ValueError("spot, strike, volatility must be positive.")
        if _ts(maturity_date) <= _ts(valuation_date):
            raise ValueError("maturity_date must be after valuation_date.")
        if explicit_sign not in ("reference", "corrected"):
            raise ValueError("explicit_sign must be 'reference' or 'corrected'")
        self.trade_id = trade_id
        self.direction = direction
        self.quantity = int(quantity)
        self.contract_multiplier = float(contract_multiplier)
        self.option_type = option_type
        self.barrier_type = barrier_type
        self.strike = float(strike)
        self.lower_barrier = lower_barrier
        self.upper_barrier = upper_barrier
        self.rebate_amount = float(rebate_amount)
        self.rebate_timing_in = rebate_timing_in
        self.rebate_timing_out = rebate_timing_out
        self.barrier_status = barrier_status
        self.spot = float(spot)
        self.sigma = float(volatility)
        self.valuation_date = _ts(valuation_date)
        self.maturity_date = _ts(maturity_date)
        self.monitoring_dates = sorted(_ts(d) for d in (monitoring_dates or []))
        self.discount_curve = self._curve_table(discount_curve)
        self.forward_curve = self._curve_table(forward_curve)
        self.dividend_schedule = [(_ts(d), float(a)) for d, a in (dividend_schedule or [])]
        self.day_count = day_count.upper()
        self.time_steps = int(time_steps)
        self.space_nodes = int(space_nodes)
        self.rannacher_steps = int(rannacher_steps)
        self.snap_strike_and_barrier = bool(snap_strike_and_barrier)
        self.n_desired_for_decision = int(n_desired_for_decision)
        self.n_min_steps_per_interval = int(n_min_steps_per_interval)
        self.n_lim_multiplier = int(n_lim_multiplier)
        self.explicit_sign = explicit_sign
        self.double_barrier_analytic = bool(double_barrier_analytic)
        self.engine = engine

        self.tenor_years = self._year_fraction(self.valuation_date, self.maturity_date)
        self.flat_rate_r = self._flat_r_from_curve()
        self.flat_dividend_q = self._flat_q_from_dividends()
        self.flat_carry_b = self.flat_rate_r - self.flat_dividend_q
        self.spot_grid = self._build_space_grid()
        self.grid_step_dS = self.spot_grid[1] - self.spot_grid[0]
        (self.use_continuous_window, self.window_k0, self.window_k1, self.bgk_lower_barrier,
         self.bgk_upper_barrier, self.monitor_steps_discrete,
         self.monitor_steps_continuous) = self._monitoring_decision_and_bgk_shift()

    # ------------------------------------------------------------ dates, curves
    def _year_fraction(self, d0, d1) -> float:
        """:173-183."""
        days = max(0, int((_ts(d1) - _ts(d0)).days))
        if self.day_count in ("ACT/365", "ACT/365F", "ACT/365 FIXED"):
            return days / 365.0
        if self.day_count == "ACT/360":
            return days / 360.0
        if self.day_count in ("30/360", "30E/360"):
            y0, m0, dd0 = d0.year, d0.month, min(d0.day, 30)
            y1, m1, dd1 = d1.year, d1.month, min(d1.day, 30)
            return ((y1 - y0) * 360 + (m1 - m0) * 30 + (dd1 - dd0)) / 360.0
        return days / 365.0

    @staticmethod
    def _curve_table(df) -> Optional[Dict[str, float]]:
        """Date string (YYYY-mm-dd) -> NACA, first row per date (the reference
        filters the DataFrame on every lookup and takes values[0])."""
        if df is None:
            return None
        import pandas as pd
        dates = df["Date"]
        if not pd.api.types.is_string_dtype(dates):
            dates = pd.to_datetime(dates).dt.strftime("%Y-%m-%d")
        out: Dict[str, float] = {}
        for d, v in zip(dates.tolist(), df["NACA"].tolist()):
            out.setdefault(d, float(v))
        return out

    def _naca_on(self, d) -> float:
        if self.discount_curve is None:
            return 0.0
        return self.discount_curve.get(_ts(d).strftime("%Y-%m-%d"), 0.0)

    @staticmethod
    def _df_from_naca(naca: float, tau: float) -> float:
        return (1.0 + naca) ** (-tau)

    def _flat_r_from_curve(self) -> float:
        """:199-204."""
        tau = max(1e-12, self.tenor_years)
        df_T = self._df_from_naca(self._naca_on(self.maturity_date), tau)
        return -math.log(max(df_T, 1e-16)) / tau

    def _pv_dividends(self) -> float:
        """:206-215: cash dividends paid in (valuation, maturity]."""
        pv = 0.0
        for pay, amount in self.dividend_schedule:
            if self.valuation_date < pay <= self.maturity_date:
                tau = self._year_fraction(self.valuation_date, pay)
                pv += amount * self._df_from_naca(self._naca_on(pay), tau)
        return pv

    def _flat_q_from_dividends(self) -> float:
        pv = self._pv_dividends()
        if pv <= 0.0:
            return 0.0
        if pv >= self.spot:
            raise ValueError("PV(dividends) >= spot; cannot back out flat dividend yield.")
        return -math.log((self.spot - pv) / self.spot) / max(1e-12, self.tenor_years)

    # ------------------------------------------------------------------ grid
    def _build_space_grid(self) -> List[float]:
        """:229-245."""
        anchors = [self.spot, self.strike]
        anchors += [b for b in (self.lower_barrier, self.upper_barrier) if b]
        s_max = 4.0 * max(anchors) * math.exp(self.sigma * math.sqrt(max(self.tenor_years, 1e-12)))
        snap = (self.strike, self.lower_barrier, self.upper_barrier) \
            if self.snap_strike_and_barrier else ()
        return uniform_spot_grid(s_max, self.space_nodes, snap).tolist()

    # ------------------------------------------------------- FIS n_lim + BGK
    def _monitoring_decision_and_bgk_shift(self):
        """:278-342."""
        if self.barrier_type == "none" or not self.monitoring_dates:
            return (False, None, None, self.lower_barrier, self.upper_barrier, {}, {})
        md = sorted(d for d in self.monitoring_dates
                    if self.valuation_date < d <= self.maturity_date)
        if not md:
            return (False, None, None, self.lower_barrier, self.upper_barrier, {}, {})
        T, M = self.tenor_years, self.time_steps
        dt_eq = T / max(1, self.n_desired_for_decision)
        intervals = [self._year_fraction(a, b) for a, b in zip(md[:-1], md[1:])] \
            or [T / len(md)]
        n_total = sum(max(self.n_min_steps_per_interval, int(round(t / max(1e-12, dt_eq))))
                      for t in intervals)
        cont = n_total > self.n_lim_multiplier * self.n_desired_for_decision

        def slice_of(d) -> int:
            return max(0, min(M, int(round(self._year_fraction(self.valuation_date, d) / (T / M)))))
        discrete = {slice_of(d): True for d in md}
        if not cont:
            return (False, None, None, self.lower_barrier, self.upper_barrier, discrete, {})
        k0, k1 = slice_of(md[0]), slice_of(md[-1])
        lo_k, hi_k = min(k0, k1), max(k0, k1)
        continuous = {k: True for k in range(lo_k, hi_k + 1)}
        adj = math.exp(self.BGK_BETA * self.sigma *
                       math.sqrt(max(1e-12, sum(intervals) / len(intervals))))
        lo = self.lower_barrier / adj if self.lower_barrier is not None else None
        up = self.upper_barrier * adj if self.upper_barrier is not None else None
        return (True, lo_k, hi_k, lo, up, discrete, continuous)

    # -------------------------------------------------------------- CN overlay
    def _cn_solve(self, grid: np.ndarray, sigma: float, eff_lower, eff_upper,
                  monitor_map: Dict[int, bool]) -> VcSolve:
        """One _cn_stepper call (:384-432) as a fdcn_vc scenario.  The
        reference marches m = M..1 (theta = 1 while M - m < rannacher_steps);
        march step k = M - m solves for the slice at tau = T - (m - 1) dt with
        the Dirichlet rows lower/upper(tau), and projects after it when
        m - 1 is a monitored slice."""
        M = self.time_steps
        N = len(grid) - 1
        dt = self.tenor_years / M
        r, q = self.flat_rate_r, self.flat_dividend_q
        sgn = 1.0 if self.explicit_sign == "corrected" else -1.0
        sig2S2 = float(_sq(sigma)) * _sq(grid[1:N])  # (sig ** 2) * (S ** 2)
        diag = np.stack([theta_rows(grid, sig2S2, dt, th, r, r - q, sgn) for th in (1.0, 0.5)])
        tau = self.tenor_years - (M - np.arange(M) - 1).astype(np.float64) * dt
        disc_K = self.strike * capi.vmath(capi.VM_EXP, -r * tau)
        bnd = np.zeros((M, 2))
        if self.option_type == "put":
            bnd[:, 0] = disc_K
        else:
            bnd[:, 1] = grid[-1] * capi.vmath(capi.VM_EXP, -q * tau) - disc_K
        sv = VcSolve(n_time=M, n_ranna=min(self.rannacher_steps, M), diag=diag, bnd=bnd,
                     v_init=smoothed_payoff(grid, self.strike, self.option_type == "call", 2,
                                            keep_if_flat=True))
        steps = sorted(M - k for k in monitor_map if 0 <= k <= M - 1)
        if steps:
            sv.ko_lo, sv.ko_hi = ko_thresholds(grid, self.barrier_type, eff_lower, eff_upper)
            sv.mon_steps = steps
            sv.mon_rebates = [0.0] * len(steps)
        return sv

    # ---------------------------------------------------------- analytic legs
    def _single_barrier_analytic_ok(self) -> bool:
        """:454-471."""
        if self.barrier_type not in ("down-and-out", "up-and-out", "down-and-in", "up-and-in"):
            return False
        H = self.lower_barrier if "down" in self.barrier_type else self.upper_barrier
        if H is None or H <= 0.0 or self.barrier_status is not None:
            return False
        return (self.rebate_timing_in in (None, "hit", "expiry")
                and self.rebate_timing_out in (None, "hit", "expiry"))

    def _continuous_leg(self, S_eff: float, sigma: float):
        """The continuous-window leg (:473-529): ("rr", contract),
        ("douady", contract) or ("cn", None) for the every-step CN overlay.
        The reference wraps both engine calls in try/except and takes the CN
        overlay when they raise (:486-519).  BarrierEngine raises on a
        non-positive sigma or T and on the log of a non-positive level, so
        such a contract goes to the overlay here -- e.g. greeks() with
        abs_vol_bump >= volatility -- instead of failing the whole batch.
        DoubleBarrier computes through NumPy and returns a number for a
        negative sigma (no exception, no fallback): kept, fixture
        dko_daily_douady_vol_bump_past_zero."""
        def positive(*xs):
            return all(math.isfinite(x) and x > 0.0 for x in xs)
        if self.barrier_type in ("double-out", "double-in"):
            if (not self.double_barrier_analytic or self.bgk_lower_barrier is None
                    or self.bgk_upper_barrier is None):
                return ("cn", None)
            return ("douady", dict(S=S_eff, X=self.strike, L=self.bgk_lower_barrier,
                                   U=self.bgk_upper_barrier, sigma=sigma,
                                   callflag="c" if self.option_type == "call" else "p",
                                   inflag="in" if "in" in self.barrier_type else "out",
                                   b=self.flat_carry_b, r=self.flat_rate_r, T=self.tenor_years))
        if not self._single_barrier_analytic_ok():
            return ("cn", None)
        down = "down" in self.barrier_type
        H = self.bgk_lower_barrier if down else self.bgk_upper_barrier
        if H is None or not positive(S_eff, self.strike, H, sigma, self.tenor_years):
            return ("cn", None)
        return ("rr", dict(s=S_eff, b=self.flat_carry_b, r=self.flat_rate_r, t=self.tenor_years,
                           x=self.strike, sigma=sigma, h=H,
                           optionflag="c" if self.option_type == "call" else "p",
                           directionflag="d" if down else "u",
                           in_out_flag="i" if "in" in self.barrier_type else "o",
                           k=self.rebate_amount, barrier_status=self.barrier_status,
                           rebate_timing_in=self.rebate_timing_in,
                           rebate_timing_out=self.rebate_timing_out))

    # ------------------------------------------------------------------ plans
    def _plan(self, spot: float, sigma: float):
        """One price() evaluation as legs: [(sign, kind, key_or_contract,
        S_eff)], kind "cn" (key into the solve table) / "rr" / "douady"."""
        S_eff = spot - self._pv_dividends()
        shift = spot - S_eff
        legs = []

        def cn(which: str):
            return ("cn", (sigma, shift, which))
        if self.barrier_type in KNOCK_INS:
            legs.append((1.0,) + cn("vanilla") + (S_eff,))
            if self.use_continuous_window:
                kind, c = self._continuous_leg(S_eff, sigma)
                legs.append((-1.0,) + (cn("continuous") if kind == "cn" else (kind, c)) + (S_eff,))
            else:
                legs.append((-1.0,) + cn("discrete") + (S_eff,))
        elif self.use_continuous_window:
            kind, c = self._continuous_leg(S_eff, sigma)
            legs.append((1.0,) + (cn("continuous") if kind == "cn" else (kind, c)) + (S_eff,))
        else:
            legs.append((1.0,) + cn("discrete") + (S_eff,))
        return legs

    def _escrowed_grid(self, shift: float) -> np.ndarray:
        e = np.asarray(self.spot_grid, np.float64) - shift
        return np.where(0.0 > e, 0.0, e)  # max(0.0, s - shift)

    def _cn_for_key(self, key) -> VcSolve:
        sigma, shift, which = key
        grid = self._escrowed_grid(shift)
        if which == "vanilla":
            return self._cn_solve(grid, sigma, None, None, {})
        if which == "continuous":
            return self._cn_solve(grid, sigma, self.bgk_lower_barrier, self.bgk_upper_barrier,
                                  self.monitor_steps_continuous)
        return self._cn_solve(grid, sigma, self.lower_barrier, self.upper_barrier,
                              self.monitor_steps_discrete)

    def _engine(self) -> Engine:
        return self.engine if self.engine is not None else default_engine()

    def _evaluate(self, plans) -> List[float]:
        """Unscaled base prices of several plans: every distinct CN solve in
        one fdcn_vc launch, the analytic legs in one batch per engine."""
        eng = self._engine()
        keys, rr, db = [], [], []
        for legs in plans:
            for _, kind, item, _ in legs:
                if kind == "cn" and item not in keys:
                    keys.append(item)
                elif kind == "rr":
                    rr.append(item)
                elif kind == "douady":
                    db.append(item)
        V = dict(zip(keys, eng.run_vc([self._cn_for_key(k) for k in keys]))) if keys else {}
        rr_out = iter(eng.run_rr(rr)) if rr else iter(())
        db_out = iter(eng.run_double(db, 6)) if db else iter(())
        out = []
        for legs in plans:
            vals = []
            for sign, kind, item, S_eff in legs:
                if kind == "cn":
                    grid = self._escrowed_grid(item[1])
                    vals.append((sign, interp_linear(S_eff, grid, V[item])))
                else:
                    vals.append((sign, float(next(rr_out if kind == "rr" else db_out))))
            if len(vals) == 1:
                out.append(vals[0][1])
            else:  # knock-in: vanilla - knock-out leg
                out.append(vals[0][1] - vals[1][1])
        return out

    def _scale(self) -> float:
        return (1.0 if self.direction == "long" else -1.0) * self.quantity * \
            self.contract_multiplier

    # ------------------------------------------------------------ public API
    def price(self) -> float:
        """:538-571."""
        return float(self._scale() * self._evaluate([self._plan(self.spot, self.sigma)])[0])

    def greeks(self, rel_spot_bump: float = 1e-4, abs_vol_bump: float = 1e-4) -> Dict[str, float]:
        """:573-616: bump and reprice on a long 1 x 1 position, all five
        repricings evaluated together."""
        s0, sig0 = self.spot, self.sigma
        ds = max(1e-8, rel_spot_bump * s0)
        base, up, dn, upv, dnv = self._evaluate([
            self._plan(s0, sig0), self._plan(s0 + ds, sig0), self._plan(s0 - ds, sig0),
            self._plan(s0, sig0 + abs_vol_bump), self._plan(s0, sig0 - abs_vol_bump)])
        tol = 2 * self.grid_step_dS
        Hdn = self.bgk_lower_barrier if self.use_continuous_window else self.lower_barrier
        Hup = self.bgk_upper_barrier if self.use_continuous_window else self.upper_barrier
        near = (Hdn is not None and abs(s0 - Hdn) <= tol) or \
            (Hup is not None and abs(s0 - Hup) <= tol)
        if self.use_continuous_window and near:
            delta = (base - dn) / ds
        else:
            delta = (up - dn) / (2 * ds)
        gamma = (up - 2 * base + dn) / (ds * ds)
        vega = (upv - dnv) / (2 * abs_vol_bump)
        scale = self._scale()
        return {"delta": scale * float(delta), "gamma": scale * float(gamma),
                "vega": scale * float(vega)}

    def print_details(self) -> None:
        info = {
            "Trade ID": self.trade_id, "Direction": self.direction, "Quantity": self.quantity,
            "Contract Multiplier": self.contract_multiplier, "Option Type": self.option_type,
            "Barrier Type": self.barrier_type,
            "Lower Barrier": self.lower_barrier if self.lower_barrier is not None else "-",
            "Upper Barrier": self.upper_barrier if self.upper_barrier is not None else "-",
            "Rebate Amount": self.rebate_amount,
            "Rebate Timing (in/out)": f"{self.rebate_timing_in} / {self.rebate_timing_out}",
            "Barrier Status": self.barrier_status, "Spot (S0)": self.spot,
            "Strike (K)": self.strike, "Valuation Date": self.valuation_date.date().isoformat(),
            "Maturity Date": self.maturity_date.date().isoformat(), "T (years)": self.tenor_years,
            "Volatility (sigma)": self.sigma, "Flat r (cont)": self.flat_rate_r,
            "Flat q (cont)": self.flat_dividend_q, "Carry (b=r-q)": self.flat_carry_b,
            "Time steps (M)": self.time_steps, "Space nodes (N)": self.space_nodes,
            "Rannacher steps": self.rannacher_steps,
            "Monitoring dates (#)": len([d for d in self.monitoring_dates
                                         if self.valuation_date < d <= self.maturity_date]),
            "Use continuous window?": self.use_continuous_window,
            "BGK Lower / Upper": f"{self.bgk_lower_barrier} / {self.bgk_upper_barrier}",
            "Decision (n_lim)": f"n={self.n_desired_for_decision}, "
                                f"n_min={self.n_min_steps_per_interval}, n_lim={self.n_lim_multiplier}",
        }
        print("==== Discrete Barrier Option (Hybrid Analytic + CN) ====")
        for k, v in info.items():
            print(f"{k:28s}: {v:.10g}" if isinstance(v, float) else f"{k:28s}: {v}")
        px = self.price()
        g = self.greeks()
        print(f"\nPrice : {px:.10g}")
        print(f"Greeks: { {k: float(f'{v:.10g}') for k, v in g.items()} }")
