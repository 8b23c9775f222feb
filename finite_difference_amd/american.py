"""American vanilla pricer: CN + Rannacher + Ikonen-Toivanen in log-spot.

Drop-in for ``AmericanFDMPricer`` (fd_american_equity.py:42-1068; the twin
file fd_american_option_pricer.py computes bit-identical numbers).  Same
constructor arguments, same public methods (``price_log``, ``price_log2``,
``greeks_log2``) and the same numerics; the difference is where the time
march runs:

* every ``_solve_segment`` (fd_american_equity.py:559-726) becomes one
  scenario of a batched Ikonen-Toivanen launch on the MI355X
  (libfdcn ``fdcn_it_batch``);
* ``price_log2`` + ``greeks_log2`` need up to 8 grid solves (N, 2*num_space
  _nodes, 2N, sigma +-h, +-2h); the unique ones are solved together, segment
  by segment in lock-step, and cached, so the pair costs 2 launches instead
  of 8 sequential Python marches.

On the GPU (the default engine) ``price_log2`` / ``greeks_log2`` /
``prefetch_many`` run in a device session (session.py): the segments of all
grids march in lock-step launches, the discrete-dividend jump between
segments (natural cubic spline, fd_american_equity.py:479-553, 732-772) runs
on the device, and the Richardson / vega / theta epilogue (:925-1068) too;
six numbers per trade come back.  With another engine (the CPU oracle in the
tests) the host-side jump and epilogue below are used.
"""
from __future__ import annotations

import datetime as _dt
import math
from typing import Dict, List, Literal, Optional, Sequence, Tuple

import numpy as np

from . import capi, market
from .engine import FORM_SUM, Boundary, Engine, Solve, default_engine, operator_coefficients
from .session import GK_AMERICAN, GK_READOUT, Session, readout

OptionType = Literal["call", "put"]


def _pmax(x: float, y: float) -> float:
    """Python's max(x, y) (keeps x unless y > x)."""
    return y if y > x else x


def _one_of(name_a: str, a, name_b: str, b):
    """The value of whichever of two keyword spellings was given (the two
    reference files spell the American pricer's arguments differently)."""
    if a is not None and b is not None and a != b:
        raise TypeError(f"got both {name_a}={a!r} and {name_b}={b!r}")
    return a if a is not None else b


class AmericanFDMPricer:
    """American vanilla option, Crank-Nicolson in log S with IT early exercise."""

    def __init__(
        self,
        spot: float,
        strike: float,
        valuation_date: _dt.date,
        maturity_date: _dt.date,
        sigma: float,
        option_type: OptionType,
        discount_curve,
        forward_curve=None,
        dividend_schedule: Optional[List[Tuple[_dt.date, float]]] = None,
        trade_id: Optional[int] = None,
        direction: str = "long",
        quantity: int = 1,
        contract_multiplier: float = 1.0,
        underlying_spot_days: int = 0,
        option_days: int = 0,
        option_settlement_days: int = 0,
        day_count: str = "ACT/365",
        grid_type: str = "uniform",
        num_space_nodes: int = 400,
        num_time_steps: int = 400,
        rannacher_steps: int = 2,
        s_max_mult: float = 4.5,
        engine: Optional[Engine] = None,
    ) -> None:
        if spot <= 0.0 or strike <= 0.0 or sigma <= 0.0:
            raise ValueError("spot, strike and sigma must be positive.")
        if maturity_date <= valuation_date:
            raise ValueError("maturity_date must be after valuation_date.")
        self.spot = float(spot)
        self.strike = float(strike)
        self.valuation_date = valuation_date
        self.maturity_date = maturity_date
        self.sigma = float(sigma)
        self.option_type: str = option_type.lower()
        if self.option_type not in ("call", "put"):
            raise ValueError("option_type must be 'call' or 'put'.")

        self.discount_curve_df = discount_curve.copy()
        self.forward_curve_df = forward_curve.copy() if forward_curve is not None else None
        self._curve = market.NacaCurve(self.discount_curve_df)
        self.dividend_schedule = sorted(dividend_schedule or [], key=lambda x: x[0])

        self.trade_id = trade_id
        self.direction = direction
        self.quantity = int(quantity)
        self.contract_multiplier = float(contract_multiplier)

        self.calendar = market.SouthAfrica()
        self.underlying_spot_days = int(underlying_spot_days)
        self.option_days = int(option_days)
        self.option_settlement_days = int(option_settlement_days)

        self.day_count = market.normalise_day_count(day_count)
        self._year_denominator = market.year_denominator(self.day_count)
        self.grid_type = grid_type.lower()

        cal = self.calendar
        self.carry_start_date = cal.add_working_days(valuation_date, self.underlying_spot_days)
        self.carry_end_date = cal.add_working_days(maturity_date, self.underlying_spot_days)
        self.discount_start_date = cal.add_working_days(valuation_date, self.option_days)
        self.discount_end_date = cal.add_working_days(maturity_date, self.option_settlement_days)

        self.time_to_expiry = self._year_fraction(valuation_date, maturity_date)
        self.time_to_carry = self._year_fraction(self.carry_start_date, self.carry_end_date)
        self.time_to_discount = self._year_fraction(self.discount_start_date,
                                                    self.discount_end_date)
        if self.time_to_expiry <= 0.0:
            raise ValueError("time_to_expiry must be positive.")

        self.discount_rate_nacc = self.get_forward_nacc_rate(self.discount_start_date,
                                                             self.discount_end_date)
        # fd_american_equity.py:235-240: the carry rate is read off the discount
        # curve over the carry window whenever a forward curve is supplied.
        if self.forward_curve_df is not None:
            self.carry_rate_nacc = self.get_forward_nacc_rate(self.carry_start_date,
                                                              self.carry_end_date)
        else:
            self.carry_rate_nacc = self.discount_rate_nacc
        self.div_yield_nacc = 0.0

        self.num_space_nodes = max(int(num_space_nodes), 3)
        self.num_time_steps = max(int(num_time_steps), 4)
        self.rannacher_steps = max(int(rannacher_steps), 0)
        self.s_max_mult = float(s_max_mult)

        self.snap_spot_to_grid: bool = True
        self.snap_strike_to_grid: bool = True
        self.spot_grid_index: Optional[int] = None
        self.spot_snapped: Optional[float] = None
        self.strike_grid_index: Optional[int] = None
        self.strike_snapped: Optional[float] = None

        self.s_nodes: List[float] = []
        self.x_nodes: List[float] = []
        self._S_min = 0.0
        self._S_max = 0.0
        self._dx = 0.0

        self.engine = engine
        self._cache: Dict[tuple, Tuple[np.ndarray, dict]] = {}
        self._dev_cache: Dict[tuple, Dict[str, float]] = {}

    def _reset_trade(self, spot: float, strike: float, sigma: float) -> None:
        """Re-point this pricer at another trade with the same dates, curves,
        dividends, option type and numerics (the constructor's trade lines,
        fd_american_equity.py:159-175); cached grids are kept, keyed by trade."""
        if spot <= 0.0 or strike <= 0.0 or sigma <= 0.0:
            raise ValueError("spot, strike and sigma must be positive.")
        self.spot, self.strike, self.sigma = float(spot), float(strike), float(sigma)
        self.spot_grid_index = self.spot_snapped = None
        self.strike_grid_index = self.strike_snapped = None
        self.s_nodes, self.x_nodes = [], []
        self._S_min = self._S_max = self._dx = 0.0

    # ------------------------------------------------------------------ dates
    def _infer_denominator(self, day_count: str) -> int:
        return market.year_denominator(day_count)

    def _year_fraction(self, start_date: _dt.date, end_date: _dt.date) -> float:
        return market.year_fraction(self.day_count, start_date, end_date)

    def get_discount_factor(self, lookup_date: _dt.date) -> float:
        return market.discount_factor(self._curve, self.day_count, self.valuation_date,
                                      lookup_date)

    def get_forward_nacc_rate(self, start_date: _dt.date, end_date: _dt.date) -> float:
        return market.forward_nacc(self._curve, self.day_count, self.valuation_date,
                                   start_date, end_date)

    # ------------------------------------------------------------------- grid
    def _configure_grid(self) -> None:
        """Log-S band around sqrt(S K) (fd_american_equity.py:340-361)."""
        T = self.time_to_expiry
        sig = self.sigma
        s_low = min(self.spot, self.strike)
        s_high = max(self.spot, self.strike)
        s_c = math.sqrt(max(s_low * s_high, 1e-12))
        band = self.s_max_mult * sig * math.sqrt(max(T, 1e-12))
        x_c = math.log(s_c)
        s_min = math.exp(x_c - 0.5 * band)
        s_max = math.exp(x_c + 0.5 * band)
        s_min = min(s_min, 0.5 * s_low)
        s_max = max(s_max, 2.0 * s_high)
        self._S_min = max(s_min, 1e-8)
        self._S_max = s_max

    def _build_log_grid(self) -> float:
        """Uniform log grid + critical-level snapping (fd_american_equity.py:363-407)."""
        self._configure_grid()
        x_min = math.log(self._S_min)
        x_max = math.log(self._S_max)
        n = self.num_space_nodes
        dx = (x_max - x_min) / float(n)
        # [x_min + i * dx ...] and math.exp of each (…equity.py:372-373), in libfdcn
        x, s = capi.log_grid(x_min, dx, n)
        self.x_nodes = x.tolist()
        self.s_nodes = s.tolist()
        self._dx = dx
        self._snap_critical_levels_to_grid()
        return dx

    def _s_array(self) -> np.ndarray:
        """self.s_nodes as float64 array, converted once per grid list."""
        if getattr(self, "_s_arr_src", None) is not self.s_nodes:
            self._s_arr = np.asarray(self.s_nodes, dtype=np.float64)
            self._s_arr_src = self.s_nodes
        return self._s_arr

    def _snap_critical_levels_to_grid(self) -> None:
        s = self._s_array()
        if s.size == 0:
            return
        if self.snap_spot_to_grid:
            i = int(np.argmin(np.abs(s - self.spot)))
            self.spot_grid_index, self.spot_snapped = i, self.s_nodes[i]
        else:
            self.spot_grid_index = self.spot_snapped = None
        if self.snap_strike_to_grid:
            i = int(np.argmin(np.abs(s - self.strike)))
            self.strike_grid_index, self.strike_snapped = i, self.s_nodes[i]
        else:
            self.strike_grid_index = self.strike_snapped = None

    # ------------------------------------------------------- payoff / bounds
    def _strike_for_pde(self) -> float:
        if self.snap_strike_to_grid and self.strike_snapped is not None:
            return self.strike_snapped
        return self.strike

    def _intrinsic_payoff(self, spot: float) -> float:
        k = self._strike_for_pde()
        if self.option_type == "call":
            return _pmax(spot - k, 0.0)
        return _pmax(k - spot, 0.0)

    def _payoff_array(self) -> np.ndarray:
        """Vectorised _intrinsic_payoff over the grid; np.where(0.0 > e, 0.0, e)
        is exactly Python's max(e, 0.0)."""
        s = self._s_array()
        k = self._strike_for_pde()
        e = s - k if self.option_type == "call" else k - s
        return np.where(0.0 > e, 0.0, e)

    def _terminal_payoff(self) -> List[float]:
        return self._payoff_array().tolist()

    def _boundary_values(self, tau: float) -> Tuple[float, float]:
        lo, hi = self._boundaries()
        return lo.value(tau), hi.value(tau)

    def _operator_rates(self) -> Tuple[float, float]:
        """(b, q) of the log-S operator: carry, and q = 0 (discrete dividends
        are jumps, fd_american_equity.py:242-249)."""
        return self.carry_rate_nacc, 0.0

    def _boundaries(self) -> Tuple[Boundary, Boundary]:
        """Dirichlet values of fd_american_equity.py:430-448 as kernel forms."""
        r, b = self.discount_rate_nacc, self.carry_rate_nacc
        k = self._strike_for_pde()
        if self.option_type == "call":
            return Boundary(), Boundary(FORM_SUM, self.s_nodes[-1], b - r, -k, -r)
        return Boundary(FORM_SUM, k, -r, 0.0, 0.0), Boundary()

    # -------------------------------------------------------------- dividends
    def _div_times_tau(self) -> List[Tuple[float, float]]:
        """(tau_div, cash) of dividends strictly inside (valuation, maturity)."""
        out = []
        for pay_date, amount in self.dividend_schedule:
            if self.valuation_date < pay_date < self.maturity_date:
                t_rel = self._year_fraction(self.valuation_date, pay_date)
                if 0.0 < t_rel < self.time_to_expiry:
                    out.append((self.time_to_expiry - t_rel, float(amount)))
        out.sort(key=lambda x: x[0])
        return out

    @staticmethod
    def _build_natural_cubic_spline(x: Sequence[float], y: Sequence[float]):
        """Natural cubic spline S(x) (fd_american_equity.py:479-553), returned
        as a vectorised evaluator with the same arithmetic per point."""
        xa = np.asarray(x, dtype=float)
        ya = np.asarray(y, dtype=float)
        n = xa.size
        if n < 2:
            raise ValueError("Need at least two points for spline.")
        h = np.diff(xa)
        if np.any(h <= 0.0):
            raise ValueError("x must be strictly increasing.")
        alpha = np.zeros(n)
        dy = ya[1:] - ya[:-1]
        alpha[1:-1] = 3.0 / h[1:] * dy[1:] - 3.0 / h[:-1] * dy[:-1]
        l_ = np.ones(n)
        mu = np.zeros(n)
        z = np.zeros(n)
        for i in range(1, n - 1):
            l_[i] = 2.0 * (xa[i + 1] - xa[i - 1]) - h[i - 1] * mu[i - 1]
            mu[i] = h[i] / l_[i]
            z[i] = (alpha[i] - h[i - 1] * z[i - 1]) / l_[i]
        c = np.zeros(n)
        b = np.zeros(n - 1)
        d = np.zeros(n - 1)
        for j in range(n - 2, -1, -1):
            c[j] = z[j] - mu[j] * c[j + 1]
            b[j] = (ya[j + 1] - ya[j]) / h[j] - h[j] * (c[j + 1] + 2.0 * c[j]) / 3.0
            d[j] = (c[j + 1] - c[j]) / (3.0 * h[j])
        a = ya[:-1]

        def evaluate(q: np.ndarray) -> np.ndarray:
            q = np.asarray(q, dtype=float)
            j = np.searchsorted(xa, q, side="right") - 1
            j = np.where(q <= xa[0], 0, np.where(q >= xa[-1], n - 2, j))
            t = q - xa[j]
            return a[j] + b[j] * t + c[j] * t * t + d[j] * t * t * t

        return evaluate

    def _apply_dividend_jump(self, v_after: Sequence[float], cash_div: float) -> List[float]:
        """V(t_d-, S) = V(t_d+, S - D), plus exercise for calls (…equity.py:732-772).

        Runs in libfdcn (fdcn_dividend_jump: the same spline and operation
        order in C, ~1000x faster than the Python loop of the spline solve);
        _apply_dividend_jump_numpy below is the NumPy restatement it is
        tested against."""
        k = self._strike_for_pde() if self.option_type == "call" else -1.0
        return capi.dividend_jump(self.s_nodes, v_after, cash_div, k).tolist()

    def _apply_dividend_jump_numpy(self, v_after: Sequence[float],
                                   cash_div: float) -> List[float]:
        s = np.asarray(self.s_nodes)
        v = np.asarray(v_after, dtype=float)
        spline = self._build_natural_cubic_spline(s, v)
        q = s - cash_div
        cont = np.where(q <= s[0], v[0], np.where(q >= s[-1], v[-1], spline(q)))
        if self.option_type == "call":
            k = self._strike_for_pde()
            ex = np.array([_pmax(x - k, 0.0) for x in s])
            return [_pmax(float(cv), float(e)) for cv, e in zip(cont, ex)]
        return [float(x) for x in cont]

    # ------------------------------------------------------------ the solves
    def _segment_solve(self, v_init: Sequence[float], tau_start: float, tau_end: float,
                       n_steps: int, restart_rannacher: bool) -> Solve:
        """The work of one _solve_segment call as a kernel scenario."""
        dt = (tau_end - tau_start) / float(n_steps)
        b, q = self._operator_rates()
        coeffs = operator_coefficients(self.sigma, b, q, self.discount_rate_nacc, self._dx)
        lower, upper = self._boundaries()
        pay = self._payoff_array()
        return Solve(it=True, n_time=int(n_steps),
                     n_ranna=self.rannacher_steps if restart_rannacher else 0, dt=dt,
                     coeffs=coeffs, v_init=np.asarray(v_init, dtype=np.float64), lower=lower,
                     upper=upper, tau0=tau_start, tau_accumulate=True, payoff=pay)

    def _engine(self) -> Engine:
        return self.engine if self.engine is not None else default_engine()

    def _solve_segment(self, v_init: List[float], tau_start: float, tau_end: float,
                       n_steps: int, restart_rannacher: bool) -> List[float]:
        """fd_american_equity.py:559-726 on the GPU (one-scenario launch)."""
        if n_steps < 1:
            return v_init
        if len(self.s_nodes) - 1 < 2:
            raise RuntimeError("Spatial grid too coarse.")
        s = self._segment_solve(v_init, tau_start, tau_end, n_steps, restart_rannacher)
        return self._engine().run([s])[0].tolist()

    def _segments(self, n_time: int):
        total_tau = self.time_to_expiry
        divs = self._div_times_tau()
        base_n = int(n_time)
        base_dt = total_tau / float(base_n)
        pts = [0.0] + [t for t, _ in divs] + [total_tau]
        steps: List[int] = []
        remaining = base_n
        for i in range(len(pts) - 2):
            ns = max(1, int(round((pts[i + 1] - pts[i]) / base_dt)))
            steps.append(ns)
            remaining -= ns
        steps.append(max(1, remaining))
        return divs, pts, steps

    def _state_key(self, sigma: float, n_time: int) -> tuple:
        return (float(sigma), int(n_time), self.spot, self.strike, self.time_to_expiry,
                self.discount_rate_nacc, self.carry_rate_nacc, self.num_space_nodes,
                self.rannacher_steps, self.s_max_mult, self.option_type,
                tuple(self.dividend_schedule), self.snap_spot_to_grid, self.snap_strike_to_grid)

    def _grid_state(self) -> dict:
        return dict(s_nodes=self.s_nodes, x_nodes=self.x_nodes, _S_min=self._S_min,
                    _S_max=self._S_max, _dx=self._dx, spot_grid_index=self.spot_grid_index,
                    spot_snapped=self.spot_snapped, strike_grid_index=self.strike_grid_index,
                    strike_snapped=self.strike_snapped)

    def _restore(self, st: dict) -> None:
        for k, v in st.items():
            setattr(self, k, v)

    def _pending_jobs(self, requests: Sequence[Tuple[float, int]]) -> list:
        """Grid jobs (one per uncached (sigma, n_time)) with their segments."""
        pending, seen = [], set()
        for sig, nt in requests:
            key = self._state_key(sig, nt)
            if key in self._cache or key in seen:
                continue
            seen.add(key)
            pending.append((key, float(sig), int(nt)))
        jobs = []
        if not pending:
            return jobs
        sigma0, saved = self.sigma, self._grid_state()
        try:
            for key, sig, nt in pending:
                self.sigma = sig
                self._build_log_grid()
                divs, pts, steps = self._segments(nt)
                jobs.append(dict(owner=self, key=key, sigma=sig, grid=self._grid_state(),
                                 divs=divs, pts=pts, steps=steps, v=self._payoff_array()))
        finally:
            self.sigma = sigma0
            self._restore(saved)
        return jobs

    @staticmethod
    def _march_jobs(jobs: list, engine: Engine) -> None:
        """March grid jobs of any number of trades in segment lock-step: every
        job's segment i goes into one engine.run (one launch per distinct
        (n_nodes, n_time)), then each job's dividend jump, then segment i+1;
        finally each job's value vector is cached on its owner."""
        if not jobs:
            return
        n_seg = max(len(j["steps"]) for j in jobs)
        for seg in range(n_seg):
            solves, owners = [], []
            for j in jobs:
                if seg >= len(j["steps"]) or j["steps"][seg] < 1:
                    continue
                p = j["owner"]
                sigma0, saved = p.sigma, p._grid_state()
                try:
                    p.sigma = j["sigma"]
                    p._restore(j["grid"])
                    if len(p.s_nodes) - 1 < 2:
                        raise RuntimeError("Spatial grid too coarse.")
                    restart = seg == 0 or (seg > 0 and p.option_type == "call")
                    solves.append(p._segment_solve(j["v"], j["pts"][seg], j["pts"][seg + 1],
                                                   j["steps"][seg], restart))
                finally:
                    p.sigma = sigma0
                    p._restore(saved)
                owners.append(j)
            if solves:
                for j, v in zip(owners, engine.run(solves)):
                    j["v"] = v
            for j in jobs:
                if seg < len(j["divs"]):
                    p = j["owner"]
                    sigma0, saved = p.sigma, p._grid_state()
                    try:
                        p.sigma = j["sigma"]
                        p._restore(j["grid"])
                        j["v"] = p._apply_dividend_jump(j["v"], j["divs"][seg][1])
                    finally:
                        p.sigma = sigma0
                        p._restore(saved)
        for j in jobs:
            j["owner"]._cache[j["key"]] = (np.asarray(j["v"], dtype=np.float64), j["grid"])

    def prefetch(self, requests: Sequence[Tuple[float, int]]) -> None:
        """Solve the (sigma, n_time) grids not yet cached, all together.

        Segments are marched in lock-step: every pending request's segment i
        goes into one batched launch (grouped by step count), then the host
        applies the dividend jump, then segment i+1."""
        self._march_jobs(self._pending_jobs(requests), self._engine())

    def _solve_grid(self, n_time: Optional[int] = None, *,
                    N_time: Optional[int] = None) -> List[float]:
        """Value vector at valuation (fd_american_equity.py:778-843).  Takes
        the fd_american_equity.py spelling (n_time) and the
        fd_american_option_pricer.py one (N_time, :659)."""
        n_time = _one_of("n_time", n_time, "N_time", N_time)
        nt = self.num_time_steps if n_time is None else int(n_time)
        self.prefetch([(self.sigma, nt)])
        V, grid = self._cache[self._state_key(self.sigma, nt)]
        self._restore(grid)
        return V.tolist()

    # ------------------------------------------------- device (session) path
    def _price2_ntime(self) -> int:
        """Step count of price_log2's second grid: 2 * num_space_nodes (the
        reference's quirk, fd_american_equity.py:950)."""
        return 2 * self.num_space_nodes

    def _theta_inputs(self) -> Tuple[float, float]:
        """(spot, carry) of greeks_log2's theta identity (:1060-1068)."""
        return self.spot, self.carry_rate_nacc

    def _dev_key(self, dv_sigma: float) -> tuple:
        return (float(dv_sigma), self._state_key(self.sigma, self.num_time_steps))

    def _job_readout(self, job: dict, slot: int, cubic: bool):
        """_interp_price (+ _local_cubic_delta_gamma) positions on a job's grid
        (fd_american_equity.py:855-907): the snapped spot, and for the cubic
        the node nearest to it clamped to [1, n-2]."""
        st = job["grid"]
        s = st["s_nodes"]
        s0 = (st["spot_snapped"] if self.snap_spot_to_grid and st["spot_snapped"] is not None
              else self.spot)
        if not cubic:
            return readout(slot, s, s0)
        n = len(s) - 1
        i = int(np.argmin(np.abs(np.asarray(s) - s0)))
        i = 1 if i < 1 else (n - 2 if i > n - 2 else i)
        return readout(slot, s, s0, s0, dg_mode=2, idx=i)

    @staticmethod
    def _march_jobs_device(jobs: list, engine: Engine, sess: Session) -> None:
        """_march_jobs with the value vectors in HBM: segment i of every job in
        lock-step launches (initial vectors: the payoff, then the previous
        segment's slots), the dividend jumps on the device between segments.
        Leaves each job's final slot in job["slot"]."""
        n_seg = max(len(j["steps"]) for j in jobs)
        for seg in range(n_seg):
            solves, owners = [], []
            for j in jobs:
                if seg >= len(j["steps"]) or j["steps"][seg] < 1:
                    continue
                p = j["owner"]
                sigma0, saved = p.sigma, p._grid_state()
                try:
                    p.sigma = j["sigma"]
                    p._restore(j["grid"])
                    if len(p.s_nodes) - 1 < 2:
                        raise RuntimeError("Spatial grid too coarse.")
                    restart = seg == 0 or (seg > 0 and p.option_type == "call")
                    solves.append(p._segment_solve(j["v"], j["pts"][seg], j["pts"][seg + 1],
                                                   j["steps"][seg], restart))
                finally:
                    p.sigma = sigma0
                    p._restore(saved)
                owners.append(j)
            if solves:
                vs = None if seg == 0 else [j["slot"] for j in owners]
                for j, sl in zip(owners, engine.march_slots(sess, solves, vs)):
                    j["slot"] = int(sl)
            jump = [j for j in jobs if seg < len(j["divs"])]
            by_n: Dict[int, list] = {}
            for j in jump:
                by_n.setdefault(len(j["grid"]["s_nodes"]), []).append(j)
            for js in by_n.values():
                S = np.array([j["grid"]["s_nodes"] for j in js], dtype=np.float64)
                cash = [j["divs"][seg][1] for j in js]
                kc = [(j["owner"]._strike_snapped_for(j) if j["owner"].option_type == "call"
                       else -1.0) for j in js]
                for j, sl in zip(js, sess.dividend_jump([j["slot"] for j in js], S, cash, kc)):
                    j["slot"] = int(sl)

    def _strike_snapped_for(self, job: dict) -> float:
        st = job["grid"]
        if self.snap_strike_to_grid and st["strike_snapped"] is not None:
            return st["strike_snapped"]
        return self.strike

    def _device_requests(self, dv_sigma: float, price_only: bool):
        N, s0, h = self.num_time_steps, self.sigma, dv_sigma
        if price_only:
            return [(s0, N), (s0, self._price2_ntime())]
        return [(s0, N), (s0, 2 * N), (s0 + h, N), (s0 - h, N), (s0 + 2.0 * h, N),
                (s0 - 2.0 * h, N), (s0, self._price2_ntime())]

    def _device_jobs(self, requests) -> Tuple[list, List[int]]:
        """One job per distinct (sigma, n_time) grid of `requests` and, per
        request, the index of its job."""
        keys, jobs, index = {}, [], []
        sigma0, saved = self.sigma, self._grid_state()
        try:
            for sig, nt in requests:
                key = self._state_key(sig, nt)
                if key not in keys:
                    self.sigma = float(sig)
                    self._build_log_grid()
                    divs, pts, steps = self._segments(int(nt))
                    keys[key] = len(jobs)
                    jobs.append(dict(owner=self, key=key, sigma=float(sig), grid=self._grid_state(),
                                     divs=divs, pts=pts, steps=steps, v=self._payoff_array()))
                index.append(keys[key])
        finally:
            self.sigma = sigma0
            self._restore(saved)
        return jobs, index

    # ----------------------------------------------------- price and greeks
    def _spot_for_interp(self) -> float:
        if self.snap_spot_to_grid and self.spot_snapped is not None:
            return self.spot_snapped
        return self.spot

    def _interp_price(self, v_values: Sequence[float]) -> float:
        s = self.s_nodes
        s0 = self._spot_for_interp()
        if s0 <= s[0]:
            return float(v_values[0])
        if s0 >= s[-1]:
            return float(v_values[-1])
        hi = int(np.searchsorted(np.asarray(s), s0, side="right"))
        lo = hi - 1
        w = (s0 - s[lo]) / (s[hi] - s[lo])
        return float((1.0 - w) * v_values[lo] + w * v_values[hi])

    def _local_cubic_delta_gamma(self, v_values: Sequence[float]) -> Tuple[float, float]:
        """Four-point cubic fit around the snapped spot (…equity.py:876-907)."""
        s = self.s_nodes
        s0 = self._spot_for_interp()
        n = len(s) - 1
        i = int(np.argmin(np.abs(np.asarray(s) - s0)))
        i = 1 if i < 1 else (n - 2 if i > n - 2 else i)
        idx = [i - 1, i, i + 1, i + 2]
        xv = np.array([s[j] for j in idx], dtype=float)
        yv = np.array([v_values[j] for j in idx], dtype=float)
        z = xv - s0
        design = np.vstack([z ** 3, z ** 2, z, np.ones_like(z)]).T
        _, b_coef, c_coef, _ = np.linalg.solve(design, yv)
        return float(c_coef), float(2.0 * b_coef)

    def price_log(self, n_time: Optional[int] = None, *, N_time: Optional[int] = None) -> float:
        """fd_american_equity.py:913 (n_time) and fd_american_option_pricer.py
        :659 (N_time) spellings."""
        return self._interp_price(self._solve_grid(n_time=_one_of("n_time", n_time,
                                                                  "N_time", N_time)))

    def price_log2(self, apply_ko: bool = True, use_richardson: bool = True, *,
                   apply_KO: Optional[bool] = None) -> float:
        """Richardson N vs 2*num_space_nodes (the reference's quirk, :950).
        apply_ko / apply_KO (fd_american_option_pricer.py:663) are ignored,
        as in both references."""
        if not use_richardson:
            return self.price_log(n_time=self.num_time_steps)
        if self._engine().on_device:
            hit = self._dev_cache.get(("price2",) + self._dev_key(0.0))
            if hit is None:
                greeks_many([self], price_only=True)
                hit = self._dev_cache[("price2",) + self._dev_key(0.0)]
            return hit["price_log2"]
        self.prefetch([(self.sigma, self.num_time_steps), (self.sigma, 2 * self.num_space_nodes)])
        p_n = self.price_log(n_time=self.num_time_steps)
        p_2n = self.price_log(n_time=2 * self.num_space_nodes)
        return (4.0 * p_2n - p_n) / 3.0

    def _price_for_sigma(self, sigma: float, n_time: Optional[int] = None, *,
                         N_time: Optional[int] = None) -> float:
        n_time = _one_of("n_time", n_time, "N_time", N_time)
        original = self.sigma
        try:
            self.sigma = sigma
            return self.price_log(n_time=n_time)
        finally:
            self.sigma = original

    def greeks_requests(self, dv_sigma: float = 0.01, use_richardson: bool = True,
                        with_price: bool = True):
        """(sigma, n_time) grids price_log2 + greeks_log2 will ask for."""
        N, s0, h = self.num_time_steps, self.sigma, dv_sigma
        req = [(s0, N)]
        if use_richardson:
            req += [(s0, 2 * N), (s0 + h, N), (s0 - h, N), (s0 + 2.0 * h, N), (s0 - 2.0 * h, N)]
            if with_price:
                req.append((s0, 2 * self.num_space_nodes))
        else:
            req += [(s0 + h, N), (s0 - h, N)]
        return req

    def greeks_log2(self, dv_sigma: float = 0.01, use_richardson: bool = True) -> Dict[str, float]:
        """Price and Greeks as fd_american_equity.py:970-1068."""
        if use_richardson and self._engine().on_device:
            hit = self._dev_cache.get(self._dev_key(dv_sigma))
            if hit is None:
                greeks_many([self], dv_sigma)
                hit = self._dev_cache[self._dev_key(dv_sigma)]
            return {k: hit[k] for k in ("price", "delta", "gamma", "vega", "theta")}
        self.prefetch(self.greeks_requests(dv_sigma, use_richardson, with_price=False))
        v_n = self._solve_grid(n_time=self.num_time_steps)
        price_n = self._interp_price(v_n)
        delta_n, gamma_n = self._local_cubic_delta_gamma(v_n)
        if use_richardson:
            v_2n = self._solve_grid(n_time=2 * self.num_time_steps)
            price_2n = self._interp_price(v_2n)
            delta_2n, gamma_2n = self._local_cubic_delta_gamma(v_2n)
            price = (4.0 * price_2n - price_n) / 3.0
            delta = (4.0 * delta_2n - delta_n) / 3.0
            gamma = (4.0 * gamma_2n - gamma_n) / 3.0
        else:
            price, delta, gamma = price_n, delta_n, gamma_n
        sigma0 = self.sigma
        h = dv_sigma
        N = self.num_time_steps
        if use_richardson:
            first_h = (self._price_for_sigma(sigma0 + h, N)
                       - self._price_for_sigma(sigma0 - h, N)) / (2.0 * h)
            first_2h = (self._price_for_sigma(sigma0 + 2.0 * h, N)
                        - self._price_for_sigma(sigma0 - 2.0 * h, N)) / (4.0 * h)
            dvds = (4.0 * first_h - first_2h) / 3.0
        else:
            dvds = (self._price_for_sigma(sigma0 + h, N)
                    - self._price_for_sigma(sigma0 - h, N)) / (2.0 * h)
        vega = dvds / 100.0
        r, b, q, s0 = self.discount_rate_nacc, self.carry_rate_nacc, 0.0, self.spot
        theta = -(0.5 * sigma0 * sigma0 * s0 * s0 * gamma + (b - q) * s0 * delta - r * price)
        return {"price": float(price), "delta": float(delta), "gamma": float(gamma),
                "vega": float(vega), "theta": float(theta)}


def greeks_many(pricers: Sequence[AmericanFDMPricer], dv_sigma: float = 0.01,
                price_only: bool = False) -> None:
    """price_log2 (+ greeks_log2 unless price_only) of many trades in one
    device session: every trade's grids (N, 2N, sigma +-h, +-2h and price_log2's
    second grid; dividend segments in lock-step with the spline jumps on the
    device) march in shared launches, and the readouts, Richardson
    extrapolations, vega and theta run on the device (FDCN_GK_AMERICAN);
    six numbers per trade come back.  Results land in each pricer's cache."""
    if not pricers:
        return
    engine = pricers[0]._engine()
    jobs, plan = [], []
    for p in pricers:
        pj, idx = p._device_jobs(p._device_requests(dv_sigma, price_only))
        plan.append((p, [len(jobs) + i for i in idx]))
        jobs.extend(pj)
    with Session() as S:
        AmericanFDMPricer._march_jobs_device(jobs, engine, S)
        trades = []
        for p, ji in plan:
            if price_only:
                trades.append((GK_READOUT, [p._job_readout(jobs[ji[0]], jobs[ji[0]]["slot"], False)],
                               ()))
                trades.append((GK_READOUT, [p._job_readout(jobs[ji[1]], jobs[ji[1]]["slot"], False)],
                               ()))
                continue
            rds = [p._job_readout(jobs[k], jobs[k]["slot"], cubic=(n < 2))
                   for n, k in enumerate(ji)]
            spot, carry = p._theta_inputs()
            trades.append((GK_AMERICAN, rds, (p.sigma, spot, carry, p.discount_rate_nacc,
                                              dv_sigma)))
        out = S.greeks(trades)
    for t, (p, ji) in enumerate(plan):
        if price_only:
            p_n, p_2 = float(out[2 * t, 0]), float(out[2 * t + 1, 0])
            p._dev_cache[("price2",) + p._dev_key(0.0)] = {"price_log2": (4.0 * p_2 - p_n) / 3.0}
            continue
        o = out[t]
        p._dev_cache[p._dev_key(dv_sigma)] = {
            "price": float(o[0]), "delta": float(o[1]), "gamma": float(o[2]),
            "vega": float(o[3]), "theta": float(o[4])}
        p._dev_cache[("price2",) + p._dev_key(0.0)] = {"price_log2": float(o[5])}


def prefetch_many(pricers: Sequence[AmericanFDMPricer], dv_sigma: float = 0.01,
                  use_richardson: bool = True) -> None:
    """Solve every grid that price_log2 + greeks_log2 of many trades will need.

    All trades' unique (sigma, n_time) grids are marched together in
    segment lock-step (AmericanFDMPricer._march_jobs): trades without
    dividends are one segment, so the whole set is one engine.run (one launch
    per distinct (n_nodes, n_time)); trades with dividends add one round per
    extra segment, shared by every trade, with the host's spline jumps in
    between."""
    if not pricers:
        return
    if use_richardson and pricers[0]._engine().on_device:
        greeks_many([p for p in pricers if p._dev_key(dv_sigma) not in p._dev_cache], dv_sigma)
        return
    jobs = []
    for p in pricers:
        jobs.extend(p._pending_jobs(p.greeks_requests(dv_sigma, use_richardson)))
    AmericanFDMPricer._march_jobs(jobs, pricers[0]._engine())
