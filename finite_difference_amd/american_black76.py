"""American option on the forward (Black-76 PDE): CN + Rannacher + IT in log F.

Drop-in for ``AmericanFwdFDMPricer`` (fd_american_black76.py:12-625).  The
time march is the same Ikonen-Toivanen kernel as the spot pricer's
(``american.AmericanFDMPricer``); what changes is the operator and the
boundaries:

* drift in log F: ``mu_x = -sigma^2 / 2`` (fd_american_black76.py:351), i.e.
  the spot operator with carry b = q = 0, discounting at r;
* Dirichlet values ``e^{-r tau} (F_max - K)`` (call, top) and
  ``e^{-r tau} K`` (put, bottom) (fd_american_black76.py:291-314);
* no dividends (they live in the forward), a single segment with Rannacher;
* ``price_log2`` uses ``2 * num_time_steps`` (not the spot pricer's
  ``2 * num_space_nodes``), and theta has no drift term
  (fd_american_black76.py:537-625).

The constructor keywords, method names and keyword spellings (``N_time``,
``apply_KO``) follow the reference class.
"""
from __future__ import annotations

import datetime as _dt
from typing import Dict, List, Optional, Tuple

from .american import AmericanFDMPricer, OptionType
from .engine import FORM_PROD, Boundary, Engine


class AmericanFwdFDMPricer(AmericanFDMPricer):
    """American vanilla on the forward F (``spot`` is F0), Black-76 dynamics."""

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
            raise ValueError("spot (forward), strike and sigma must be positive.")
        super().__init__(spot, strike, valuation_date, maturity_date, sigma, option_type,
                         discount_curve, forward_curve, None, trade_id, direction, quantity,
                         contract_multiplier, underlying_spot_days, option_days,
                         option_settlement_days, day_count, grid_type, num_space_nodes,
                         num_time_steps, rannacher_steps, s_max_mult, engine)
        self.forward0 = float(spot)
        # fd_american_black76.py:133-146: r from the discount curve; the carry
        # attribute mirrors it, and the PDE has neither carry nor dividends
        self.carry_rate_nacc = self.discount_rate_nacc
        self.dividend_schedule = []

    # ----------------------------------------------------- operator / bounds
    def _operator_rates(self) -> Tuple[float, float]:
        """(b, q) of the log-F operator: mu_x = (0 - 0) - sigma^2/2."""
        return 0.0, 0.0

    def _boundaries(self) -> Tuple[Boundary, Boundary]:
        """fd_american_black76.py:291-314: disc * (F_max - K) / disc * K with
        disc = exp(-r tau); FORM_PROD evaluates ((1 * e^{-r tau}) * c) * e^{0}."""
        r = self.discount_rate_nacc
        k = self._strike_for_pde()
        if self.option_type == "call":
            return Boundary(), Boundary(FORM_PROD, 1.0, -r, self.s_nodes[-1] - k, 0.0)
        return Boundary(FORM_PROD, 1.0, -r, k, 0.0), Boundary()

    def _div_times_tau(self):
        return []

    def _price2_ntime(self) -> int:
        """price_log2 uses 2 * num_time_steps here (fd_american_black76.py:537-546)."""
        return 2 * self.num_time_steps

    def _theta_inputs(self):
        """theta = -(1/2 sigma^2 F0^2 Gamma - r P) (fd_american_black76.py:620):
        the spot form with zero carry."""
        return self.forward0, 0.0

    # ----------------------------------------------------------- public API
    def _solve_grid(self, N_time: Optional[int] = None) -> List[float]:
        return super()._solve_grid(n_time=N_time)

    def price_log(self, N_time: Optional[int] = None) -> float:
        return self._interp_price(self._solve_grid(N_time=N_time))

    def price_log2(self, apply_KO: bool = True, use_richardson: bool = True) -> float:
        """Richardson N vs 2N (fd_american_black76.py:537-546)."""
        if not use_richardson:
            return self.price_log(N_time=self.num_time_steps)
        if self._engine().on_device:
            return super().price_log2(apply_KO, use_richardson)
        self.prefetch([(self.sigma, self.num_time_steps), (self.sigma, 2 * self.num_time_steps)])
        p_n = self.price_log(N_time=self.num_time_steps)
        p_2n = self.price_log(N_time=2 * self.num_time_steps)
        return (4.0 * p_2n - p_n) / 3.0

    def _price_for_sigma(self, sigma: float, N_time: Optional[int] = None) -> float:
        original = self.sigma
        try:
            self.sigma = sigma
            return self.price_log(N_time=N_time)
        finally:
            self.sigma = original

    def greeks_requests(self, dv_sigma: float = 0.01, use_richardson: bool = True,
                        with_price: bool = True):
        N, s0, h = self.num_time_steps, self.sigma, dv_sigma
        if use_richardson:
            return [(s0, N), (s0, 2 * N), (s0 + h, N), (s0 - h, N), (s0 + 2.0 * h, N),
                    (s0 - 2.0 * h, N)]
        return [(s0, N), (s0 + h, N), (s0 - h, N)]

    def greeks_log2(self, dv_sigma: float = 0.01, use_richardson: bool = True) -> Dict[str, float]:
        """Price and Greeks as fd_american_black76.py:556-625 (Delta/Gamma in F)."""
        if use_richardson and self._engine().on_device:
            return super().greeks_log2(dv_sigma, use_richardson)
        self.prefetch(self.greeks_requests(dv_sigma, use_richardson))
        N = self.num_time_steps
        v_n = self._solve_grid(N_time=N)
        price_n = self._interp_price(v_n)
        delta_n, gamma_n = self._local_cubic_delta_gamma(v_n)
        if use_richardson:
            v_2n = self._solve_grid(N_time=2 * N)
            price_2n = self._interp_price(v_2n)
            delta_2n, gamma_2n = self._local_cubic_delta_gamma(v_2n)
            price = (4.0 * price_2n - price_n) / 3.0
            delta = (4.0 * delta_2n - delta_n) / 3.0
            gamma = (4.0 * gamma_2n - gamma_n) / 3.0
        else:
            price, delta, gamma = price_n, delta_n, gamma_n
        sigma0 = self.sigma
        h = dv_sigma
        if use_richardson:
            p_up_h = self._price_for_sigma(sigma0 + h, N_time=N)
            p_dn_h = self._price_for_sigma(sigma0 - h, N_time=N)
            d_h = (p_up_h - p_dn_h) / (2.0 * h)
            p_up_2h = self._price_for_sigma(sigma0 + 2.0 * h, N_time=N)
            p_dn_2h = self._price_for_sigma(sigma0 - 2.0 * h, N_time=N)
            d_2h = (p_up_2h - p_dn_2h) / (4.0 * h)
            dv_dsigma = (4.0 * d_h - d_2h) / 3.0
        else:
            p_up = self._price_for_sigma(sigma0 + h, N_time=N)
            p_dn = self._price_for_sigma(sigma0 - h, N_time=N)
            dv_dsigma = (p_up - p_dn) / (2.0 * h)
        vega = dv_dsigma / 100.0
        r = self.discount_rate_nacc
        F0 = self.forward0
        theta = -(0.5 * sigma0 * sigma0 * F0 * F0 * gamma - r * price)
        return {"price": float(price), "delta": float(delta), "gamma": float(gamma),
                "vega": float(vega), "theta": float(theta)}
