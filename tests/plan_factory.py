"""Seeded random plans (lists of engine.Solve) for kernel parity tests.

Coefficients, grids, boundaries and knock-out data are drawn in the ranges
the reference's scenarios use (config_scenarios*.csv, fd_american_equity.py
defaults), so the systems have the same conditioning as the real workload.
"""
from __future__ import annotations

import math

import numpy as np

from finite_difference_amd.engine import (FORM_PROD, FORM_SUM, Boundary, Solve,
                                          operator_coefficients)


def log_grid(s_min: float, s_max: float, n_space: int):
    x_min, x_max = math.log(s_min), math.log(s_max)
    dx = (x_max - x_min) / n_space
    s = np.array([math.exp(x_min + i * dx) for i in range(n_space + 1)])
    return dx, s


def random_solve(rng: np.random.Generator, n_nodes: int, n_time: int, n_ranna: int, it: bool,
                 ko: bool = True, drop_top: bool = False) -> Solve:
    S0 = 100.0
    sigma = float(rng.uniform(0.12, 0.45))
    r = float(rng.uniform(0.0, 0.1))
    b = r - float(rng.uniform(0.0, 0.04))
    T = float(rng.uniform(0.05, 0.6))
    s_lo = float(rng.uniform(25.0, 60.0))
    s_hi = float(rng.uniform(180.0, 400.0))
    n_space = n_nodes if drop_top else n_nodes - 1
    dx, s = log_grid(s_lo, s_hi, n_space)
    K = float(rng.uniform(80.0, 125.0))
    call = bool(rng.integers(0, 2))
    pay = np.maximum(s - K, 0.0) if call else np.maximum(K - s, 0.0)
    dt = T / max(n_time, 1)
    a, c, bc = operator_coefficients(sigma, b, 0.0, r, dx)
    if call:
        lower = Boundary(FORM_SUM, 0.0, 0.0, 0.0, 0.0)
        upper = Boundary(FORM_SUM, float(s[-1]), b - r, -K, -r)
    else:
        upper = Boundary()
        if rng.integers(0, 2):
            lower = Boundary(FORM_PROD, K, -r, float(s[0]), b - r)  # pricer.py:391 form
        else:
            lower = Boundary(FORM_SUM, K, -r, 0.0, 0.0)
    v0 = pay[:n_nodes].copy()
    sv = Solve(it=it, n_time=n_time, n_ranna=n_ranna, dt=dt, coeffs=(a, c, bc), v_init=v0,
               lower=lower, upper=upper, tau0=0.0)
    if it:
        sv.payoff = pay[:n_nodes].copy()
    elif ko:
        kind = int(rng.integers(0, 4))
        if kind in (0, 2):
            sv.ko_lo = int(rng.integers(0, n_nodes // 3))
        if kind in (1, 2):
            sv.ko_hi = int(rng.integers(2 * n_nodes // 3, n_nodes))
        nm = int(rng.integers(1, 25))
        steps = sorted(set(int(x) for x in rng.integers(1, n_time + 1, nm)))
        sv.mon_steps = steps
        sv.mon_rebates = [float(rng.choice([0.0, 0.0, 1.5])) for _ in steps]
    return sv
