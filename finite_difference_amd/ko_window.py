"""Active window of a march that knocks out on every time step.

A barrier projected on every step (the FD engines' continuous-monitoring
mode, config 5's double knock-out) resets every node beyond a barrier to the
projection value after each step (discrete_barrier_fdm_pricer.py:413-440,
:545).  Those nodes then influence the live ones only through the step's
tridiagonal solve, and that influence decays geometrically with the
distance: the solve's Green's function falls off like rho^d with rho =
max(|fm|, |bm|) of the converged LU factors (the decay the kernel's
Sherman-Morrison extent and scan stages already cut at 1e-18).  So the live
nodes are the same, to 1e-18 of the values, if the march runs on the live
range widened by a margin of K nodes (rho^K <= 1e-18) on each cut side, with
the projection value as the Dirichlet value at the cut.  Every node outside
the window holds the projection value after the last step, exactly as in the
full march.

Config 5 (4 097 nodes, barriers at nodes 1 799 / 2 297, rho <= 0.37) marches
about 640 nodes instead of 4 097.  Only for every-step projection: between
discrete monitoring dates the knocked-out region evolves and feeds back.

The bench's throughput lines keep the configured grid (BASELINE's node-step
unit); the façades (FDDoubleBarrier.price, FDBarrierEngine.price) use the
window unless constructed with ``active_window=False``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import Optional

import numpy as np

from .engine import Boundary, Solve

# relative weight below which the cut side's influence is dropped (the
# kernel's truncation criterion), and extra nodes on top of that distance
DECAY_TOL = 1e-18
MARGIN_EXTRA = 8
# skip the window when it would keep more than this share of the grid
MAX_KEEP = 0.9


def decay_rate(sv: Solve) -> float:
    """max(|fm|, |bm|) over the theta phases the march uses (make_phase in
    csrc/fdcn_kernels.hip; A_L, A_C, A_U of discrete_barrier_fdm_pricer.py:475-484)."""
    a, c, bc = sv.coeffs
    rho = 0.0
    thetas = ([1.0] if sv.n_ranna > 0 else []) + ([0.5] if sv.n_ranna < sv.n_time else [])
    for th in thetas:
        AL, AC, AU = -th * sv.dt * a, 1.0 - th * sv.dt * bc, -th * sv.dt * c
        disc = AC * AC - 4.0 * AL * AU
        if disc < 0.0 or AC <= 0.0:
            return 1.0
        r = 0.5 * (AC + math.sqrt(disc))
        rho = max(rho, abs(AL / r), abs(AU / r))
    return rho


def margin_nodes(sv: Solve) -> Optional[int]:
    """Nodes beyond the barrier kept in the window (None: no usable decay)."""
    rho = decay_rate(sv)
    if not (0.0 <= rho < 0.999):
        return None
    if rho == 0.0:
        return MARGIN_EXTRA
    return int(math.ceil(math.log(DECAY_TOL) / math.log(rho))) + MARGIN_EXTRA


@dataclass
class KoWindow:
    """A windowed march and how to put its result back on the full grid."""
    solve: Solve
    a: int          # first node of the window on the full grid
    n_nodes: int    # full grid
    fill: float     # projection value after the last step

    def expand(self, v: np.ndarray) -> np.ndarray:
        out = np.full(self.n_nodes, self.fill)
        out[self.a:self.a + self.solve.n_nodes] = v
        return out


def ko_window(sv: Solve, ko_value: Boundary) -> Optional[KoWindow]:
    """The window of an every-step knock-out march, or None when it does not
    apply (American IT, discrete monitoring, nothing knocked out, too little
    to cut).  ``ko_value`` is the projection value as a function of tau,
    the value sv.mon_rebates holds at tau = k dt for step k."""
    n = sv.n_nodes
    if sv.it or sv.n_time < 1 or list(sv.mon_steps) != list(range(1, sv.n_time + 1)):
        return None
    if sv.ko_lo < 0 and sv.ko_hi >= n:
        return None
    K = margin_nodes(sv)
    if K is None:
        return None
    a = max(0, sv.ko_lo + 1 - K) if sv.ko_lo >= 0 else 0
    b = min(n - 1, sv.ko_hi - 1 + K) if sv.ko_hi < n else n - 1
    if b - a + 1 < 3 or b - a + 1 > MAX_KEEP * n:
        return None
    w = replace(sv, v_init=np.ascontiguousarray(sv.v_init[a:b + 1]),
                lower=ko_value if a > 0 else sv.lower,
                upper=ko_value if b < n - 1 else sv.upper,
                ko_lo=sv.ko_lo - a if sv.ko_lo >= 0 else -1,
                ko_hi=sv.ko_hi - a if sv.ko_hi < n else 1 << 30)
    return KoWindow(solve=w, a=a, n_nodes=n, fill=float(sv.mon_rebates[-1]))
