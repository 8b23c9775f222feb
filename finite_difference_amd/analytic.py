"""Closed-form barrier engines (host-side, scalar): the analytic boundary of
the hot path and the cross-checks for the FD kernels.

* ``BarrierEngine``: Reiner-Rubinstein / Merton A-F factors for a single
  continuously monitored barrier with rebate timing and "crossed" status --
  same constructor, attributes and results as barrier_engine.py:17-190.
* ``DoubleBarrier``: Ikeda-Kunitomo / Douady series for double knock-out /
  knock-in calls and puts (double _barrier.py:6-134).  The reference's put
  branch sets the lower integration limit to the constant 1 (:95) instead of
  the log-barrier l; that is kept by default for parity
  (``corrected_put=False``) and fixed with ``corrected_put=True``.
* ``black_scholes``: generalized Black-Scholes with carry b.
* ``barrier_engine_batch`` / ``double_barrier_batch``: the same two engines
  for many contracts at once, one GPU thread per contract (libfdcn
  ``fdcn_rr_barrier_batch`` / ``fdcn_double_barrier_batch``).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
from scipy.special import ndtr


class norm:  # noqa: N801 - scipy.stats.norm.cdf is ndtr((x - 0) / 1); called directly
    cdf = staticmethod(ndtr)


def _norm_rebate_timing(s: Optional[str], default: str) -> str:
    if s is None:
        return default
    s = s.strip().lower()
    if s in ("hit", "pay at hit", "at hit"):
        return "hit"
    if s in ("expiry", "exp", "maturity", "pay at expiry", "at expiry", "expiary",
             "pay at expiary"):
        return "expiry"
    raise ValueError("rebate timing must be 'hit' or 'expiry'")


def black_scholes(callput: str, S: float, K: float, r: float, b: float, sigma: float,
                  T: float) -> float:
    """Generalized Black-Scholes (cost of carry b)."""
    sq = np.sqrt(T)
    d1 = (np.log(S / K) + (b + 0.5 * sigma ** 2) * T) / (sigma * sq)
    d2 = d1 - sigma * sq
    if callput == "c":
        return S * np.exp((b - r) * T) * norm.cdf(d1) - K * np.exp(-r * T) * norm.cdf(d2)
    return K * np.exp(-r * T) * norm.cdf(-d2) - S * np.exp((b - r) * T) * norm.cdf(-d1)


class BarrierEngine:
    """Single continuous barrier, Reiner & Rubinstein (1991) factors.

    optionflag 'c'/'p', directionflag 'u'/'d', in_out_flag 'i'/'o';
    k is the cash rebate; rebate_timing_in default 'expiry', rebate_timing_out
    default 'hit'; barrier_status None/'not_crossed'/'crossed'."""

    def __init__(self, s: float, b: float, r: float, t: float, x: float, sigma: float, h: float,
                 optionflag: str, directionflag: str, in_out_flag: str, k: float,
                 barrier_status: Optional[str] = None, rebate_timing_in: Optional[str] = None,
                 rebate_timing_out: Optional[str] = None):
        self.s, self.b, self.r, self.t = float(s), float(b), float(r), float(t)
        self.x, self.sigma, self.h, self.k = float(x), float(sigma), float(h), float(k)
        if self.sigma <= 0 or self.t <= 0:
            raise ValueError("sigma and t must be positive.")
        if optionflag.lower() not in ("c", "p"):
            raise ValueError("optionflag must be 'c' or 'p'.")
        if directionflag.lower() not in ("u", "d"):
            raise ValueError("directionflag must be 'u' or 'd'.")
        if in_out_flag.lower() not in ("i", "o"):
            raise ValueError("in_out_flag must be 'i' or 'o'.")
        if barrier_status not in (None, "crossed", "not_crossed"):
            raise ValueError("barrier_status must be None, 'crossed', or 'not_crossed'.")
        self.optionflag = optionflag.lower()
        self.directionflag = directionflag.lower()
        self.in_out_flag = in_out_flag.lower()
        self.barrier_status = barrier_status
        self.phi = 1 if self.optionflag == "c" else -1
        self.eta = -1 if self.directionflag == "u" else 1
        self.rebate_timing_in = _norm_rebate_timing(rebate_timing_in, "expiry")
        self.rebate_timing_out = _norm_rebate_timing(rebate_timing_out, "hit")

        N = norm.cdf
        s, x, h, t, r, b, sig = self.s, self.x, self.h, self.t, self.r, self.b, self.sigma
        phi, eta, K = self.phi, self.eta, self.k
        sqrtT = np.sqrt(t)
        sigRT = sig * sqrtT
        ebmt = np.exp((b - r) * t)
        erT = np.exp(-r * t)
        mu = (b - 0.5 * sig ** 2) / sig ** 2
        lam = np.sqrt(mu ** 2 + 2.0 * r / sig ** 2)
        lead = (1.0 + mu) * sigRT
        x1 = np.log(s / x) / sigRT + lead
        x2 = np.log(s / h) / sigRT + lead
        y1 = np.log(h ** 2 / (s * x)) / sigRT + lead
        y2 = np.log(h / s) / sigRT + lead
        z = np.log(h / s) / sigRT + lam * sigRT
        hs = h / s
        p2mu1, p2mu = hs ** (2.0 * (mu + 1.0)), hs ** (2.0 * mu)
        pml, pmnl = hs ** (mu + lam), hs ** (mu - lam)

        def leg(w, arg_s, arg_x, pw_s=1.0, pw_x=1.0):
            return phi * s * ebmt * pw_s * N(w * arg_s) - phi * x * erT * pw_x * N(w * arg_x)

        A = leg(phi, x1, x1 - sigRT)
        B = leg(phi, x2, x2 - sigRT)
        C = leg(eta, y1, y1 - sigRT, p2mu1, p2mu)
        D = leg(eta, y2, y2 - sigRT, p2mu1, p2mu)
        E = K * erT * (N(eta * (x2 - sigRT)) - p2mu * N(eta * (y2 - sigRT)))
        F = K * (pml * N(eta * z) + pmnl * N(eta * (z - 2.0 * lam * sigRT)))
        self.elements = {"x1": x1, "x2": x2, "y1": y1, "y2": y2, "z": z, "mu": mu,
                         "lambda": lam}
        self.factors = {"A": A, "B": B, "C": C, "D": D, "E": E, "F": F}
        self.vanilla_value = A

        reb_in = E if self.rebate_timing_in == "expiry" else F
        reb_out = F if self.rebate_timing_out == "hit" else (K * erT - E)
        if barrier_status == "crossed":
            if self.in_out_flag == "i":
                self.price_value = A
            else:
                self.price_value = K if self.rebate_timing_out == "hit" else K * erT
            return
        x_gt_h = (self.x - self.h) > 1e-14
        table = {  # (option, direction, in/out) -> (value if X > H, value otherwise)
            ("c", "d", "i"): (C, A - B + D), ("c", "d", "o"): (A - C, B - D),
            ("c", "u", "i"): (A, B - C + D), ("c", "u", "o"): (0.0, A - B + C - D),
            ("p", "d", "i"): (B - C + D, A), ("p", "d", "o"): (A - B + C - D, 0.0),
            ("p", "u", "i"): (A - B + D, C), ("p", "u", "o"): (B - D, A - C),
        }
        hi_lo = table[(self.optionflag, self.directionflag, self.in_out_flag)]
        base = hi_lo[0] if x_gt_h else hi_lo[1]
        self.price_value = base + (reb_in if self.in_out_flag == "i" else reb_out)

    def get_factors(self) -> Dict[str, float]:
        return self.factors

    def get_elements(self) -> Dict[str, float]:
        return self.elements

    def price(self) -> float:
        return self.price_value

    def vanilla(self) -> float:
        return self.vanilla_value


class DoubleBarrier:
    """Double barrier knock-in / knock-out, Douady-style series in
    sigma-scaled log coordinates, terms n = -m..m."""

    def __init__(self, S, X, L, U, sigma, callflag: str, inflag: str, m: int = 4,
                 corrected_put: bool = False):
        self.S, self.X, self.L, self.U = float(S), float(X), float(L), float(U)
        self.sigma = float(sigma)
        self.callflag = callflag.lower()
        self.inflag = inflag.lower()
        self.m = int(m)
        self.corrected_put = corrected_put

    @staticmethod
    def _bs_price(callput: str, S: float, K: float, r: float, b: float, sigma: float,
                  T: float) -> float:
        return black_scholes(callput, S, K, r, b, sigma, T)

    def _series(self, lam: float, alpha: float, beta: float, u: float, delta: float,
                T: float) -> float:
        sq = np.sqrt(T)
        tot = []
        for n in range(-self.m, self.m + 1):
            sh = 2 * n * delta
            I_ = np.exp(-2 * n * lam * delta) * (norm.cdf((beta + sh) / sq - lam * sq)
                                                 - norm.cdf((alpha + sh) / sq - lam * sq))
            J_ = np.exp(2 * lam * (n * delta + u)) * (norm.cdf((2 * u - alpha + sh) / sq + lam * sq)
                                                      - norm.cdf((2 * u - beta + sh) / sq + lam * sq))
            tot.append(I_ - J_)
        return np.sum(tot)

    def price(self, b: float, r: float, T: float) -> float:
        bs = self._bs_price(self.callflag, self.S, self.X, r, b, self.sigma, T)
        u = np.log(self.U / self.S) / self.sigma
        k = np.log(self.X / self.S) / self.sigma
        l_ = np.log(self.L / self.S) / self.sigma
        lam = b / self.sigma - self.sigma / 2.0
        lam_p = b / self.sigma + self.sigma / 2.0
        delta = u - l_
        if self.callflag == "c":
            if self.X < self.U:
                alpha, beta = max(k, l_), u
                p1 = self._series(lam_p, alpha, beta, u, delta, T)
                p2 = self._series(lam, alpha, beta, u, delta, T)
                out = np.exp((b - r) * T) * self.S * p1 - np.exp(-r * T) * self.X * p2
            else:
                out = 0.0
        elif self.callflag == "p":
            if self.X > self.L:
                alpha = l_ if self.corrected_put else 1  # reference :95 uses 1
                beta = min(k, u)
                p1 = self._series(lam, alpha, beta, u, delta, T)
                p2 = self._series(lam_p, alpha, beta, u, delta, T)
                out = np.exp(-r * T) * self.X * p1 - np.exp((b - r) * T) * self.S * p2
            else:
                out = 0.0
        else:
            raise ValueError("Incorrect callflag (use 'c' or 'p')")
        if self.inflag == "out":
            return out
        if self.inflag == "in":
            return bs - out
        raise ValueError("Incorrect inflag")


def _rr_encode(optionflag, directionflag, in_out_flag, barrier_status=None,
               rebate_timing_in=None, rebate_timing_out=None):
    if optionflag.lower() not in ("c", "p") or directionflag.lower() not in ("u", "d") or \
            in_out_flag.lower() not in ("i", "o"):
        raise ValueError("flags must be optionflag c/p, directionflag u/d, in_out_flag i/o")
    if barrier_status not in (None, "crossed", "not_crossed"):
        raise ValueError("barrier_status must be None, 'crossed', or 'not_crossed'.")
    bits = (1 if _norm_rebate_timing(rebate_timing_in, "expiry") == "hit" else 0) | \
        (2 if _norm_rebate_timing(rebate_timing_out, "hit") == "expiry" else 0)
    return [0 if optionflag.lower() == "c" else 1, 0 if directionflag.lower() == "u" else 1,
            0 if in_out_flag.lower() == "i" else 1, 1 if barrier_status == "crossed" else 0,
            bits]


def barrier_engine_batch(contracts):
    """BarrierEngine(**c).price() / .vanilla() for every dict ``c`` in
    ``contracts`` (BarrierEngine's keyword names), on the GPU.
    Returns (price, vanilla) arrays."""
    from . import capi
    P = np.empty((len(contracts), capi.RR_NPARAM), dtype=np.float64)
    F = np.empty((len(contracts), capi.RR_NFLAG), dtype=np.int32)
    for i, c in enumerate(contracts):
        if float(c["sigma"]) <= 0 or float(c["t"]) <= 0:
            raise ValueError("sigma and t must be positive.")
        P[i] = (c["s"], c["b"], c["r"], c["t"], c["x"], c["sigma"], c["h"], c["k"])
        F[i] = _rr_encode(c["optionflag"], c["directionflag"], c["in_out_flag"],
                          c.get("barrier_status"), c.get("rebate_timing_in"),
                          c.get("rebate_timing_out"))
    return capi.rr_barrier_batch(P, F)


def double_barrier_batch(contracts, m: int = 4):
    """DoubleBarrier(S, X, L, U, sigma, callflag, inflag, m,
    corrected_put).price(b, r, T) for every dict in ``contracts``, on the GPU."""
    from . import capi
    P = np.empty((len(contracts), capi.DB_NPARAM), dtype=np.float64)
    F = np.empty((len(contracts), capi.DB_NFLAG), dtype=np.int32)
    for i, c in enumerate(contracts):
        cf, io = c["callflag"].lower(), c["inflag"].lower()
        if cf not in ("c", "p"):
            raise ValueError("Incorrect callflag (use 'c' or 'p')")
        if io not in ("in", "out"):
            raise ValueError("Incorrect inflag")
        P[i] = (c["S"], c["X"], c["L"], c["U"], c["sigma"], c["b"], c["r"], c["T"])
        F[i] = (0 if cf == "c" else 1, 0 if io == "in" else 1,
                1 if c.get("corrected_put", False) else 0)
    return capi.double_barrier_batch(P, F, m)
