"""ctypes loader for the CPU oracle (oracle/fdcn_oracle.c).

TEST INFRASTRUCTURE ONLY.  Importable by tests/, by __graft_entry__.smoke()
and by bench.py's cpu_baseline leg, where it is the checker or the timed CPU
baseline.  The product package (finite_difference_amd) never imports it.

Parity status: PINNED.  ``ref_*`` restate the reference's loops literally and
are checked bit-for-bit against tests/golden/*.json (vectors produced by the
reference itself, see tests/golden/make_golden.py) and against the reference's
committed scenario_results*.csv.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

_lib: Optional[ctypes.CDLL] = None

_D = ctypes.c_double
_I = ctypes.c_int
_I32 = ctypes.c_int32
_PD = ctypes.POINTER(ctypes.c_double)
_PI = ctypes.POINTER(ctypes.c_int)
_PI32 = ctypes.POINTER(ctypes.c_int32)

# barrier type codes of fdcn_oracle.c
BT_CODES = {"none": 0, "down-and-out": 1, "up-and-out": 2, "double-out": 3,
            "down-and-in": 4, "up-and-in": 4, "double-in": 4}


def build() -> str:
    """Compile oracle/build/liboracle.so (gcc, no GPU needed)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_ref_barrier_solve.restype = _I
        L.oracle_ref_barrier_solve.argtypes = [
            _PD, _I, _I, _D, _D, _D, _D, _D, _D, _I, _I, _D, _I, _I, _D, _I, _D, _D, _I, _D,
            _PI, _I, _I, _PD]
        L.oracle_ref_cnlog_solve.restype = _I
        L.oracle_ref_cnlog_solve.argtypes = [
            _PD, _I, _I, _D, _D, _D, _D, _D, _I, _D, _I, _I, _D, _I, _D, _D, _PI, _I, _I, _PD]
        L.oracle_ref_american_segment.restype = _I
        L.oracle_ref_american_segment.argtypes = [
            _PD, _I, _D, _PD, _D, _D, _I, _I, _I, _D, _D, _D, _I, _D, _PD]
        L.oracle_cn_batch.restype = _I
        L.oracle_cn_batch.argtypes = [_I32, _I32, _I32, _I32, _PD, _PI32, _PD, _I32, _PI32, _PD,
                                      _PD, _I32]
        L.oracle_it_batch.restype = _I
        L.oracle_it_batch.argtypes = [_I32, _I32, _I32, _I32, _PD, _PI32, _PD, _PD, _PD, _I32]
        L.oracle_vc_batch.restype = _I
        L.oracle_vc_batch.argtypes = [_I32, _I32, _I32, _I32, _PD, _PD, _PD, _PI32, _I32, _PI32,
                                      _PD, _PD, _I32]
        L.oracle_max_threads.restype = _I
        _lib = L
    return _lib


def _pd(a: np.ndarray):
    return a.ctypes.data_as(_PD)


def _pi(a: np.ndarray):
    return a.ctypes.data_as(_PI)


def _f64(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


def _i32(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32))


# ---------------------------------------------------------------------------
# literal restatements (reference inputs)
# ---------------------------------------------------------------------------
def ref_barrier_solve(s_nodes: Sequence[float], n_time: int, T: float, dx: float, sigma: float,
                      r: float, b: float, q: float, rannacher_steps: int, option_type: str,
                      K: float, barrier_type: str, lower_barrier, upper_barrier,
                      rebate_amount: float, rebate_at_hit: bool, carry: float,
                      monitor_idx: Sequence[int], apply_KO: bool) -> np.ndarray:
    """discrete_barrier_fdm_pricer.py:442-547 -> list of length N_s."""
    s = _f64(s_nodes)
    n_space = len(s) - 1
    mon = _i32(sorted(monitor_idx)) if len(monitor_idx) else _i32([0])
    out = np.empty(n_space + 1, dtype=np.float64)
    n = lib().oracle_ref_barrier_solve(
        _pd(s), n_space, int(n_time), T, dx, sigma, r, b, q, int(rannacher_steps),
        1 if option_type == "call" else 0, K, BT_CODES[barrier_type],
        lower_barrier is not None, float(lower_barrier or 0.0), upper_barrier is not None,
        float(upper_barrier or 0.0), rebate_amount, bool(rebate_at_hit), carry,
        _pi(mon), len(monitor_idx), bool(apply_KO), _pd(out))
    if n < 0:
        raise RuntimeError("oracle_ref_barrier_solve failed")
    return out[:n]


def ref_cnlog_solve(s_nodes: Sequence[float], n_time: int, T: float, dx: float, sigma: float,
                    r_disc: float, b_carry: float, option_type: str, K: float,
                    barrier_type: str, lower_barrier, upper_barrier, rebate: float,
                    monitor_idx: Sequence[int], apply_KO: bool) -> np.ndarray:
    """discrete_barrier_fdm_pricer_cn.py:219-302 -> list of length N+1."""
    s = _f64(s_nodes)
    N = len(s) - 1
    mon = _i32(sorted(monitor_idx)) if len(monitor_idx) else _i32([0])
    out = np.empty(N + 1, dtype=np.float64)
    n = lib().oracle_ref_cnlog_solve(
        _pd(s), N, int(n_time), T, dx, sigma, r_disc, b_carry,
        1 if option_type.lower() == "call" else 0, K, BT_CODES[barrier_type.lower()],
        lower_barrier is not None, float(lower_barrier or 0.0), upper_barrier is not None,
        float(upper_barrier or 0.0), rebate, _pi(mon), len(monitor_idx), bool(apply_KO),
        _pd(out))
    if n < 0:
        raise RuntimeError("oracle_ref_cnlog_solve failed")
    return out


def ref_american_segment(s_nodes: Sequence[float], dx: float, v_init: Sequence[float],
                         tau_start: float, tau_end: float, n_steps: int,
                         restart_rannacher: bool, rannacher_steps: int, sigma: float,
                         r: float, b: float, option_type: str, strike_pde: float) -> np.ndarray:
    """fd_american_equity.py:559-726."""
    s = _f64(s_nodes)
    v = _f64(v_init)
    out = np.empty_like(s)
    rc = lib().oracle_ref_american_segment(
        _pd(s), len(s) - 1, dx, _pd(v), tau_start, tau_end, int(n_steps),
        bool(restart_rannacher), int(rannacher_steps), sigma, r, b,
        1 if option_type == "call" else 0, strike_pde, _pd(out))
    if rc < 0:
        raise RuntimeError("oracle_ref_american_segment failed")
    return out


# ---------------------------------------------------------------------------
# plan-level solvers (same inputs as the C ABI in include/fdcn.h)
# ---------------------------------------------------------------------------
def cn_batch(n_nodes: int, n_time: int, n_ranna: int, params, iparams, v_init, mon_step,
             mon_rebate, nthreads: int = 1) -> np.ndarray:
    P, I, V = _f64(params), _i32(iparams), _f64(v_init)
    B = V.shape[0]
    ms = _i32(mon_step) if len(mon_step) else _i32([0])
    mr = _f64(mon_rebate) if len(mon_rebate) else _f64([0.0])
    out = np.empty((B, n_nodes), dtype=np.float64)
    rc = lib().oracle_cn_batch(B, n_nodes, n_time, n_ranna, _pd(P), I.ctypes.data_as(_PI32),
                               _pd(V), len(mon_step), ms.ctypes.data_as(_PI32), _pd(mr),
                               _pd(out), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle_cn_batch failed ({rc})")
    return out


def it_batch(n_nodes: int, n_time: int, n_ranna: int, params, iparams, v_init, payoff,
             nthreads: int = 1) -> np.ndarray:
    P, I, V, F = _f64(params), _i32(iparams), _f64(v_init), _f64(payoff)
    B = V.shape[0]
    out = np.empty((B, n_nodes), dtype=np.float64)
    rc = lib().oracle_it_batch(B, n_nodes, n_time, n_ranna, _pd(P), I.ctypes.data_as(_PI32),
                               _pd(V), _pd(F), _pd(out), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle_it_batch failed ({rc})")
    return out


def vc_batch(n_nodes: int, n_time: int, n_ranna: int, diag, bnd, v_init, iparams, mon_step,
             mon_rebate, nthreads: int = 1) -> np.ndarray:
    """Spot-space CN with per-row coefficients on the fdcn_vc_batch plan
    (discrete_barrier_fdm_pricer_2.py:336-428): sequential Thomas per step."""
    D, Bd, V, I = _f64(diag), _f64(bnd), _f64(v_init), _i32(iparams)
    B = V.shape[0]
    ms = _i32(mon_step) if len(mon_step) else _i32([0])
    mr = _f64(mon_rebate) if len(mon_rebate) else _f64([0.0])
    if Bd.size == 0:
        Bd = _f64([0.0, 0.0])
    out = np.empty((B, n_nodes), dtype=np.float64)
    rc = lib().oracle_vc_batch(B, n_nodes, n_time, n_ranna, _pd(D), _pd(Bd), _pd(V),
                               I.ctypes.data_as(_PI32), len(mon_step), ms.ctypes.data_as(_PI32),
                               _pd(mr), _pd(out), int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle_vc_batch failed ({rc})")
    return out


def max_threads() -> int:
    return int(lib().oracle_max_threads())
