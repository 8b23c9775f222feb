"""ctypes binding of libfdcn.so (include/fdcn.h).

This is the product's only route to the time-stepping hot path.  There is no
CPU fallback: if the library is missing, or no gfx950 device is visible when a
solve is requested, the call raises.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "_lib")
# the in-tree build; bench.py --lib points it at an A/B build before the
# first load (timing of kernel variants only)
LIB_PATH = os.path.join(LIB_DIR, "libfdcn.so")
REPO_ROOT = os.path.dirname(HERE)
HEADER_PATH = os.path.join(REPO_ROOT, "include", "fdcn.h")
DIAG_HEADER_PATH = os.path.join(REPO_ROOT, "include", "fdcn_diag.h")

# mirrors of the enums in include/fdcn.h
P_DT, P_A, P_C, P_BC, P_TAU0 = 0, 1, 2, 3, 4
P_LO_C0, P_LO_E0, P_LO_C1, P_LO_E1 = 5, 6, 7, 8
P_HI_C0, P_HI_E0, P_HI_C1, P_HI_E1 = 9, 10, 11, 12
NPARAM = 13
I_LO_FORM, I_HI_FORM, I_KO_LO, I_KO_HI, I_MON_START, I_MON_COUNT, I_TAU_MODE = range(7)
NIPARAM = 7
ABI_VERSION = 5

EXPORTED = ("fdcn_cn_batch", "fdcn_it_batch", "fdcn_cn_batch_dev", "fdcn_it_batch_dev",
            "fdcn_plan", "fdcn_sm_extent", "fdcn_log_grid", "fdcn_dividend_jump",
            "fdcn_rr_barrier_batch",
            "fdcn_rr_barrier_batch_dev", "fdcn_double_barrier_batch",
            "fdcn_double_barrier_batch_dev", "fdcn_last_error", "fdcn_device_count",
            "fdcn_abi_version", "fdcn_select_device", "fdcn_current_device",
            "fdcn_tau_sequence", "fdcn_tau_runs", "fdcn_session_create",
            "fdcn_session_destroy", "fdcn_session_slots", "fdcn_session_host_buffer",
            "fdcn_session_march",
            "fdcn_session_dividend_jump", "fdcn_session_greeks", "fdcn_session_fetch",
            "fdcn_vc_batch", "fdcn_vc_batch_dev", "fdcn_vc_plan", "fdcn_barrier_plan",
            "fdcn_vmath", "fdcn_american_plan", "fdcn_device_ordinals")
# include/fdcn_diag.h: test / tuning entry points, not the product boundary
DIAG_EXPORTED = ("fdcn_force_variant", "fdcn_forced_variant", "fdcn_variant_name",
                 "fdcn_vc_force_variant", "fdcn_vc_variant_name", "fdcn_vc_forms")
FLAVOUR_THROUGHPUT, FLAVOUR_LATENCY, FLAVOUR_PAIRED = 0, 1, 2
VC_NDIAG = 6
RR_NPARAM, RR_NFLAG = 8, 5
DB_NPARAM, DB_NFLAG = 8, 3


class FdcnError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

_PD = ctypes.POINTER(ctypes.c_double)
_PI = ctypes.POINTER(ctypes.c_int32)
_I = ctypes.c_int32
_V = ctypes.c_void_p
_I64 = ctypes.c_int64


def elf_dynamic_names(path: str) -> dict:
    """{"soname": str | None, "needed": [str]} from an ELF64 shared object's
    dynamic section (read from the file; nothing is loaded)."""
    import struct
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError(f"{path}: not an ELF64 object")
    e_phoff, = struct.unpack_from("<Q", data, 0x20)
    e_phentsize, e_phnum = struct.unpack_from("<HH", data, 0x36)
    loads, dyn = [], None
    for i in range(e_phnum):
        p_type, _, p_offset, p_vaddr, _, p_filesz = struct.unpack_from(
            "<IIQQQQ", data, e_phoff + i * e_phentsize)
        if p_type == 1:
            loads.append((p_vaddr, p_offset, p_filesz))
        elif p_type == 2:
            dyn = (p_offset, p_filesz)
    if dyn is None:
        return {"soname": None, "needed": []}

    def file_off(vaddr):
        for va, off, sz in loads:
            if va <= vaddr < va + sz:
                return off + vaddr - va
        raise ValueError("address outside the loaded segments")
    entries, strtab = [], None
    for k in range(dyn[1] // 16):
        tag, val = struct.unpack_from("<qQ", data, dyn[0] + 16 * k)
        if tag == 0:
            break
        if tag == 5:  # DT_STRTAB
            strtab = file_off(val)
        entries.append((tag, val))

    def cstr(o):
        return data[strtab + o:data.index(b"\0", strtab + o)].decode()
    return {"soname": next((cstr(v) for t, v in entries if t == 14), None),  # DT_SONAME
            "needed": [cstr(v) for t, v in entries if t == 1]}              # DT_NEEDED


def _torch_hip_runtime() -> Optional[str]:
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except Exception:
        return None
    if spec is None or not spec.origin:
        return None
    path = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    return path if os.path.exists(path) else None


def _preload_hip_runtime() -> None:
    """Load the HIP runtime PyTorch ships (torch/lib/libamdhip64.so) before
    libfdcn, so a process that uses both -- device tensors for the _dev entry
    points, torch.distributed over RCCL -- has ONE HIP runtime.  libfdcn's
    dependency (soname libamdhip64.so.7) then binds to the copy already
    loaded; loading libfdcn first would map /opt/rocm's copy and torch would
    later add a second one (its NEEDED entry is the unversioned name).
    Only when torch's copy carries the SONAME libfdcn needs: another major
    version would not satisfy libfdcn's dependency, and preloading it would
    itself make two runtimes.  torch is not imported."""
    path = _torch_hip_runtime()
    if path is None:
        return
    try:
        want = [n for n in elf_dynamic_names(LIB_PATH)["needed"] if n.startswith("libamdhip64")]
        have = elf_dynamic_names(path)["soname"]
    except (OSError, ValueError):
        return
    if want and have == want[0]:
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def lib() -> ctypes.CDLL:
    """Load libfdcn.so (raises FdcnError if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise FdcnError(
                    f"{LIB_PATH} is missing: build it with `python -c 'import "
                    f"__graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
            _preload_hip_runtime()
            L = ctypes.CDLL(LIB_PATH)
            # the version first: a stale build (or bench.py --lib pointing at
            # an older A/B build) fails here with a clear message rather than
            # with an AttributeError on a symbol it does not export
            ver = getattr(L, "fdcn_abi_version", None)
            if ver is None:
                raise FdcnError(f"{LIB_PATH} exports no fdcn_abi_version: ABI version "
                                f"mismatch; rebuild")
            ver.restype = ctypes.c_int
            ver.argtypes = []
            got = int(ver())
            if got != ABI_VERSION:
                raise FdcnError(f"libfdcn.so ABI version mismatch (library {got}, package "
                                f"{ABI_VERSION}); rebuild")
            L.fdcn_cn_batch.restype = _I
            L.fdcn_cn_batch.argtypes = [_I, _I, _I, _I, _PD, _PI, _PD, _I, _PI, _PD, _PD]
            L.fdcn_it_batch.restype = _I
            L.fdcn_it_batch.argtypes = [_I, _I, _I, _I, _PD, _PI, _PD, _PD, _PD]
            L.fdcn_cn_batch_dev.restype = _I
            L.fdcn_cn_batch_dev.argtypes = [_I, _I, _I, _I, _V, _V, _V, _I, _V, _V, _V, _I, _V,
                                            _I64, _V]
            L.fdcn_it_batch_dev.restype = _I
            L.fdcn_it_batch_dev.argtypes = [_I, _I, _I, _I, _V, _V, _V, _V, _V, _I, _V, _I64, _V]
            L.fdcn_plan.restype = _I
            L.fdcn_plan.argtypes = [_I, _I, _I, _I, _I, _PI, _PI, _PI, _PI,
                                    ctypes.POINTER(ctypes.c_int64)]
            L.fdcn_sm_extent.restype = _I
            L.fdcn_sm_extent.argtypes = [_I, _I, _I, _I, _PD]
            L.fdcn_log_grid.restype = _I
            L.fdcn_log_grid.argtypes = [ctypes.c_double, ctypes.c_double, _I, _V, _V]
            L.fdcn_dividend_jump.restype = _I
            L.fdcn_dividend_jump.argtypes = [_I, _V, _V, ctypes.c_double, ctypes.c_double, _V]
            L.fdcn_rr_barrier_batch.restype = _I
            L.fdcn_rr_barrier_batch.argtypes = [_I, _V, _V, _V, _V]
            L.fdcn_rr_barrier_batch_dev.restype = _I
            L.fdcn_rr_barrier_batch_dev.argtypes = [_I, _V, _V, _V, _V, _V]
            L.fdcn_double_barrier_batch.restype = _I
            L.fdcn_double_barrier_batch.argtypes = [_I, _I, _V, _V, _V]
            L.fdcn_double_barrier_batch_dev.restype = _I
            L.fdcn_double_barrier_batch_dev.argtypes = [_I, _I, _V, _V, _V, _V]
            L.fdcn_last_error.restype = ctypes.c_char_p
            L.fdcn_last_error.argtypes = []
            L.fdcn_device_count.restype = ctypes.c_int
            L.fdcn_device_count.argtypes = []
            L.fdcn_device_ordinals.restype = ctypes.c_int
            L.fdcn_device_ordinals.argtypes = [_PI, _I]
            L.fdcn_abi_version.restype = ctypes.c_int
            L.fdcn_abi_version.argtypes = []
            L.fdcn_tau_sequence.restype = _I
            L.fdcn_tau_sequence.argtypes = [ctypes.c_double, ctypes.c_double, _I, _V]
            L.fdcn_tau_runs.restype = _I
            L.fdcn_tau_runs.argtypes = [ctypes.c_double, ctypes.c_double, _I]
            L.fdcn_vc_batch.restype = _I
            L.fdcn_vc_batch.argtypes = [_I, _I, _I, _I, _V, _V, _V, _V, _I, _V, _V, _V]
            L.fdcn_vc_batch_dev.restype = _I
            L.fdcn_vc_batch_dev.argtypes = [_I, _I, _I, _I, _V, _V, _V, _V, _I, _V, _V, _V, _V,
                                            _I64, _V]
            L.fdcn_vc_plan.restype = _I
            L.fdcn_vc_plan.argtypes = [_I, _I, _PI, _PI, ctypes.POINTER(ctypes.c_int64)]
            L.fdcn_barrier_plan.restype = _I
            L.fdcn_barrier_plan.argtypes = [_I, _V, _V, ctypes.c_double, _I, _I, _I, _I,
                                            ctypes.c_double, ctypes.c_double, _I, _I, _V, _V,
                                            _V, _V, _V, _V, _V, _V, _V]
            L.fdcn_american_plan.restype = _I
            L.fdcn_american_plan.argtypes = [_I, _V, _V, _I, ctypes.c_double, ctypes.c_double,
                                             _V, _V, _V, _V, _V, _V, _V]
            L.fdcn_vmath.restype = _I
            L.fdcn_vmath.argtypes = [_I, ctypes.c_int64, _V, _V]
            L.fdcn_select_device.restype = ctypes.c_int
            L.fdcn_select_device.argtypes = [_I]
            L.fdcn_current_device.restype = ctypes.c_int
            L.fdcn_current_device.argtypes = []
            L.fdcn_force_variant.restype = _I
            L.fdcn_force_variant.argtypes = [_I, _I, _I]
            L.fdcn_forced_variant.restype = _I
            L.fdcn_forced_variant.argtypes = [_PI, _PI, _PI]
            L.fdcn_variant_name.restype = _I
            L.fdcn_variant_name.argtypes = [_I, _I, _I, _I, ctypes.c_char_p, _I]
            L.fdcn_vc_force_variant.restype = _I
            L.fdcn_vc_force_variant.argtypes = [_I, _I, _I]
            L.fdcn_vc_variant_name.restype = _I
            L.fdcn_vc_variant_name.argtypes = [_I, _I, ctypes.c_char_p, _I]
            L.fdcn_vc_forms.restype = _I
            L.fdcn_vc_forms.argtypes = [_I, _I, _I, _I, _PD, _PI]
            _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        msg = lib().fdcn_last_error().decode(errors="replace")
        raise FdcnError(f"fdcn error {rc}: {msg}")


_n_devices: Optional[int] = None


def device_count() -> int:
    """gfx950 devices visible (queried once per process)."""
    global _n_devices
    if _n_devices is None:
        _n_devices = int(lib().fdcn_device_count())
    return _n_devices


def device_ordinals() -> list:
    """HIP ordinals of the visible gfx950 devices (ascending)."""
    buf = (ctypes.c_int32 * 64)()
    n = int(lib().fdcn_device_ordinals(buf, 64))
    return [int(buf[i]) for i in range(min(n, 64))]


def require_device() -> None:
    if device_count() < 1:
        raise FdcnError("no gfx950 (MI355X) device visible; the CN engine has no CPU path")


def select_device(ordinal: int) -> None:
    """Make `ordinal` the calling thread's HIP device (one process per GPU:
    the local rank).  The host-array entry points run there."""
    _check(lib().fdcn_select_device(int(ordinal)))


def current_device() -> int:
    d = int(lib().fdcn_current_device())
    if d < 0:
        _check(d)
    return d


def force_variant(waves: int, npt: int = 0, flavour: int = FLAVOUR_THROUGHPUT) -> None:
    """Diagnostics (include/fdcn_diag.h): pin every later march launch of this
    process to the compiled variant (waves, npt, flavour) where it fits;
    waves = 0 clears.  Tests and A/B tools only -- the product never calls it."""
    _check(lib().fdcn_force_variant(int(waves), int(npt), int(flavour)))


def forced_variant() -> tuple:
    w, n, f = (ctypes.c_int32() for _ in range(3))
    _check(lib().fdcn_forced_variant(ctypes.byref(w), ctypes.byref(n), ctypes.byref(f)))
    return w.value, n.value, f.value


def variant_name(n_nodes: int, it_mode: bool, k_cap: int = 0, *, B: int) -> str:
    """The kernel instance ("fdcn_march<IT,W,NPT,ZG>") a launch of B scenarios
    runs, the override included (diagnostics, include/fdcn_diag.h)."""
    buf = ctypes.create_string_buffer(64)
    _check(lib().fdcn_variant_name(int(B), int(n_nodes), 1 if it_mode else 0, int(k_cap), buf, 64))
    return buf.value.decode()


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def plan(n_nodes: int, it_mode: bool, k_cap: int = 0, n_time: int = 1, *, B: int) -> dict:
    """Launch geometry for a launch of B scenarios.  B is required: the kernel
    variant -- and so ws_bytes_per_scen -- depends on it (small batches spread
    a scenario over more waves), and a workspace sized for another B is
    rejected by the _dev entry points."""
    w, npt, spb, lds = (ctypes.c_int32() for _ in range(4))
    ws = ctypes.c_int64()
    _check(lib().fdcn_plan(B, n_nodes, n_time, 1 if it_mode else 0, k_cap, ctypes.byref(w),
                           ctypes.byref(npt), ctypes.byref(spb), ctypes.byref(lds),
                           ctypes.byref(ws)))
    return dict(waves=w.value, npt=npt.value, scen_per_block=spb.value, lds_bytes=lds.value,
                ws_bytes_per_scen=ws.value)


def sm_extent(n_nodes: int, n_time: int, n_ranna: int, params: np.ndarray) -> int:
    P = _f64(params).reshape(-1, NPARAM)
    rc = lib().fdcn_sm_extent(P.shape[0], n_nodes, n_time, n_ranna, P.ctypes.data_as(_PD))
    if rc < 0:
        _check(rc)
    return int(rc)


def _out_array(out, B: int, n_nodes: int) -> np.ndarray:
    """v_out: a new array, or the caller's own (C-contiguous float64 [B,
    n_nodes]) -- a caller that launches repeatedly reuses one buffer instead
    of paying first-touch page faults on a fresh one per call."""
    if out is None:
        return np.empty((B, n_nodes), dtype=np.float64)
    if (not isinstance(out, np.ndarray) or out.dtype != np.float64 or out.shape != (B, n_nodes)
            or not out.flags["C_CONTIGUOUS"] or not out.flags["WRITEABLE"]):
        raise FdcnError(f"out must be a writeable C-contiguous float64 array of shape {(B, n_nodes)}")
    return out


def cn_batch(n_nodes: int, n_time: int, n_ranna: int, params, iparams, v_init, mon_step,
             mon_rebate, out=None) -> np.ndarray:
    """Host-array European/KO batch solve -> v_out [B, n_nodes] (into `out`
    when given)."""
    require_device()
    P, I, V = _f64(params), _i32(iparams), _f64(v_init)
    B = V.shape[0]
    ms = _i32(mon_step if len(mon_step) else [0])
    mr = _f64(mon_rebate if len(mon_rebate) else [0.0])
    out = _out_array(out, B, n_nodes)
    _check(lib().fdcn_cn_batch(B, n_nodes, n_time, n_ranna, P.ctypes.data_as(_PD),
                               I.ctypes.data_as(_PI), V.ctypes.data_as(_PD), len(mon_step),
                               ms.ctypes.data_as(_PI), mr.ctypes.data_as(_PD),
                               out.ctypes.data_as(_PD)))
    return out


def it_batch(n_nodes: int, n_time: int, n_ranna: int, params, iparams, v_init,
             payoff, out=None) -> np.ndarray:
    """Host-array American (Ikonen-Toivanen) batch solve -> v_out [B, n_nodes]
    (into `out` when given)."""
    require_device()
    P, I, V, F = _f64(params), _i32(iparams), _f64(v_init), _f64(payoff)
    B = V.shape[0]
    out = _out_array(out, B, n_nodes)
    _check(lib().fdcn_it_batch(B, n_nodes, n_time, n_ranna, P.ctypes.data_as(_PD),
                               I.ctypes.data_as(_PI), V.ctypes.data_as(_PD),
                               F.ctypes.data_as(_PD), out.ctypes.data_as(_PD)))
    return out


def cn_batch_dev(B: int, n_nodes: int, n_time: int, n_ranna: int, params_ptr: int,
                 iparams_ptr: int, v_init_ptr: int, n_mon: int, mon_step_ptr: int,
                 mon_rebate_ptr: int, v_out_ptr: int, k_cap: int, workspace_ptr: int,
                 workspace_bytes: int, stream_ptr: int) -> None:
    """Device-pointer launch (asynchronous on `stream_ptr`)."""
    _check(lib().fdcn_cn_batch_dev(B, n_nodes, n_time, n_ranna, params_ptr, iparams_ptr,
                                   v_init_ptr, n_mon, mon_step_ptr, mon_rebate_ptr, v_out_ptr,
                                   k_cap, workspace_ptr, workspace_bytes, stream_ptr))


def it_batch_dev(B: int, n_nodes: int, n_time: int, n_ranna: int, params_ptr: int,
                 iparams_ptr: int, v_init_ptr: int, payoff_ptr: int, v_out_ptr: int,
                 k_cap: int, workspace_ptr: int, workspace_bytes: int, stream_ptr: int) -> None:
    _check(lib().fdcn_it_batch_dev(B, n_nodes, n_time, n_ranna, params_ptr, iparams_ptr,
                                   v_init_ptr, payoff_ptr, v_out_ptr, k_cap, workspace_ptr,
                                   workspace_bytes, stream_ptr))


def vc_batch(n_nodes: int, n_time: int, n_ranna: int, diag, bnd, v_init, iparams, mon_step,
             mon_rebate) -> np.ndarray:
    """Spot-space CN with per-row coefficients (fdcn_vc_batch) -> v_out [B, n_nodes].
    diag [B, 2, VC_NDIAG, n_nodes], bnd [B, n_time, 2]."""
    require_device()
    D, Bd, V, I = _f64(diag), _f64(bnd), _f64(v_init), _i32(iparams)
    B = V.shape[0]
    ms = _i32(mon_step if len(mon_step) else [0])
    mr = _f64(mon_rebate if len(mon_rebate) else [0.0])
    out = np.empty((B, n_nodes), dtype=np.float64)
    _check(lib().fdcn_vc_batch(B, n_nodes, n_time, n_ranna, D.ctypes.data, Bd.ctypes.data,
                               V.ctypes.data, I.ctypes.data, len(mon_step), ms.ctypes.data,
                               mr.ctypes.data, out.ctypes.data))
    return out


def vc_batch_dev(B: int, n_nodes: int, n_time: int, n_ranna: int, diag_ptr: int, bnd_ptr: int,
                 v_init_ptr: int, iparams_ptr: int, n_mon: int, mon_step_ptr: int,
                 mon_rebate_ptr: int, v_out_ptr: int, workspace_ptr: int, workspace_bytes: int,
                 stream_ptr: int) -> None:
    """fdcn_vc_batch_dev: every array already on the device (bench, sessions)."""
    _check(lib().fdcn_vc_batch_dev(B, n_nodes, n_time, n_ranna, diag_ptr, bnd_ptr, v_init_ptr,
                                   iparams_ptr, n_mon, mon_step_ptr, mon_rebate_ptr, v_out_ptr,
                                   workspace_ptr, workspace_bytes, stream_ptr))


def vc_plan(n_nodes: int, *, B: int) -> dict:
    w, npt = ctypes.c_int32(), ctypes.c_int32()
    ws = ctypes.c_int64()
    _check(lib().fdcn_vc_plan(B, n_nodes, ctypes.byref(w), ctypes.byref(npt), ctypes.byref(ws)))
    return dict(waves=w.value, npt=npt.value, ws_bytes_per_scen=ws.value)


def vc_force_variant(waves: int = 0, npt: int = 0, stencil_only: bool = False) -> None:
    """Diagnostics (include/fdcn_diag.h): pin later fdcn_vc launches to the
    compiled variant (waves, npt) where it fits, and/or make every scenario
    take the stencil form; (0, 0, False) clears.  Tests and A/B tools only."""
    _check(lib().fdcn_vc_force_variant(int(waves), int(npt), 1 if stencil_only else 0))


def vc_variant_name(n_nodes: int, *, B: int) -> str:
    buf = ctypes.create_string_buffer(64)
    _check(lib().fdcn_vc_variant_name(int(B), int(n_nodes), buf, 64))
    return buf.value.decode()


def vc_forms(n_nodes: int, n_time: int, n_ranna: int, diag: np.ndarray) -> np.ndarray:
    """Form each scenario of a fdcn_vc launch takes (1 pointwise, 0 stencil):
    the factor kernel's classification of diag [B, 2, 6, n_nodes], on the host."""
    D = _f64(diag)
    B = D.shape[0]
    out = np.zeros(B, np.int32)
    _check(lib().fdcn_vc_forms(B, int(n_nodes), int(n_time), int(n_ranna),
                               D.ctypes.data_as(_PD), out.ctypes.data_as(_PI)))
    return out


VM_EXP, VM_LOG, VM_SQRT, VM_SQUARE = 0, 1, 2, 3


def vmath(op: int, x) -> np.ndarray:
    """libm exp / log / sqrt / pow(x, 2) elementwise (bit-identical to CPython's
    math.exp / math.log / math.sqrt and float ** 2), host only."""
    X = _f64(x)
    Y = np.empty_like(X)
    _check(lib().fdcn_vmath(int(op), X.size, X.ctypes.data, Y.ctypes.data))
    return Y


BP_NROW, BP_NFLAG = 10, 4  # FDCN_BP_NROW / FDCN_BP_NFLAG
AP_NJOB, AP_NOUT = 5, 4    # FDCN_AP_NJOB / FDCN_AP_NOUT


def american_plan(job: np.ndarray, call: np.ndarray, n_space: int, s_max_mult: float,
                  T: float, with_grids: bool = False, payoff_out=None) -> dict:
    """fdcn_american_plan: grid, payoff, coefficients and readouts of J
    American (row, sigma) jobs, host only (see include/fdcn.h).
    ``payoff_out`` (optional): a callable n -> float64 array of n elements
    the payoffs are written into (a session's pinned host buffer)."""
    job = np.ascontiguousarray(job, np.float64)
    call = np.ascontiguousarray(call, np.int32)
    J = job.shape[0]
    if job.shape != (J, AP_NJOB) or call.shape != (J,):
        raise ValueError("american_plan: job [J, 5] and call [J] expected")
    n1 = int(n_space) + 1
    out = dict(params=np.empty((J, NPARAM)), iparams=np.empty((J, NIPARAM), np.int32),
               payoff=(np.empty(J * n1) if payoff_out is None
                       else payoff_out(J * n1)).reshape(J, n1), s_nodes=np.empty((J, n1)) if with_grids else None,
               rint=np.empty((2 * J, GK_NRINT), np.int32), rdbl=np.empty((2 * J, GK_NRDBL)),
               gout=np.empty((J, AP_NOUT)))
    _check(lib().fdcn_american_plan(
        J, job.ctypes.data, call.ctypes.data, int(n_space), float(s_max_mult), float(T),
        out["params"].ctypes.data, out["iparams"].ctypes.data, out["payoff"].ctypes.data,
        out["s_nodes"].ctypes.data if with_grids else None, out["rint"].ctypes.data,
        out["rdbl"].ctypes.data, out["gout"].ctypes.data))
    return out
GK_NPARAM, GK_NRINT, GK_NRDBL = 8, 5, 8


def barrier_plan(row: np.ndarray, flag: np.ndarray, T: float, n_space: int, n_time: int,
                 grid_mode: int, k_tail: float, dv_sigma: float,
                 rebate_at_hit: bool, mon_k: np.ndarray, v_init_out=None) -> dict:
    """fdcn_barrier_plan: base and sigma-bumped solve of every row (solve
    q = 2 row + bump), host only.  Returns the launch arrays (params, iparams,
    v_init, mon_rebate), the readouts (rint with the solve index in column 0,
    rdbl), the per-row epilogue parameters and n_nodes.  ``v_init_out``
    (optional): a callable n -> float64 array of n elements the initial
    vectors are written into (a session's pinned host buffer)."""
    row = np.ascontiguousarray(row, np.float64)
    flag = np.ascontiguousarray(flag, np.int32)
    R = row.shape[0]
    if row.shape != (R, BP_NROW) or flag.shape != (R, BP_NFLAG):
        raise ValueError("barrier_plan: row [R, 10] and flag [R, 4] expected")
    mon = np.ascontiguousarray(mon_k, np.int32)
    if grid_mode == 0:
        n_max = int(math.ceil(k_tail * n_time)) + 2
    else:
        n_max = int(n_space)
    Q = 2 * R
    out = dict(params=np.empty((Q, NPARAM)), iparams=np.empty((Q, NIPARAM), np.int32),
               v_init=np.empty(Q * n_max) if v_init_out is None else v_init_out(Q * n_max),
               mon_rebate=np.empty(max(1, Q * mon.size)),
               rint=np.empty((Q, GK_NRINT), np.int32), rdbl=np.empty((Q, GK_NRDBL)),
               tparams=np.empty((R, GK_NPARAM)))
    nn = np.zeros(1, np.int32)
    _check(lib().fdcn_barrier_plan(
        R, row.ctypes.data, flag.ctypes.data, float(T), int(n_space), int(n_time),
        int(grid_mode), n_max, float(k_tail), float(dv_sigma), 1 if rebate_at_hit else 0,
        mon.size, mon.ctypes.data if mon.size else None, out["params"].ctypes.data,
        out["iparams"].ctypes.data, out["v_init"].ctypes.data, out["mon_rebate"].ctypes.data,
        out["rint"].ctypes.data, out["rdbl"].ctypes.data, out["tparams"].ctypes.data,
        nn.ctypes.data))
    N = int(nn[0])
    out["n_nodes"] = N
    out["v_init"] = out["v_init"][:Q * N].reshape(Q, N)
    out["mon_rebate"] = out["mon_rebate"][:Q * mon.size]
    return out


def log_grid(x_min: float, dx: float, n: int):
    """(x, s) with x[i] = x_min + i*dx and s = exp(x) for i = 0..n, computed in
    libfdcn with the C library's exp -- bit-identical to the reference's
    ``[math.exp(x_min + i * dx) for i in range(n + 1)]`` (host only, no device)."""
    x = np.empty(n + 1, dtype=np.float64)
    s = np.empty(n + 1, dtype=np.float64)
    _check(lib().fdcn_log_grid(float(x_min), float(dx), int(n), x.ctypes.data, s.ctypes.data))
    return x, s


def tau_sequence(tau0: float, dt: float, n: int) -> np.ndarray:
    """tau after each of n steps of `tau = tau + dt` (FDCN_I_TAU_MODE = 1), as
    the kernels evaluate it (host only)."""
    out = np.empty(max(n, 0), dtype=np.float64)
    _check(lib().fdcn_tau_sequence(float(tau0), float(dt), int(n), out.ctypes.data))
    return out


def tau_runs(tau0: float, dt: float, n: int) -> int:
    rc = int(lib().fdcn_tau_runs(float(tau0), float(dt), int(n)))
    if rc < 0:
        _check(rc)
    return rc


def rr_barrier_batch(params, flags):
    """Reiner-Rubinstein barrier batch on the GPU -> (price[B], vanilla[B]).
    params [B, RR_NPARAM] = s, b, r, t, x, sigma, h, k; flags [B, RR_NFLAG]."""
    require_device()
    P = _f64(params).reshape(-1, RR_NPARAM)
    F = _i32(flags).reshape(-1, RR_NFLAG)
    if P.shape[0] != F.shape[0]:
        raise ValueError("params and flags disagree on B")
    B = P.shape[0]
    price = np.empty(B, dtype=np.float64)
    vanilla = np.empty(B, dtype=np.float64)
    _check(lib().fdcn_rr_barrier_batch(B, P.ctypes.data, F.ctypes.data, price.ctypes.data,
                                       vanilla.ctypes.data))
    return price, vanilla


def double_barrier_batch(params, flags, m: int = 4):
    """Double-barrier (Douady series) batch on the GPU -> price[B].
    params [B, DB_NPARAM] = S, X, L, U, sigma, b, r, T; flags [B, DB_NFLAG]."""
    require_device()
    P = _f64(params).reshape(-1, DB_NPARAM)
    F = _i32(flags).reshape(-1, DB_NFLAG)
    if P.shape[0] != F.shape[0]:
        raise ValueError("params and flags disagree on B")
    B = P.shape[0]
    price = np.empty(B, dtype=np.float64)
    _check(lib().fdcn_double_barrier_batch(B, int(m), P.ctypes.data, F.ctypes.data,
                                           price.ctypes.data))
    return price


def dividend_jump(s_nodes, v, cash_div: float, strike_call: float = -1.0) -> np.ndarray:
    """V(t_d-, S) = V(t_d+, S - D) through the natural cubic spline, and for
    calls (strike_call >= 0) max with the payoff -- in libfdcn, bit-identical to
    fd_american_equity.py:479-553/732-772 (host only, no device)."""
    S = _f64(s_nodes)
    V = _f64(v)
    if S.shape != V.shape or S.ndim != 1:
        raise ValueError("s_nodes and v must be 1-D arrays of the same length")
    out = np.empty_like(V)
    rc = lib().fdcn_dividend_jump(S.shape[0], S.ctypes.data, V.ctypes.data, float(cash_div),
                                  float(strike_call), out.ctypes.data)
    if rc != 0:
        msg = lib().fdcn_last_error().decode(errors="replace")
        raise ValueError(msg)
    return out
