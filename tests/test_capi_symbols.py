"""The C-ABI library loads on a CPU-only host and exports every symbol the
header declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from finite_difference_amd import capi


def _header_symbols(path=None):
    """Functions declared by include/fdcn.h (or `path`); with path="all",
    every header under include/."""
    if path == "all":
        inc = os.path.dirname(capi.HEADER_PATH)
        return sorted(set().union(*(_header_symbols(os.path.join(inc, f))
                                    for f in os.listdir(inc) if f.endswith(".h"))))
    txt = open(path or capi.HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fdcn_[a-z_]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert _header_symbols() == sorted(capi.EXPORTED)
    assert _header_symbols(capi.DIAG_HEADER_PATH) == sorted(capi.DIAG_EXPORTED)
    assert _header_symbols("all") == sorted(capi.EXPORTED + capi.DIAG_EXPORTED)


def test_launch_path_reads_no_environment():
    """The variant choice depends on the arguments and the explicit
    diagnostics override only: no getenv in libfdcn."""
    csrc = os.path.join(os.path.dirname(capi.__file__), "csrc")
    for f in os.listdir(csrc):
        assert "getenv" not in open(os.path.join(csrc, f)).read(), f


def test_force_variant_pins_and_clears():
    big = capi.variant_name(1024, False, B=10000)
    assert big == "fdcn_march<0,1,16,0>", big
    # small batches: the single-trade flavour for the IT march only (the CN
    # flavour measured slower at every batch size, fdcn_kernels.hip choose())
    assert capi.variant_name(1024, False, B=8) == big
    assert capi.variant_name(1024, True, B=8) == "fdcn_march<1,1,16,2>"
    try:
        capi.force_variant(1, 16, 1)
        assert capi.forced_variant() == (1, 16, 1)
        assert capi.variant_name(1024, False, B=8) == "fdcn_march<0,1,16,2>"
        capi.force_variant(1, 16)
        assert capi.forced_variant() == (1, 16, 0)
        assert capi.variant_name(1024, True, B=8) == "fdcn_march<1,1,16,0>"
        assert capi.plan(1024, False, B=8)["npt"] == 16
        with pytest.raises(capi.FdcnError):
            capi.force_variant(3, 16)  # not compiled
        assert capi.forced_variant() == (1, 16, 0)  # unchanged by the failed call
    finally:
        capi.force_variant(0)
    assert capi.forced_variant() == (0, 0, 0)
    assert capi.variant_name(1024, True, B=8) == "fdcn_march<1,1,16,2>"


def test_library_exports_all_symbols():
    assert os.path.exists(capi.LIB_PATH), "run __graft_entry__.build() first"
    L = ctypes.CDLL(capi.LIB_PATH)
    for name in _header_symbols("all"):
        assert hasattr(L, name), name


def test_abi_version_and_plan_without_gpu():
    L = capi.lib()
    assert L.fdcn_abi_version() == capi.ABI_VERSION
    p = capi.plan(2049, True, B=4096)
    assert p["waves"] >= 1 and p["npt"] * 64 * p["waves"] >= 2047
    p = capi.plan(1024, False, B=10000)
    assert p["npt"] * 64 * p["waves"] >= 1022


def test_plan_depends_on_batch_size():
    """The variant, and with it the workspace, depends on B: a workspace
    planned for a large batch is too small for a single solve of the same
    grid (the _dev entry points reject it, see test_gpu_boundary.py)."""
    big = capi.plan(4097, False, n_time=4096, B=4096)
    one = capi.plan(4097, False, n_time=4096, B=1)
    assert (big["waves"], one["waves"]) == (1, 4)
    assert one["ws_bytes_per_scen"] > big["ws_bytes_per_scen"]


def test_every_grid_from_five_nodes_has_a_variant():
    """Every grid the ABI accepts (n_nodes >= 5) gets a kernel instance, at
    batch sizes that reach the single-trade, throughput and paired choices.
    (5, 7, 8 and 11 nodes had none before the two-node-chunk variants: no
    chunk length of 4+ lays 3, 5, 6 or 9 interior nodes out with at most one
    phantom slot per lane and the last lane full.)"""
    for it in (False, True):
        for n in range(5, 4200):
            for B in (1, 4096):
                p = capi.plan(n, it, B=B)
                assert p["npt"] * 64 * p["waves"] >= n - 2, (n, it, B, p)
    assert capi.plan(8, True, B=1)["npt"] == 2 and capi.plan(12, True, B=1)["npt"] == 4
    # up to the largest layout (16 waves x 64 lanes x 40 nodes + 2), and no further
    for n in list(range(4200, 40963, 97)) + [40962]:
        p = capi.plan(n, n % 2 == 0, B=1)
        assert p["npt"] * 64 * p["waves"] >= n - 2, (n, p)
    with pytest.raises(capi.FdcnError):
        capi.plan(40963, False, B=1)


def test_invalid_size_reports_error():
    import pytest
    with pytest.raises(capi.FdcnError):
        capi.plan(3, False, B=1)
    with pytest.raises(TypeError):
        capi.plan(2049, True)  # B is required


def test_log_grid_is_bitwise_math_exp():
    """fdcn_log_grid (host helper) reproduces the reference's
    [math.exp(x_min + i*dx) for i in range(n+1)] bit for bit."""
    import math
    import numpy as np
    rng = np.random.default_rng(5)
    for _ in range(20):
        x_min = float(rng.uniform(-2.0, 6.0))
        dx = float(rng.uniform(1e-5, 1e-2))
        n = int(rng.integers(1, 5000))
        x, s = capi.log_grid(x_min, dx, n)
        ref_x = [x_min + i * dx for i in range(n + 1)]
        assert x.tolist() == ref_x
        assert s.tolist() == list(map(math.exp, ref_x))


def _raw_cn(iparams, mon_step, n_time=10, B=1, n_nodes=20):
    """fdcn_cn_batch straight through ctypes: argument validation happens
    before any device is touched, so it is testable on a CPU-only host."""
    import numpy as np
    P = np.zeros((B, capi.NPARAM))
    P[:, capi.P_DT] = 0.01
    I = np.ascontiguousarray(np.asarray(iparams, dtype=np.int32).reshape(B, capi.NIPARAM))
    V = np.zeros((B, n_nodes))
    ms = np.ascontiguousarray(np.asarray(mon_step, dtype=np.int32))
    mr = np.zeros(max(1, len(ms)))
    out = np.empty_like(V)
    rc = capi.lib().fdcn_cn_batch(B, n_nodes, n_time, 2, P.ctypes.data_as(capi._PD),
                                  I.ctypes.data_as(capi._PI), V.ctypes.data_as(capi._PD),
                                  len(ms), ms.ctypes.data_as(capi._PI),
                                  mr.ctypes.data_as(capi._PD), out.ctypes.data_as(capi._PD))
    return rc, capi.lib().fdcn_last_error().decode()


def _ip(start=0, count=0, tau_mode=0):
    return [0, 0, -1, 1 << 20, start, count, tau_mode]


import pytest  # noqa: E402


@pytest.mark.parametrize("steps", [[0, 3], [3, 3], [5, 2], [4, 11]],
                         ids=["zero", "repeat", "descending", "beyond_n_time"])
def test_host_entry_rejects_bad_monitor_steps(steps):
    rc, msg = _raw_cn(_ip(0, len(steps)), steps)
    assert rc == -1 and "monitor steps" in msg, (rc, msg)


def test_host_entry_rejects_bad_tau_mode():
    rc, msg = _raw_cn(_ip(tau_mode=2), [])
    assert rc == -1 and "TAU_MODE" in msg, (rc, msg)


def test_host_entry_accepts_valid_plan_until_the_device():
    """A valid plan passes validation; without a GPU the call then fails with
    FDCN_ENODEV (or runs, on a GPU host)."""
    rc, msg = _raw_cn(_ip(0, 3, tau_mode=1), [1, 4, 10])
    assert rc in (0, -3), (rc, msg)


def test_select_device_without_gpu_is_an_error_not_a_crash():
    if capi.device_count() > 0:
        pytest.skip("GPU host")
    rc = capi.lib().fdcn_select_device(0)
    assert rc != 0


def test_concurrent_groups_reuse_the_launch_threads():
    """Engine.run issues groups of different shapes from the process-wide
    launch pool (libfdcn keeps one stream per calling thread): repeated runs
    reuse the same threads instead of creating new ones each call."""
    import threading

    import numpy as np

    from finite_difference_amd import capi, engine

    class Recording(engine.HipBackend):  # takes the concurrent path, no GPU call
        def __init__(self):
            self.threads = set()

        def run_group(self, g):
            self.threads.add(threading.get_ident())
            return g.v_init * 2.0

    solves = [engine.Solve(it=False, n_time=4, n_ranna=0, dt=0.01, coeffs=(1.0, 1.0, -2.0),
                           v_init=np.full(n, float(n)), lower=engine.Boundary(),
                           upper=engine.Boundary()) for n in (16, 32, 48)]
    be = Recording()
    eng = engine.Engine(backend=be)
    saved = capi.current_device, capi.select_device
    capi.current_device, capi.select_device = (lambda: 0), (lambda d: None)
    try:
        for _ in range(20):
            out = eng.run(solves)
            assert [float(o[0]) for o in out] == [32.0, 64.0, 96.0]
    finally:
        capi.current_device, capi.select_device = saved
    assert 1 <= len(be.threads) <= 8


def test_one_hip_runtime_after_load():
    """capi.lib() preloads torch's HIP runtime only when its SONAME
    is the one libfdcn needs, so the process maps exactly one
    libamdhip64 (checked in a fresh interpreter: this one may have loaded
    other builds)."""
    import subprocess
    import sys
    code = ("from finite_difference_amd import capi; capi.lib(); import torch; "
            "maps = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}; "
            "print(len(maps), sorted(maps))")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(capi.__file__)))
    assert p.returncode == 0, p.stderr[-2000:]
    n = int(p.stdout.split()[0])
    assert n == 1, p.stdout


def test_elf_dynamic_names_reads_needed_and_soname():
    names = capi.elf_dynamic_names(capi.LIB_PATH)
    assert any(n.startswith("libamdhip64.so") for n in names["needed"])
    torch_rt = capi._torch_hip_runtime()
    if torch_rt:
        assert capi.elf_dynamic_names(torch_rt)["soname"].startswith("libamdhip64.so")


def test_out_buffer_validation():
    """The host-array wrappers' out= must be a writeable C-contiguous float64
    [B, n_nodes] array; anything else is refused before any launch."""
    import numpy as np
    from finite_difference_amd import capi
    ok = np.empty((3, 5))
    assert capi._out_array(ok, 3, 5) is ok
    assert capi._out_array(None, 3, 5).shape == (3, 5)
    bad = [np.empty((3, 4)), np.empty((3, 5), dtype=np.float32), np.empty((5, 3)).T,
           [[0.0] * 5] * 3]
    ro = np.empty((3, 5))
    ro.flags.writeable = False
    for b in bad + [ro]:
        with pytest.raises(capi.FdcnError):
            capi._out_array(b, 3, 5)
