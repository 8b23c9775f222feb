"""The C-ABI library loads on a CPU-only host and exports every symbol the
header declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from finite_difference_amd import capi


def _header_symbols():
    txt = open(capi.HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(fdcn_[a-z_]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert _header_symbols() == sorted(capi.EXPORTED)


def test_library_exports_all_symbols():
    assert os.path.exists(capi.LIB_PATH), "run __graft_entry__.build() first"
    L = ctypes.CDLL(capi.LIB_PATH)
    for name in _header_symbols():
        assert hasattr(L, name), name


def test_abi_version_and_plan_without_gpu():
    L = capi.lib()
    assert L.fdcn_abi_version() == capi.ABI_VERSION
    p = capi.plan(2049, True)
    assert p["waves"] >= 1 and p["npt"] * 64 * p["waves"] >= 2047
    p = capi.plan(1024, False)
    assert p["npt"] * 64 * p["waves"] >= 1022


def test_invalid_size_reports_error():
    import pytest
    with pytest.raises(capi.FdcnError):
        capi.plan(3, False)


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
