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
