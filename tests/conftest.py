"""Shared pytest configuration.

Markers:
  gpu  -- needs an MI355X (gfx950) and the built HIP library; run with -m gpu.
Everything else runs on CPU (no GPU in the build container).
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--fdcn-lib", default="",
                     help="run against this build of libfdcn.so (the sanitizer build of "
                          "`make sanitize`); default: the in-tree library")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X GPU and libfdcn.so")
    alt = config.getoption("--fdcn-lib")
    if alt:
        from finite_difference_amd import capi
        capi.LIB_PATH = os.path.abspath(alt)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture
def force_variant():
    """Pin the march kernel variant (include/fdcn_diag.h) for one test:
    force_variant(waves, npt, flavour=0); cleared afterwards."""
    from finite_difference_amd import capi

    def pin(waves, npt, flavour=0):
        capi.force_variant(waves, npt, flavour)
    yield pin
    capi.force_variant(0)
