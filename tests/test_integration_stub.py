"""The reference-side ctypes stub of INTEGRATION.md, run as written.

The stub ("Reference-side ctypes stub") replaces
DiscreteBarrierFDMPricer._solve_grid (discrete_barrier_fdm_pricer.py:442-547)
and AmericanFDMPricer._solve_segment (fd_american_equity.py:559-726) with a
one-scenario call into libfdcn's host-array entry points.  Two checks, each on
the exact code block the document carries:

* CPU, build container only (skipped where /root/reference is absent, e.g.
  on the GPU box): the stub's library handle answered by the C oracle (same
  ABI arrays, the reference's arithmetic), patched into the REFERENCE classes
  and compared with their own loops -- bit for bit.  That proves the stub
  hands the library exactly the problem the reference solves.
* GPU: the stub on the real libfdcn.so (FDCN_LIB), called on this package's
  facade objects, which carry the reference's attribute names, for the
  inputs of tests/golden/barrier_cases.json (KO and no-KO) and
  american_cases.json (0/1/2 dividends: the reference's segment loop with
  the dividend jump between segments); every node against the vectors the
  reference itself produced, within the GPU bound of DESIGN.md §5.
"""
import ctypes
import math
import os
import re
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, load_golden

REFERENCE = "/root/reference"
TOL = 1e-10  # |GPU - reference| <= TOL * max(1, max|V|), tests/test_gpu_kernels.py


def stub_source() -> str:
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.search(r'```python\n("""ctypes binding of libfdcn.*?)```', text, re.S).group(1)


def load_stub(lib=None) -> dict:
    """Execute the stub; with `lib` its CDLL line is replaced by that object,
    otherwise it loads FDCN_LIB as written."""
    code = stub_source()
    ns = {}
    if lib is not None:
        code = code.replace('_L = ctypes.CDLL(os.environ["FDCN_LIB"])', "_L = _FAKE")
        ns["_FAKE"] = lib
    exec(compile(code, "INTEGRATION.md:stub", "exec"), ns)
    return ns


def test_stub_declares_the_current_abi():
    from finite_difference_amd import capi
    m = re.search(r"assert _L.fdcn_abi_version\(\) == (\d+)", stub_source())
    assert m and int(m.group(1)) == capi.ABI_VERSION


# ---------------------------------------------------------------------------
# CPU: the stub against the reference's own loops (oracle as the library)
# ---------------------------------------------------------------------------
class _OracleAsFdcn:
    """libfdcn's host entry points, answered by the C oracle."""

    def __init__(self, oracle):
        from finite_difference_amd import capi
        self._o = ctypes.CDLL(oracle.LIB_PATH)
        self.fdcn_cn_batch = self._wrap(self._o.oracle_cn_batch)
        self.fdcn_it_batch = self._wrap(self._o.oracle_it_batch)
        self.fdcn_last_error = lambda: b"oracle"
        self.fdcn_abi_version = lambda: capi.ABI_VERSION

    @staticmethod
    def _wrap(fn):
        class F:
            argtypes = None
            restype = None

            def __call__(self, *a):
                return fn(*a, ctypes.c_int32(1))
        return F()


@pytest.fixture(scope="module")
def reference_loaders():
    if not os.path.isdir(REFERENCE):
        pytest.skip("/root/reference is absent (the GPU box): the build container runs this")
    sys.path.insert(0, GOLDEN)
    import make_golden as G
    return G


BARRIER_SPECS = [
    dict(spot=229.74, strike=190.0, sigma=0.287899982, option_type="put",
         barrier_type="up-and-out", upper_barrier=260.0, rate=0.073086, num_time_steps=40),
    dict(spot=229.74, strike=190.0, sigma=0.287899982, option_type="put",
         barrier_type="down-and-out", lower_barrier=200.0, rate=0.073086, num_time_steps=40),
    dict(spot=229.74, strike=220.0, sigma=0.25, option_type="call",
         barrier_type="up-and-out", upper_barrier=250.0, rate=0.07, rebate_amount=2.0,
         rebate_at_hit=False, num_time_steps=40),
    dict(spot=229.74, strike=220.0, sigma=0.25, option_type="call",
         barrier_type="double-out", lower_barrier=205.0, upper_barrier=255.0, rate=0.07,
         rebate_amount=1.0, rebate_at_hit=True, num_time_steps=30),
]


@pytest.mark.parametrize("spec", BARRIER_SPECS, ids=lambda s: f"{s['option_type']}_"
                         f"{s['barrier_type']}")
def test_stub_barrier_reproduces_reference_loop(reference_loaders, oracle_lib, spec):
    G = reference_loaders
    stub = load_stub(_OracleAsFdcn(oracle_lib))
    bm = G.load_barrier()
    cls = bm.DiscreteBarrierFDMPricer
    orig = cls._solve_grid
    for ko in (True, False):
        p = G.make_barrier(bm, **dict(spec))
        ref = orig(p, ko)
        cls._solve_grid = stub["solve_grid_fdcn"]
        try:
            got = p._solve_grid(ko)
        finally:
            cls._solve_grid = orig
        assert got == ref, (ko, sum(1 for x, y in zip(got, ref) if x != y))


@pytest.mark.parametrize("opt,ndiv", [("put", 0), ("call", 1)])
def test_stub_american_reproduces_reference_loop(reference_loaders, oracle_lib, opt, ndiv):
    import datetime as dt
    G = reference_loaders
    stub = load_stub(_OracleAsFdcn(oracle_lib))
    am = G.load_american()
    A = am.AmericanFDMPricer
    orig = A._solve_segment
    c = G.curve(0.073)
    kw = dict(spot=176.39, strike=172.0, valuation_date=G.VAL, maturity_date=G.MAT, sigma=0.3,
              option_type=opt, discount_curve=c, forward_curve=c,
              dividend_schedule=[(dt.date(2025, 8, 10), 1.5)][:ndiv], num_space_nodes=120,
              num_time_steps=90, rannacher_steps=2)
    ref = A(**kw)._solve_grid()
    A._solve_segment = stub["solve_segment_fdcn"]
    try:
        got = A(**kw)._solve_grid()
    finally:
        A._solve_segment = orig
    assert list(got) == list(ref)


# ---------------------------------------------------------------------------
# GPU: the stub on libfdcn.so, on this package's facades
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu_stub():
    from finite_difference_amd import capi
    capi.lib()  # the package's load order (HIP runtime first), same library
    capi.require_device()
    old = os.environ.get("FDCN_LIB")
    os.environ["FDCN_LIB"] = capi.LIB_PATH
    try:
        yield load_stub()
    finally:
        if old is None:
            os.environ.pop("FDCN_LIB", None)
        else:
            os.environ["FDCN_LIB"] = old


def _close(got, ref):
    got, ref = np.asarray(got, dtype=float), np.asarray(ref, dtype=float)
    assert got.shape == ref.shape
    err = float(np.max(np.abs(got - ref))) / max(1.0, float(np.max(np.abs(ref))))
    assert err <= TOL, err
    return err


@pytest.mark.gpu
@pytest.mark.parametrize("case", load_golden("barrier_cases.json")["cases"],
                         ids=lambda c: c["name"])
def test_stub_barrier_on_libfdcn(gpu_stub, case):
    """solve_grid_fdcn on the facade DiscreteBarrierFDMPricer: the knock-out
    march (V_ko, the in-types as their out twins as the reference pricer
    marches them) and the plain one (V_noko), against the reference's own
    _solve_grid vectors."""
    from test_barrier_host import make
    p = make(case["inputs"], None)
    bt = p.barrier_type
    p.barrier_type = bt.replace("-in", "-out")
    _close(gpu_stub["solve_grid_fdcn"](p, True), case["V_ko"])
    p.barrier_type = bt
    _close(gpu_stub["solve_grid_fdcn"](p, False), case["V_noko"])
    assert p.s_nodes == case["s_nodes"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", load_golden("american_cases.json")["cases"],
                         ids=lambda c: c["name"])
def test_stub_american_on_libfdcn(gpu_stub, case):
    """solve_segment_fdcn in the reference's segment loop
    (fd_american_equity.py:778-843: Rannacher restarted in every segment of
    a call, the first of a put; the dividend jump between segments) on the
    facade AmericanFDMPricer, against the reference's _solve_grid vector."""
    from test_american_host import make
    p = make(case, None)
    p._build_log_grid()
    divs, pts, steps = p._segments(p.num_time_steps)
    v = p._payoff_array().tolist()
    for seg, ns in enumerate(steps):
        restart = seg == 0 or p.option_type == "call"
        v = gpu_stub["solve_segment_fdcn"](p, v, pts[seg], pts[seg + 1], ns, restart)
        if seg < len(divs):
            v = list(p._apply_dividend_jump(np.asarray(v), divs[seg][1]))
    assert p.s_nodes == case["s_nodes"]
    _close(v, case["V"])
