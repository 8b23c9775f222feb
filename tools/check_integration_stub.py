"""Check the reference-side ctypes stub of INTEGRATION.md (build container only).

The stub is taken verbatim from INTEGRATION.md.  Its library handle is pointed
at the CPU oracle (oracle/build/liboracle.so: same ABI arrays, plus a thread
count), so the arrays the stub builds are solved by the reference's own
arithmetic.  The patched reference methods must then return the same lists as
the unpatched ones, bit for bit -- which proves the stub hands libfdcn exactly
the problem the reference solves.

Needs /root/reference (loaded as in tests/golden/make_golden.py); never runs
on the GPU box.  Usage:  python tools/check_integration_stub.py
"""
import ctypes
import math
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, ROOT)

import make_golden as G  # noqa: E402
from oracle import oracle  # noqa: E402


class _OracleAsFdcn:
    """libfdcn's host entry points, answered by the C oracle."""

    def __init__(self):
        self._o = ctypes.CDLL(oracle.build_lib_path() if hasattr(oracle, "build_lib_path")
                              else oracle.LIB_PATH)
        self.fdcn_cn_batch = self._wrap(self._o.oracle_cn_batch)
        self.fdcn_it_batch = self._wrap(self._o.oracle_it_batch)
        self.fdcn_last_error = lambda: b"oracle"
        self.fdcn_abi_version = lambda: 4

    @staticmethod
    def _wrap(fn):
        class F:
            argtypes = None
            restype = None

            def __call__(self, *a):
                return fn(*a, ctypes.c_int32(1))
        return F()


def load_stub():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.search(r'```python\n("""ctypes binding of libfdcn.*?)```', text, re.S).group(1)
    code = code.replace('_L = ctypes.CDLL(os.environ["FDCN_LIB"])', "_L = _FAKE")
    ns = {"_FAKE": _OracleAsFdcn()}
    exec(compile(code, "INTEGRATION.md:stub", "exec"), ns)
    return ns


def main():
    oracle.build()
    stub = load_stub()
    worst = 0
    bm = G.load_barrier()
    cls = bm.DiscreteBarrierFDMPricer
    orig = cls._solve_grid
    specs = [
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
    for s in specs:
        for ko in (True, False):
            p = G.make_barrier(bm, **dict(s))
            ref = orig(p, ko)
            cls._solve_grid = stub["solve_grid_fdcn"]
            try:
                got = p._solve_grid(ko)
            finally:
                cls._solve_grid = orig
            assert len(got) == len(ref), (len(got), len(ref))
            bad = sum(1 for x, y in zip(got, ref) if x != y)
            worst = max(worst, bad)
            print(f"barrier {s['option_type']} {s['barrier_type']} ko={ko}: n={len(ref)} "
                  f"mismatches={bad}")
    am = G.load_american()
    A = am.AmericanFDMPricer
    orig_seg = A._solve_segment
    import datetime as dt
    for opt, divs in (("put", []), ("call", [(dt.date(2025, 8, 10), 1.5)])):
        c = G.curve(0.073)
        kw = dict(spot=176.39, strike=172.0, valuation_date=G.VAL, maturity_date=G.MAT,
                  sigma=0.3, option_type=opt, discount_curve=c, forward_curve=c,
                  dividend_schedule=divs, num_space_nodes=120, num_time_steps=90,
                  rannacher_steps=2)
        ref = A(**kw)._solve_grid()
        A._solve_segment = stub["solve_segment_fdcn"]
        try:
            got = A(**kw)._solve_grid()
        finally:
            A._solve_segment = orig_seg
        # the stub asks for tau accumulation (TAU_MODE=1), as the reference does
        bad = sum(1 for x, y in zip(got, ref) if x != y)
        worst = max(worst, bad)
        print(f"american {opt} divs={len(divs)}: n={len(ref)} mismatches={bad}")
    print("OK: stub reproduces the reference bit for bit" if worst == 0 else "MISMATCH")
    return 0 if worst == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
