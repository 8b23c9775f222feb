"""Parity of the exact kernels bench.py times, at the lengths it times them.

The bench launches thousands of scenarios; the kernel variant depends on the
batch size, and a small test batch would normally get another one (the
single-trade flavour below 1024 waves).  Here a sample of the bench's OWN
scenarios (bench.build_*, same draws, same façades) is marched on the full
BASELINE grid with the variant pinned (include/fdcn_diag.h) to the instance
the bench's batch size selects -- asserted by name -- and every node of every
output is compared with the C oracle (oracle/fdcn_oracle.c):

  config 2  American IT put 2048 x 4096, accumulated tau (TAU_MODE = 1), the
            two-pass IT solve (fd_american_equity.py:559-726)
  config 3  discrete barrier KO 1024 x 2000, daily monitoring, the capped
            4-wave split-form variant with its block-start boundary loads
            (discrete_barrier_fdm_pricer.py:442-547)
  config 5  double knock-out 4096 x 8192, projection on every step, the
            recovery-form variant

Tolerance: max_j |V_gpu - V_oracle| <= 1e-10 * max(1, max_j |V_oracle|) per
scenario (test_gpu_kernels.py); bench.py applies the same bound to the timed
launch's own output in its "parity" record.
"""
import os
import sys

import numpy as np
import pytest

from finite_difference_amd import capi
from finite_difference_amd.engine import Engine

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import bench  # noqa: E402

TOL = 1e-10


def _oracle(g):
    from oracle import oracle
    if g.it:
        return oracle.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                               g.payoff, 16)
    return oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                           g.mon_step, g.mon_rebate, 16)


def _gpu(g):
    from finite_difference_amd.engine import HipBackend
    return HipBackend().run_group(g)


# (workload, bench batch, sample of scenario indices)
CASES = [("american", 4096, [0, 1, 700, 1401, 2100, 2801, 3500, 4095]),
         ("barrier", 10000, [0, 1, 2, 3, 4, 5, 6, 7, 2501, 5002, 7503, 9999]),
         ("double", 2048, [0, 511, 1024, 2047])]


@pytest.mark.parametrize("workload,B,sample", CASES, ids=[c[0] for c in CASES])
def test_bench_kernel_vs_oracle_full_length(workload, B, sample, force_variant):
    builder, ns, nt, is_it, _ = bench.WORKLOADS[workload]
    g = builder(B, ns, nt, seed=0, select=sample)
    assert g.B == len(sample) and g.n_time == nt
    if is_it:
        assert np.all(g.iparams[:, capi.I_TAU_MODE] == 1)  # the American accumulated tau
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    timed = capi.variant_name(g.n_nodes, is_it, k_cap, B=B)
    p = capi.plan(g.n_nodes, is_it, k_cap, n_time=nt, B=B)
    force_variant(p["waves"], p["npt"], 0)
    assert capi.variant_name(g.n_nodes, is_it, k_cap, B=g.B) == timed, timed
    got = _gpu(g)
    ref = _oracle(g)
    assert np.all(np.isfinite(got))
    scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
    rel = np.max(np.abs(got - ref), axis=1) / scale
    print(f"[{workload} {timed} {g.n_nodes}x{nt} B={g.B}] max_rel_err={rel.max():.3e}")
    assert rel.max() <= TOL, rel


def test_timed_instances_are_the_throughput_variants():
    """The instances the bench times at its default batches (VERDICT r2
    item 1 names them)."""
    assert capi.variant_name(2049, True, B=4096) == "fdcn_march<1,1,32,0>"
    assert capi.variant_name(1024, False, B=10000) == "fdcn_march<0,1,16,0>"
    assert capi.variant_name(4097, False, B=2048) == "fdcn_march<0,1,64,0>"


def test_bench_spot_vc_kernel_vs_oracle_full_length():
    """bench.py --workload spot_vc times fdcn_vc_march<1,16> on 4 096
    Pricer2 knock-outs (1 025 nodes, 2 000 steps); every one of its trades
    takes the pointwise form.  A sample of the bench's own trades on that
    instance (pinned: a small batch would take shorter chunks), at full
    length, every node vs the C oracle (oracle_vc_batch, the reference's
    per-step Thomas, discrete_barrier_fdm_pricer_2.py:336-428)."""
    from oracle import oracle
    B = bench.DEFAULT_BATCH["spot_vc"]
    full = bench.build_spot_vc(24, 1024, 2000)
    timed = capi.vc_variant_name(full.n_nodes, B=B)
    assert timed == "fdcn_vc_march<1,16>"
    assert np.all(capi.vc_forms(full.n_nodes, full.n_time, full.n_ranna, full.diag) == 1)
    p = capi.vc_plan(full.n_nodes, B=B)
    capi.vc_force_variant(p["waves"], p["npt"], False)
    try:
        assert capi.vc_variant_name(full.n_nodes, B=full.B) == timed
        got = _gpu_vc(full)
    finally:
        capi.vc_force_variant(0, 0, False)
    ref = oracle.vc_batch(full.n_nodes, full.n_time, full.n_ranna, full.diag, full.bnd,
                          full.v_init, full.iparams, full.mon_step, full.mon_rebate, 16)
    scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
    rel = np.max(np.abs(got - ref), axis=1) / scale
    print(f"[spot_vc {timed} {full.n_nodes}x{full.n_time} B={full.B}] max_rel_err={rel.max():.3e}")
    assert rel.max() <= TOL, rel


def _gpu_vc(g):
    from finite_difference_amd.engine import HipBackend
    return HipBackend().run_vc_group(g)
