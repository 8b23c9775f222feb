"""Out-of-bounds write guard for the timed march instances.

Round 4 lost one A/B build of the config-5 kernel to hipErrorIllegalAddress
(gpurun_out/r04y.err; DESIGN.md §9 records what is known).  GPU address
sanitizing is not available on this pool, so the indexing of the kept
kernels is checked the deterministic way: every buffer the march writes
(v_out and the workspace: boundary table or Rannacher save slice, knock-out
mask row) is allocated exactly as the plan sizes it, between two 64 KiB guard
regions filled with a canary bit pattern, and after the launch

* both guards of both buffers are bit-for-bit intact (no store left its
  buffer, before or after), and
* every node of v_out agrees with the C oracle (the reads that feed them
  were the right ones).

Cases: the three bench instances pinned as the bench selects them
(fdcn_march<0,1,64,0> config 5, <0,1,16,0> config 3, <1,1,32,0> config 2),
each on a step count that fills whole 64-step chunks and on a ragged one
(the last chunk partly past n_time), on the first and last scenario of the
bench's own batch; the workspace ends at the last scenario's row, so a row
offset or length past its end lands in the tail guard.

Round 6: the same guard over EVERY compiled variant the
planner can return -- each (waves, chunk, flavour) of kVariants, CN and IT:
the multi-wave latency variants, the single-trade flavour, the paired
flavour, and the variants with the correction table in the workspace --
pinned with fdcn_force_variant on a grid that fills it, over 128 steps
(two whole chunks) and 130 (a ragged third), three scenarios each (an odd
batch: the paired flavour's last wave has no second scenario).
"""
import os
import sys

import numpy as np
import pytest
import torch

from finite_difference_amd import capi

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import bench  # noqa: E402

TOL = 1e-10
GUARD = 8192  # doubles = 64 KiB each side
CANARY = np.int64(0x7FF4DEADBEEF5A5A)  # a signalling-NaN bit pattern no march produces

# (workload, bench batch, step counts, pinned instance)
CASES = [("double", 2048, (8192, 130), "fdcn_march<0,1,64,0>"),
         ("barrier", 10000, (2000, 67), "fdcn_march<0,1,16,0>"),
         ("american", 4096, (4096, 100), "fdcn_march<1,1,32,0>")]


class Guarded:
    """n doubles between two guard regions on the device."""

    def __init__(self, n, dev):
        self.n = n
        self.buf = torch.full((GUARD + max(n, 1) + GUARD,), int(CANARY), dtype=torch.int64,
                              device=dev)

    @property
    def ptr(self):
        return self.buf.data_ptr() + GUARD * 8

    def guards_intact(self):
        b = self.buf.cpu().numpy()
        return bool(np.all(b[:GUARD] == CANARY) and np.all(b[GUARD + max(self.n, 1):] == CANARY))

    def values(self):
        return self.buf.cpu().numpy()[GUARD:GUARD + self.n].view(np.float64)


def _oracle(g):
    from oracle import oracle
    if g.it:
        return oracle.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                               g.payoff, 16)
    return oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                           g.mon_step, g.mon_rebate, 16)


@pytest.mark.parametrize("workload,B,steps,instance", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("which", [0, 1], ids=["full_chunks", "ragged"])
def test_march_stores_stay_in_their_buffers(workload, B, steps, instance, which, force_variant):
    builder, ns, _, is_it, _ = bench.WORKLOADS[workload]
    nt = steps[which]
    g = builder(B, ns, nt, seed=0, select=[0, B - 1])
    assert g.B == 2 and g.n_time == nt
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    p = capi.plan(g.n_nodes, is_it, k_cap, n_time=nt, B=B)
    force_variant(p["waves"], p["npt"], 0)
    assert capi.variant_name(g.n_nodes, is_it, k_cap, B=g.B) == instance
    p = capi.plan(g.n_nodes, is_it, k_cap, n_time=nt, B=g.B)
    dev = torch.device("cuda", 0)
    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    out = Guarded(g.B * g.n_nodes, dev)
    ws_bytes = p["ws_bytes_per_scen"] * g.B
    assert ws_bytes % 8 == 0
    ws = Guarded(ws_bytes // 8, dev)
    stream = torch.cuda.current_stream()
    if is_it:
        F = torch.from_numpy(g.payoff).to(dev)
        capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                          V0.data_ptr(), F.data_ptr(), out.ptr, k_cap, ws.ptr, ws_bytes,
                          stream.cuda_stream)
    else:
        MS = torch.from_numpy(g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)).to(dev)
        MR = torch.from_numpy(g.mon_rebate if len(g.mon_rebate) else np.zeros(1)).to(dev)
        capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                          V0.data_ptr(), len(g.mon_step), MS.data_ptr(), MR.data_ptr(), out.ptr,
                          k_cap, ws.ptr, ws_bytes, stream.cuda_stream)
    torch.cuda.synchronize()
    assert out.guards_intact(), "a store left v_out"
    assert ws.guards_intact(), "a store left the workspace"
    got = out.values().reshape(g.B, g.n_nodes)
    ref = _oracle(g)
    scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
    rel = np.max(np.abs(got - ref), axis=1) / scale
    print(f"[{workload} {instance} {g.n_nodes}x{nt} ws={ws_bytes}] max_rel_err={rel.max():.3e}")
    assert rel.max() <= TOL, rel


# every compiled variant (fdcn_kernels.hip kVariants): (waves, npt, flavour,
# table in the workspace); flavour 1 single-trade, 2 paired (CN only)
ALL_VARIANTS = [(1, 2, 0), (1, 4, 0), (1, 8, 0), (1, 12, 0), (1, 16, 0), (1, 24, 0), (1, 32, 0),
                (1, 40, 0), (1, 48, 0), (1, 64, 0), (2, 8, 0), (2, 16, 0), (2, 32, 0), (2, 40, 0),
                (4, 8, 0), (4, 16, 0), (4, 24, 0), (4, 40, 0), (8, 8, 0), (8, 16, 0), (8, 40, 0),
                (16, 8, 0), (16, 24, 0), (16, 40, 0), (1, 8, 1), (1, 16, 1), (1, 32, 1), (1, 8, 2)]
ZG_VARIANTS = [(1, 64), (4, 40), (8, 40), (16, 40)]


def _guarded_launch(g, k_cap, p):
    dev = torch.device("cuda", 0)
    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    out = Guarded(g.B * g.n_nodes, dev)
    ws_bytes = p["ws_bytes_per_scen"] * g.B
    assert ws_bytes % 8 == 0
    ws = Guarded(ws_bytes // 8, dev)
    stream = torch.cuda.current_stream()
    if g.it:
        F = torch.from_numpy(g.payoff).to(dev)
        capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                          V0.data_ptr(), F.data_ptr(), out.ptr, k_cap, ws.ptr, ws_bytes,
                          stream.cuda_stream)
    else:
        MS = torch.from_numpy(g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)).to(dev)
        MR = torch.from_numpy(g.mon_rebate if len(g.mon_rebate) else np.zeros(1)).to(dev)
        capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                          V0.data_ptr(), len(g.mon_step), MS.data_ptr(), MR.data_ptr(), out.ptr,
                          k_cap, ws.ptr, ws_bytes, stream.cuda_stream)
    torch.cuda.synchronize()
    return out, ws


def _check_guarded(g, out, ws, label, tol):
    assert out.guards_intact(), f"{label}: a store left v_out"
    assert ws.guards_intact(), f"{label}: a store left the workspace"
    got = out.values().reshape(g.B, g.n_nodes)
    ref = _oracle(g)
    scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
    rel = np.max(np.abs(got - ref), axis=1) / scale
    print(f"[{label}] max_rel_err={rel.max():.3e}")
    assert rel.max() <= tol, rel


@pytest.mark.parametrize("n_time", [128, 130], ids=["full_chunks", "ragged"])
@pytest.mark.parametrize("it", [False, True], ids=["cn", "it"])
@pytest.mark.parametrize("w,npt,fl", ALL_VARIANTS, ids=[f"w{w}n{n}f{f}" for w, n, f in ALL_VARIANTS])
def test_every_variant_stores_stay_in_their_buffers(w, npt, fl, it, n_time, force_variant):
    if it and fl == 2:
        pytest.skip("the paired flavour is compiled for the CN march only")
    from finite_difference_amd.engine import pack
    from plan_factory import random_solve
    force_variant(w, npt, fl)
    n_nodes = (32 if fl == 2 else 64 * w) * npt - 3 + 2
    # (few steps on a 40k-node grid: |fm| near 1 can need the correction
    # table in the workspace -- the variant's ZG twin, also compiled -- or
    # more LDS than the variant has: the first seeded batch that the pinned
    # variant (or its twin) takes; checked on the host by the planner)
    zg = 2 * fl if fl < 2 else 4
    want = (f"fdcn_march<{int(it)},{w},{npt},{zg}>", f"fdcn_march<{int(it)},{w},{npt},{zg | 1}>")
    for seed in range(8):
        rng = np.random.default_rng(9000 + 31 * w + npt + 7 * fl + int(it) + n_time + 1000 * seed)
        solves = [random_solve(rng, n_nodes, n_time, 2, it=it, drop_top=(i == 1))
                  for i in range(3)]
        for i, sv in enumerate(solves):
            sv.tau_accumulate = i == 2
        g = pack(solves, list(range(3)))
        k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
        name = capi.variant_name(g.n_nodes, it, k_cap, B=g.B)
        if name in want:
            break
    assert name in want, name
    p = capi.plan(g.n_nodes, it, k_cap, n_time=n_time, B=g.B)
    out, ws = _guarded_launch(g, k_cap, p)
    _check_guarded(g, out, ws, f"{name} n={n_nodes} m={n_time}",
                   TOL * max(1.0, n_nodes / 2048))


@pytest.mark.parametrize("it", [False, True], ids=["cn", "it"])
@pytest.mark.parametrize("w,npt", ZG_VARIANTS, ids=[f"w{w}n{n}" for w, n in ZG_VARIANTS])
def test_workspace_table_variants_stores_stay_in_their_buffers(w, npt, it, force_variant):
    """The ZG variants (Sherman-Morrison table in the workspace, after the
    boundary row): |fm| -> 1 on a grid that fills the variant, so the
    correction extent needs more LDS than a CU has."""
    from finite_difference_amd.engine import pack
    from plan_factory import random_solve
    force_variant(w, npt, 0)
    n_nodes, n_time = 64 * w * npt - 3 + 2, 3
    rng = np.random.default_rng(77 + w + int(it))
    solves = [random_solve(rng, n_nodes, n_time, 2, it=it) for _ in range(3)]
    g = pack(solves, list(range(3)))
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    name = capi.variant_name(g.n_nodes, it, k_cap, B=g.B)
    if name != f"fdcn_march<{int(it)},{w},{npt},1>":
        pytest.skip(f"{name}: this grid's correction extent ({k_cap}) fits LDS")
    p = capi.plan(g.n_nodes, it, k_cap, n_time=n_time, B=g.B)
    out, ws = _guarded_launch(g, k_cap, p)
    _check_guarded(g, out, ws, f"{name} n={n_nodes} k_cap={k_cap}", TOL * n_nodes / 2048)
