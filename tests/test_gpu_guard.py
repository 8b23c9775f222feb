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
