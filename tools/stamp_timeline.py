#!/usr/bin/env python3
"""Per-phase timeline of the config-5 march from in-kernel s_memtime stamps.

Needs a diagnostic build of the library (the product build has no stamps):
    ABFLAGS=-DFDCN_STAMPS bash tools/build_ab.sh st
then, on the GPU box:
    python tools/stamp_timeline.py ab/st/libfdcn.so [B] > gpurun_out/.../timeline.json

The march (fdcn_march<0,1,64,0>, the recovery form) stamps eight points of
each of steps 1024..1055 for the first 64 scenarios (FDCN_STAMP in
fdcn_kernels.hip) into the scenario's Rannacher save slice of the workspace:
0 step start, 1 forward pass 1 + join done, 2 first-half chain done, 3 second
half + backward aggregate done, 4 fused backward pass done, 5 Sherman-Morrison
/ bookkeeping done, 6 knock-out done, 7 step end.  Printed: the median cycles
of each phase per step, and for the waves that shared a SIMD (same XCC, SE,
CU, SIMD from HW_ID / XCC_ID) how their phases overlapped.  Stamps perturb
the timing (each costs an s_memtime wait and a store): read the phase shares,
not the absolute step time.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["pass1+join", "first-half chain", "second half + bwd agg", "fused backward",
          "SM / bookkeeping", "knock-out", "advance / loop"]
STEP0, NSTEPS, NSCEN = 1024, 32, 64


def main():
    lib = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    from finite_difference_amd import capi
    capi.LIB_PATH = os.path.abspath(lib)
    import torch
    import bench
    g = bench.build_double(B, 4096, 8192, seed=0)
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    plan = capi.plan(g.n_nodes, False, k_cap, n_time=g.n_time, B=g.B)
    assert (plan["waves"], plan["npt"]) == (1, 64), plan
    dev = torch.device("cuda", 0)
    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    MS = torch.from_numpy(g.mon_step).to(dev)
    MR = torch.from_numpy(g.mon_rebate).to(dev)
    out = torch.empty_like(V0)
    wsb = plan["ws_bytes_per_scen"] * g.B
    ws = torch.zeros(wsb // 8, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()

    def launch():
        capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                          V0.data_ptr(), len(g.mon_step), MS.data_ptr(), MR.data_ptr(),
                          out.data_ptr(), k_cap, ws.data_ptr(), wsb, stream.cuda_stream)
    launch()
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record(stream)
    launch()
    t1.record(stream)
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1)
    # the save slice is the workspace's last region: 64 x NPT doubles per
    # scenario after the rows (boundary table, if any, and knock-out masks)
    w = ws.cpu().numpy()
    save = 64 * plan["npt"]
    vs = w[g.B * (plan["ws_bytes_per_scen"] // 8 - save):].reshape(g.B, save)[:NSCEN]
    stamps = vs[:, :NSTEPS * 16].reshape(NSCEN, NSTEPS, 16)[:, :, :8].view(np.int64)
    hw = vs[:, 15].astype(np.int64)
    xcc = vs[:, 14].astype(np.int64)
    # gfx9 HW_ID: wave [3:0], simd [5:4], cu [11:8], sh [12], se [15:13]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    d = np.diff(stamps, axis=2)           # [scen, step, 7] phase durations
    step = stamps[:, 1:, 0] - stamps[:, :-1, 0]
    rec = {"lib": lib, "B": g.B, "kernel_ms": ms,
           "median_step_cycles": float(np.median(step)),
           "median_phase_cycles": {n: float(np.median(d[:, :, i])) for i, n in enumerate(PHASES)},
           "mean_phase_cycles": {n: float(np.mean(d[:, :, i])) for i, n in enumerate(PHASES)}}
    # waves sharing a SIMD among the stamped scenarios
    pairs = []
    key = list(zip(xcc, se, cu, simd))
    for a in range(NSCEN):
        for b in range(a + 1, NSCEN):
            if key[a] == key[b]:
                pairs.append((a, b))
    rec["simd_pairs"] = len(pairs)
    if pairs:
        # fraction of wave a's fused-backward phase (VALU-dense) that overlaps
        # wave b's knock-out or first-half chain (VALU-light), and vice versa
        def spans(s, i):
            return [(int(s[j, i]), int(s[j, i + 1])) for j in range(NSTEPS)]
        ov = []
        for a, b in pairs[:16]:
            for (i_dense, i_light) in ((3, 5), (3, 1)):
                A = spans(stamps[a], i_dense)
                Bs = spans(stamps[b], i_light)
                tot = sum(e - s for s, e in A)
                hit = sum(max(0, min(e1, e2) - max(s1, s2)) for s1, e1 in A for s2, e2 in Bs)
                ov.append({"pair": [a, b], "dense": PHASES[i_dense], "light": PHASES[i_light],
                           "overlap_frac": hit / max(tot, 1)})
        rec["overlap"] = ov
        a, b = pairs[0]
        base = min(stamps[a, 0, 0], stamps[b, 0, 0])
        rec["pair0_first4_steps"] = {
            "a": (stamps[a, :4] - base).tolist(), "b": (stamps[b, :4] - base).tolist()}
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
