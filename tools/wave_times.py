#!/usr/bin/env python3
"""When each wave of the config-5 launch starts and ends (diagnostic build).

    ABFLAGS=-DFDCN_WAVE_TIMES bash tools/build_ab.sh wt
    python tools/wave_times.py ab/wt/libfdcn.so > gpurun_out/.../wave_times.json

fdcn_march<0,1,64,0> (the recovery form) writes, per scenario, its wave's
s_memtime at entry and after the march plus HW_ID / XCC_ID into the
scenario's Rannacher save slice (FDCN_WAVE_TIMES in fdcn_kernels.hip).  One
launch of the bench's 2 048-scenario batch (two waves per SIMD, one round):
the spread of the start and end times, the waves' durations, and for the
waves that shared a SIMD how far apart they finished -- the time the SIMD
ran one wave alone at the end of the launch -- and the durations per XCD
and shader engine.  s_memtime is a per-XCD counter: only times on one XCD
are compared with each other.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = sys.argv[1]
    from finite_difference_amd import capi
    capi.LIB_PATH = os.path.abspath(lib)
    import torch
    import bench
    g = bench.build_double(2048, 4096, 8192, seed=0)
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
    for _ in range(40):  # past the clock ramp
        launch()
    torch.cuda.synchronize()
    recs = []
    for _ in range(3):
        launch()
        torch.cuda.synchronize()
        w = ws.cpu().numpy()
        # the save slice is the workspace's last region (64 x NPT doubles a
        # scenario, after the knock-out mask rows)
        save = 64 * plan["npt"]
        vs = w[g.B * (plan["ws_bytes_per_scen"] // 8 - save):].reshape(g.B, save)
        t0 = vs[:, 0].view(np.int64).astype(np.float64)
        t1 = vs[:, 1].view(np.int64).astype(np.float64)
        hw = vs[:, 2].astype(np.int64)
        xcc = vs[:, 3].astype(np.int64)
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        se = (hw >> 13) & 7
        base = t0.min()
        dur = t1 - t0
        key = xcc * 1000 + se * 100 + cu * 4 + simd
        pairs = {}
        for i, k in enumerate(key):
            pairs.setdefault(int(k), []).append(i)
        gaps = [abs(t1[v[0]] - t1[v[1]]) for v in pairs.values() if len(v) == 2]
        starts = [abs(t0[v[0]] - t0[v[1]]) for v in pairs.values() if len(v) == 2]
        pct = lambda a: [float(np.percentile(a, q)) for q in (0, 10, 50, 90, 100)]
        recs.append({
            "duration_pct": pct(dur),
            "simds": len(pairs), "simds_with_two": len(gaps),
            "pair_end_gap_pct": pct(gaps) if gaps else None,
            "pair_start_gap_pct": pct(starts) if starts else None,
            "per_xcc_duration": {int(x): {"median": float(np.median(dur[xcc == x])),
                                          "min": float(dur[xcc == x].min()),
                                          "max": float(dur[xcc == x].max()),
                                          "waves": int(np.sum(xcc == x))}
                                 for x in np.unique(xcc)},
            "per_se_duration_median": {f"{int(x)}.{int(e)}": float(np.median(
                dur[(xcc == x) & (se == e)])) for x in np.unique(xcc) for e in np.unique(se)
                if np.any((xcc == x) & (se == e))}})
    raw = {"duration": dur.tolist(), "xcc": xcc.tolist(), "hw_id": hw.tolist(),
           "start_in_xcc": [float(t0[i] - t0[xcc == xcc[i]].min()) for i in range(g.B)]}
    print(json.dumps({"lib": lib, "units": "s_memtime ticks", "launches": recs,
                      "last_launch_per_scenario": raw}, indent=1))


if __name__ == "__main__":
    main()
