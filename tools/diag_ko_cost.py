#!/usr/bin/env python3
"""Diagnostic (not a benchmark line): kernel time of a bench workload's
launch with and without its knock-out schedule, to price the projection.
Usage: python tools/diag_ko_cost.py WORKLOAD [--batch B] [--steps K]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from finite_difference_amd import capi, distributed
    dev = torch.device("cuda", distributed.bind_device())
    builder, ns, nt, is_it, _ = bench.WORKLOADS[a.workload]
    B = a.batch or bench.DEFAULT_BATCH[a.workload]
    g = builder(B, ns, nt, seed=0)
    out = {}
    for label, strip in (("with_ko", False), ("no_ko", True)):
        I = g.iparams.copy()
        if strip:
            I[:, capi.I_MON_COUNT] = 0
        k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
        plan = capi.plan(g.n_nodes, False, k_cap, n_time=g.n_time, B=g.B)
        P = torch.from_numpy(g.params).to(dev)
        It = torch.from_numpy(I).to(dev)
        V0 = torch.from_numpy(g.v_init).to(dev)
        o = torch.empty_like(V0)
        MS = torch.from_numpy(g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)).to(dev)
        MR = torch.from_numpy(g.mon_rebate if len(g.mon_rebate) else np.zeros(1)).to(dev)
        wsb = max(8, plan["ws_bytes_per_scen"] * g.B)
        ws = torch.empty(wsb // 8, dtype=torch.float64, device=dev)
        st = torch.cuda.current_stream()

        def step():
            capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), It.data_ptr(),
                              V0.data_ptr(), len(g.mon_step), MS.data_ptr(), MR.data_ptr(),
                              o.data_ptr(), k_cap, ws.data_ptr(), wsb, st.cuda_stream)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            step()
        e1.record(st)
        torch.cuda.synchronize()
        out[label] = e0.elapsed_time(e1) / a.steps
    print(json.dumps({"workload": a.workload, "B": B, "kernel_ms": out,
                      "variant": capi.variant_name(g.n_nodes, False, B=g.B)}))


if __name__ == "__main__":
    main()
