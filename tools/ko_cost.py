"""Diagnostic (GPU box): config-5 kernel time with and without the
every-step knock-out projection, for the library FDCN_LIB points at.
Prints one JSON line: ms per launch with KO, without KO (n_mon = 0)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from finite_difference_amd import capi  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    g = bench.build_double(B, 4096, 8192, seed=0)
    dev = torch.device("cuda:0")
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    plan = capi.plan(g.n_nodes, False, k_cap, n_time=g.n_time, B=g.B)
    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    out = torch.empty_like(V0)
    ws = torch.empty(plan["ws_bytes_per_scen"] * g.B // 8, dtype=torch.float64, device=dev)
    MS = torch.from_numpy(g.mon_step).to(dev)
    MR = torch.from_numpy(g.mon_rebate).to(dev)
    s = torch.cuda.current_stream()
    res = {"lib": os.environ.get("FDCN_LIB", "in-tree"), "plan": plan}
    for label, n_mon in (("ko", len(g.mon_step)), ("no_ko", 0)):
        def step():
            capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                              V0.data_ptr(), n_mon, MS.data_ptr(), MR.data_ptr(),
                              out.data_ptr(), k_cap, ws.data_ptr(), s.cuda_stream)
        step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(5):
            step()
        e1.record(s)
        torch.cuda.synchronize()
        res[label] = e0.elapsed_time(e1) / 5
    print(json.dumps(res))


if __name__ == "__main__":
    main()
