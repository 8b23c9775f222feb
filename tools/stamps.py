"""Per-phase cycle shares of the time loop (GPU box, diagnostic build).

Builds nothing: expects finite_difference_amd/_lib/libfdcn_stamps.so compiled
with -DFDCN_STAMPS (see __graft_entry__.build_stamps).  Runs the bench
workload once through the host entry point and prints each phase's share of
the summed wave cycles.  The stamps serialise the phases, so only the SHARES
mean anything.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["IT/KO + loop top", "halo + RHS", "fwd pass 1", "fwd scan", "fwd pass 2",
         "bwd pass 1", "bwd scan", "bwd pass 2", "Sherman-Morrison"]


def main():
    import numpy as np
    import bench
    wl = sys.argv[1] if len(sys.argv) > 1 else "american"
    builder, ns, nt, it, _ = bench.WORKLOADS[wl]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else bench.DEFAULT_BATCH[wl]
    L = ctypes.CDLL(os.environ.get("FDCN_STAMPS_LIB") or
                    os.path.join(ROOT, "finite_difference_amd", "_lib", "libfdcn_stamps.so"))
    g = builder(B, ns, nt, seed=0)
    D, I = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
    out = np.empty_like(g.v_init)
    st = (ctypes.c_ulonglong * 10)()
    L.fdcn_debug_stamps(st, 1)
    if it:
        rc = L.fdcn_it_batch(g.B, g.n_nodes, g.n_time, g.n_ranna, g.params.ctypes.data_as(D),
                             g.iparams.ctypes.data_as(I), g.v_init.ctypes.data_as(D),
                             g.payoff.ctypes.data_as(D), out.ctypes.data_as(D))
    else:
        ms = g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)
        mr = g.mon_rebate if len(g.mon_rebate) else np.zeros(1)
        rc = L.fdcn_cn_batch(g.B, g.n_nodes, g.n_time, g.n_ranna, g.params.ctypes.data_as(D),
                             g.iparams.ctypes.data_as(I), g.v_init.ctypes.data_as(D),
                             len(g.mon_step), ms.ctypes.data_as(I), mr.ctypes.data_as(D),
                             out.ctypes.data_as(D))
    assert rc == 0, rc
    L.fdcn_debug_stamps(st, 0)
    vals = [st[i] for i in range(9)]
    tot = sum(vals)
    res = {"waves": st[9], "cycles_per_wave_step": tot / max(1, st[9]) / g.n_time,
           "shares": {n: v / tot for n, v in zip(NAMES, vals)}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
