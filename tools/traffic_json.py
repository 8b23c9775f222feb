#!/usr/bin/env python3
"""Rebuild profiles/pmc_traffic.json from tools/pmc_traffic.sh output.

Usage: python tools/traffic_json.py TAG [WORKLOAD...]   (default: all three)

Per workload, reads gpurun_out/<TAG>_<wl>/{FETCH_SIZE,WRITE_SIZE}/*counter_collection.csv
(separate rocprofv3 passes), sums each fdcn_march dispatch's rows and averages
over the dispatches.  HBM bytes per launch = FETCH_SIZE x 2 (gfx950 counts half
of wide coalesced reads, MI355X_MICROARCH.md) + WRITE_SIZE, both KiB -> B.
The expected bytes are the launch's compulsory traffic: params/iparams,
v_init (+ payoff for IT) and the monitor entries read once, v_out written
once, the Dirichlet table (16 B per padded step per wave) written and read
once, and for the knock-out variants with NPT >= 48 the mask row (8 B per
slot per wave) written and read once.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def kib_per_launch(d):
    per = defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "fdcn_march" in row["Kernel_Name"]:
                per[int(row["Dispatch_Id"])] += float(row["Counter_Value"])
    if not per:
        raise SystemExit(f"no fdcn_march rows under {d}")
    return sum(per.values()) / len(per), len(per)


def expected(wl):
    import bench
    from finite_difference_amd import capi
    builder, ns, nt, is_it, label = bench.WORKLOADS[wl]
    B = bench.DEFAULT_BATCH[wl]
    g = builder(B, ns, nt, seed=0)
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    plan = capi.plan(g.n_nodes, is_it, k_cap, n_time=g.n_time, B=g.B)
    n_pad = (max(g.n_time, 1) + 63) // 64 * 64
    waves = plan["waves"]
    vec = g.B * g.n_nodes * 8
    rd = g.params.nbytes + g.iparams.nbytes + vec * (2 if is_it else 1)
    rd += len(g.mon_step) * 12
    bnd = g.B * waves * n_pad * 16
    ko_row = g.B * waves * plan["npt"] * 8 if (not is_it and plan["npt"] >= 48) else 0
    # recovery-form variants (CN, W = 1, NPT > 40): the old V of each
    # Rannacher step is written and read back once (64 x NPT doubles per wave)
    rec = (g.B * 64 * plan["npt"] * 8 * min(g.n_ranna, g.n_time)
           if (not is_it and waves == 1 and plan["npt"] > 40) else 0)
    key = f"{label}_{ns}x{nt}_batch{B}"
    return key, rd + bnd + ko_row + rec, vec + bnd + ko_row + rec, plan


def main():
    tag = sys.argv[1]
    wls = sys.argv[2:] or ["american", "barrier", "double"]
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for wl in wls:
        base = os.path.join(ROOT, "gpurun_out", f"{tag}_{wl}")
        fk, nf = kib_per_launch(os.path.join(base, "FETCH_SIZE"))
        wk, nw = kib_per_launch(os.path.join(base, "WRITE_SIZE"))
        key, exp_rd, exp_wr, plan = expected(wl)
        rd, wr = fk * 2 * 1024, wk * 1024
        out[key] = {
            "hbm_bytes_per_launch": rd + wr,
            "read_bytes": rd,
            "write_bytes": wr,
            "fetch_size_kib_raw": fk,
            "write_size_kib_raw": wk,
            "launches_averaged": min(nf, nw),
            "correction": "FETCH_SIZE x2 (gfx950 counts half of wide coalesced reads); KiB -> B",
            "expected_read_bytes": exp_rd,
            "expected_write_bytes": exp_wr,
            "plan": {"waves": plan["waves"], "npt": plan["npt"]},
            "note": ("compulsory bytes: inputs and monitor entries read once, v_out written "
                     "once, Dirichlet table (16 B per padded step per wave) and, for NPT >= 48 "
                     "knock-out variants, the mask row written and read once (plus, for the "
                     "recovery-form variants, the old V of each Rannacher step); the march "
                     "itself moves no HBM bytes per step"),
            "source": (f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                       f"python bench.py --workload {wl} --steps 2 --warmup 1 "
                       f"(tools/pmc_traffic.sh {tag}; tools/traffic_json.py)"),
        }
        print(f"{key}: {(rd + wr) / 1e6:.1f} MB measured, "
              f"{(exp_rd + exp_wr) / 1e6:.1f} MB expected")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
