#!/usr/bin/env python3
"""profiles/pmc_counters.json from tools/pmc_counters.sh output.

Usage: python tools/counters_json.py TAG [WORKLOAD...]   (default: all three)

Per workload, reads gpurun_out/<TAG>_<wl>/<pass>/*counter_collection.csv,
sums each fdcn_march dispatch's rows per counter, averages over the
dispatches, and records:
  hbm_bytes_per_launch  FETCH_SIZE x 2 (gfx950 counts half of wide coalesced
                        reads, MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> B
  valu_insts_per_launch SQ_INSTS_VALU (wave-level instructions)
  gpu_clock_ghz         GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration
  valu_issue_utilisation  4 x SQ_INSTS_VALU / (1024 SIMDs x GUI cycles): a
                        wave64 fp64 VALU op holds a 16-lane SIMD for 4 cycles
plus the compulsory bytes the launch must move, and the sha of the kernel
source the counters were measured on: bench.py reports these numbers only
while fdcn_kernels.hip is unchanged.
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
XCD = 8


def per_launch(d, kernel="fdcn_march"):
    """Average per dispatch of the kernels whose name contains `kernel`."""
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel not in row["Kernel_Name"]:
                continue
            k = int(row["Dispatch_Id"])
            per[k][row["Counter_Name"]] += float(row["Counter_Value"])
            per[k]["_ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    if not per:
        raise SystemExit(f"no {kernel} rows under {d}")
    acc = defaultdict(list)
    for cs in per.values():
        for c, v in cs.items():
            acc[c].append(v)
    return {c: sum(v) / len(v) for c, v in acc.items()}, len(per)


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
    if not is_it and waves == 1 and plan["npt"] > 40:
        bnd = 0  # the recovery form evaluates its boundary terms in the march (round 5)
    raw_wr = 0
    if not is_it and waves == 1 and plan["npt"] <= 40:
        # the one-scenario split form (round 6): one-sided tables and the raw
        # values of the steps read after an edge knock-out (fdcn_kernels.hip kTab1)
        bnd, raw_wr = one_sided_table_bytes(g, n_pad)
    ko_row = g.B * waves * plan["npt"] * 8 if (not is_it and plan["npt"] >= 48) else 0
    rec = (g.B * 64 * plan["npt"] * 8 * min(g.n_ranna, g.n_time)
           if (not is_it and waves == 1 and plan["npt"] > 40) else 0)
    key = f"{label}_{ns}x{nt}_batch{B}"
    node_steps = g.B * bench.node_units(g) * g.n_time
    return key, rd + bnd + ko_row + rec, vec + bnd + raw_wr + ko_row + rec, plan, node_steps


def one_sided_table_bytes(g, n_pad):
    """(table bytes written = read, raw-value bytes written) of the kTab1
    variants: a scenario whose lower / upper Dirichlet side has zero
    coefficients keeps the other side alone (8 B a step); the raw values are
    stored for the steps after the monitor dates of a scenario whose
    knock-out reaches an edge node, and for the last step."""
    import math
    from finite_difference_amd import capi
    P, I = g.params, g.iparams
    table = raw = 0
    for b in range(g.B):
        t_a, t_b = P[b, capi.P_TAU0], P[b, capi.P_TAU0] + 1.01 * g.n_time * P[b, capi.P_DT]

        def const(form, c0, e0, c1, e1):
            zero = (c0 == 0 or c1 == 0) if form == 1 else (c0 == 0 and c1 == 0)
            return (zero and math.isfinite(c0) and math.isfinite(c1) and
                    max(e0 * t_a, e0 * t_b, e1 * t_a, e1 * t_b) <= 700.0)
        lo = const(I[b, capi.I_LO_FORM], *P[b, capi.P_LO_C0:capi.P_LO_E1 + 1])
        hi = const(I[b, capi.I_HI_FORM], *P[b, capi.P_HI_C0:capi.P_HI_E1 + 1])
        w = 8 if (lo or hi) else 16
        table += n_pad * w
        edge = I[b, capi.I_KO_LO] >= 0 or g.n_nodes - 1 >= I[b, capi.I_KO_HI]
        ms, mc = I[b, capi.I_MON_START], I[b, capi.I_MON_COUNT]
        need = {g.n_time - 1}
        if edge:
            need |= {int(s) for s in g.mon_step[ms:ms + mc] if 0 <= s < n_pad}
        raw += len(need) * w
    return table, raw


def spot_vc(tag, out):
    """The spot-space march (bench.py --workload spot_vc): the pointwise
    march kernel (the planner's form for every bench trade) and the factor
    kernel, each per launch; keyed like the bench line's workload."""
    import bench
    import numpy as np
    from finite_difference_amd import capi
    base = os.path.join(ROOT, "gpurun_out", f"{tag}_spot_vc")
    B = bench.DEFAULT_BATCH["spot_vc"]
    g = bench.build_spot_vc(B, 1024, 2000)
    plan = capi.vc_plan(g.n_nodes, B=B)
    name = f"fdcn_vc_march<{plan['waves']}, {plan['npt']}, true>"
    node_steps = g.B * (g.n_nodes - 1) * g.n_time
    rec = {}
    for kern, label in ((name, "march"), ("fdcn_vc_factor", "factor")):
        fe, n1 = per_launch(os.path.join(base, "fetch"), kern)
        wr, n2 = per_launch(os.path.join(base, "write"), kern)
        sq, _ = per_launch(os.path.join(base, "sq"), kern)
        gr, _ = per_launch(os.path.join(base, "grbm"), kern)
        clk = gr["GRBM_GUI_ACTIVE"] / XCD / gr["_ns"]
        rec[label] = {
            "kernel": kern,
            "hbm_bytes_per_launch": fe["FETCH_SIZE"] * 2 * 1024 + wr["WRITE_SIZE"] * 1024,
            "read_bytes": fe["FETCH_SIZE"] * 2 * 1024, "write_bytes": wr["WRITE_SIZE"] * 1024,
            "valu_insts_per_launch": sq["SQ_INSTS_VALU"],
            "valu_insts_per_lane_node_step": 64.0 * sq["SQ_INSTS_VALU"] / node_steps,
            "salu_insts_per_launch": sq.get("SQ_INSTS_SALU"),
            "lds_insts_per_launch": sq.get("SQ_INSTS_LDS"),
            "wait_inst_any_per_launch": sq.get("SQ_WAIT_INST_ANY"),
            "gpu_clock_ghz": clk, "profiled_launch_ms": gr["_ns"] * 1e-6,
            "valu_issue_utilisation": 4.0 * sq["SQ_INSTS_VALU"] / (
                gr["GRBM_GUI_ACTIVE"] / XCD * 256 * 4),
            "launches_averaged": min(n1, n2)}
    # compulsory: diag [B][2][6][n], bnd [B][n_time][2], v_init, v_out
    compulsory = (g.diag.nbytes + g.bnd.nbytes + 2 * g.v_init.nbytes)
    key = f"spot_vc_1024x2000_batch{B}"
    out[key] = dict(rec, kernel_src_sha=bench.file_sha("fdcn_vc.hip"),
                    compulsory_bytes_per_launch=compulsory,
                    source=(f"rocprofv3 --pmc, one counter group per pass, python bench.py "
                            f"--workload spot_vc --steps 2 --warmup 1 (tools/pmc_counters.sh {tag})"))
    m = rec["march"]
    print(f"{key}: march VALU per lane node-step {m['valu_insts_per_lane_node_step']:.2f}, issue "
          f"{m['valu_issue_utilisation']:.2f} at {m['gpu_clock_ghz']:.2f} GHz, HBM march "
          f"{m['hbm_bytes_per_launch'] / 1e6:.0f} MB + factor "
          f"{rec['factor']['hbm_bytes_per_launch'] / 1e6:.0f} MB (compulsory {compulsory / 1e6:.0f})")


def main():
    import bench
    tag = sys.argv[1]
    wls = sys.argv[2:] or ["american", "barrier", "double"]
    path = os.path.join(ROOT, "profiles", "pmc_counters.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    if "spot_vc" in wls:
        spot_vc(tag, out)
        wls = [w for w in wls if w != "spot_vc"]
    for wl in wls:
        base = os.path.join(ROOT, "gpurun_out", f"{tag}_{wl}")
        fe, n1 = per_launch(os.path.join(base, "fetch"))
        wr, n2 = per_launch(os.path.join(base, "write"))
        sq, _ = per_launch(os.path.join(base, "sq"))
        gr, _ = per_launch(os.path.join(base, "grbm"))
        key, exp_rd, exp_wr, plan, node_steps = expected(wl)
        rd, wb = fe["FETCH_SIZE"] * 2 * 1024, wr["WRITE_SIZE"] * 1024
        clk = gr["GRBM_GUI_ACTIVE"] / XCD / gr["_ns"]
        f64 = sum(gr.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64",
                                            "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
        out[key] = {
            "kernel_src_sha": bench.kernel_src_sha(),
            "hbm_bytes_per_launch": rd + wb,
            "read_bytes": rd, "write_bytes": wb,
            "expected_read_bytes": exp_rd, "expected_write_bytes": exp_wr,
            "valu_insts_per_launch": sq["SQ_INSTS_VALU"],
            "valu_insts_per_node_step": sq["SQ_INSTS_VALU"] / node_steps,
            # per lane: a wave instruction advances 64 lanes' chunks
            "valu_insts_per_lane_node_step": 64.0 * sq["SQ_INSTS_VALU"] / node_steps,
            "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"],
            "f64_valu_insts_per_launch": f64,
            "fma_f64_per_launch": gr.get("SQ_INSTS_VALU_FMA_F64", 0.0),
            "wait_inst_any_per_launch": sq.get("SQ_WAIT_INST_ANY"),
            "lds_insts_per_launch": sq.get("SQ_INSTS_LDS"),
            "gpu_clock_ghz": clk,
            "profiled_launch_ms": gr["_ns"] * 1e-6,
            "valu_issue_utilisation": 4.0 * sq["SQ_INSTS_VALU"] / (
                gr["GRBM_GUI_ACTIVE"] / XCD * 256 * 4),
            "plan": {"waves": plan["waves"], "npt": plan["npt"]},
            "launches_averaged": min(n1, n2),
            "source": (f"rocprofv3 --pmc, one counter group per pass, python bench.py "
                       f"--workload {wl} --steps 2 --warmup 1 (tools/pmc_counters.sh {tag})"),
        }
        print(f"{key}: HBM {(rd + wb) / 1e6:.1f} MB (expected {(exp_rd + exp_wr) / 1e6:.1f}), "
              f"VALU per lane node-step {out[key]['valu_insts_per_lane_node_step']:.2f}, "
              f"issue {out[key]['valu_issue_utilisation']:.2f} at {clk:.2f} GHz")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
