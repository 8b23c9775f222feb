#!/usr/bin/env python3
"""Per-launch averages of rocprofv3 --pmc counter CSVs (tools/pmc.sh output).

Usage: python tools/pmc_summary.py gpurun_out/<tag>   -> JSON on stdout
Counters are summed over a dispatch's rows, then averaged over the march
launches (the kernel named fdcn_march).  Derived: the shader clock during the
launch (GRBM_GUI_ACTIVE / 8 XCDs / duration) and the VALU issue utilisation:
a wave64 VALU instruction occupies a 16-lane SIMD for 4 cycles, so the chip
issues at most 1024 SIMDs x cycles / 4 of them.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))  # (pass, dispatch) -> counter -> value
    names = {}
    for f in glob.glob(os.path.join(d, "*", "*_counter_collection.csv")):
        pas = os.path.basename(os.path.dirname(f))
        for row in csv.DictReader(open(f)):
            if "fdcn_march" not in row["Kernel_Name"]:
                continue
            key = (pas, int(row["Dispatch_Id"]))
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
            names[key] = row["Kernel_Name"]
            per[key]["_ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    avg = defaultdict(list)
    for key, cs in per.items():
        for c, v in cs.items():
            avg[c].append(v)
    return {c: sum(v) / len(v) for c, v in avg.items()}, sorted(set(names.values()))


def main():
    d = sys.argv[1]
    a, kernels = load(d)
    out = {"kernels": kernels, "per_launch": a}
    if "SQ_INSTS_VALU" in a and "SQ_WAVES" in a:
        out["valu_insts_per_wave"] = a["SQ_INSTS_VALU"] / a["SQ_WAVES"]
    xcc = 8  # MI355X: GRBM_GUI_ACTIVE accumulates over the 8 XCDs
    if "GRBM_GUI_ACTIVE" in a and "_ns" in a:
        out["gpu_clock_ghz"] = a["GRBM_GUI_ACTIVE"] / xcc / a["_ns"]
    f64 = sum(a.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64",
                                       "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
    if f64:
        out["f64_valu_insts"] = f64
    if "SQ_INSTS_VALU" in a and "GRBM_GUI_ACTIVE" in a:
        # wave64 VALU instruction = 4 cycles of one SIMD (16 lanes x 4 passes);
        # 256 CUs x 4 SIMDs issue at most one every 4 cycles each
        simd_cycles = a["GRBM_GUI_ACTIVE"] / xcc * 256 * 4
        out["valu_issue_utilisation"] = 4.0 * a["SQ_INSTS_VALU"] / simd_cycles
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
