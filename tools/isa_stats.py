#!/usr/bin/env python3
"""Instruction mix of a kernel's time loop, from a hipcc --save-temps .s file.

Usage: python tools/isa_stats.py FILE.s IT W NPT [ZG]

Finds the kernel fdcn_march<IT,W,NPT,ZG>, takes the instructions between the
longest backward branch's target and the branch (the time loop), and counts
them by class.  Static counts: conditional blocks inside the loop (Rannacher
switch, Dirichlet refill, knock-out) are counted once.  Also prints the
kernel's VGPR/AGPR/scratch/occupancy lines from the assembler comments.
"""
import re
import sys
from collections import Counter


def kernel_lines(path, it, w, npt, zg):
    name = f"_ZN12_GLOBAL__N_110fdcn_marchILi{it}ELi{w}ELi{npt}ELi{zg}EEEvNS_5KArgsE:"
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(name))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    meta = []
    for l in lines[end:end + 80]:
        if any(k in l for k in ("NumVgprs:", "NumAgprs:", "ScratchSize:", "Occupancy:", "codeLenInByte")):
            meta.append(l.strip())
    return lines[start:end + 1], meta


def classify(op):
    if "_dpp" in op:
        return "valu_dpp"
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "valu_lane"
    if op.startswith("v_cndmask"):
        return "valu_cndmask"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, it, w, npt = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    zg = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    ks, meta = kernel_lines(path, it, w, npt, zg)
    labels = {l.split(":")[0]: i for i, l in enumerate(ks) if re.match(r"^\.LBB\d+_\d+:", l)}
    best = None
    for i, l in enumerate(ks):
        m = re.match(r"\s+s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            span = i - labels[m.group(1)]
            if best is None or span > best[0]:
                best = (span, labels[m.group(1)], i)
    _, a, b = best
    cnt = Counter()
    for l in ks[a:b + 1]:
        s = l.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        cnt[classify(s.split()[0])] += 1
    total = sum(cnt.values())
    print(f"fdcn_march<{it},{w},{npt},{zg}> loop: {total} instructions (static)")
    for k, v in cnt.most_common():
        print(f"  {k:14s} {v:6d}")
    print("  f64 VALU per node:", round(cnt["valu_f64"] / npt, 2))
    for l in meta:
        print("  " + l)


if __name__ == "__main__":
    main()
