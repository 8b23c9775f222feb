#!/usr/bin/env python3
"""Generate finite_difference_amd/csrc/fdcn_ko_res.h: the resident-mask
knock-out projection of the recovery-form march (config 5) as one inline-asm
block per chunk length (NPT = 48, 64).

Why one generated block.  The projection sets V[k] = rebate on the lanes of
mask M(k) for every slot k.  The masks are constant for the march and take at
most three values over slots 0 .. NPT-2 (q0, q1, q2: the lower side's partial
lane leaves after its last knocked slot, the upper side's joins at its first),
plus the last slot's own value (qd: a short lane's phantom slot is never
knocked out).  The slots are walked in groups of eight (the last group
seven).  Each group has a code, fixed for the march (kernel prologue):

  0                      no change inside: exec = q0, one move per slot
  1 + o                  one change at offset o: q0 on [0, o), q1 on [o, G),
                         then the queue shifts (q0 = q1, q1 = q2)
  G + 1 + pair(o1, o2)   two changes: q0 / q1 / q2 on the three runs, then
                         q0 = q1 = q2
  63                     masks from the workspace row, slot by slot
                         (the prologue sets it on every group if a march ever
                         had more than two changes: never, by construction)

Groups with code 0 run straight through (no taken branch): the special
groups branch out to a binary tree over their code placed after the block's
main path, whose leaf branches back.  Written as C++ switch cases (one asm
statement per case) the same logic made the register allocator split the
value vector's live ranges: 353 registers (97 AGPRs) and one wave per SIMD.
One asm statement sees the vector as 64 in-place operands.

Usage: python tools/gen_ko_res.py  (rewrites the header; the build does not
run it).
"""
import os

OUT = os.path.join(os.path.dirname(__file__), "..", "finite_difference_amd", "csrc",
                   "fdcn_ko_res.h")


def pair_index(g, o1, o2):
    """Index of the two-change case (o1 < o2) among a G-slot group's pairs,
    in (o1, o2) lexicographic order -- fdcn_kernels.hip computes the same."""
    return o1 * (2 * g - o1 - 1) // 2 + (o2 - o1 - 1)


def leaves(gsz):
    """(code, runs) of every special case of a GSZ-slot group; runs are
    (mask operand, first slot, end slot)."""
    out = []
    for o in range(gsz):
        out.append((1 + o, [("q0", 0, o), ("q1", o, gsz)], 1))
    for o1 in range(gsz):
        for o2 in range(o1 + 1, gsz):
            code = gsz + 1 + pair_index(gsz, o1, o2)
            out.append((code, [("q0", 0, o1), ("q1", o1, o2), ("q2", o2, gsz)], 2))
    assert max(c for c, _, _ in out) < 63
    return out


def gen_block(npt, blk, mode, gpb):
    """Groups gpb blk .. gpb blk + gpb - 1 of a chunk of NPT slots (slots
    8 gpb blk .. 8 gpb (blk + 1) - 1): one asm statement.  Several statements
    per projection because the front end counts a tied "+v" operand twice
    against the 256-VGPR file (64 doubles in place would ask for 256 + 256).
    The v_mov_b64 form (A/B only) runs in statements of 32 slots (gpb 4), the
    product's LDS form at NPT 64 in statements of 16 (gpb 2): config 5
    13.05-13.12 ms with 32-slot statements, 12.30-12.34 with 16, 12.94-12.99
    with 8, 13.25-13.29 with 24 (24 + 24 + 16), 13.50-13.55 with the first
    of two 32-slot statements left undrained, all bitwise equal
    (profiles/r06/config5_ko/r06j_1drain, r06k_gpb, r06l_g16, r06m_g24).  At NPT 48 statements of 16 measured 0.6 % slower
    (11.17-11.20 against 11.10 ms on a 3 073-node grid): it keeps 32.

    mode "v": each slot's rebate is a v_mov_b64 (VALU).  mode "l": an
    exec-masked ds_read_b64 of the rebate from one LDS slot ([la]), which
    the kernel writes (lane 0) in the statement that loads the run masks, so
    the write's latency hides under theirs (12.40 -> 12.35 ms over four
    interleaved pairs, r06aa/r06ab) -- the LDS unit writes the VGPRs, so
    the projection takes no VALU issue slot; each statement drains its reads
    (lgkmcnt(0)) before it ends, so its outputs are complete for the
    compiler."""
    mov = ("v_mov_b64 %[v{}], %[rb]" if mode == "v" else "ds_read_b64 %[v{}], %[la]").format
    ng = npt // 8
    groups = range(gpb * blk, min(gpb * blk + gpb, ng))
    main, special = [], []
    for g in groups:
        gsz = 7 if g == ng - 1 else 8
        base = 8 * g
        word, bit = ("c0", 6 * g) if g < 5 else ("c1", 6 * (g - 5))
        r_lab, s_lab = 100 + g, 200 + g
        main += [f"s_bfe_u32 %[cd], %[{word}], {hex((6 << 16) | bit)}",
                 "s_cmp_lg_u32 %[cd], 0",
                 f"s_cbranch_scc1 {s_lab}f",
                 "s_and_b64 exec, %[q0], %[sv]"]
        main += [mov(base + i) for i in range(gsz)]
        main.append(f"{r_lab}:")
        # special region of this group: binary search over the codes
        lv = leaves(gsz)
        lv.append((63, None, 0))
        lv.sort(key=lambda x: x[0])
        special.append(f"{s_lab}:")
        counter = [0]

        def label():
            counter[0] += 1
            return 1000 + 100 * g + counter[0]

        def emit(lo, hi):  # leaves lv[lo:hi]
            if hi - lo == 1:
                code, runs, nshift = lv[lo]
                if runs is None:  # the workspace row, slot by slot
                    for i in range(gsz):
                        special.extend([f"s_load_dwordx2 %[mt], %[ka], {8 * (base + i)}",
                                        "s_waitcnt lgkmcnt(0)",
                                        "s_and_b64 exec, %[mt], %[sv]",
                                        mov(base + i)])
                    special.append("s_mov_b64 %[q0], %[q2]")
                    special.append("s_mov_b64 %[q1], %[q2]")
                else:
                    for q, a, b in runs:
                        if a == b:
                            continue
                        special.append(f"s_and_b64 exec, %[{q}], %[sv]")
                        special.extend(mov(base + i) for i in range(a, b))
                    if nshift == 1:
                        special.extend(["s_mov_b64 %[q0], %[q1]", "s_mov_b64 %[q1], %[q2]"])
                    else:
                        special.extend(["s_mov_b64 %[q0], %[q2]", "s_mov_b64 %[q1], %[q2]"])
                special.append(f"s_branch {r_lab}b")
                return
            mid = (lo + hi) // 2
            right = label()
            special.extend([f"s_cmp_lt_u32 %[cd], {lv[mid][0]}", f"s_cbranch_scc0 {right}f"])
            emit(lo, mid)
            special.append(f"{right}:")
            emit(mid, hi)

        emit(0, len(lv))
    last = groups[-1] == ng - 1
    if last:  # the chunk's last slot under its own mask
        main += ["s_and_b64 exec, %[qd], %[sv]", mov(npt - 1)]
    main += ["s_mov_b64 exec, %[sv]", "s_branch 99f"]
    head = []  # (the LDS form's rebate word is written by the kernel's mask-load statement)
    tail = ["s_waitcnt lgkmcnt(0)"] if mode == "l" else []
    lines = head + main + special + ["99:"] + tail
    body = "".join(f'  "{l}\\n\\t" \\\n' for l in lines)
    lo_slot, hi_slot = 8 * gpb * blk, min(8 * gpb * (blk + 1), npt)
    ops = ", ".join(f'[v{i}] "+v"(V[{i}])' for i in range(lo_slot, hi_slot))
    tag = "" if mode == "v" else "L"
    return (f"#define FDCN_KO_RES{tag}_ASM_{npt}_{blk} \\\n{body}  \"\"\n"
            f"#define FDCN_KO_RES{tag}_VOPS_{npt}_{blk} {ops}\n")


def gen(npt):
    ng = npt // 8
    lg = 2 if npt == 64 else 4  # groups per statement of the LDS form
    return ("".join(gen_block(npt, b, "v", 4) for b in range((ng + 3) // 4))
            + "".join(gen_block(npt, b, "l", lg) for b in range((ng + lg - 1) // lg)))


def render():
    txt = ["// Generated by tools/gen_ko_res.py -- do not edit.",
           "// The resident-mask knock-out projection of the recovery-form march",
           "// (fdcn_march, kKoRes): one asm block per chunk length; see the generator",
           "// for the group codes.  Operands: the value vector [v0]..[vNPT-1] (in",
           "// place), [rb] the rebate (VGPR), [sv] the saved exec, [q0] [q1] (in/out",
           "// copies of the first two run masks), [q2], [qd] the last slot's mask,",
           "// [c0] [c1] the packed group codes, [ka] the mask row, [cd] [mt] scratch.",
           "#pragma once",
           ""]
    for npt in (48, 64):
        txt.append(gen(npt))
    txt.append('#define FDCN_KO_RES_INS(RB_, SV_, Q2_, QD_, C0_, C1_, KA_, LA_) \\\n'
               '  [rb] "v"(RB_), [sv] "s"(SV_), [q2] "s"(Q2_), [qd] "s"(QD_), [c0] "s"(C0_), '
               '[c1] "s"(C1_), [ka] "s"(KA_), [la] "v"(LA_)\n')
    return "\n".join(txt)


def main():
    with open(OUT, "w") as f:
        f.write(render())
    print(OUT)


if __name__ == "__main__":
    main()
