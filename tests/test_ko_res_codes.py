"""CPU checks of the resident-mask knock-out projection (fdcn_ko_res.h).

1. The committed header is what tools/gen_ko_res.py generates.
2. The generated asm, run by a small interpreter of the instructions it uses,
   with the group codes and run masks computed as the kernel prologue computes
   them (fdcn_kernels.hip, kKoRes), moves the rebate into exactly the
   (lane, slot) positions of the interior nodes the reference knocks out --
   j <= KO_LO or j >= KO_HI (discrete_barrier_fdm_pricer.py:413-440) -- and
   into no phantom slot or inactive lane, for every layout class: one change
   per side at every offset, two changes in one group, one partial lane for
   both sides, one side only, sides covering whole lanes.

The GPU twin (tests/test_gpu_ko_resident.py) runs the kernel itself against
the oracle on the same layouts.
"""
import importlib.util
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "finite_difference_amd", "csrc", "fdcn_ko_res.h")


def _gen():
    spec = importlib.util.spec_from_file_location("gen_ko_res",
                                                  os.path.join(ROOT, "tools", "gen_ko_res.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_header_is_generated():
    with open(HEADER) as f:
        assert f.read() == _gen().render(), "run python tools/gen_ko_res.py"


def _blocks(npt, form=""):
    """The instruction lists of the projection's asm statements for NPT
    (form "": the v_mov_b64 form, "L": the ds_read_b64 form the kernel runs)."""
    text = _gen().render()
    out = []
    # statements of 32 slots, or of 16 (the LDS form at NPT 64, gen_ko_res.py)
    nblk = (npt + 15) // 16 if (form == "L" and npt == 64) else (npt + 31) // 32
    for blk in range(nblk):
        m = re.search(rf"#define FDCN_KO_RES{form}_ASM_{npt}_{blk} \\\n((?:  \".*\" \\\n)+)",
                      text)
        assert m, (npt, blk)
        out.append([re.match(r'  "(.*)\\n\\t" \\', ln).group(1)
                    for ln in m.group(1).splitlines() if ln.strip() != '"" \\'])
    return out


def lane_slot(i, npt, ls):
    split = ls * (npt - 1)
    if i < split:
        return i // (npt - 1), i % (npt - 1)
    return ls + (i - split) // npt, (i - split) % npt


def slot_masks(npt, n_nodes, klo, khi):
    """The kernel's per-slot masks (fdcn_march: masks / slot_mask)."""
    n_int = n_nodes - 2
    l_act = -(-n_int // npt)
    ls = l_act * npt - n_int
    act = (1 << l_act) - 1 if l_act < 64 else (1 << 64) - 1
    allm = (1 << 64) - 1
    ml = dict(full=0, part=0, k0=0, k1=-1)
    mh = dict(full=0, part=0, k0=0, k1=-1)
    if klo >= 1:
        tl, sl = (l_act, 0) if klo >= n_int else lane_slot(klo - 1, npt, ls)
        ml["full"] = (0 if tl <= 0 else (allm if tl >= 64 else (1 << tl) - 1)) & act
        if klo < n_int and 0 <= tl < 64:
            ml.update(part=act & (1 << tl), k0=0, k1=sl)
    if khi <= n_int:
        th, sh = (0, 0) if khi <= 1 else lane_slot(khi - 1, npt, ls)
        mh["full"] = (0 if th >= 63 else (allm if th < 0 else allm & ~((2 << th) - 1))) & act
        if 0 <= th < 64:
            mh.update(part=act & (1 << th), k0=sh, k1=npt - 1)
    shrt = (1 << ls) - 1
    out = []
    for k in range(npt):
        m = ml["full"] | mh["full"]
        if ml["k0"] <= k <= ml["k1"]:
            m |= ml["part"]
        if mh["k0"] <= k <= mh["k1"]:
            m |= mh["part"]
        if k == npt - 1:
            m &= ~shrt
        out.append(m)
    return out


def prologue(npt, masks):
    """Run masks and packed codes, as the kernel prologue computes them."""
    chg = 0
    for k in range(1, npt - 1):
        if masks[k] != masks[k - 1]:
            chg |= 1 << k
    nchg = bin(chg).count("1")
    pos = [k for k in range(64) if chg >> k & 1]
    q0 = masks[0]
    q1 = masks[pos[0]] if nchg >= 1 else q0
    q2 = masks[pos[1]] if nchg >= 2 else q1
    c = [0, 0]
    for g in range(npt // 8):
        gsz = 7 if g + 1 == npt // 8 else 8
        bits = (chg >> (8 * g)) & ((1 << gsz) - 1)
        if nchg > 2:
            code = 63
        elif bits == 0:
            code = 0
        elif bits & (bits - 1) == 0:
            code = 1 + (bits & -bits).bit_length() - 1
        else:
            o1 = (bits & -bits).bit_length() - 1
            b2 = bits & (bits - 1)
            o2 = (b2 & -b2).bit_length() - 1
            code = gsz + 1 + o1 * (2 * gsz - o1 - 1) // 2 + (o2 - o1 - 1)
        if g < 5:
            c[0] |= code << (6 * g)
        else:
            c[1] |= code << (6 * (g - 5))
    return dict(q0=q0, q1=q1, q2=q2, qd=masks[npt - 1], c0=c[0], c1=c[1]), nchg


def run_block(ins, regs, row, moved):
    """Interpret one asm statement of the projection."""
    labels = {}
    for i, s in enumerate(ins):
        if re.fullmatch(r"\d+:", s):
            labels.setdefault(int(s[:-1]), []).append(i)

    def target(ref, at):
        n, d = int(ref[:-1]), ref[-1]
        cands = labels[n]
        return min(x for x in cands if x > at) if d == "f" else max(x for x in cands if x < at)

    op = re.compile(r"%\[(\w+)\]")
    pc, scc, exec_ = 0, False, (1 << 64) - 1
    steps = 0
    while pc < len(ins):
        steps += 1
        assert steps < 10000
        s = ins[pc]
        if re.fullmatch(r"\d+:", s):
            pc += 1
            continue
        name = s.split()[0]
        args = op.findall(s)
        if name == "s_bfe_u32":
            imm = int(s.split(",")[-1], 0)
            regs[args[0]] = (regs[args[1]] >> (imm & 31)) & ((1 << ((imm >> 16) & 0x7F)) - 1)
        elif name in ("s_cmp_lg_u32", "s_cmp_lt_u32"):
            n = int(s.split(",")[-1])
            scc = regs[args[0]] != n if name == "s_cmp_lg_u32" else regs[args[0]] < n
        elif name in ("s_cbranch_scc1", "s_cbranch_scc0"):
            if scc == (name == "s_cbranch_scc1"):
                pc = target(s.split()[1], pc)
                continue
        elif name == "s_branch":
            pc = target(s.split()[1], pc)
            continue
        elif name == "s_and_b64":
            assert s.startswith("s_and_b64 exec,") and args[1] == "sv"
            exec_ = regs[args[0]]
        elif name == "s_mov_b64":
            if s == "s_mov_b64 exec, 1":
                exec_ = 1
            elif s.startswith("s_mov_b64 exec,"):
                assert args == ["sv"]
                exec_ = (1 << 64) - 1
            else:
                regs[args[0]] = regs[args[1]]
        elif name in ("v_mov_b64", "ds_read_b64"):
            # ds_read_b64: the rebate slot, written by lane 0 before any read
            assert name == "v_mov_b64" or regs.get("_lds_written")
            k = int(args[0][1:])
            moved[k] |= exec_
        elif name == "ds_write_b64":
            assert exec_ == 1 and args == ["la", "rb"]
            regs["_lds_written"] = True
        elif name == "s_load_dwordx2":
            regs[args[0]] = row[int(s.split(",")[-1]) // 8]
        elif name == "s_waitcnt":
            pass
        else:
            raise AssertionError(f"unmodelled instruction {s!r}")
        pc += 1
    return exec_


def truth(npt, n_nodes, klo, khi):
    """(lane, slot) positions of the knocked-out interior nodes."""
    n_int = n_nodes - 2
    ls = -(-n_int // npt) * npt - n_int
    out = [0] * npt
    for i in range(n_int):
        if i <= klo - 1 or i >= khi - 1:
            t, k = lane_slot(i, npt, ls)
            out[k] |= 1 << t
    return out


def _cases(npt):
    from test_gpu_ko_resident import layouts, thresholds
    n_nodes = 64 * npt
    cs = [thresholds(npt, n_nodes, *lay) for lay in layouts(npt)]
    rng = np.random.default_rng(npt)
    n_int = n_nodes - 2
    for _ in range(300):
        a, b = sorted(int(x) for x in rng.integers(-2, n_int + 4, 2))
        cs.append((a, b))
    cs += [(-1, 1 << 30), (0, n_int + 1), (n_int, n_int + 1), (5, 6), (n_int - 1, 1)]
    return n_nodes, cs


@pytest.mark.parametrize("form", ["", "L"], ids=["vmov", "lds"])
@pytest.mark.parametrize("npt", [64, 48])
def test_projection_moves_exactly_the_knocked_nodes(npt, form):
    blocks = _blocks(npt, form)
    n_nodes, cases = _cases(npt)
    seen = set()
    for klo, khi in cases:
        masks = slot_masks(npt, n_nodes, klo, khi)
        regs, nchg = prologue(npt, masks)
        assert nchg <= 2, (klo, khi)
        row = masks + [0] * (64 - npt)
        regs.update(rb=0, sv=(1 << 64) - 1, cd=0, mt=0, ka=0, la=0)
        if form == "L":  # the kernel's mask-load statement wrote the rebate word
            regs["_lds_written"] = True
        moved = [0] * npt
        for ins in blocks:
            assert run_block(ins, regs, row, moved) == (1 << 64) - 1  # exec restored
        assert moved == truth(npt, n_nodes, klo, khi), (klo, khi)
        for g in range(npt // 8):
            word = regs["c0"] if g < 5 else regs["c1"]
            seen.add((g, (word >> (6 * (g if g < 5 else g - 5))) & 63))
    # every special code of groups 0, 3 and the last was exercised
    g_last = npt // 8 - 1
    for g in (0, 3, g_last):
        gsz = 7 if g == g_last else 8
        # (group 0 has no change at its slot 0: change points start at slot 1)
        want = {1 + o for o in range(gsz) if g or o}
        want |= {gsz + 1 + o1 * (2 * gsz - o1 - 1) // 2 + (o2 - o1 - 1)
                 for o1 in range(gsz) for o2 in range(o1 + 1, gsz) if g or o1}
        assert want <= {c for gg, c in seen if gg == g}, (g, sorted(want - {c for gg, c in seen if gg == g}))


@pytest.mark.parametrize("form", ["", "L"], ids=["vmov", "lds"])
def test_row_fallback_path(form):
    """Code 63 (masks from the workspace row) on every group reproduces the
    per-slot masks exactly, whatever the queue holds."""
    npt = 64
    blocks = _blocks(npt, form)
    rng = np.random.default_rng(5)
    masks = [int(x) for x in rng.integers(0, 1 << 62, npt)]
    regs = dict(q0=1, q1=2, q2=3, qd=masks[-1], c0=sum(63 << (6 * g) for g in range(5)),
                c1=sum(63 << (6 * g) for g in range(3)), rb=0, sv=(1 << 64) - 1, cd=0, mt=0, ka=0,
                la=0, _lds_written=(form == "L"))  # (the kernel's mask-load statement)
    moved = [0] * npt
    for ins in blocks:
        run_block(ins, regs, masks, moved)
    assert moved == masks


def test_lds_form_rebate_written_by_the_mask_load_statement():
    """The LDS form's statements only read the rebate word; the kernel writes
    it (lane 0, exec = 1, then exec restored) inside the statement that loads
    the run masks, ahead of that statement's lgkmcnt(0) -- so the write has
    landed before the first ds_read (LDS operations complete in order)."""
    for npt in (64, 48):
        for ins in _blocks(npt, "L"):
            assert not any(i.startswith("ds_write") for i in ins), npt
    src = open(os.path.join(ROOT, "finite_difference_amd", "csrc", "fdcn_kernels.hip")).read()
    w = src.index("#define FDCN_KO_RB_WRITE \\")
    body = src[w:src.index("#endif", w)]
    assert "s_mov_b64 exec, 1" in body and "ds_write_b64 %14, %15" in body
    assert "s_mov_b64 exec, %6" in body
    load = src.index('FDCN_KO_RB_WRITE "s_waitcnt lgkmcnt(0)"')
    assert load > w
