"""GPU parity of the resident-mask knock-out projection (round 6; the
recovery-form variants fdcn_march<0,1,48|64,*>, config 5's layout).

The projection walks the slots in groups of eight with a per-group code that
the kernel prologue derives from the knock-out thresholds (fdcn_ko_res.h,
tools/gen_ko_res.py): no change inside the group, one change at each offset
0..7 (the lower side's partial lane leaving, the upper side's joining), two
changes in one group (28 cases), the last group of seven, the last slot under
its own mask (the short lanes' phantom).  Each case here puts the partial
lanes' last / first knocked slot where it lands in a chosen group and offset,
with a knock-out on every step and a non-zero rebate (a missed or extra node
is then a visible error), and compares every node with the C oracle
(reference: discrete_barrier_fdm_pricer.py:413-440, :517-546).

Tolerance: 1e-10 relative, as test_gpu_kernels.py.
"""
import numpy as np
import pytest

from finite_difference_amd import capi
from plan_factory import random_solve
from test_gpu_kernels import _compare

pytestmark = pytest.mark.gpu

N_TIME = 24


def lane_start(t, npt, ls):
    """First interior index of lane t (the first ls lanes hold npt-1 nodes)."""
    return t * (npt - 1) if t < ls else ls * (npt - 1) + (t - ls) * npt


def thresholds(npt, n_nodes, tl, sl, th, sh):
    """KO_LO / KO_HI putting the lower side's last knocked node at slot sl of
    lane tl and the upper side's first at slot sh of lane th (None: side
    absent)."""
    n_int = n_nodes - 2
    ls = -(-n_int // npt) * npt - n_int
    klo = -1 if tl is None else lane_start(tl, npt, ls) + sl + 1
    khi = 1 << 30 if th is None else lane_start(th, npt, ls) + sh + 1
    return klo, khi


def layouts(npt):
    """(tl, sl, th, sh) cases covering every group code at least once."""
    out = []
    # one change per side, in different groups: every offset of every group
    for sl in range(npt):
        out.append((10, sl, 50 if npt == 64 else 40, (5 * sl + 3) % npt))
    # both changes in one group: every (o1, o2) pair of groups 0, 3 and the last
    g_last = npt // 8 - 1
    for g in (0, 3, g_last):
        gsz = 7 if g == g_last else 8
        for o1 in range(gsz):
            for o2 in range(o1 + 1, gsz):
                # c1 = sl + 1, c2 = sh
                c1, c2 = 8 * g + o1, 8 * g + o2
                if c1 >= 1:
                    out.append((12, c1 - 1, 45 if npt == 64 else 35, c2))
                    out.append((12, c2 - 1, 45 if npt == 64 else 35, c1))  # upper joins first
    # one partial lane serving both sides (a window inside one lane)
    for sl, sh in ((3, 9), (0, 63 if npt == 64 else 47), (20, 21), (40, 44)):
        if sh < npt:
            out.append((30, sl, 30, sh))
    # one side only; a side covering the short lanes only; lane-aligned sides
    out += [(None, 0, 40, 17), (9, 33, None, 0), (1, 5, None, 0), (0, npt - 3, 60 if npt == 64 else 44, 0),
            (20, npt - 1, 41, 0)]
    return out


@pytest.mark.parametrize("npt", [64, 48])
def test_resident_ko_groups_vs_oracle(npt, force_variant):
    force_variant(1, npt)
    n_nodes = 64 * npt - 2 + 2  # two short lanes: the phantom slot is in play
    cases = layouts(npt)
    rng = np.random.default_rng(640 + npt)
    solves = []
    for i, (tl, sl, th, sh) in enumerate(cases):
        s = random_solve(rng, n_nodes, N_TIME, 2, it=False, ko=False, drop_top=(i % 3 == 0))
        s.ko_lo, s.ko_hi = thresholds(npt, n_nodes, tl, sl, th, sh)
        s.mon_steps = list(range(1, N_TIME + 1))
        s.mon_rebates = [0.75 + 0.01 * (i % 7)] * N_TIME
        solves.append(s)
    plan = capi.plan(n_nodes, False, B=len(solves))
    assert (plan["waves"], plan["npt"]) == (1, npt), plan
    assert capi.variant_name(n_nodes, False, B=len(solves)) == f"fdcn_march<0,1,{npt},0>"
    _compare(solves, f"resident KO NPT={npt} cases={len(solves)}")


def test_resident_ko_monitor_dates_subset(force_variant):
    """Discrete monitoring (knock-outs on a subset of steps) on the same
    layout: the projection runs only on monitor steps, the codes stay."""
    force_variant(1, 64)
    n_nodes = 4096
    rng = np.random.default_rng(4242)
    solves = []
    for i, (tl, sl, th, sh) in enumerate(layouts(64)[:40]):
        s = random_solve(rng, n_nodes, 70, 2, it=False, ko=False)
        s.ko_lo, s.ko_hi = thresholds(64, n_nodes, tl, sl, th, sh)
        s.mon_steps = sorted(set(int(x) for x in rng.integers(1, 71, 12)))
        s.mon_rebates = [float(rng.choice([0.0, 1.5])) for _ in s.mon_steps]
        solves.append(s)
    _compare(solves, "resident KO, discrete monitoring")
