"""GPU parity: libfdcn (HIP, gfx950) vs the CPU oracle on identical plans.

Tolerance (fp64): max_j |V_gpu - V_oracle| <= 1e-10 * max(1, max_j |V_oracle|)
per solve.  The kernel reassociates the Thomas solve (converged-LU scan +
Sherman-Morrison, FMA), so results agree to rounding, not bitwise; the bound
leaves >100x margin over the observed error (printed with -s).
"""
import numpy as np
import pytest

from finite_difference_amd import capi
from finite_difference_amd.engine import Engine, group_solves
from plan_factory import random_solve

pytestmark = pytest.mark.gpu

TOL = 1e-10


class OracleBackend:
    name = "oracle"

    def run_group(self, g):
        from oracle import oracle
        if g.it:
            return oracle.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                   g.v_init, g.payoff, 8)
        return oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                               g.mon_step, g.mon_rebate, 8)


def _compare(solves, label, tol=TOL):
    gpu = Engine().run(solves)
    ref = Engine(OracleBackend()).run(solves)
    worst = 0.0
    for g, r in zip(gpu, ref):
        assert np.all(np.isfinite(g)), f"{label}: non-finite GPU output"
        scale = max(1.0, float(np.max(np.abs(r))))
        err = float(np.max(np.abs(g - r))) / scale
        worst = max(worst, err)
    print(f"[{label}] solves={len(solves)} worst_rel_err={worst:.3e}")
    assert worst <= tol, f"{label}: {worst:.3e} > {tol}"
    return worst


# (n_nodes, n_time, n_ranna): covers every W=1 NPT variant, short/phantom lanes,
# inactive lanes, multi-wave variants, Rannacher on/off, n_ranna >= n_time.
CASES = [
    (6, 20, 2), (20, 37, 2), (67, 50, 0), (130, 64, 2), (257, 100, 2), (513, 200, 0),
    (769, 120, 2), (1024, 150, 2), (1500, 90, 2), (2049, 128, 2), (2134, 60, 2),
    (2600, 40, 2), (3000, 30, 2), (4097, 24, 2), (4265, 20, 2), (9000, 12, 2),
    (300, 3, 5),
    (5, 10, 2), (7, 30, 2), (8, 25, 0), (11, 40, 2),  # two-node chunks (NPT = 2)
]


@pytest.mark.parametrize("n_nodes,n_time,n_ranna", CASES)
def test_cn_ko_vs_oracle(n_nodes, n_time, n_ranna):
    rng = np.random.default_rng(1000 + n_nodes)
    B = 9
    solves = [random_solve(rng, n_nodes, n_time, n_ranna, it=False, drop_top=(i % 2 == 0))
              for i in range(B)]
    _compare(solves, f"cn n={n_nodes} m={n_time} r={n_ranna} {capi.plan(n_nodes, False, B=B)}")


@pytest.mark.parametrize("n_nodes,n_time,n_ranna", CASES)
def test_it_vs_oracle(n_nodes, n_time, n_ranna):
    rng = np.random.default_rng(2000 + n_nodes)
    B = 7
    solves = [random_solve(rng, n_nodes, n_time, n_ranna, it=True) for _ in range(B)]
    _compare(solves, f"it n={n_nodes} m={n_time} r={n_ranna} {capi.plan(n_nodes, True, B=B)}")


# Every compiled (W, NPT, flavour) variant, forced (fdcn_force_variant) on a
# grid that fills it (64*W*NPT - 3 interior nodes: 3 short lanes, no idle
# wave), over 130 steps: three 64-step blocks of boundary terms, so every
# block-start load and the block loop's carried state are exercised, with
# half the solves on accumulated tau (TAU_MODE = 1, the American reference's
# tau += dt) from a non-zero tau0.  The default choice depends on the batch
# size, so small test batches alone would not reach the throughput variants
# the bench uses.
VARIANTS = [(1, 2, 0), (1, 4, 0), (1, 8, 0), (1, 12, 0), (1, 16, 0), (1, 24, 0), (1, 32, 0), (1, 40, 0),
            (1, 48, 0), (1, 64, 0), (2, 8, 0), (2, 16, 0), (2, 32, 0), (2, 40, 0), (4, 8, 0), (4, 16, 0),
            (4, 24, 0), (4, 40, 0), (8, 8, 0), (8, 16, 0), (8, 40, 0), (16, 8, 0), (16, 24, 0),
            (16, 40, 0), (1, 8, 1), (1, 16, 1), (1, 32, 1)]
N_TIME_BLOCKS = 130


@pytest.mark.parametrize("it", [False, True], ids=["cn", "it"])
@pytest.mark.parametrize("w,npt,fl", VARIANTS, ids=[f"w{w}n{n}f{f}" for w, n, f in VARIANTS])
def test_every_variant_vs_oracle(w, npt, fl, it, force_variant):
    force_variant(w, npt, fl)
    n_nodes = 64 * w * npt - 3 + 2
    n_time = N_TIME_BLOCKS
    plan = capi.plan(n_nodes, it, B=4)
    assert (plan["waves"], plan["npt"]) == (w, npt), plan
    assert capi.variant_name(n_nodes, it, B=4) == f"fdcn_march<{int(it)},{w},{npt},{2 * fl}>"
    rng = np.random.default_rng(3000 + 7 * w + npt + 11 * fl + (1 if it else 0))
    solves = [random_solve(rng, n_nodes, n_time, 2, it=it, drop_top=(i == 1)) for i in range(4)]
    for i, s in enumerate(solves):
        s.tau_accumulate = i % 2 == 1
        s.tau0 = 0.0 if i < 2 else 0.037
    # these grids reach 40k nodes with few steps (dt sigma^2/dx^2 up to ~1e5, |fm|
    # within 1e-3 of 1): rounding in the O(n) recurrences of both solvers then
    # grows with n, so the bound scales with n / 2048 above 2048 nodes
    _compare(solves, f"{'it' if it else 'cn'} forced W={w} NPT={npt} F={fl} n={n_nodes} m={n_time}",
             tol=TOL * max(1.0, n_nodes / 2048))


@pytest.mark.parametrize("it", [False, True], ids=["cn", "it"])
def test_correction_table_in_workspace(it):
    """|fm| -> 1 (huge dt sigma^2/dx^2): the Sherman-Morrison extent covers the
    whole 10k-node grid, its table no longer fits LDS, and the launch falls
    back to a ZG variant that keeps it in the global workspace."""
    n_nodes, n_time = 64 * 4 * 40 - 3 + 2, 3
    rng = np.random.default_rng(77 + int(it))
    solves = [random_solve(rng, n_nodes, n_time, 2, it=it) for _ in range(3)]
    from finite_difference_amd.engine import pack
    g = pack(solves, list(range(3)))
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    assert k_cap > 5000, k_cap
    plan = capi.plan(n_nodes, it, k_cap=k_cap, B=3)
    assert plan["ws_bytes_per_scen"] > 16 * 64 * plan["waves"], plan  # table in the workspace
    _compare(solves, f"{'it' if it else 'cn'} ZG n={n_nodes} k_cap={k_cap} {plan}",
             tol=TOL * n_nodes / 2048)


def test_batch_size_picks_variant():
    assert (capi.plan(2049, True, B=4096)["waves"], capi.plan(2049, True, B=4096)["npt"]) == (1, 32)
    large = capi.plan(4097, False, B=4096)
    small = capi.plan(4097, False, B=1)
    assert (large["waves"], large["npt"]) == (1, 64)
    # a single solve of 64-node chunks is split over 4 waves (latency)
    assert (small["waves"], small["npt"]) == (4, 16)
    # a single 2049-node IT solve keeps W = 1 NPT = 32 (single-trade flavour)
    one = capi.plan(2049, True, B=1)
    assert (one["waves"], one["npt"]) == (1, 32)


def test_large_batch_partial_block():
    # B not a multiple of the 4 scenarios per workgroup; mixed KO layouts
    rng = np.random.default_rng(7)
    solves = [random_solve(rng, 1024, 40, 2, it=False) for _ in range(203)]
    _compare(solves, "cn batch 203")


def test_zero_steps_is_identity():
    rng = np.random.default_rng(3)
    s = random_solve(rng, 300, 0, 2, it=False, ko=False)
    out = Engine().run([s])[0]
    assert np.array_equal(out, s.v_init)


def test_device_visible():
    assert capi.device_count() >= 1


@pytest.mark.parametrize("ko_lo", [-1, 30, 1500], ids=["none", "inside_table", "covers_table"])
def test_rec_form_every_step_knockout_vs_oracle(ko_lo, force_variant):
    """Config-5 layout (W=1, NPT=64, recovery form) with a knock-out on every
    step.  When the lower side covers the Sherman-Morrison lanes the kernel
    skips the correction on those steps (the projection overwrites it)."""
    force_variant(1, 64)
    n_nodes, n_time = 4096, 96
    rng = np.random.default_rng(4096 + ko_lo)
    solves = []
    for i in range(4):
        s = random_solve(rng, n_nodes, n_time, 2, it=False, ko=False)
        s.ko_lo, s.ko_hi = ko_lo, 3500 if i % 2 else 1 << 30
        s.mon_steps = list(range(1, n_time + 1))
        s.mon_rebates = [0.0 if i < 2 else 0.75] * n_time
        solves.append(s)
    assert capi.plan(n_nodes, False, B=4)["npt"] == 64
    _compare(solves, f"rec every-step KO ko_lo={ko_lo}")


# The paired flavour (two scenarios per wave, lanes 0-31 and 32-63), forced:
# full and partial lane use, an odd batch (the last wave's second scenario is
# missing), per-scenario monitoring schedules and knock-out layouts, both
# top-node layouts, accumulated tau.
PAIR_CASES = [(8, 32 * 8 - 1, 5), (8, 32 * 8 + 1, 6), (8, 150, 4), (8, 97, 7), (8, 42, 1)]


@pytest.mark.parametrize("npt,n_nodes,B", PAIR_CASES,
                         ids=[f"n{npt}_{n}_{b}" for npt, n, b in PAIR_CASES])
def test_paired_variant_vs_oracle(npt, n_nodes, B, force_variant):
    force_variant(1, npt, 2)
    plan = capi.plan(n_nodes, False, B=B)
    assert (plan["waves"], plan["npt"], plan["scen_per_block"]) == (1, npt, 2), plan
    rng = np.random.default_rng(5000 + npt + n_nodes + B)
    solves = []
    for i in range(B):
        s = random_solve(rng, n_nodes, 60, 2, it=False, drop_top=(i % 3 == 0))
        s.tau_accumulate = (i % 4 == 1)
        solves.append(s)
    _compare(solves, f"cn paired NPT={npt} n={n_nodes} B={B}")


def test_paired_every_step_knockout_vs_oracle(force_variant):
    """Knock-out schedules that differ between the two scenarios of a wave:
    every step on one, sparse on the other, rebates on both sides."""
    force_variant(1, 8, 2)
    n_nodes, n_time = 256, 80
    rng = np.random.default_rng(99)
    solves = []
    for i in range(6):
        s = random_solve(rng, n_nodes, n_time, 2, it=False, ko=False)
        s.ko_lo, s.ko_hi = (10 + 9 * i, 225 - 3 * i) if i % 2 else (-1, 175)
        s.mon_steps = list(range(1, n_time + 1)) if i % 2 == 0 else [5, 17, 18, 60, n_time]
        s.mon_rebates = [0.5 * (i % 3)] * len(s.mon_steps)
        solves.append(s)
    _compare(solves, "cn paired, mixed knock-out schedules")


def test_large_batch_picks_paired_variant():
    big = capi.plan(256, False, B=10000)
    assert (big["waves"], big["npt"], big["scen_per_block"]) == (1, 8, 2), big
    small = capi.plan(256, False, B=100)
    assert (small["waves"], small["npt"], small["scen_per_block"]) == (1, 4, 1), small
    # config-3 grids keep one scenario per wave (the paired flavour loses there)
    c3 = capi.plan(1024, False, B=10000)
    assert (c3["waves"], c3["npt"], c3["scen_per_block"]) == (1, 16, 1), c3


@pytest.mark.parametrize("ko_lo", [-1, 20, 600], ids=["none", "inside_table", "covers_table"])
def test_split_two_pass_every_step_knockout_vs_oracle(ko_lo, force_variant):
    """Config-3 layout (CN split form on the two-pass solve, DPP-broadcast
    tables, W=1 NPT=16) with a knock-out on every step, rebates on both sides,
    accumulated tau on half the solves, both top-node layouts: the carried
    boundary terms after a knock-out (ko_prev) and the folded
    Sherman-Morrison correction under a projection that covers its lanes."""
    force_variant(1, 16)
    n_nodes, n_time = 1024, 150
    rng = np.random.default_rng(1600 + ko_lo)
    solves = []
    for i in range(6):
        s = random_solve(rng, n_nodes, n_time, 2, it=False, ko=False, drop_top=(i % 2 == 0))
        s.ko_lo, s.ko_hi = ko_lo, (900 if i % 3 else 1 << 30)
        s.mon_steps = list(range(1, n_time + 1)) if i < 3 else list(range(2, n_time + 1, 7))
        s.mon_rebates = [0.0 if i % 2 else 1.25] * len(s.mon_steps)
        s.tau_accumulate = i % 2 == 1
        solves.append(s)
    assert capi.variant_name(n_nodes, False, B=6) == "fdcn_march<0,1,16,0>"
    _compare(solves, f"split two-pass every-step KO ko_lo={ko_lo}")


def _fm(a, c, bc, dt, theta):
    """The converged forward multiplier fm = -A_L / r of A = I - theta dt L
    (r: the larger root of r^2 - A_C r + A_L A_U = 0), as the kernel's phase."""
    AL, AC, AU = -theta * dt * a, 1.0 - theta * dt * bc, -theta * dt * c
    r = 0.5 * (AC + np.sqrt(AC * AC - 4.0 * AL * AU))
    return -AL / r


@pytest.mark.parametrize("n_nodes", [4096, 4097, 3000], ids=["short2", "full", "npt48"])
def test_rec_form_half_chunk_aggregates_vs_oracle(n_nodes, force_variant):
    """The recovery form's half-chunk aggregates (solve_rec, rec_half): grids
    with dt sigma^2 / dx^2 ~ 1 (config 5's regime), so the Crank-Nicolson
    phase's |fm|^(NPT/2) is below 1e-18 (aggregates over half a chunk, no
    scan stages) while the two Rannacher steps' is not (the uniform branch
    that adds the other halves): both paths in one march, with a knock-out
    on every step, short lanes (4096 nodes: two), a full layout (4097) and
    the 48-node chunks (3000 nodes)."""
    npt = 48 if n_nodes == 3000 else 64
    force_variant(1, npt)
    rng = np.random.default_rng(77 + n_nodes)
    solves = []
    for i in range(6):
        s = random_solve(rng, n_nodes, 80, 2, it=False, ko=False)
        a, c, bc = s.coeffs
        # dt a in a band where the CN phase's |fm|^(NPT/2) is < 1e-18 and the
        # Rannacher phase's is not
        s.dt = ((0.6 + 0.04 * i) if npt == 64 else (0.3 + 0.03 * i)) / a
        fm_cn, fm_r = _fm(a, c, bc, s.dt, 0.5), _fm(a, c, bc, s.dt, 1.0)
        bm_cn = _fm(c, a, bc, s.dt, 0.5)
        assert abs(fm_cn) ** (npt // 2) < 1e-18 and abs(bm_cn) ** (npt // 2) < 1e-18, (fm_cn, bm_cn)
        assert abs(fm_r) ** (npt // 2) > 1e-18, fm_r  # the Rannacher steps take the branch
        s.ko_lo, s.ko_hi = int(rng.integers(-1, 600)), int(rng.integers(n_nodes - 700, n_nodes + 2))
        s.mon_steps = list(range(1, s.n_time + 1))
        s.mon_rebates = [0.0 if i % 2 else 0.4] * s.n_time
        solves.append(s)
    assert capi.plan(n_nodes, False, B=6)["npt"] == npt
    _compare(solves, f"rec half-chunk aggregates n={n_nodes}")


@pytest.mark.parametrize("n_nodes,npt", [(1024, 16), (513, 8), (2134, 40)])
def test_one_sided_table_batch_vs_oracle(n_nodes, npt):
    """The one-sided boundary table (round 6; fdcn_march kTab1: chunks of 16
    to 40 nodes, batches of kTab1MinBatch = 256 and more; the 513-node grid's
    8-node chunks keep the two-sided table): calls (constant lower side), puts
    (constant upper side, both Dirichlet forms), knock-outs that reach an
    edge node or not, sparse and every-step monitoring, accumulated tau --
    the raw values kept only for the steps after an edge knock-out, every
    node against the oracle."""
    rng = np.random.default_rng(777 + n_nodes)
    B = 300
    solves = []
    for i in range(B):
        s = random_solve(rng, n_nodes, 150, 2, it=False, drop_top=(i % 2 == 0))
        s.tau_accumulate = i % 5 == 1
        if i % 7 == 3:  # a knock-out on every step reaching node 0 / the last node
            s.ko_lo, s.ko_hi = int(rng.integers(0, 40)), n_nodes - int(rng.integers(1, 40))
            s.mon_steps = list(range(1, 151))
            s.mon_rebates = [0.25] * 150
        solves.append(s)
    plan = capi.plan(n_nodes, False, B=B)
    assert (plan["waves"], plan["npt"]) == (1, npt), plan
    _compare(solves, f"one-sided table n={n_nodes} B={B}", tol=TOL * max(1.0, n_nodes / 2048))


@pytest.mark.parametrize("n_nodes,B,n_ranna,variant", [
    (2049, 2048, 2, "fdcn_march<1,1,32,0>"),   # config 2's instance
    (1500, 300, 2, "fdcn_march<1,1,24,0>"),
    (1500, 300, 0, "fdcn_march<1,1,24,0>")], ids=["config2", "npt24", "npt24_no_rannacher"])
def test_it_throughput_batch_vs_oracle(n_nodes, B, n_ranna, variant):
    """The IT throughput variants on throughput-sized batches (the planner's
    own choice at these B, asserted): puts (both lower-boundary forms) and
    calls, accumulated tau on a fifth of the solves, a non-zero tau0 on a
    third, every node against the oracle over three 64-step blocks.  (Round 6
    ran a one-sided-table build of these variants through it, measured and
    not kept: profiles/r06/config2_tab1/.)"""
    assert capi.variant_name(n_nodes, True, B=B) == variant
    rng = np.random.default_rng(2049 + n_nodes + B + n_ranna)
    solves = []
    for i in range(B):
        s = random_solve(rng, n_nodes, 150, n_ranna, it=True)
        s.tau_accumulate = i % 5 == 1
        s.tau0 = 0.0 if i % 3 else 0.021
        solves.append(s)
    _compare(solves, f"it throughput batch n={n_nodes} B={B} r={n_ranna}")
