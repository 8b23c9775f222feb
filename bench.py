#!/usr/bin/env python3
"""Benchmark: CN grid-node-steps/sec on the BASELINE workloads.

Default workload (BASELINE.json configs[1], the metric's config): American put,
fd_american_equity.py, num_space_nodes=2048, num_time_steps=4096, Rannacher 2,
Ikonen-Toivanen early exercise, the notebook trade (S0=176.39, 2025-07-28 ->
2025-08-28, flat NACA e^0.07053828272-1).  A "step" is one pass of the hot
path over one batch: one launch of the batched IT march over B independent
scenarios of that trade swept over strike and volatility (the scenario-batch
axis of the north star).  Inputs are built by the product's AmericanFDMPricer
facade and are resident in HBM before the timed region.

Other workloads (--workload, same JSON line format):
  barrier  configs[2]: 10 000 discrete-barrier scenarios (config_scenarios.csv
           trade, K/sigma/barrier sweep, up/down out/in x call/put), explicit
           1024 x 2000 grid, daily KO monitoring (run_config_scenarios.py).
  double   configs[4]: double knock-out call of double _barrier.py:139-146 on a
           4096 x 8192 grid, projection every step; --batch B sweeps sigma and
           the barriers.
  analytic SURVEY §8(f) row 4, not a BASELINE config: 2^20 Reiner-Rubinstein
           barrier contracts (barrier_engine.py) per launch, one GPU thread
           each; its own metric line (contracts/s).
Single-trade latency (one trade end to end through the drop-in facade, host
plan building, launches, copies and the Greeks epilogue included; their own
metric line, ms per trade):
  trade_cnlog     configs[0]: DiscreteBarrierCrankNicolsonLog.price() of the
                  discrete_barrier_fdm_main_cn.py trade, 512 x 1000 (3 solves)
  trade_american  configs[1]: AmericanFDMPricer price_log2() + greeks_log2()
                  of the notebook trade, 2048 x 4096 (6 unique solves)
  trade_double    configs[4]: FDDoubleBarrier.price(b, r, T), 4096 x 8192
Whole scenario file (run_all_scenarios' pricing, ms per file; host time split
out -- VERDICT r1 item 7):
  scenario_file   configs[2] numerics: 10 000 rows (KO / KI / vanilla, one
                  option type per file), explicit 1024 x 2000, priced by
                  scenario_batch.price_columns + result_columns
  american_file   configs[1] numerics: 2 000 American put rows (strike / vol /
                  spot sweep, two curves), 2048 x 4096, price_log2 +
                  greeks_log2 of every row by american_batch.price_columns

value = total node-steps (configured nodes x steps x B x ranks) / max-over-
ranks wall time of the K timed launches (whole-job aggregate).

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank; `--gpus N` without WORLD_SIZE spawns the N ranks
itself (torch.multiprocessing, spawn start method) before anything touches a
GPU.  Each rank binds GPU LOCAL_RANK and marches its own B scenarios (weak
scaling, no collective in the data path; the only RCCL calls are the timing
barrier and the max over ranks).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                       [--workload NAME] [--dry-run]
"""
from __future__ import annotations

import argparse
import datetime as dt
import hashlib
import json
import math
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md chip table (spec)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X spec sheet, FP64 vector (FMA = 2 flops)
VALU_CLOCK_GHZ = 2.4          # peak engine clock: 1024 SIMDs x 1 wave64 fp64 op / 4 clk
N_SIMD = 1024
# algorithmic flops per node-step of the reference
# algorithm (DESIGN.md §4 derives them from fd_american_equity.py:681-717 and
# discrete_barrier_fdm_pricer.py:531-546: RHS 5 (+2 for dt*lambda), Thomas
# with the factorisation hoisted 5, IT update 5).  (§8(d)'s bytes per
# node-step -- 32 IT, 16 CN, V (and lambda) in and out as if streamed every
# step -- are not an HBM quantity here: the vector stays in VGPRs; the line
# reports the measured HBM bytes instead, roofline_records.)
FLOPS_PER_NODE_STEP = {True: 17, False: 10}
DEFAULT_BATCH = {"american": 4096, "barrier": 10000, "double": 2048, "analytic": 1 << 20,
                 "spot_vc": 4096}
TRADE_WORKLOADS = ("trade_cnlog", "trade_american", "trade_double", "scenario_file",
                   "american_file")
KERNEL_SRC = os.path.join(ROOT, "finite_difference_amd", "csrc", "fdcn_kernels.hip")
# GPU vs oracle bound of the parity record (tests/test_gpu_kernels.py TOL)
PARITY_TOL = 1e-10


WARM_SECONDS = 1.0


def warm_up(step, args, sync=None) -> int:
    """Run the untimed warm-up and return the number of steps it ran.  An
    explicit --warmup W runs exactly W.  The default runs 2, then more until
    WARM_SECONDS of wall time have passed (at most 2000 steps): on a fresh
    box the first launches run below the steady clock (config 3, 10 000
    scenarios: 5.2 ms falling to 4.2 over the first ~1 s; --warmup 2 timed
    4.44 ms, --warmup 40 4.22)."""
    if args.warmup is not None:
        for _ in range(args.warmup):
            step()
        return args.warmup
    sync = sync or (lambda: None)
    n = 0
    t0 = time.perf_counter()
    while n < 2 or (time.perf_counter() - t0 < WARM_SECONDS and n < 2000):
        step()
        n += 1
        if n % 4 == 0:
            sync()  # bound the queue so the wall clock tracks the GPU
    sync()
    return n


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warm-up steps (default: at least 2, continued until "
                         "WARM_SECONDS of them have run: the clock ramps over the first ~1 s "
                         "of work, profiles/r05/tail/)")
    ap.add_argument("--workload", choices=sorted(DEFAULT_BATCH) + list(TRADE_WORKLOADS),
                    default="american")
    ap.add_argument("--batch", type=int, default=0, help="scenarios per GPU (0: workload default)")
    ap.add_argument("--total", type=int, default=0,
                    help="strong scaling (BASELINE config 4): ONE batch of this many scenarios, "
                         "built identically on every rank; rank r marches its contiguous "
                         "shard (distributed.shard_range)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group of the N>1 ranks: nccl (RCCL over xGMI, one GPU per "
                         "rank) or gloo (host collectives: ranks rehearsing the sharded path "
                         "on one GPU with FDCN_SHARE_DEVICE=1, tests/test_gpu_multirank.py)")
    ap.add_argument("--lib", default="", help="A/B timing: load this build of libfdcn.so")
    ap.add_argument("--force-variant", default="",
                    help="A/B timing: W,NPT[,FLAVOUR] pinned through fdcn_force_variant "
                         "(include/fdcn_diag.h)")
    ap.add_argument("--n-space", type=int, default=0, help="0: workload default")
    ap.add_argument("--n-time", type=int, default=0, help="0: workload default")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--overlap-streams", action="store_true",
                    help="also time the same batch launched on two streams in turn (each "
                         "launch with its own v_out / workspace, consecutive launches "
                         "overlapping): reported beside the line as overlapped_streams, "
                         "never its value (DESIGN.md §6, one launch and what concurrency "
                         "recovers)")
    ap.add_argument("--pcie-launches", type=int, default=2,
                    help="launches timed through the host-array ABI (pcie_inclusive; 0: skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="exercise the rank spawn / gloo / timing / gather plumbing without "
                         "a GPU (no march; the line is marked dry_run and is not a measurement)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
def build_american(B: int, n_space: int, n_time: int, seed: int, select=None):
    """B American puts of the notebook trade over a strike x vol sweep
    (scenarios `select` of them only, default all)."""
    from finite_difference_amd import market
    from finite_difference_amd.american import AmericanFDMPricer
    from finite_difference_amd.engine import pack
    val, mat = dt.date(2025, 7, 28), dt.date(2025, 8, 28)
    curve = market.iso_curve(market.create_rate_df(math.exp(0.07053828272) - 1.0))
    solves = []
    p = None  # one pricer, re-pointed per scenario (same dates and curve)
    for i in (range(B) if select is None else select):
        j = (i * 2654435761 + seed * 97) % B  # deterministic shuffle
        strike = 140.0 + 70.0 * (j % 64) / 63.0
        sigma = 0.18 + 0.30 * ((j // 64) % 64) / 63.0
        if p is None:
            p = AmericanFDMPricer(spot=176.39, strike=strike, valuation_date=val,
                                  maturity_date=mat, sigma=sigma, option_type="put",
                                  discount_curve=curve, forward_curve=curve,
                                  num_space_nodes=n_space, num_time_steps=n_time,
                                  rannacher_steps=2)
        p._reset_trade(176.39, strike, sigma)
        p._build_log_grid()
        solves.append(p._segment_solve(p._payoff_array(), 0.0, p.time_to_expiry, n_time, True))
    return pack(solves, list(range(len(solves))))


def build_barrier(B: int, n_space: int, n_time: int, seed: int, select=None):
    """the config_scenarios.csv trade swept over strike,
    vol and barrier; types cycle up/down-out/in x call/put; explicit grid.  A
    knock-in's march is its knock-out twin's (in/out parity), so every
    scenario contributes one KO march."""
    import numpy as np
    from finite_difference_amd import scenarios
    from finite_difference_amd.engine import pack
    rng = np.random.default_rng(20250728 + seed)
    base = scenarios.runner_base_params("put", n_space)
    base.update(num_time_steps=n_time, grid_mode="explicit")
    kinds = ["up-and-out", "down-and-out", "up-and-in", "down-and-in"]
    solves = []
    S0 = 229.74
    calc = {}  # one pricer per option type, re-pointed per scenario (scenarios.run_rows_batched)
    sel = range(B) if select is None else select
    for i in range(B):  # the draws of every scenario, so a shard sees the same batch
        bt = kinds[i % 4]
        K, sig = float(rng.uniform(150, 300)), float(rng.uniform(0.15, 0.45))
        up = float(rng.uniform(1.02, 1.5) * S0) if "up" in bt else None
        lo = float(rng.uniform(0.6, 0.98) * S0) if "down" in bt else None
        if i not in sel:
            continue
        opt = ("call", "put")[(i // 4) % 2]
        p = calc.get(opt)
        if p is None:
            p = calc[opt] = scenarios.make_barrier_pricer(
                S0, K, sig, 0.073086, bt, up, lo, base["valuation"], base["maturity"],
                base["monitor_dates"], opt_type=opt, num_space_nodes=n_space,
                num_time_steps=n_time, grid_mode="explicit")
        p._reset_trade(S0, K, sig, bt, lo, up)
        p.barrier_type = p._map_KI_to_KO() or p.barrier_type
        solves.append(p._make_solve(True, p.sigma)[0])
    grp = pack(solves, list(range(len(solves))))
    grp.top_dropped = True  # n_nodes = N_s configured nodes (…pricer.py:449, :543)
    return grp


def build_double(B: int, n_space: int, n_time: int, seed: int, select=None):
    """BASELINE config 5: double knock-out call of double _barrier.py:139-146,
    knock-out projected every step; B > 1 sweeps sigma and the barriers."""
    from finite_difference_amd.engine import pack
    from finite_difference_amd.fd_barrier import FDDoubleBarrier
    b, r, T = 0.049493018, 0.0709454892, 49 / 365
    solves = []
    for i in (range(B) if select is None else select):
        j = (i * 2654435761 + seed * 97) % max(B, 1)
        f = j / max(B - 1, 1)
        sig = 0.10994120968 * (0.8 + 0.4 * f) if B > 1 else 0.10994120968
        lo = 19.0 - (0.5 * f if B > 1 else 0.0)
        hi = 23.0 + (0.5 * f if B > 1 else 0.0)
        d = FDDoubleBarrier(20.786, 21.0, lo, hi, sig, "c", "out", n_space=n_space,
                            n_time=n_time)
        solves.append(d.solve_for(b, r, T))
    return pack(solves, list(range(len(solves))))


WORKLOADS = {  # name -> (builder, n_space, n_time, IT?, config label)
    "american": (build_american, 2048, 4096, True, "american_it_put"),
    "barrier": (build_barrier, 1024, 2000, False, "discrete_barrier_ko"),
    "double": (build_double, 4096, 8192, False, "double_barrier_ko"),
}


def node_units(group) -> int:
    """Configured asset nodes of one solve: N_s for the
    top-node-dropping barrier march (n_nodes = N_s), n_nodes - 1 otherwise."""
    return group.n_nodes if getattr(group, "top_dropped", False) else group.n_nodes - 1


# ---------------------------------------------------------------------------
# counters measured by tools/pmc_*.sh for THIS kernel source
# ---------------------------------------------------------------------------
def file_sha(name: str) -> str:
    """sha256 prefix of a kernel source file in finite_difference_amd/csrc/."""
    with open(os.path.join(os.path.dirname(KERNEL_SRC), name), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def kernel_src_sha() -> str:
    return file_sha(os.path.basename(KERNEL_SRC))


def load_counters(workload: str):
    """{hbm_bytes_per_launch, valu_insts_per_launch, ...} from
    profiles/pmc_counters.json for this workload -- only if they were measured
    on the current kernel source (sha of fdcn_kernels.hip); stale numbers are
    dropped (null), never reported."""
    path = os.path.join(ROOT, "profiles", "pmc_counters.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(workload)
    except Exception:
        return None
    if not rec or rec.get("kernel_src_sha") != kernel_src_sha():
        return None
    return rec


def roofline_records(fps: float, node_steps_launch: float, kernel_s: float, ctr) -> dict:
    """The measurement records of a march line,
    each against the peak of the resource it measures, so that no achieved
    figure can exceed its stated peak:

    roofline       the reference algorithm's fp64 flops (fps per node-step:
                   17 IT, 10 CN) / kernel time, against the fp64 VALU peak --
                   the binding roof (the value vector never leaves VGPRs);
    fp64_executed  the fp64 work the hardware actually issued (PMC:
                   SQ_INSTS_VALU_FMA_F64 x 2 + the other f64 VALU
                   instructions x 1, x 64 lanes) / kernel time, against the
                   same peak -- what the fp64 pipe was busy with, whatever the
                   reference's operation count;
    hbm            the measured HBM bytes (PMC FETCH_SIZE x 2 + WRITE_SIZE,
                   profiles/pmc_counters.json) / kernel time, against the
                   HBM peak (round 5's algorithmic-bytes rate, 32 B per
                   node-step as if V were streamed every step, reached 12.8x
                   the HBM peak: it was not an HBM quantity and is gone);
    valu_issue     SQ_INSTS_VALU per lane node-step and the issue fraction.

    The PMC-derived records are null unless the counters were measured on the
    current kernel source (load_counters)."""
    achieved_tf = fps * node_steps_launch / kernel_s / 1e12
    out = {"roofline": {"bound": "fp64_valu", "achieved": achieved_tf,
                        "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": achieved_tf / FP64_VALU_PEAK_TFLOPS,
                        "traffic": ctr.get("hbm_bytes_per_launch") if ctr else None,
                        "flops_per_node_step": fps},
           "fp64_executed": None, "hbm": None, "valu_issue": None}
    if ctr and ctr.get("f64_valu_insts_per_launch") and ctr.get("fma_f64_per_launch") is not None:
        fma = float(ctr["fma_f64_per_launch"])
        other = float(ctr["f64_valu_insts_per_launch"]) - fma
        flops = 64.0 * (2.0 * fma + other)
        tf = flops / kernel_s / 1e12
        out["fp64_executed"] = {
            "flops_per_node_step": flops / node_steps_launch, "achieved": tf,
            "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_VALU_PEAK_TFLOPS,
            "note": "PMC of this kernel source: (2 x SQ_INSTS_VALU_FMA_F64 + other f64 VALU "
                    "instructions) x 64 lanes per launch / kernel time"}
    if ctr and ctr.get("hbm_bytes_per_launch"):
        gbs = float(ctr["hbm_bytes_per_launch"]) / kernel_s / 1e9
        out["hbm"] = {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": gbs / HBM_PEAK_GBS,
                      "bytes_per_launch": float(ctr["hbm_bytes_per_launch"]),
                      "note": "measured HBM traffic (PMC FETCH_SIZE x 2 + WRITE_SIZE, "
                              "profiles/pmc_counters.json) / kernel time"}
    if ctr and ctr.get("valu_insts_per_launch"):
        insts = float(ctr["valu_insts_per_launch"])
        out["valu_issue"] = {
            "valu_insts_per_lane_node_step": 64 * insts / node_steps_launch,
            "issue_frac": insts * 4 / (N_SIMD * VALU_CLOCK_GHZ * 1e9 * kernel_s),
            "note": "SQ_INSTS_VALU (wave instructions) of this kernel source "
                    "(profiles/pmc_counters.json) x 64 lanes / node-steps; issue: x 4 clk "
                    "per wave64 fp64 op / (1024 SIMDs x 2.4 GHz x launch time)"}
    return out


# ---------------------------------------------------------------------------
# CPU baselines (rank 0, N = 1): the oracle restatements on the host cores
# ---------------------------------------------------------------------------
def _cpu_model() -> str:
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        return next((l.split(":", 1)[1].strip() for l in out.splitlines()
                     if l.startswith("Model name")), "") or platform.processor()
    except Exception:
        return platform.processor()


def host_cores():
    """(threads to use, record) for the CPU baseline: every core of the
    process's affinity set, capped by the cgroup CPU quota when one is set
    (a GPU box grants one-GPU jobs a share of its CPUs; threads beyond the
    quota only time-slice).  The record lists all three numbers."""
    affinity = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) / float(period)))
    except Exception:
        pass
    n = min(affinity, quota) if quota else affinity
    return n, {"affinity_cpus": affinity, "cgroup_cpu_quota": quota,
               "omp_max_threads_env": os.environ.get("OMP_NUM_THREADS")}


# scenarios per rank in the sampled parity record of multi-GPU runs
PARITY_SAMPLE = 8


def sample_parity(group, res, k: int) -> dict:
    """The parity record of the first k scenarios of `res` (this rank's timed
    output) against the C oracle, every node (cpu_baseline's rule)."""
    import numpy as np
    from oracle import oracle
    k = min(k, group.B)
    nthreads, _ = host_cores()
    sl = slice(0, k)
    if group.it:
        ref = oracle.it_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                              group.iparams[sl], group.v_init[sl], group.payoff[sl], nthreads)
    else:
        ref = oracle.cn_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                              group.iparams[sl], group.v_init[sl], group.mon_step,
                              group.mon_rebate, nthreads)
    got = np.asarray(res[:k])
    scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
    rel = np.max(np.abs(got - ref), axis=1) / scale
    rel = np.where(np.isnan(rel), np.inf, rel)  # a NaN must not vanish in the MAX reduction
    return {"max_rel_err": float(np.max(rel)) if rel.size else 0.0, "n_compared": int(k),
            "nodes_per_scenario": int(group.n_nodes), "tol": PARITY_TOL,
            "ok": bool(np.all(rel <= PARITY_TOL)), "all_finite": bool(np.all(np.isfinite(got))),
            "rule": "per scenario max_j |V_gpu - V_oracle| / max(1, max_j |V_oracle|), every "
                    "node of the timed launch's output vs the C oracle (oracle/fdcn_oracle.c)"}


def reduce_parity(part: dict, world: int, device) -> dict:
    """Every rank's sample_parity record -> the job's: the worst error and
    finiteness over the ranks (MAX), the compared scenarios summed."""
    import torch
    import torch.distributed as dist
    worst = torch.tensor([part["max_rel_err"], 0.0 if part["all_finite"] else 1.0],
                         dtype=torch.float64, device=device)
    cnt = torch.tensor([float(part["n_compared"])], dtype=torch.float64, device=device)
    dist.all_reduce(worst, op=dist.ReduceOp.MAX)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    err = float(worst[0].item())
    return dict(part, max_rel_err=err, all_finite=not worst[1].item() > 0,
                n_compared=int(cnt.item()), ok=bool(err <= PARITY_TOL),
                rule=part["rule"] + f"; the first {PARITY_SAMPLE} scenarios of every rank's "
                                    f"shard, worst over the {world} ranks")


def cpu_baseline(group, seconds: float, res=None):
    """Two variants of the reference algorithm, each on a
    bounded sample of the same batch:
      (i)  C oracle: sequential Thomas (+ IT / KO) per scenario, the
           reference's loops, OpenMP over scenarios on every host core the
           process may use (host_cores);
      (ii) NumPy batched over scenarios: the same loops with every per-node
           operation vectorised across scenarios (one core).
    The line's value is the faster one; both are listed.  The C oracle's
    outputs are the parity check of the GPU outputs `res` of the same
    scenarios (whole grid, every node): the "parity" record."""
    import numpy as np
    from oracle import batched_numpy, oracle
    nthreads, cores_rec = host_cores()
    model = _cpu_model()
    # (i) C oracle over whole scenarios, doubling the sample until `seconds`
    done, t_total, m = 0, 0.0, nthreads
    ref_parts = []
    while t_total < seconds and done < group.B:
        m = min(m, group.B - done)
        sl = slice(done, done + m)
        t0 = time.perf_counter()
        if group.it:
            out = oracle.it_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                                  group.iparams[sl], group.v_init[sl], group.payoff[sl],
                                  nthreads)
        else:
            # monitor runs are addressed by MON_START/MON_COUNT: pass the full arrays
            out = oracle.cn_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                                  group.iparams[sl], group.v_init[sl], group.mon_step,
                                  group.mon_rebate, nthreads)
        t_total += time.perf_counter() - t0
        ref_parts.append(out)
        done += m
        m *= 2
    c_rate = done * node_units(group) * group.n_time / t_total
    c_var = {"value": c_rate, "unit": "node-steps/s", "cores": nthreads, "kind": "port",
             "variant": "C oracle, per-scenario Thomas, OpenMP over scenarios",
             "sample": f"{done} of the {group.B} scenarios, full {node_units(group)}x"
                       f"{group.n_time} grid, {t_total:.1f} s"}
    parity = None
    if res is not None:
        ref = np.concatenate(ref_parts)
        got = res[:done]
        scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
        rel = np.max(np.abs(got - ref), axis=1) / scale
        parity = {"max_rel_err": float(np.max(rel)) if rel.size else None,
                  "n_compared": int(done), "nodes_per_scenario": int(group.n_nodes),
                  "tol": PARITY_TOL, "ok": bool(np.all(rel <= PARITY_TOL)),
                  "all_finite": bool(np.all(np.isfinite(got))),
                  "rule": "per scenario max_j |V_gpu - V_oracle| / max(1, max_j |V_oracle|), "
                          "every node of the timed launch's output vs the C oracle "
                          "(oracle/fdcn_oracle.c) on the same scenarios"}
    # (ii) NumPy batched over up to 4096 scenarios, a prefix of the time steps
    nb = min(group.B, 4096)
    kw = dict(payoff=group.payoff[:nb]) if group.it else dict(
        mon_step=group.mon_step, mon_rebate=group.mon_rebate)
    steps, t_np = 1, 0.0
    while True:
        t0 = time.perf_counter()
        batched_numpy.march(group.it, group.n_nodes, group.n_time, group.n_ranna,
                            group.params[:nb], group.iparams[:nb], group.v_init[:nb],
                            max_steps=steps, **kw)
        t_np = time.perf_counter() - t0
        if t_np > seconds / 3 or steps >= group.n_time:
            break
        steps = min(group.n_time, steps * 4)
    np_rate = nb * node_units(group) * steps / t_np
    np_var = {"value": np_rate, "unit": "node-steps/s", "cores": 1, "kind": "port",
              "variant": "NumPy, Thomas vectorised over scenarios",
              "sample": f"{nb} scenarios x first {steps} of {group.n_time} steps, full "
                        f"{node_units(group)}-node grid, {t_np:.1f} s"}
    best = c_var if c_rate >= np_rate else np_var
    cpu = {"value": best["value"], "unit": "node-steps/s", "cores": best["cores"],
           "kind": "port",
           "sample": best["sample"] + f"; {best['variant']} ("
                     + ("fd_american_equity.py:559-726" if group.it else
                        "discrete_barrier_fdm_pricer.py:442-547")
                     + f") on {model}",
           **cores_rec, "variants": [c_var, np_var]}
    return cpu, parity


# ---------------------------------------------------------------------------
# ranks
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_entry(local_rank: int, argv, port: int, world: int) -> None:
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    args = parse(argv)
    if args.lib:
        from finite_difference_amd import capi
        capi.LIB_PATH = os.path.abspath(args.lib)
    rc = run_rank(args)
    if rc:
        raise SystemExit(rc)


def spawn_ranks(args, argv) -> int:
    """`--gpus N` without a launcher: start N rank processes (spawn: fresh
    interpreters; this parent never touches a GPU) and wait for them."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_entry, args=(argv, _free_port(), args.gpus), nprocs=args.gpus,
                       join=True, start_method="spawn")
    return 0


def run_rank(args):
    if args.workload == "analytic":
        return bench_analytic(args)
    if args.workload == "spot_vc":
        return bench_spot_vc(args)
    if args.workload == "scenario_file":
        return bench_scenario_file(args)
    if args.workload == "american_file":
        return bench_american_file(args)
    if args.workload in TRADE_WORKLOADS:
        return bench_trade(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
        return dry_run_rank(args, world, rank, local)
    from finite_difference_amd import capi, distributed
    # this rank's GPU for libfdcn and torch; with several ranks a local
    # failure is reported through the group's binding check, so every rank
    # raises together instead of the others waiting for it in a collective
    bound = distributed.bind_device(raise_local=world == 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl" and bound is not None:
            dist.init_process_group("nccl", device_id=torch.device("cuda", bound))
        elif args.backend == "nccl":
            dist.init_process_group("nccl")
        else:
            dist.init_process_group("gloo")
        err = distributed.bind_error() or (
            None if bound is not None else "no gfx950 device visible to this rank")
        distributed.check_device_binding(bound, err)  # no two ranks on one GPU unless shared
    if bound is None:
        raise capi.FdcnError("no gfx950 device visible; the benchmark needs an MI355X")
    if args.force_variant:
        capi.force_variant(*[int(x) for x in args.force_variant.split(",")])
    dev = torch.device("cuda", bound)
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # collective tensors
    builder, ns0, nt0, is_it, label = WORKLOADS[args.workload]
    n_space, n_time = args.n_space or ns0, args.n_time or nt0
    t_build = time.perf_counter()
    if args.total:
        # config 4: one batch of `total` scenarios (the same draws on every
        # rank), rank r marches its contiguous shard -- strong scaling
        mine = distributed.shard_range(args.total, rank, world)
        g = builder(args.total, n_space, n_time, seed=0, select=mine)
        B = g.B
    else:
        B = args.batch or DEFAULT_BATCH[args.workload]
        g = builder(B, n_space, n_time, seed=rank)
    t_build = time.perf_counter() - t_build
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    plan = capi.plan(g.n_nodes, is_it, k_cap, n_time=g.n_time, B=g.B)

    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    out = torch.empty_like(V0)
    ws_bytes = max(8, plan["ws_bytes_per_scen"] * g.B)
    ws = torch.empty(ws_bytes // 8, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()
    if is_it:
        F = torch.from_numpy(g.payoff).to(dev)

        def step():
            capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                              V0.data_ptr(), F.data_ptr(), out.data_ptr(), k_cap,
                              ws.data_ptr(), ws_bytes, stream.cuda_stream)
    else:
        MS = torch.from_numpy(g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)).to(dev)
        MR = torch.from_numpy(g.mon_rebate if len(g.mon_rebate) else np.zeros(1)).to(dev)

        def step():
            capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                              V0.data_ptr(), len(g.mon_step), MS.data_ptr(), MR.data_ptr(),
                              out.data_ptr(), k_cap, ws.data_ptr(), ws_bytes,
                              stream.cuda_stream)

    args.warmup = warm_up(step, args, torch.cuda.synchronize)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # HIP events on the launch stream (the kernel runs on torch's current stream)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    # whole-job node-steps: every rank's batch (they differ by one scenario
    # at most under --total), summed over the ranks
    node_steps_launch = g.B * node_units(g) * g.n_time  # configured nodes x steps x solves
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tot = torch.tensor([float(node_steps_launch)], dtype=torch.float64, device=cdev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed = float(t.item())
        job_node_steps = float(tot.item())
    else:
        job_node_steps = float(node_steps_launch)

    res = out.cpu().numpy()
    finite = bool(np.all(np.isfinite(res)))
    total = job_node_steps * args.steps
    value = total / elapsed
    workload = (f"{label}_{n_space}x{n_time}_total{args.total}" if args.total
                else f"{label}_{n_space}x{n_time}_batch{B}")
    fps = FLOPS_PER_NODE_STEP[is_it]
    kernel_s = kernel_ms * 1e-3
    ctr = load_counters(workload)
    recs = roofline_records(fps, node_steps_launch, kernel_s, ctr)

    # the PCIe-inclusive rate of the host-array boundary (fdcn_it_batch /
    # fdcn_cn_batch with NumPy arrays: H2D of the plan, the march, D2H of
    # v_out): reported beside the line, never its value
    pcie = None
    if rank == 0 and world == 1 and args.pcie_launches > 0 and not args.total:
        # the caller's v_out buffer, reused across launches as a caller
        # launching repeatedly would (a fresh 82 MB array per call pays ~20 k
        # first-touch page faults inside the D2H copy)
        v_host = np.empty((g.B, g.n_nodes), dtype=np.float64)
        host_call = ((lambda: capi.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                            g.v_init, g.payoff, out=v_host)) if is_it else
                     (lambda: capi.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams,
                                            g.v_init, g.mon_step, g.mon_rebate, out=v_host)))
        host_call()  # warm (allocations, pinned staging, v_host's pages)
        tp0 = time.perf_counter()
        for _ in range(args.pcie_launches):
            host_call()
        pcie_ms = (time.perf_counter() - tp0) / args.pcie_launches * 1e3
        pcie = {"ms_per_launch": pcie_ms, "node_steps_per_s": node_steps_launch / (pcie_ms * 1e-3),
                "launches": args.pcie_launches,
                "bytes_each_way": {"in": int(g.params.nbytes + g.iparams.nbytes + g.v_init.nbytes +
                                             (g.payoff.nbytes if is_it else 0)),
                                   "out": int(g.v_init.nbytes)},
                "note": "host arrays through the C ABI (fdcn_it_batch / fdcn_cn_batch): H2D, "
                        "march, D2H per launch into one reused v_out buffer; value is the "
                        "HBM-resident rate"}

    # consecutive launches on two streams in turn: a serving loop with two
    # streams, where one launch's drain overlaps the next one's start
    overlapped = None
    if args.overlap_streams and world == 1:
        # two non-default streams: the default stream would serialise with them
        sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
        outs = (torch.empty_like(V0), torch.empty_like(V0))
        wss = (torch.empty_like(ws), torch.empty_like(ws))

        def launch(j):
            if is_it:
                capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(),
                                  I.data_ptr(), V0.data_ptr(), F.data_ptr(), outs[j].data_ptr(),
                                  k_cap, wss[j].data_ptr(), ws_bytes, (sa, sb)[j].cuda_stream)
            else:
                capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(),
                                  I.data_ptr(), V0.data_ptr(), len(g.mon_step), MS.data_ptr(),
                                  MR.data_ptr(), outs[j].data_ptr(), k_cap, wss[j].data_ptr(),
                                  ws_bytes, (sa, sb)[j].cuda_stream)
        for k in range(4):  # the two streams' first launches out of the timed region
            launch(k % 2)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sa)
        sb.wait_event(e0)
        for k in range(args.steps):
            launch(k % 2)
        j = torch.cuda.Event()
        j.record(sb)
        sa.wait_event(j)
        e1.record(sa)
        torch.cuda.synchronize()
        ms2 = e0.elapsed_time(e1) / max(1, args.steps)
        same = all(bool(np.array_equal(o.cpu().numpy().view(np.int64), res.view(np.int64)))
                   for o in outs)
        overlapped = {"ms_per_step": ms2, "node_steps_per_s": node_steps_launch / (ms2 * 1e-3),
                      "frac": fps * node_steps_launch / (ms2 * 1e-3) / 1e12 / FP64_VALU_PEAK_TFLOPS,
                      "steps": args.steps, "outputs_bitwise_equal": same,
                      "note": "the K launches alternate between two streams, each its own "
                              "v_out and workspace, timed from the first launch to the last "
                              "one's end; value is one launch at a time"}

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(g, args.cpu_seconds, res)
    elif world > 1 and not args.no_cpu_baseline:
        # every rank checks a sample of its own timed output against the C
        # oracle on its host cores; the record is the worst over the ranks
        parity = reduce_parity(sample_parity(g, res, PARITY_SAMPLE), world, cdev)

    if rank == 0:
        config = {"workload": workload, "scenarios_per_gpu": g.B, "grid": [n_space, n_time],
                  "parallelism": f"scenario-sharded x{world}"}
        if world > 1:
            config["process_group"] = args.backend
        if args.total:
            config.update(total_scenarios=args.total, shard="contiguous (shard_range)")
        if is_it:
            config.update(option="american put", exercise="ikonen-toivanen", rannacher_steps=2)
        elif args.workload == "barrier":
            config.update(option="discrete barrier (up/down out/in, call/put)",
                          monitoring="daily", rannacher_steps=2, grid_mode="explicit")
        else:
            config.update(option="double knock-out call", monitoring="every step",
                          rannacher_steps=2)
        fv = capi.forced_variant()
        line = {
            "metric": "CN grid-node-steps/sec/GPU (2048x4096 grid); achieved HBM GB/s vs peak",
            "value": value,
            "unit": "node-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.total else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (" + {"american": "strike x vol sweep of the notebook American put",
                                     "barrier": "strike/vol/barrier sweep of the config_scenarios trade",
                                     "double": "vol/barrier sweep of the double _barrier.py trade"}[
                args.workload] + ")",
            "config": config,
            # the binding roof: the march keeps V in VGPRs, so HBM never binds
            # (DESIGN.md §4); fp64 FMA throughput does -- beside it the fp64
            # work actually executed and the measured HBM rate (roofline_records)
            **recs,
            "value_per_gpu": value / world,
            "kernel_ms_per_launch": kernel_ms,
            "pcie_inclusive": pcie,
            "overlapped_streams": overlapped,
            "kernel": {"name": f"fdcn_march<IT={int(is_it)}>", **plan, "k_cap": k_cap,
                       "src_sha": kernel_src_sha(),
                       "forced": list(fv) if fv[0] else None,
                       "lib": capi.LIB_PATH if args.lib else None},
            "outputs_finite": finite,
            # bits of the last launch's v_out: A/B builds of the kernel that
            # must agree bitwise compare this
            "out_sha": hashlib.sha256(np.ascontiguousarray(res).tobytes()).hexdigest()[:16],
            "parity": parity,
            "host_build_s": t_build,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and not (parity["ok"] and parity["all_finite"]):
        print(f"bench.py: PARITY FAILURE {parity}", file=sys.stderr, flush=True)
        return 3
    return 0


def dry_run_rank(args, world: int, rank: int, local: int):
    """The multi-rank plumbing without a GPU: spawn, process group, barrier,
    max-over-ranks timing and a gather of every rank's identity."""
    import torch
    import torch.distributed as dist
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ranks = [{"rank": rank, "local_rank": local, "pid": os.getpid()}]
    if args.total:  # the shard this rank would march (config 4), built
        from finite_difference_amd.distributed import shard_range
        r = shard_range(args.total, rank, world)
        ranks[0]["shard"] = [r.start, r.stop]
        builder, ns0, nt0, _, _ = WORKLOADS[args.workload]
        g = builder(args.total, args.n_space or ns0, args.n_time or nt0, seed=0, select=r)
        ranks[0]["batch"] = int(g.B)
        ranks[0]["params_sha"] = hashlib.sha256(g.params.tobytes()).hexdigest()[:16]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        box = [None] * world if rank == 0 else None
        dist.gather_object(ranks[0], box, dst=0)
        ranks = box
    if rank == 0:
        print(json.dumps({"metric": "dry run (no march)", "value": None, "unit": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed / max(1, args.steps) * 1e3, "dry_run": True,
                          "ranks": ranks}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# single-trade latency through the drop-in facades
# ---------------------------------------------------------------------------
def bench_scenario_file(args):
    """A 10 000-row scenario file priced end to end per step: native plan
    build for every row, one launch of the 2R solves, the device Greeks
    epilogue, the vectorised Black-76 legs and the result columns."""
    import numpy as np
    from finite_difference_amd import capi, distributed, scenario_batch, scenarios
    from finite_difference_amd.engine import Engine
    if distributed.bind_device() is None:
        raise capi.FdcnError("no gfx950 device visible; the benchmark needs an MI355X")
    R = args.batch or 10000
    N, M = args.n_space or 1024, args.n_time or 2000
    rng = np.random.default_rng(20250728)
    kinds = ["up-and-out", "down-and-out", "up-and-in", "down-and-in", "none"]
    S0 = 229.74
    bt = [kinds[i % 5] for i in range(R)]
    cols = {"scenario_name": [f"s{i}" for i in range(R)], "S0": [S0] * R,
            "K": rng.uniform(150, 300, R).tolist(), "sigma": rng.uniform(0.15, 0.45, R).tolist(),
            "rate": [(0.073086, 0.065)[i % 2] for i in range(R)], "barrier_type": bt,
            "upper_barrier": [float(x) if "up" in b else None
                              for b, x in zip(bt, rng.uniform(1.02, 1.5, R) * S0)],
            "lower_barrier": [float(x) if "down" in b else None
                              for b, x in zip(bt, rng.uniform(0.6, 0.98, R) * S0)],
            "FA_price": [1.0] * R, "FA_delta": [0.5] * R, "FA_gamma": [0.01] * R,
            "FA_vega": [0.2] * R}
    # the columns as run_all_scenarios hands them over (DataFrame columns as
    # NumPy arrays; a missing barrier level is NaN, as pandas reads the CSV)
    cols = {k: np.asarray([np.nan if v is None else v for v in c],
                          dtype=object if k in ("scenario_name", "barrier_type") else np.float64)
            for k, c in cols.items()}
    base = scenarios.runner_base_params("put", N)
    base.update(num_time_steps=M, grid_mode="explicit")
    eng = Engine()

    def one(timing):
        res = scenario_batch.price_columns(cols, base, eng, timing=timing)
        return scenario_batch.result_columns(cols, res)
    args.warmup = warm_up(lambda: one({}), args)
    walls, parts = [], {}
    out = None
    for _ in range(args.steps):
        tm = {}
        t0 = time.perf_counter()
        out = one(tm)
        walls.append(time.perf_counter() - t0)
        for k, v in tm.items():
            parts.setdefault(k, []).append(v)
    ms = sum(walls) / len(walls) * 1e3
    avg = {k: sum(v) / len(v) * 1e3 for k, v in parts.items()}
    march_ms = avg["march"]
    n_pde = sum(1 for b in bt if b != "none")
    print(json.dumps({
        "metric": "scenario file wall time (run_all_scenarios pricing)",
        "value": ms, "unit": "ms/file", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "ms_min": min(walls) * 1e3,
        "higher_is_better": False, "scaling": "none", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic scenario file (config_scenarios.csv trade swept over K, sigma, "
                "barriers; two curves)",
        "config": {"workload": f"scenario_file_{R}rows_{N}x{M}", "config": "BASELINE configs[2]",
                   "rows": R, "pde_rows": n_pde, "solves": 2 * n_pde,
                   "plan_chunks": max(1, min(scenario_batch.MAX_CHUNKS,
                                             n_pde // scenario_batch.CHUNK_ROWS))},
        "host_ms": ms - march_ms, "plan_ms": avg["plan"], "march_and_epilogue_ms": march_ms,
        "host_parts_ms": {k: avg[k] for k in ("prep", "plan", "free") if k in avg},
        "outputs_finite": bool(np.all(np.isfinite(out["model_price"])))}), flush=True)


def bench_american_file(args):
    """A 2 000-row American scenario file priced end to end per step
    (price_log2 + greeks_log2 of every row: six unique grids each)."""
    import numpy as np
    from finite_difference_amd import american_batch, capi, distributed
    from finite_difference_amd.engine import Engine
    if distributed.bind_device() is None:
        raise capi.FdcnError("no gfx950 device visible; the benchmark needs an MI355X")
    R = args.batch or 2000
    N, M = args.n_space or 2048, args.n_time or 4096
    rng = np.random.default_rng(20250728)
    cols = {"scenario_name": [f"a{i}" for i in range(R)],
            "S0": (176.39 * rng.uniform(0.9, 1.1, R)).tolist(),
            "K": rng.uniform(150, 200, R).tolist(), "sigma": rng.uniform(0.2, 0.4, R).tolist(),
            "rate": [(0.0705, 0.065)[i % 2] for i in range(R)],
            "FA_price": [5.0] * R, "FA_delta": [-0.4] * R, "FA_gamma": [0.02] * R,
            "FA_vega": [0.2] * R}
    base = dict(valuation=dt.date(2025, 7, 28), maturity=dt.date(2025, 8, 28), opt_type="put",
                num_space_nodes=N, num_time_steps=M)
    eng = Engine()

    def one(timing):
        res = american_batch.price_columns(cols, base, eng, timing=timing)
        return american_batch.result_columns(cols, res)
    args.warmup = warm_up(lambda: one({}), args)
    walls, parts = [], {}
    out = None
    for _ in range(args.steps):
        tm = {}
        t0 = time.perf_counter()
        out = one(tm)
        walls.append(time.perf_counter() - t0)
        for k, v in tm.items():
            parts.setdefault(k, []).append(v)
    ms = sum(walls) / len(walls) * 1e3
    avg = {k: sum(v) / len(v) * 1e3 for k, v in parts.items()}
    march_ms = avg["march"]
    node_steps = R * (5 * N * M + N * 2 * M)  # N, sigma +-h, +-2h at M steps; 2M
    print(json.dumps({
        "metric": "American scenario file wall time (run_all_american_scenarios pricing)",
        "value": ms, "unit": "ms/file", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "ms_min": min(walls) * 1e3,
        "higher_is_better": False, "scaling": "none", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic American put file (notebook trade swept over spot, strike, vol; "
                "two curves)",
        "config": {"workload": f"american_file_{R}rows_{N}x{M}", "config": "BASELINE configs[1]",
                   "rows": R, "grids_per_row": 6,
                   "plan_chunks": max(1, min(american_batch.MAX_CHUNKS,
                                             R // american_batch.CHUNK_ROWS))},
        "host_ms": ms - march_ms, "plan_ms": avg["plan"], "march_and_epilogue_ms": march_ms,
        "host_parts_ms": {k: avg[k] for k in ("prep", "plan", "free") if k in avg},
        "node_steps_per_s": node_steps / (ms * 1e-3),
        "outputs_finite": bool(np.all(np.isfinite(out["model_price"])))}), flush=True)


def bench_trade(args):
    """One trade end to end per step: construct the facade, price (and for
    the American trade the Greeks), read the result -- host plan building,
    H2D, launches, D2H and the epilogue all inside the timed region."""
    from finite_difference_amd import capi, distributed
    if distributed.bind_device() is None:
        raise capi.FdcnError("no gfx950 device visible; the benchmark needs an MI355X")
    if args.force_variant:  # A/B: every launch of the trade on that instance
        capi.force_variant(*[int(x) for x in args.force_variant.split(",")])
    from finite_difference_amd import market
    from finite_difference_amd.american import AmericanFDMPricer, prefetch_many
    from finite_difference_amd.cn_log import DiscreteBarrierCrankNicolsonLog
    from finite_difference_amd.fd_barrier import FDDoubleBarrier

    if args.workload == "trade_cnlog":
        N, M = args.n_space or 512, args.n_time or 1000
        mon = [d / 365 for d in (7, 10, 15, 21, 25, 30, 31)]

        def trade():
            p = DiscreteBarrierCrankNicolsonLog(
                S0=229.74, K=220.0, T=31 / 365, sigma=0.261319016, r_disc=0.070538822,
                b_carry=0.070538822, option_type="call", barrier_type="up-and-out",
                upper_barrier=270.0, rebate=0.0, monitor_times=mon, N_space=N, N_time=M)
            return {"price": p.price()}
        solves, node_steps = 3, 3 * N * M
        cfg = {"workload": f"trade_cnlog_{N}x{M}", "config": "BASELINE configs[0]",
               "facade": "DiscreteBarrierCrankNicolsonLog.price() (base, sigma +- 1e-3)"}
    elif args.workload == "trade_american":
        N, M = args.n_space or 2048, args.n_time or 4096
        val, mat = dt.date(2025, 7, 28), dt.date(2025, 8, 28)
        curve = market.iso_curve(market.create_rate_df(math.exp(0.07053828272) - 1.0))

        def trade():
            p = AmericanFDMPricer(spot=176.39, strike=170.0, valuation_date=val,
                                  maturity_date=mat, sigma=0.296783211249, option_type="put",
                                  discount_curve=curve, forward_curve=curve,
                                  num_space_nodes=N, num_time_steps=M, rannacher_steps=2)
            prefetch_many([p])
            g = p.greeks_log2()
            g["price_log2"] = p.price_log2()
            return g
        grids = {(0, M), (0, 2 * N), (0, 2 * M), (1, M), (-1, M), (2, M), (-2, M)}
        solves = len(grids)
        node_steps = sum(N * nt for _, nt in grids)
        cfg = {"workload": f"trade_american_{N}x{M}", "config": "BASELINE configs[1]",
               "facade": "AmericanFDMPricer price_log2() + greeks_log2() "
                         f"({solves} unique grids, one launch per step count)"}
    else:
        N, M = args.n_space or 4096, args.n_time or 8192

        def trade(window=True):
            d = FDDoubleBarrier(20.786, 21.0, 19.0, 23.0, 0.10994120968, "c", "out",
                                n_space=N, n_time=M, active_window=window)
            return {"price": d.price(0.049493018, 0.0709454892, 49 / 365)}
        solves, node_steps = 1, N * M
        cfg = {"workload": f"trade_double_{N}x{M}", "config": "BASELINE configs[4]",
               "facade": "FDDoubleBarrier.price(b, r, T), knock-out every step; the "
                         "façade marches the knock-out window (ko_window.py), "
                         "full_grid_ms times active_window=False"}
        from finite_difference_amd.ko_window import ko_window
        _sv = FDDoubleBarrier(20.786, 21.0, 19.0, 23.0, 0.10994120968, "c", "out",
                              n_space=N, n_time=M).solve_for(0.049493018, 0.0709454892, 49 / 365)
        _w = ko_window(_sv, _sv.ko_value)
        cfg["window_nodes"] = _w.solve.n_nodes if _w else None
        cfg["grid_nodes"] = _sv.n_nodes
        cfg["configured_node_steps"] = node_steps
        if _w:  # node_steps_per_s counts the nodes the window marches
            node_steps = _w.solve.n_nodes * M

    args.warmup = warm_up(trade, args)
    times = []
    res = None
    for _ in range(args.steps):
        t0 = time.perf_counter()
        res = trade()
        times.append(time.perf_counter() - t0)
    times.sort()
    ms = sum(times) / len(times) * 1e3
    cfg["solves_per_trade"] = solves
    if args.workload == "trade_double":  # the same trade on the whole grid
        full = []
        for _ in range(max(1, args.steps // 2)):
            t0 = time.perf_counter()
            rf = trade(window=False)
            full.append(time.perf_counter() - t0)
        cfg["full_grid_ms"] = sum(full) / len(full) * 1e3
        cfg["full_grid_price"] = rf["price"]
    print(json.dumps({
        "metric": "single-trade latency through the drop-in facade",
        "value": ms, "unit": "ms/trade", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "ms_min": times[0] * 1e3,
        "ms_median": times[len(times) // 2] * 1e3, "higher_is_better": False,
        "scaling": "none", "vs_baseline": None, "dtype": "f64",
        "data": "the reference's own trade parameters", "config": cfg,
        "node_steps_per_s": node_steps / (ms * 1e-3), "result": res}), flush=True)


def build_spot_vc(B: int, n_space: int, n_time: int, seed: int = 0):
    """SURVEY §8(f)3 workload: B DiscreteBarrierFDMPricer2 trades (uniform S
    grid, per-row CN coefficients, FIS barrier rows; discrete_barrier_fdm_
    pricer_2.py:336-428) over a strike / vol / barrier sweep, up / down /
    double knock-out, call and put, daily monitoring over one year.  The
    explicit terms take the corrected sign (the reference's own sign makes
    the march diverge, tests/test_spot_barrier.py).  One march per trade."""
    import numpy as np
    from finite_difference_amd.engine import pack_vc
    from finite_difference_amd.spot_barrier import DiscreteBarrierFDMPricer2
    rng = np.random.default_rng(20250106 + seed)
    v0, v1 = dt.date(2025, 1, 6), dt.date(2026, 1, 6)
    daily = [v0 + dt.timedelta(days=i) for i in range(1, (v1 - v0).days + 1)]
    kinds = ["up-and-out", "down-and-out", "double-out"]
    solves = []
    for i in range(B):
        bt = kinds[i % 3]
        lo = float(rng.uniform(60.0, 92.0)) if bt != "up-and-out" else None
        hi = float(rng.uniform(108.0, 150.0)) if bt != "down-and-out" else None
        p = DiscreteBarrierFDMPricer2(
            spot=100.0, strike=float(rng.uniform(80.0, 120.0)), valuation_date=v0,
            maturity_date=v1, volatility=float(rng.uniform(0.15, 0.45)),
            option_type=("call", "put")[(i // 3) % 2], barrier_type=bt, lower_barrier=lo,
            upper_barrier=hi, monitoring_dates=daily, flat_rate_nacc=0.05,
            num_space_nodes=n_space, num_time_steps=n_time, explicit_sign="corrected")
        solves.extend(p._grid_solves()[2])
    return pack_vc(solves, list(range(len(solves))))


def vc_cpu_baseline(group, seconds: float, res=None):
    """The C oracle's spot-space march (oracle_vc_batch: the reference's
    per-step Thomas, discrete_barrier_fdm_pricer_2.py:336-428) on a bounded
    sample of the same batch, OpenMP over scenarios on the host cores, and
    the parity record of the GPU outputs `res` of those scenarios."""
    import numpy as np
    from oracle import oracle
    nthreads, cores_rec = host_cores()
    done, t_total, m, parts = 0, 0.0, nthreads, []
    while t_total < seconds and done < group.B:
        m = min(m, group.B - done)
        sl = slice(done, done + m)
        t0 = time.perf_counter()
        parts.append(oracle.vc_batch(group.n_nodes, group.n_time, group.n_ranna, group.diag[sl],
                                     group.bnd[sl], group.v_init[sl], group.iparams[sl],
                                     group.mon_step, group.mon_rebate, nthreads))
        t_total += time.perf_counter() - t0
        done += m
        m *= 2
    units = group.n_nodes - 1
    cpu = {"value": done * units * group.n_time / t_total, "unit": "node-steps/s",
           "cores": nthreads, "kind": "port",
           "sample": f"{done} of the {group.B} scenarios, full {units}x{group.n_time} grid, "
                     f"{t_total:.1f} s; C oracle (oracle_vc_batch, per-step Thomas of "
                     f"discrete_barrier_fdm_pricer_2.py:336-428), OpenMP over scenarios on "
                     f"{_cpu_model()}", **cores_rec}
    parity = None
    if res is not None:
        ref = np.concatenate(parts)
        got = np.asarray(res[:done])
        scale = np.maximum(1.0, np.max(np.abs(ref), axis=1))
        rel = np.max(np.abs(got - ref), axis=1) / scale
        rel = np.where(np.isnan(rel), np.inf, rel)
        parity = {"max_rel_err": float(np.max(rel)), "n_compared": int(done),
                  "nodes_per_scenario": int(group.n_nodes), "tol": PARITY_TOL,
                  "ok": bool(np.all(rel <= PARITY_TOL)),
                  "all_finite": bool(np.all(np.isfinite(got))),
                  "rule": "per scenario max_j |V_gpu - V_oracle| / max(1, max_j |V_oracle|), "
                          "every node of the timed launch's output vs the C oracle"}
    return cpu, parity


def bench_spot_vc(args):
    """the spot-space per-row CN march (fdcn_vc_batch_dev) of
    B Pricer2 trades, node-steps/s, with the fp64-VALU roofline, the C
    oracle's CPU rate and the parity record of the timed output."""
    import numpy as np
    import torch
    from finite_difference_amd import capi, distributed
    capi.require_device()
    dev = torch.device("cuda", distributed.bind_device())
    n_space, n_time = args.n_space or 1024, args.n_time or 2000
    B = args.batch or DEFAULT_BATCH["spot_vc"]
    if args.force_variant:  # A/B: W,NPT of fdcn_vc_march pinned
        capi.vc_force_variant(*[int(x) for x in args.force_variant.split(",")[:2]])
    t_build = time.perf_counter()
    g = build_spot_vc(B, n_space, n_time)
    t_build = time.perf_counter() - t_build
    plan = capi.vc_plan(g.n_nodes, B=g.B)
    ws_bytes = max(8, plan["ws_bytes_per_scen"] * g.B)
    D, Bd = torch.from_numpy(g.diag).to(dev), torch.from_numpy(g.bnd).to(dev)
    V0, I = torch.from_numpy(g.v_init).to(dev), torch.from_numpy(g.iparams).to(dev)
    MS = torch.from_numpy(g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)).to(dev)
    MR = torch.from_numpy(g.mon_rebate if len(g.mon_rebate) else np.zeros(1)).to(dev)
    out = torch.empty_like(V0)
    ws = torch.empty(ws_bytes // 8, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        capi.vc_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, D.data_ptr(), Bd.data_ptr(),
                          V0.data_ptr(), I.data_ptr(), len(g.mon_step), MS.data_ptr(),
                          MR.data_ptr(), out.data_ptr(), ws.data_ptr(), ws_bytes,
                          stream.cuda_stream)
    args.warmup = warm_up(step, args, torch.cuda.synchronize)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    res = out.cpu().numpy()
    cpu = parity = None
    if not args.no_cpu_baseline:
        cpu, parity = vc_cpu_baseline(g, args.cpu_seconds, res)
    units = g.n_nodes - 1
    node_steps = g.B * units * g.n_time
    fps = FLOPS_PER_NODE_STEP[False]
    tf = fps * node_steps / (kernel_ms * 1e-3) / 1e12
    slots = 64 * plan["waves"] * plan["npt"]
    # PMC of this workload (profiles/pmc_counters.json), only if measured on
    # the current fdcn_vc.hip
    ctr = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_counters.json")) as f:
            rec = json.load(f).get(f"spot_vc_{n_space}x{n_time}_batch{g.B}")
        if rec and rec.get("kernel_src_sha") == file_sha("fdcn_vc.hip"):
            ctr = rec
    except (OSError, ValueError):
        pass
    print(json.dumps({
        "metric": "spot-space CN grid-node-steps/sec/GPU (DiscreteBarrierFDMPricer2 march)",
        "value": node_steps * args.steps / elapsed, "unit": "node-steps/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (strike/vol/barrier sweep of Pricer2 knock-outs, daily monitoring)",
        "config": {"workload": f"spot_vc_{n_space}x{n_time}_batch{g.B}", "scenarios": g.B,
                   "grid": [n_space, n_time], "n_nodes": g.n_nodes, "rannacher_steps": 2,
                   "explicit_sign": "corrected"},
        "roofline": {"bound": "fp64_valu", "achieved": tf, "peak": FP64_VALU_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": tf / FP64_VALU_PEAK_TFLOPS,
                     "traffic": (ctr["march"]["hbm_bytes_per_launch"]
                                 + ctr["factor"]["hbm_bytes_per_launch"]) if ctr else None,
                     "flops_per_node_step": fps},
        "valu_issue": ({"march_valu_insts_per_lane_node_step":
                        ctr["march"]["valu_insts_per_lane_node_step"],
                        "march_issue_frac": ctr["march"]["valu_issue_utilisation"],
                        "note": "profiles/pmc_counters.json, measured on this fdcn_vc.hip"}
                       if ctr else None),
        # measured HBM bytes of both kernels per launch / launch time (PMC)
        "hbm": ({"achieved": (ctr["march"]["hbm_bytes_per_launch"]
                              + ctr["factor"]["hbm_bytes_per_launch"]) / (kernel_ms * 1e-3) / 1e9,
                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": (ctr["march"]["hbm_bytes_per_launch"]
                          + ctr["factor"]["hbm_bytes_per_launch"]) / (kernel_ms * 1e-3) / 1e9
                         / HBM_PEAK_GBS,
                 "note": "PMC FETCH_SIZE x 2 + WRITE_SIZE of the march and factor kernels"}
                if ctr else None),
        "kernel_ms_per_launch": kernel_ms,
        "kernel": {"name": f"fdcn_vc_march<{plan['waves']},{plan['npt']}>", **plan,
                   "slots": slots, "slot_use": g.n_nodes / slots},
        "outputs_finite": bool(np.all(np.isfinite(res))), "parity": parity,
        "out_sha": hashlib.sha256(np.ascontiguousarray(res).tobytes()).hexdigest()[:16],
        "host_build_s": t_build, "cpu_baseline": cpu}), flush=True)
    if parity is not None and not (parity["ok"] and parity["all_finite"]):
        print(f"bench.py: PARITY FAILURE {parity}", file=sys.stderr, flush=True)
        return 3
    return 0


def bench_analytic(args):
    """Closed-form barrier batch (fdcn_rr_barrier_batch_dev): contracts/s."""
    import numpy as np
    import torch
    from finite_difference_amd import capi, distributed
    from finite_difference_amd.analytic import BarrierEngine
    capi.require_device()
    dev = torch.device("cuda", distributed.bind_device())
    B = args.batch or DEFAULT_BATCH["analytic"]
    rng = np.random.default_rng(20250728)
    s = rng.uniform(50, 150, B)
    up = rng.integers(0, 2, B).astype(bool)
    P = np.stack([s, rng.uniform(-0.02, 0.08, B), rng.uniform(0.0, 0.1, B),
                  rng.uniform(0.05, 2.0, B), s * rng.uniform(0.7, 1.3, B),
                  rng.uniform(0.1, 0.6, B),
                  s * np.where(up, rng.uniform(1.02, 1.4, B), rng.uniform(0.6, 0.98, B)),
                  rng.uniform(0.0, 3.0, B)], axis=1)
    F = np.zeros((B, capi.RR_NFLAG), dtype=np.int32)
    F[:, 0] = np.arange(B) % 2
    F[:, 1] = np.where(up, 0, 1)
    F[:, 2] = (np.arange(B) // 2) % 2
    dP = torch.from_numpy(P).to(dev)
    dF = torch.from_numpy(F).to(dev)
    price = torch.empty(B, dtype=torch.float64, device=dev)
    van = torch.empty(B, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        capi._check(capi.lib().fdcn_rr_barrier_batch_dev(B, dP.data_ptr(), dF.data_ptr(),
                                                         price.data_ptr(), van.data_ptr(),
                                                         stream.cuda_stream))
    args.warmup = warm_up(step, args, torch.cuda.synchronize)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / max(1, args.steps)
    got = price.cpu().numpy()
    cpu = None
    if not args.no_cpu_baseline:  # the host engine (Python/NumPy/SciPy), one core
        n, t_cpu = 0, 0.0
        names = ("s", "b", "r", "t", "x", "sigma", "h", "k")
        while t_cpu < min(args.cpu_seconds, 5.0) and n < B:
            c = dict(zip(names, map(float, P[n])))
            c.update(optionflag="cp"[F[n, 0]], directionflag="ud"[F[n, 1]],
                     in_out_flag="io"[F[n, 2]])
            t1 = time.perf_counter()
            ref = BarrierEngine(**c).price()
            t_cpu += time.perf_counter() - t1
            assert abs(ref - got[n]) <= 1e-11 * abs(ref) + 1e-12, (n, ref, got[n])
            n += 1
        cpu = {"value": n / t_cpu, "unit": "contracts/s", "cores": 1, "kind": "port",
               "sample": f"first {n} contracts through analytic.BarrierEngine (host, "
                         f"NumPy/SciPy, the reference's formulas), each checked against "
                         f"the GPU result"}
    bytes_per = 8 * capi.RR_NPARAM + 4 * capi.RR_NFLAG + 16
    gbs = bytes_per * B / (kernel_ms * 1e-3) / 1e9
    print(json.dumps({
        "metric": "closed-form barrier contracts/s (Reiner-Rubinstein, barrier_engine.py)",
        "value": B * args.steps / elapsed, "unit": "contracts/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (uniform spot/strike/barrier/vol/rate/tenor sweep)",
        "config": {"workload": f"rr_barrier_batch{B}", "contracts": B},
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "traffic": None},
        "kernel_ms_per_launch": kernel_ms, "outputs_finite": bool(np.all(np.isfinite(got))),
        "cpu_baseline": cpu}), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.lib:
        from finite_difference_amd import capi
        capi.LIB_PATH = os.path.abspath(args.lib)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.workload in TRADE_WORKLOADS or args.workload in ("analytic", "spot_vc"):
            raise SystemExit(f"--workload {args.workload} is a single-GPU measurement")
        return spawn_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
              file=sys.stderr)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main() or 0)
