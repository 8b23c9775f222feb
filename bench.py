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
           the barriers (B=1 is the single-solve latency case).
  analytic SURVEY §8(f) row 4, not a BASELINE config: 2^20 Reiner-Rubinstein
           barrier contracts (barrier_engine.py) per launch, one GPU thread
           each; its own metric line (contracts/s).

value = total node-steps (configured nodes x steps x B x ranks) / max-over-
ranks wall time of the K timed launches.

Multi-GPU: one process per GPU (torch.distributed.run); each rank marches its
own B scenarios (weak scaling, no collective in the data path).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
                       [--workload american|barrier|double]
"""
from __future__ import annotations

import argparse
import datetime as dt
import json
import math
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X spec sheet, FP64 vector
# algorithmic bytes / flops per node-step
BYTES_PER_NODE_STEP = {True: 32, False: 16}   # IT: V and lambda in+out; CN: V in+out
FLOPS_PER_NODE_STEP = {True: 17, False: 10}   # RHS 5 (+2 lambda) + Thomas 5 (+ IT 5)
DEFAULT_BATCH = {"american": 4096, "barrier": 10000, "double": 2048, "analytic": 1 << 20}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(DEFAULT_BATCH), default="american")
    ap.add_argument("--batch", type=int, default=0, help="scenarios per GPU (0: workload default)")
    ap.add_argument("--n-space", type=int, default=0, help="0: workload default")
    ap.add_argument("--n-time", type=int, default=0, help="0: workload default")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def build_american(B: int, n_space: int, n_time: int, seed: int):
    """B American puts of the notebook trade over a strike x vol sweep."""
    from finite_difference_amd import market
    from finite_difference_amd.american import AmericanFDMPricer
    from finite_difference_amd.engine import pack
    val, mat = dt.date(2025, 7, 28), dt.date(2025, 8, 28)
    curve = market.iso_curve(market.create_rate_df(math.exp(0.07053828272) - 1.0))
    solves = []
    p = None  # one pricer, re-pointed per scenario (same dates and curve)
    for i in range(B):
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
    return pack(solves, list(range(B)))


def build_barrier(B: int, n_space: int, n_time: int, seed: int):
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
    for i in range(B):
        bt = kinds[i % 4]
        K, sig = float(rng.uniform(150, 300)), float(rng.uniform(0.15, 0.45))
        up = float(rng.uniform(1.02, 1.5) * S0) if "up" in bt else None
        lo = float(rng.uniform(0.6, 0.98) * S0) if "down" in bt else None
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
    grp = pack(solves, list(range(B)))
    grp.top_dropped = True  # n_nodes = N_s configured nodes (…pricer.py:449, :543)
    return grp


def build_double(B: int, n_space: int, n_time: int, seed: int):
    """BASELINE config 5: double knock-out call of double _barrier.py:139-146,
    knock-out projected every step; B > 1 sweeps sigma and the barriers."""
    from finite_difference_amd.engine import pack
    from finite_difference_amd.fd_barrier import FDDoubleBarrier
    b, r, T = 0.049493018, 0.0709454892, 49 / 365
    solves = []
    for i in range(B):
        j = (i * 2654435761 + seed * 97) % max(B, 1)
        f = j / max(B - 1, 1)
        sig = 0.10994120968 * (0.8 + 0.4 * f) if B > 1 else 0.10994120968
        lo = 19.0 - (0.5 * f if B > 1 else 0.0)
        hi = 23.0 + (0.5 * f if B > 1 else 0.0)
        d = FDDoubleBarrier(20.786, 21.0, lo, hi, sig, "c", "out", n_space=n_space,
                            n_time=n_time)
        solves.append(d.solve_for(b, r, T))
    return pack(solves, list(range(B)))


WORKLOADS = {  # name -> (builder, n_space, n_time, IT?, config label)
    "american": (build_american, 2048, 4096, True, "american_it_put"),
    "barrier": (build_barrier, 1024, 2000, False, "discrete_barrier_ko"),
    "double": (build_double, 4096, 8192, False, "double_barrier_ko"),
}


def cpu_baseline(group, seconds: float):
    """C oracle (sequential Thomas + IT per scenario, OpenMP over scenarios)
    timed on a bounded prefix of the same batch."""
    from oracle import oracle
    nthreads = oracle.max_threads()
    nthreads = min(nthreads, int(os.environ.get("OMP_NUM_THREADS", nthreads)))
    done, t_total, m = 0, 0.0, nthreads
    while t_total < seconds and done < group.B:
        m = min(m, group.B - done)
        sl = slice(done, done + m)
        t0 = time.perf_counter()
        if group.it:
            oracle.it_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                            group.iparams[sl], group.v_init[sl], group.payoff[sl], nthreads)
        else:
            # monitor runs are addressed by MON_START/MON_COUNT: pass the full arrays
            oracle.cn_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                            group.iparams[sl], group.v_init[sl], group.mon_step,
                            group.mon_rebate, nthreads)
        t_total += time.perf_counter() - t0
        done += m
        m *= 2
    units = done * node_units(group) * group.n_time
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), "")
    except Exception:
        pass
    return {"value": units / t_total, "unit": "node-steps/s", "cores": nthreads,
            "kind": "port",
            "sample": f"{done} of the {group.B} scenarios, full {node_units(group)}x"
                      f"{group.n_time} grid, C oracle ("
                      + ("Thomas + IT as fd_american_equity.py:559-726" if group.it else
                         "Thomas + KO as discrete_barrier_fdm_pricer.py:442-547")
                      + f"), {nthreads} OpenMP threads, {t_total:.1f} s on "
                      f"{model or platform.processor()}"}


def node_units(group) -> int:
    """Configured asset nodes of one solve: N_s for the
    top-node-dropping barrier march (n_nodes = N_s), n_nodes - 1 otherwise."""
    return group.n_nodes if getattr(group, "top_dropped", False) else group.n_nodes - 1


def load_traffic(workload: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        rec = d.get(workload)
        return None if rec is None else rec.get("hbm_bytes_per_launch")
    except Exception:
        return None


def bench_analytic(args):
    """Closed-form barrier batch (fdcn_rr_barrier_batch_dev): contracts/s."""
    import numpy as np
    import torch
    from finite_difference_amd import capi
    from finite_difference_amd.analytic import BarrierEngine, _rr_encode
    capi.require_device()
    dev = torch.device("cuda", 0)
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
    for _ in range(args.warmup):
        step()
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


def main():
    args = parse()
    if args.workload == "analytic":
        return bench_analytic(args)
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from finite_difference_amd import capi
    capi.require_device()
    builder, ns0, nt0, is_it, label = WORKLOADS[args.workload]
    B = args.batch or DEFAULT_BATCH[args.workload]
    n_space, n_time = args.n_space or ns0, args.n_time or nt0
    t_build = time.perf_counter()
    g = builder(B, n_space, n_time, seed=rank)
    t_build = time.perf_counter() - t_build
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    plan = capi.plan(g.n_nodes, is_it, k_cap, n_time=g.n_time, B=g.B)

    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    out = torch.empty_like(V0)
    ws = torch.empty(max(1, plan["ws_bytes_per_scen"] * g.B // 8), dtype=torch.float64,
                     device=dev)
    stream = torch.cuda.current_stream()
    if is_it:
        F = torch.from_numpy(g.payoff).to(dev)

        def step():
            capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                              V0.data_ptr(), F.data_ptr(), out.data_ptr(), k_cap,
                              ws.data_ptr(), stream.cuda_stream)
    else:
        MS = torch.from_numpy(g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)).to(dev)
        MR = torch.from_numpy(g.mon_rebate if len(g.mon_rebate) else np.zeros(1)).to(dev)

        def step():
            capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                              V0.data_ptr(), len(g.mon_step), MS.data_ptr(), MR.data_ptr(),
                              out.data_ptr(), k_cap, ws.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
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
    kernel_ms = ev0.elapsed_time(ev1) / max(1, args.steps)  # HIP events, kernel stream
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    res = out.cpu().numpy()
    finite = bool(np.all(np.isfinite(res)))
    node_steps_launch = g.B * node_units(g) * g.n_time  # configured nodes x steps x solves
    total = node_steps_launch * args.steps * world
    value = total / elapsed
    workload = f"{label}_{n_space}x{n_time}_batch{B}"
    bps, fps = BYTES_PER_NODE_STEP[is_it], FLOPS_PER_NODE_STEP[is_it]
    achieved_gbs = bps * node_steps_launch / (kernel_ms * 1e-3) / 1e9
    achieved_tf = fps * node_steps_launch / (kernel_ms * 1e-3) / 1e12

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(g, args.cpu_seconds)

    if rank == 0:
        config = {"workload": workload, "scenarios_per_gpu": g.B, "grid": [n_space, n_time],
                  "parallelism": f"scenario-sharded x{world}"}
        if is_it:
            config.update(option="american put", exercise="ikonen-toivanen", rannacher_steps=2)
        elif args.workload == "barrier":
            config.update(option="discrete barrier (up/down out/in, call/put)",
                          monitoring="daily", rannacher_steps=2, grid_mode="explicit")
        else:
            config.update(option="double knock-out call", monitoring="every step",
                          rannacher_steps=2)
        line = {
            "metric": "CN grid-node-steps/sec/GPU (2048x4096 grid); achieved HBM GB/s vs peak",
            "value": value,
            "unit": "node-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (" + {"american": "strike x vol sweep of the notebook American put",
                                     "barrier": "strike/vol/barrier sweep of the config_scenarios trade",
                                     "double": "vol/barrier sweep of the double _barrier.py trade"}[
                args.workload] + ")",
            "config": config,
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": load_traffic(workload)},
            "roofline_fp64_valu": {"achieved": achieved_tf, "peak": FP64_VALU_PEAK_TFLOPS,
                                   "unit": "TFLOP/s", "frac": achieved_tf / FP64_VALU_PEAK_TFLOPS,
                                   "flops_per_node_step": fps},
            "roofline_note": ("algorithmic bytes per node-step (SURVEY 8d) over the HBM peak; the "
                              "march keeps V in VGPRs, so HBM moves only `traffic` bytes per "
                              "launch and the binding roof is fp64 VALU issue (DESIGN.md 4)"),
            "kernel_ms_per_launch": kernel_ms,
            "kernel": {"name": f"fdcn_march<IT={int(is_it)}>", **plan, "k_cap": k_cap},
            "outputs_finite": finite,
            "host_build_s": t_build,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
