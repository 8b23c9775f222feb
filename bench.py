#!/usr/bin/env python3
"""Benchmark: CN grid-node-steps/sec on the 2048 x 4096 American grid.

Workload (BASELINE.json configs[1]): American put, fd_american_equity.py,
num_space_nodes=2048, num_time_steps=4096, Rannacher 2, Ikonen-Toivanen early
exercise, the notebook trade (S0=176.39, 2025-07-28 -> 2025-08-28, flat NACA
e^0.07053828272-1).  A "step" is one pass of the hot path over one batch: one
launch of the batched IT march over B independent scenarios of that trade
swept over strike and volatility (the scenario-batch axis of the north star).
Inputs are built by the product's AmericanFDMPricer façade and are resident
in HBM before the timed region.

value = total node-steps (2048 configured nodes x 4096 steps x B x ranks)
        / max-over-ranks wall time of the K timed launches.

Multi-GPU: one process per GPU (torch.distributed.run); each rank marches its
own B scenarios (weak scaling, no collective in the data path).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
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
BYTES_PER_NODE_STEP_IT = 32   # V and lambda in+out, fp64
FLOPS_PER_NODE_STEP_IT = 17   # RHS 5 + lambda term 2 + fwd 3 + bwd 2 + IT 5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="scenarios per GPU")
    ap.add_argument("--n-space", type=int, default=2048)
    ap.add_argument("--n-time", type=int, default=4096)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def build_workload(B: int, n_space: int, n_time: int, seed: int):
    """B American puts of the notebook trade over a strike x vol sweep."""
    from finite_difference_amd import market
    from finite_difference_amd.american import AmericanFDMPricer
    from finite_difference_amd.engine import pack
    val, mat = dt.date(2025, 7, 28), dt.date(2025, 8, 28)
    curve = market.iso_curve(market.create_rate_df(math.exp(0.07053828272) - 1.0))
    solves = []
    for i in range(B):
        j = (i * 2654435761 + seed * 97) % B  # deterministic shuffle
        strike = 140.0 + 70.0 * (j % 64) / 63.0
        sigma = 0.18 + 0.30 * ((j // 64) % 64) / 63.0
        p = AmericanFDMPricer(spot=176.39, strike=strike, valuation_date=val, maturity_date=mat,
                              sigma=sigma, option_type="put", discount_curve=curve,
                              forward_curve=curve, num_space_nodes=n_space,
                              num_time_steps=n_time, rannacher_steps=2)
        p._build_log_grid()
        solves.append(p._segment_solve(p._payoff_array(), 0.0, p.time_to_expiry, n_time, True))
    return pack(solves, list(range(B)))


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
        oracle.it_batch(group.n_nodes, group.n_time, group.n_ranna, group.params[sl],
                        group.iparams[sl], group.v_init[sl], group.payoff[sl], nthreads)
        t_total += time.perf_counter() - t0
        done += m
        m *= 2
    units = done * (group.n_nodes - 1) * group.n_time
    model = ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        model = next((l.split(":", 1)[1].strip() for l in out.splitlines()
                      if l.startswith("Model name")), "")
    except Exception:
        pass
    return {"value": units / t_total, "unit": "node-steps/s", "cores": nthreads,
            "kind": "port",
            "sample": f"{done} of the {group.B} scenarios, full {group.n_nodes - 1}x"
                      f"{group.n_time} grid, C oracle (Thomas + IT as fd_american_equity.py:"
                      f"559-726), {nthreads} OpenMP threads, {t_total:.1f} s on "
                      f"{model or platform.processor()}"}


def load_traffic(workload: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        rec = d.get(workload)
        return None if rec is None else rec.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    args = parse()
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
    t_build = time.perf_counter()
    g = build_workload(args.batch, args.n_space, args.n_time, seed=rank)
    t_build = time.perf_counter() - t_build
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    plan = capi.plan(g.n_nodes, True, k_cap, n_time=g.n_time)

    P = torch.from_numpy(g.params).to(dev)
    I = torch.from_numpy(g.iparams).to(dev)
    V0 = torch.from_numpy(g.v_init).to(dev)
    F = torch.from_numpy(g.payoff).to(dev)
    out = torch.empty_like(V0)
    ws = torch.empty(max(1, plan["ws_bytes_per_scen"] * g.B // 8), dtype=torch.float64,
                     device=dev)
    stream = torch.cuda.current_stream()

    def step():
        capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, P.data_ptr(), I.data_ptr(),
                          V0.data_ptr(), F.data_ptr(), out.data_ptr(), k_cap,
                          ws.data_ptr(),
                          stream.cuda_stream)

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
    node_steps_launch = g.B * (g.n_nodes - 1) * g.n_time  # configured nodes x steps x solves
    total = node_steps_launch * args.steps * world
    value = total / elapsed
    workload = f"american_it_put_{args.n_space}x{args.n_time}_batch{args.batch}"
    achieved_gbs = BYTES_PER_NODE_STEP_IT * node_steps_launch / (kernel_ms * 1e-3) / 1e9
    achieved_tf = FLOPS_PER_NODE_STEP_IT * node_steps_launch / (kernel_ms * 1e-3) / 1e12

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(g, args.cpu_seconds)

    if rank == 0:
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
            "data": "synthetic (strike x vol sweep of the notebook American put)",
            "config": {"workload": workload, "scenarios_per_gpu": g.B,
                       "grid": [args.n_space, args.n_time], "option": "american put",
                       "exercise": "ikonen-toivanen", "rannacher_steps": 2,
                       "parallelism": f"scenario-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": load_traffic(workload)},
            "roofline_fp64_valu": {"achieved": achieved_tf, "peak": FP64_VALU_PEAK_TFLOPS,
                                   "unit": "TFLOP/s", "frac": achieved_tf / FP64_VALU_PEAK_TFLOPS,
                                   "flops_per_node_step": FLOPS_PER_NODE_STEP_IT},
            "kernel_ms_per_launch": kernel_ms,
            "kernel": {"name": "fdcn_march<IT=1>", **plan, "k_cap": k_cap},
            "outputs_finite": finite,
            "host_build_s": t_build,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
