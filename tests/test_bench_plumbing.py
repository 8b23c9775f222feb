"""bench.py's multi-GPU plumbing on CPU (gloo, 2 ranks, 127.0.0.1).

`--dry-run` runs everything but the march: the rank processes, the process
group, the timing barrier, the max over ranks and a gather of every rank's
identity.  Covered both ways the driver may launch it: `bench.py --gpus 2`
(bench spawns the ranks itself) and torch.distributed.run (one process per
rank, WORLD_SIZE set by the launcher)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


def _check(line: dict, world: int) -> None:
    assert line["dry_run"] is True and line["n_gpus"] == world
    ranks = line["ranks"]
    assert [r["rank"] for r in ranks] == list(range(world))
    assert [r["local_rank"] for r in ranks] == list(range(world))
    assert len({r["pid"] for r in ranks}) == world  # one process per rank


def test_bench_spawns_ranks_itself():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_last_json(p.stdout), 2)


def test_bench_under_torch_distributed_run():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), "bench.py", "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_last_json(p.stdout), 2)


def test_trade_workloads_refuse_multi_gpu():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--workload", "trade_cnlog"],
                       cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "single-GPU" in p.stderr


def test_bench_total_shards_one_batch():
    """--total (config 4, strong scaling): the ranks split ONE batch into
    contiguous shards that cover it exactly once."""
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dry-run", "--steps", "1",
                        "--warmup", "0", "--workload", "barrier", "--total", "10001"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _last_json(p.stdout)
    _check(line, 2)
    assert [r["shard"] for r in line["ranks"]] == [[0, 5001], [5001, 10001]]


def test_barrier_builder_shard_equals_slice_of_full_batch():
    """A rank's shard of the config-4 batch is bit-identical to the same rows
    of the whole batch built in one process (the draws are not per rank)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    full = bench.build_barrier(40, 64, 30, seed=0)
    part = bench.build_barrier(40, 64, 30, seed=0, select=range(13, 27))
    assert np.array_equal(part.params, full.params[13:27])
    assert np.array_equal(part.v_init, full.v_init[13:27])
    ip = full.iparams[13:27].copy()
    ip[:, 4] -= ip[0, 4]  # monitor runs are re-based in the shard
    assert np.array_equal(part.iparams, ip)


def test_cpu_cores_record():
    sys.path.insert(0, ROOT)
    import bench
    n, rec = bench.host_cores()
    assert 1 <= n <= rec["affinity_cpus"]
    if rec["cgroup_cpu_quota"]:
        assert n <= rec["cgroup_cpu_quota"]


def test_parity_record_flags_a_wrong_launch():
    """cpu_baseline's parity record on CPU: the oracle's own outputs pass, a
    result off by 1e-8 of the scale in one node of one scenario fails, and a
    NaN is reported as not finite (bench.py exits 3 on either)."""
    import numpy as np
    import bench
    from oracle import oracle
    g = bench.build_barrier(6, 64, 40, seed=0)
    ref = oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                          g.mon_step, g.mon_rebate, 1)
    _, par = bench.cpu_baseline(g, 0.01, ref.copy())
    assert par["ok"] and par["all_finite"] and par["max_rel_err"] == 0.0
    n = par["n_compared"]
    bad = ref.copy()
    bad[n - 1, g.n_nodes // 2] += 1e-8 * max(1.0, float(np.max(np.abs(ref[n - 1]))))
    _, par = bench.cpu_baseline(g, 0.01, bad)
    assert not par["ok"] and par["max_rel_err"] > bench.PARITY_TOL
    nan = ref.copy()
    nan[0, 3] = np.nan
    _, par = bench.cpu_baseline(g, 0.01, nan)
    assert not par["all_finite"]


def test_sample_parity_record_of_a_rank():
    """sample_parity (the per-rank record of multi-GPU bench runs): the
    oracle's own outputs pass, one node off by 1e-8 of the scale fails, and a
    NaN turns into an infinite error (so it survives the MAX over ranks) and
    a non-finite flag; both the American and the barrier groups."""
    import numpy as np
    import bench
    from oracle import oracle
    for g in (bench.build_barrier(5, 64, 40, seed=1), bench.build_american(5, 64, 40, seed=1)):
        k = 3
        if g.it:
            ref = oracle.it_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                                  g.payoff, 1)
        else:
            ref = oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                                  g.mon_step, g.mon_rebate, 1)
        par = bench.sample_parity(g, ref.copy(), k)
        assert par["ok"] and par["all_finite"] and par["max_rel_err"] == 0.0
        assert par["n_compared"] == k
        bad = ref.copy()
        bad[k - 1, g.n_nodes // 2] += 1e-8 * max(1.0, float(np.max(np.abs(ref[k - 1]))))
        par = bench.sample_parity(g, bad, k)
        assert not par["ok"] and par["max_rel_err"] > bench.PARITY_TOL
        bad[k, 0] = np.nan  # outside the sample: not seen
        assert not bench.sample_parity(g, bad, k)["ok"]
        nan = ref.copy()
        nan[1, 3] = np.nan
        par = bench.sample_parity(g, nan, k)
        assert not par["all_finite"] and par["max_rel_err"] == float("inf") and not par["ok"]
        assert bench.sample_parity(g, ref, 99)["n_compared"] == g.B


def _parity_rank(rank, world, port, out_path):
    """One gloo rank of test_reduce_parity_over_two_ranks: rank 1's sample
    carries a wrong node (the barrier group of bench.py, seed = rank)."""
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    import bench
    from oracle import oracle
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        g = bench.build_barrier(4, 64, 40, seed=rank)
        res = oracle.cn_batch(g.n_nodes, g.n_time, g.n_ranna, g.params, g.iparams, g.v_init,
                              g.mon_step, g.mon_rebate, 1)
        good = bench.reduce_parity(bench.sample_parity(g, res, 2), world, "cpu")
        if rank == 1:
            res[1, 7] += 1e-6 * max(1.0, abs(res[1]).max())
        bad = bench.reduce_parity(bench.sample_parity(g, res, 2), world, "cpu")
        with open(f"{out_path}.{rank}", "w") as f:
            json.dump([good, bad], f)
    finally:
        dist.destroy_process_group()


def test_reduce_parity_over_two_ranks(tmp_path):
    """The multi-GPU bench's parity record (reduce_parity over gloo): the
    worst error over the ranks and the compared scenarios summed, the same on
    every rank, so a wrong node on rank 1 fails rank 0's line too."""
    import torch.multiprocessing as mp
    import bench
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "par")
    mp.start_processes(_parity_rank, args=(2, port, out), nprocs=2, join=True,
                       start_method="spawn")
    recs = [json.load(open(f"{out}.{r}")) for r in range(2)]
    for good, bad in recs:
        assert good["ok"] and good["max_rel_err"] == 0.0 and good["n_compared"] == 4
        assert not bad["ok"] and bad["max_rel_err"] > bench.PARITY_TOL and bad["n_compared"] == 4
        assert "worst over the 2 ranks" in bad["rule"]
    assert recs[0][1] == recs[1][1]


def test_spot_vc_workload_and_parity_record():
    """bench.py --workload spot_vc on CPU: the Pricer2 batch packs one march
    per trade with its knock-out lanes and daily monitoring, the device plan
    accepts it, and vc_cpu_baseline's parity record passes the oracle's own
    outputs and fails a wrong node."""
    import numpy as np
    import bench
    from finite_difference_amd import capi
    from oracle import oracle
    g = bench.build_spot_vc(6, 64, 40)  # Pricer2 takes N = max(200, num_space_nodes)
    assert g.B == 6 and g.n_nodes == 201 and g.n_time == 40 and g.n_ranna == 2
    assert g.diag.shape == (6, 2, 6, 201)
    assert len(g.mon_step) > 0 and np.all(g.iparams[:, capi.I_MON_COUNT] > 0)
    assert capi.vc_plan(g.n_nodes, B=g.B)["waves"] >= 1
    ref = oracle.vc_batch(g.n_nodes, g.n_time, g.n_ranna, g.diag, g.bnd, g.v_init, g.iparams,
                          g.mon_step, g.mon_rebate, 1)
    assert np.all(np.isfinite(ref))
    cpu, par = bench.vc_cpu_baseline(g, 0.01, ref.copy())
    assert par["ok"] and par["max_rel_err"] == 0.0 and cpu["value"] > 0
    bad = ref.copy()
    bad[0, 30] += 1e-6 * max(1.0, np.abs(ref[0]).max())
    _, par = bench.vc_cpu_baseline(g, 0.01, bad)
    assert not par["ok"]


def test_warm_up_runs_exactly_w_or_about_a_second(monkeypatch):
    """bench.warm_up: an explicit --warmup W runs exactly W steps (the
    contract); without it at least two, then more until WARM_SECONDS of wall
    time have passed (the clock ramp), syncing every four."""
    import argparse
    import time
    sys.path.insert(0, ROOT)
    import bench
    calls, syncs = [], []

    def step():
        calls.append(1)
        time.sleep(0.002)
    assert bench.warm_up(step, argparse.Namespace(warmup=3), lambda: syncs.append(1)) == 3
    assert len(calls) == 3 and not syncs
    calls.clear()
    assert bench.warm_up(step, argparse.Namespace(warmup=0)) == 0 and not calls
    monkeypatch.setattr(bench, "WARM_SECONDS", 0.05)
    t0 = time.perf_counter()
    n = bench.warm_up(step, argparse.Namespace(warmup=None), lambda: syncs.append(1))
    assert n == len(calls) and n >= 2 and time.perf_counter() - t0 >= 0.05
    assert len(syncs) == n // 4 + 1  # every fourth step, and once at the end
    calls.clear()
    monkeypatch.setattr(bench, "WARM_SECONDS", 0.0)
    assert bench.warm_up(step, argparse.Namespace(warmup=None)) == 2  # the floor


def _peaked(rec):
    """Every {achieved, peak} record nested in a bench line."""
    if isinstance(rec, dict):
        if "achieved" in rec and "peak" in rec:
            yield rec
        for v in rec.values():
            yield from _peaked(v)


def test_no_line_field_exceeds_its_peak():
    """the march line's measurement records, built from the
    committed PMC records and the round-5 kernel times of the three
    throughput configs, stay physically consistent -- every achieved figure
    at or below its stated peak, and the measured HBM rate is traffic / time,
    not the algorithmic-bytes rate (12.8x the HBM peak) it replaced."""
    sys.path.insert(0, ROOT)
    import bench
    with open(os.path.join(ROOT, "profiles", "pmc_counters.json")) as f:
        pmc = json.load(f)
    # (pmc key, is_it, node-steps per launch, round-5 kernel ms)
    cases = [("american_it_put_2048x4096_batch4096", True, 4096 * 2048 * 4096, 10.71),
             ("discrete_barrier_ko_1024x2000_batch10000", False, 10000 * 1024 * 2000, 4.13),
             ("double_barrier_ko_4096x8192_batch2048", False, 2048 * 4096 * 8192, 15.18)]
    for key, is_it, ns, ms in cases:
        ctr = pmc[key]
        recs = bench.roofline_records(bench.FLOPS_PER_NODE_STEP[is_it], ns, ms * 1e-3, ctr)
        assert recs["hbm"] and recs["fp64_executed"] and recs["valu_issue"], key
        found = list(_peaked(recs))
        assert len(found) == 3, found  # roofline, fp64_executed, hbm
        for r in found:
            assert 0.0 < r["achieved"] <= r["peak"], (key, r)
            assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-12
        assert recs["valu_issue"]["issue_frac"] <= 1.0
        hbm = recs["hbm"]
        assert abs(hbm["achieved"] - ctr["hbm_bytes_per_launch"] / (ms * 1e-3) / 1e9) < 1e-9
        assert "roofline_hbm_effective" not in recs
    # the config-2 figures VERDICT r5 recomputed: ~69 GB/s and 14.7 executed flops
    am = bench.roofline_records(17, 4096 * 2048 * 4096, 10.71e-3,
                                pmc["american_it_put_2048x4096_batch4096"])
    assert 60 < am["hbm"]["achieved"] < 80
    assert 14.0 < am["fp64_executed"]["flops_per_node_step"] < 15.5
    # stale counters (another kernel source): the PMC records are null
    none = bench.roofline_records(10, 1e12, 1e-3, None)
    assert none["hbm"] is None and none["fp64_executed"] is None and none["valu_issue"] is None
    assert none["roofline"]["traffic"] is None


# ---------------------------------------------------------------------------
# World size 8: the shapes the driver's SCALE run uses on an 8-GPU node
# (VERDICT r5 item 5), rehearsed over gloo on CPU.  The serial loop this
# replaces is run_config_scenarios.py:137-195.
# ---------------------------------------------------------------------------
def test_bench_spawns_eight_ranks_itself():
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--dry-run", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_last_json(p.stdout), 8)


def test_bench_eight_ranks_under_torch_distributed_run():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), "bench.py", "--gpus", "8", "--dry-run", "--steps", "2",
                        "--warmup", "1"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_last_json(p.stdout), 8)


def test_bench_total_10000_over_eight_ranks():
    """Config 4 at N = 8 (`--workload barrier --total 10000`): eight contiguous
    shards of 1 250 scenarios that cover the one batch exactly once, each
    rank's shard built (the draws are the whole batch's, not per rank) with
    the rows of the full batch."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import hashlib
    import bench
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--dry-run", "--steps", "1",
                        "--warmup", "0", "--workload", "barrier", "--total", "10000"],
                       cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-2000:]
    line = _last_json(p.stdout)
    _check(line, 8)
    shards = [r["shard"] for r in line["ranks"]]
    assert shards == [[1250 * k, 1250 * (k + 1)] for k in range(8)]
    assert [r["batch"] for r in line["ranks"]] == [1250] * 8
    assert len({r["params_sha"] for r in line["ranks"]}) == 8
    # rank 3's shard is rows 3750..4999 of the single-process batch
    full = bench.build_barrier(10000, 1024, 2000, seed=0, select=range(3750, 5000))
    assert hashlib.sha256(full.params.tobytes()).hexdigest()[:16] == line["ranks"][3]["params_sha"]


def test_reduce_parity_over_eight_ranks(tmp_path):
    """reduce_parity at world size 8: rank 1's wrong node fails every rank's
    record; the compared scenarios sum over the eight ranks."""
    import torch.multiprocessing as mp
    import bench
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "par")
    mp.start_processes(_parity_rank, args=(8, port, out), nprocs=8, join=True,
                       start_method="spawn")
    recs = [json.load(open(f"{out}.{r}")) for r in range(8)]
    for good, bad in recs:
        assert good["ok"] and good["max_rel_err"] == 0.0 and good["n_compared"] == 16
        assert not bad["ok"] and bad["max_rel_err"] > bench.PARITY_TOL and bad["n_compared"] == 16
        assert "worst over the 8 ranks" in bad["rule"]
    assert all(r[1] == recs[0][1] for r in recs)
