"""BASELINE config 4's sharded path with N > 1 ranks on the GPU.

The driver's scaling run puts one rank on each GPU of an 8-GPU node; this
box has one MI355X.  Two fresh rank processes (spawn) share it on purpose
(FDCN_SHARE_DEVICE=1, distributed.bind_device) over a gloo group, so the
N > 1 code path runs on the HIP engine end to end:

  * run_all_scenarios (run_config_scenarios.py:137-195): each rank prices
    its contiguous shard_range of a config-3-shaped file (1 024-node grids,
    2 000 steps, daily monitoring, explicit grids) through the whole-file
    path (scenario_batch.price_columns: native plan, one launch, device
    epilogue) and rank 0 gathers the columns.  The gathered columns equal
    the world-size-1 GPU run (`==`: both plans pick the same kernel
    instance, asserted), and a sample of rows equals the oracle-engine run
    within the GPU-vs-oracle bounds;
  * bench.py --gpus 2 --workload barrier --total N --backend gloo: the
    config-4 strong-scaling launch itself, with its reduced parity record
    (every rank's first scenarios against the C oracle) ok.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
N_SPACE, N_TIME = 1024, 2000
ROWS = 2400


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _write_file(path, rows=ROWS):
    """A config_scenarios.csv-shaped file: strike / vol / barrier sweep of
    the config-3 trade, every barrier type (bench.py scenario_file draws)."""
    import pandas as pd
    rng = np.random.default_rng(20250728)
    kinds = ["up-and-out", "down-and-out", "up-and-in", "down-and-in", "none"]
    S0 = 229.74
    bt = [kinds[i % 5] for i in range(rows)]
    up = rng.uniform(1.02, 1.5, rows) * S0
    dn = rng.uniform(0.6, 0.98, rows) * S0
    df = pd.DataFrame({
        "scenario_name": [f"s{i}" for i in range(rows)], "S0": [S0] * rows,
        "K": rng.uniform(150, 300, rows), "sigma": rng.uniform(0.15, 0.45, rows),
        "rate": [(0.073086, 0.065)[i % 2] for i in range(rows)], "barrier_type": bt,
        "upper_barrier": [float(x) if "up" in b else np.nan for b, x in zip(bt, up)],
        "lower_barrier": [float(x) if "down" in b else np.nan for b, x in zip(bt, dn)],
        "FA_price": [1.0] * rows, "FA_delta": [0.5] * rows, "FA_gamma": [0.01] * rows,
        "FA_vega": [0.2] * rows})
    df.to_csv(path, index=False)


def _base():
    from finite_difference_amd import scenarios
    base = scenarios.runner_base_params("put", N_SPACE)
    base.update(num_time_steps=N_TIME, grid_mode="explicit")
    return base


def _rank(rank, world, port, cfg, out_path):
    os.environ.update(LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), FDCN_SHARE_DEVICE="1")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from finite_difference_amd import capi, distributed, scenarios
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        df = scenarios.run_all_scenarios(cfg, None, _base(), verbose=False)
        assert capi.current_device() == capi.device_ordinals()[0]
        assert distributed.shard_range(ROWS) == distributed.shard_range(ROWS, rank, world)
        if rank == 0:
            df.to_csv(out_path, index=False)
        else:
            assert df is None
    finally:
        dist.destroy_process_group()


GREEKS = ("model_price", "model_delta", "model_gamma", "model_vega")


def test_two_ranks_on_one_gpu_equal_the_single_rank_run(tmp_path):
    import pandas as pd
    import torch.multiprocessing as mp
    from backends import oracle_engine
    from finite_difference_amd import capi, scenarios
    cfg = str(tmp_path / "config.csv")
    out = str(tmp_path / "ranked.csv")
    _write_file(cfg)
    mp.start_processes(_rank, args=(2, _free_port(), cfg, out), nprocs=2, join=True,
                       start_method="spawn")
    ranked = pd.read_csv(out, float_precision="round_trip")
    single = scenarios.run_all_scenarios(cfg, None, _base(), verbose=False)
    single = single.reset_index(drop=True)
    assert list(ranked.columns) == list(single.columns)
    assert list(ranked["scenario_name"]) == [f"s{i}" for i in range(ROWS)]
    # every grid is N_SPACE nodes, one or two solves (base + sigma bump) per
    # row: a shard's launch (1 200 - 2 400 solves) and the whole file's
    # (2 400 - 4 800) take the same kernel instance, so the columns are
    # bitwise equal
    names = {capi.variant_name(N_SPACE, False, B=b) for b in (ROWS // 2, ROWS, 2 * ROWS)}
    assert len(names) == 1, names
    for col in GREEKS:
        a, b = ranked[col].to_numpy(), single[col].to_numpy()
        assert np.all(np.isfinite(a)), col
        assert np.array_equal(a, b), (col, np.max(np.abs(a - b)))
    # a sample of rows from both shards against the oracle engine
    sample = [0, 1, 2, 3, 4, ROWS // 2 - 1, ROWS // 2, ROWS // 2 + 1, ROWS - 2, ROWS - 1]
    cfg_s = str(tmp_path / "sample.csv")
    pd.read_csv(cfg).iloc[sample].to_csv(cfg_s, index=False)
    ref = scenarios.run_all_scenarios(cfg_s, None, _base(), engine=oracle_engine(),
                                      verbose=False).reset_index(drop=True)
    got = ranked.iloc[sample].reset_index(drop=True)
    assert list(got["scenario_name"]) == list(ref["scenario_name"])
    for col, tol in zip(GREEKS, (1e-9, 1e-9, 1e-7, 1e-7)):
        a, b = got[col].to_numpy(), ref[col].to_numpy()
        err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
        assert np.all(err <= tol), (col, err.max())


def test_bench_total_two_ranks_gloo_parity_ok(tmp_path):
    """bench.py's config-4 line at --gpus 2 (the driver's N > 1 shape), the
    ranks sharing this GPU over gloo: one JSON line, n_gpus 2, strong
    scaling, the reduced parity record over both ranks ok."""
    env = dict(os.environ, FDCN_SHARE_DEVICE="1", PYTHONUNBUFFERED="1")
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(v, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload",
           "barrier", "--total", "2000", "--backend", "gloo", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["total_scenarios"] == 2000
    assert line["config"]["process_group"] == "gloo"
    assert line["config"]["scenarios_per_gpu"] == 1000
    p = line["parity"]
    assert p["ok"] and p["all_finite"] and p["n_compared"] == 16, p
    assert line["outputs_finite"]
