"""Multi-process scenario sharding on CPU (gloo, world_size 2, 127.0.0.1).

Each rank prices its contiguous block of the golden scenario file (oracle
backend: no GPU here); rank 0 gathers the rows.  The result must equal the
single-process run row for row."""
import os
import socket

import pandas as pd
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from finite_difference_amd import distributed as fdist

HERE = os.path.dirname(os.path.abspath(__file__))
CFG = os.path.join(HERE, "golden", "ref_csv", "config_scenarios_space_1.csv")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, decline_rank=-1):
    import sys
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    from backends import oracle_engine
    from finite_difference_amd import scenario_batch, scenarios
    if rank == decline_rank:  # this shard takes the per-row fallback
        scenario_batch.price_columns = lambda *a, **k: None
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        df = scenarios.run_all_scenarios(CFG, None, scenarios.runner_base_params("put", 60),
                                         engine=oracle_engine(), verbose=False)
        if rank == 0:
            df.to_csv(out_path, index=False)
        else:
            assert df is None
    finally:
        dist.destroy_process_group()


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 5, 20, 10_000):
        for w in (1, 2, 3, 8):
            got = [list(fdist.shard_range(n, r, w)) for r in range(w)]
            flat = [i for g in got for i in g]
            assert flat == list(range(n))
            sizes = [len(g) for g in got]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_matches_single_process(tmp_path):
    from backends import oracle_engine
    from finite_difference_amd import scenarios
    out = str(tmp_path / "dist.csv")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True,
                       start_method="spawn")
    single = scenarios.run_all_scenarios(CFG, None, scenarios.runner_base_params("put", 60),
                                         engine=oracle_engine(), verbose=False)
    got = pd.read_csv(out, float_precision="round_trip")
    ref = single.reset_index(drop=True)
    assert list(got["scenario_name"]) == list(ref["scenario_name"])
    for col in ("model_price", "model_delta", "model_gamma", "model_vega"):
        assert (got[col].to_numpy() == ref[col].to_numpy()).all(), col


def test_two_rank_gloo_one_shard_on_the_fallback(tmp_path):
    """Rank 1's whole-file plan is declined, so its shard goes through the
    per-row façades (run_rows_batched) while rank 0's takes price_columns:
    the merged columns have one schema and equal the single-process run."""
    from backends import oracle_engine
    from finite_difference_amd import scenarios
    out = str(tmp_path / "dist.csv")
    mp.start_processes(_worker, args=(2, _free_port(), out, 1), nprocs=2, join=True,
                       start_method="spawn")
    single = scenarios.run_all_scenarios(CFG, None, scenarios.runner_base_params("put", 60),
                                         engine=oracle_engine(), verbose=False)
    got = pd.read_csv(out, float_precision="round_trip")
    ref = single.reset_index(drop=True)
    assert list(got.columns) == list(ref.columns)
    assert list(got["scenario_name"]) == list(ref["scenario_name"])
    for col in ("model_price", "model_delta", "model_gamma", "model_vega"):
        assert (got[col].to_numpy() == ref[col].to_numpy()).all(), col


class _FakeDist:
    """Rank `rank` of a `world`-rank group whose other ranks contribute
    `others` to every all_gather_object / gather_object."""

    def __init__(self, rank, world, others):
        self.rank, self.world, self.others = rank, world, others
        self.gathers = 0

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.world

    def all_gather_object(self, out, obj):
        for r in range(self.world):
            out[r] = obj if r == self.rank else self.others[r]

    def gather_object(self, obj, out, dst=0):
        self.gathers += 1
        if out is not None:
            self.all_gather_object(out, obj)


def test_gather_columns_rejects_mismatched_parts(monkeypatch):
    """the schema check is collective -- every rank raises, before
    the gather, not rank 0 alone after it."""
    for rank in (0, 1):
        fake = _FakeDist(rank, 2, {0: ["a", "b"], 1: ["b", "a"]})
        monkeypatch.setattr(fdist, "_dist", lambda: fake)
        with pytest.raises(ValueError):
            fdist.gather_columns({"a": [1], "b": [2]} if rank == 0 else {"b": [1], "a": [2]})
        assert fake.gathers == 0
    # a rank with no rows (empty schema) is not a mismatch
    fake = _FakeDist(1, 2, {0: ["a", "b"]})
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    assert fdist.gather_columns({}) is None


def test_check_device_binding_refuses_two_ranks_on_one_gpu(monkeypatch):
    """a job-wide HIP_VISIBLE_DEVICES=0 with two local ranks makes
    both bind the one device; the collective check raises on every rank.
    Distinct per-rank visible sets, distinct ordinals or FDCN_SHARE_DEVICE=1
    on both ranks pass."""
    import socket
    from finite_difference_amd import capi
    host = socket.gethostname()
    for v in ("ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "FDCN_SHARE_DEVICE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")

    def report(vis, dev, share=False):
        return ((host, (vis, "", ""), dev), share)
    for rank in (0, 1):
        fake = _FakeDist(rank, 2, {0: report("0", 0), 1: report("0", 0)})
        monkeypatch.setattr(fdist, "_dist", lambda: fake)
        with pytest.raises(capi.FdcnError):
            fdist.check_device_binding(0)
    fake = _FakeDist(0, 2, {1: report("1", 0)})  # per-rank sets "0" / "1"
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    fdist.check_device_binding(0)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    fake = _FakeDist(0, 2, {1: report("", 1)})  # two visible devices, ordinals 0 / 1
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    fdist.check_device_binding(0)
    monkeypatch.setenv("FDCN_SHARE_DEVICE", "1")
    fake = _FakeDist(0, 2, {1: report("", 0, True)})  # shared on purpose
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    fdist.check_device_binding(0)
    fake = _FakeDist(0, 2, {1: report("", 0, False)})  # only one rank asked to share
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    with pytest.raises(capi.FdcnError):
        fdist.check_device_binding(0)
    monkeypatch.setattr(fdist, "_dist", lambda: None)
    fdist.check_device_binding(0)  # no group: nothing to check


def test_bind_device_maps_local_rank_through_gfx950_ordinals(monkeypatch):
    """local rank k binds the k-th visible gfx950 device; a rank
    that sees exactly one device binds it whatever its LOCAL_RANK only when
    the launcher gave each rank its own (per-rank HIP_VISIBLE_DEVICES, one
    rank per node) or sharing is asked for (FDCN_SHARE_DEVICE=1); too few
    devices for the rank is an error."""
    from finite_difference_amd import capi
    chosen = []
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
              "FDCN_SHARE_DEVICE", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(capi, "select_device", lambda d: chosen.append(d))
    monkeypatch.setattr(capi, "device_ordinals", lambda: [0])
    monkeypatch.setenv("LOCAL_RANK", "0")
    assert fdist.bind_device() == 0 and chosen[-1] == 0
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    with pytest.raises(capi.FdcnError):  # torchrun --nproc-per-node 2 on one visible GPU
        fdist.bind_device()
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")  # the launcher's per-rank device
    assert fdist.bind_device() == 0 and chosen[-1] == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("FDCN_SHARE_DEVICE", "1")
    assert fdist.bind_device() == 0
    monkeypatch.delenv("FDCN_SHARE_DEVICE")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert fdist.bind_device() == 0
    monkeypatch.setattr(capi, "device_ordinals", lambda: [1, 3, 4])
    assert fdist.bind_device() == 3 and chosen[-1] == 3
    monkeypatch.setenv("LOCAL_RANK", "3")
    with pytest.raises(capi.FdcnError):
        fdist.bind_device()
    monkeypatch.setattr(capi, "device_ordinals", lambda: [])
    assert fdist.bind_device() is None


def test_gather_columns_without_a_group_is_identity():
    import numpy as np
    cols = {"a": [1, 2], "b": np.arange(2.0)}
    assert fdist.gather_columns(cols) is cols


def test_bind_device_eight_gfx950_ordinals(monkeypatch):
    """An 8-GPU node: local rank k binds the k-th of eight
    stubbed gfx950 ordinals, and the group's binding check passes the eight
    distinct reports."""
    import socket
    from finite_difference_amd import capi
    host = socket.gethostname()
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
              "FDCN_SHARE_DEVICE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    chosen = []
    monkeypatch.setattr(capi, "select_device", lambda d: chosen.append(d))
    monkeypatch.setattr(capi, "device_ordinals", lambda: list(range(8)))
    reports = {r: ((host, ("", "", ""), r), False, None) for r in range(8)}
    for k in range(8):
        monkeypatch.setenv("LOCAL_RANK", str(k))
        fake = _FakeDist(k, 8, reports)
        monkeypatch.setattr(fdist, "_dist", lambda: fake)
        assert fdist.bind_device() == k and chosen[-1] == k


def test_bind_device_failure_reaches_every_rank(monkeypatch):
    """once the group exists a rank whose binding fails still
    enters the collective check with its error, and every rank raises
    together -- none waits in all_gather_object for it."""
    import socket
    from finite_difference_amd import capi
    host = socket.gethostname()
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
              "FDCN_SHARE_DEVICE"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.setattr(capi, "select_device", lambda d: None)
    monkeypatch.setattr(capi, "device_ordinals", lambda: [0])
    err = "LOCAL_RANK=1 ... only 1 gfx950 device(s) are visible"
    # rank 1 fails locally (two local ranks, one visible device): it raises,
    # and only after contributing its report to the collective
    calls = []

    class Spy(_FakeDist):
        def all_gather_object(self, out, obj):
            calls.append(obj)
            super().all_gather_object(out, obj)
    fake = Spy(1, 2, {0: ((host, ("", "", ""), 0), False, None)})
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    monkeypatch.setenv("LOCAL_RANK", "1")
    with pytest.raises(capi.FdcnError, match="rank"):
        fdist.bind_device()
    assert len(calls) == 1 and calls[0][0] is None and calls[0][2]
    # rank 0 bound its device fine, but raises with rank 1's error
    fake = _FakeDist(0, 2, {1: (None, False, err)})
    monkeypatch.setattr(fdist, "_dist", lambda: fake)
    monkeypatch.setenv("LOCAL_RANK", "0")
    with pytest.raises(capi.FdcnError, match="rank\\(s\\) 1"):
        fdist.bind_device()
    # before the group exists: raise at once, or hand the error back
    monkeypatch.setattr(fdist, "_dist", lambda: None)
    monkeypatch.setenv("LOCAL_RANK", "1")
    with pytest.raises(capi.FdcnError):
        fdist.bind_device()
    assert fdist.bind_device(raise_local=False) is None and "LOCAL_RANK=1" in fdist.bind_error()
    with pytest.raises(capi.FdcnError):
        fdist.check_device_binding(None, fdist.bind_error())
