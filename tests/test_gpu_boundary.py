"""The C-ABI boundary's contracts on the MI355X (include/fdcn.h, ABI 5).

* FDCN_I_TAU_MODE = 1 (the reference American loop's accumulated tau,
  fd_american_equity.py:664-724) is honoured on the device;
* the _dev entry points reject a workspace smaller than the launch needs;
* the host-pointer entry points are reentrant: concurrent calls from several
  threads (each on its own stream) give the single-threaded results bitwise;
* _dev monitor entries < 1 are skipped as the oracle skips them;
* the sharded scenario runner binds each rank's GPU (world size 1 here).

Tolerance: value vectors max|V - V_oracle| <= 1e-10 max(1, max|V_oracle|).
"""
import math
import os
import socket
import threading

import numpy as np
import pytest

from backends import oracle_engine
from finite_difference_amd import capi, scenarios
from finite_difference_amd.engine import FORM_SUM, Boundary, Engine, pack
from plan_factory import random_solve

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _rel(a, b):
    return float(np.max(np.abs(a - b))) / max(1.0, float(np.max(np.abs(b))))


def _accumulated_tau(tau0, dt, n):
    t = tau0
    for _ in range(n):
        t = t + dt
    return t


@pytest.mark.parametrize("it", [True, False], ids=["it", "cn"])
def test_tau_mode_accumulate_matches_oracle(it):
    """A segment starting at tau0 = 1e4 with a step that is not a binary
    fraction, and lower boundary c0 e^{0.06 tau} (c0 = 1e-260 keeps it O(1)):
    the accumulated tau (tau = tau + dt per step) and tau0 + (m+1) dt then
    differ by many ulps, which e^{0.06 tau} turns into a relative difference
    of ~1e-12 in the final Dirichlet value -- far above exp's own rounding.
    The GPU must land on the tau of the mode it was given."""
    n_nodes, n_time = 300, 700
    rng = np.random.default_rng(11 + int(it))
    c0, e0, tau0 = 1e-260, 0.06, 1.0e4
    solves = []
    for k in range(4):
        s = random_solve(rng, n_nodes, n_time, 2, it=it, ko=False)
        s.tau0 = tau0
        s.dt = 1e-3 / 3.0
        s.lower = Boundary(FORM_SUM, c0, e0, 0.0, 0.0)
        s.tau_accumulate = k % 2 == 0
        solves.append(s)
    acc = _accumulated_tau(tau0, solves[0].dt, n_time)
    closed = tau0 + n_time * solves[0].dt
    assert abs(math.exp(e0 * acc) / math.exp(e0 * closed) - 1.0) > 1e-13  # distinguishable
    gpu = Engine().run(solves)
    ref = oracle_engine().run(solves)
    for k, (g, r) in enumerate(zip(gpu, ref)):
        assert _rel(g, r) <= 1e-10, (k, _rel(g, r))
        tau = acc if k % 2 == 0 else closed
        want = c0 * math.exp(e0 * tau)  # the final lower Dirichlet value of that mode
        assert abs(g[0] / want - 1.0) <= 1e-15, (k, g[0], want)
        assert abs(g[0] / r[0] - 1.0) <= 1e-15


def _dev_setup(it, B=4, n_nodes=4097, n_time=40):
    import torch
    rng = np.random.default_rng(5)
    solves = [random_solve(rng, n_nodes, n_time, 2, it=it) for _ in range(B)]
    g = pack(solves, list(range(B)))
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(getattr(g, k))).to(dev)
         for k in ("params", "iparams", "v_init")}
    t["out"] = torch.empty_like(t["v_init"])
    if it:
        t["payoff"] = torch.from_numpy(g.payoff).to(dev)
    ms = g.mon_step if len(g.mon_step) else np.zeros(1, np.int32)
    mr = g.mon_rebate if len(g.mon_rebate) else np.zeros(1)
    t["ms"] = torch.from_numpy(ms).to(dev)
    t["mr"] = torch.from_numpy(mr).to(dev)
    return g, t


def _launch_dev(it, g, t, ws, ws_bytes, k_cap, stream):
    if it:
        capi.it_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, t["params"].data_ptr(),
                          t["iparams"].data_ptr(), t["v_init"].data_ptr(),
                          t["payoff"].data_ptr(), t["out"].data_ptr(), k_cap, ws.data_ptr(),
                          ws_bytes, stream)
    else:
        capi.cn_batch_dev(g.B, g.n_nodes, g.n_time, g.n_ranna, t["params"].data_ptr(),
                          t["iparams"].data_ptr(), t["v_init"].data_ptr(), len(g.mon_step),
                          t["ms"].data_ptr(), t["mr"].data_ptr(), t["out"].data_ptr(), k_cap,
                          ws.data_ptr(), ws_bytes, stream)


@pytest.mark.parametrize("it", [True, False], ids=["it", "cn"])
def test_dev_rejects_workspace_planned_for_another_batch(it):
    """a workspace sized for another batch size (IT: a large batch's
    plan is too small for a 4-scenario launch, which spreads each scenario
    over 4 waves), or one double short, is refused with FDCN_EINVAL before
    anything is launched; the right size runs and matches the oracle."""
    import torch
    g, t = _dev_setup(it)
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    big = capi.plan(g.n_nodes, it, k_cap, n_time=g.n_time, B=4096)["ws_bytes_per_scen"] * g.B
    right = capi.plan(g.n_nodes, it, k_cap, n_time=g.n_time, B=g.B)["ws_bytes_per_scen"] * g.B
    if it:  # IT: the large-batch plan (W=1) needs less than the 4-scenario one (W=4)
        assert big < right
    wrong = min(big, right - 8)
    ws = torch.empty(right // 8 + 1, dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    with pytest.raises(capi.FdcnError, match="workspace"):
        _launch_dev(it, g, t, ws, wrong, k_cap, stream)
    with pytest.raises(capi.FdcnError, match="workspace"):
        _launch_dev(it, g, t, ws, -1, k_cap, stream)
    _launch_dev(it, g, t, ws, right, k_cap, stream)
    torch.cuda.synchronize()
    got = t["out"].cpu().numpy()
    ref = oracle_engine().backend.run_group(g)
    assert _rel(got, ref) <= 1e-10


def test_dev_skips_monitor_entries_below_one():
    """_dev path (no host validation): leading entries <= 0 and an entry not
    above its predecessor are skipped, as the oracle's `while` skips them."""
    import torch
    g, t = _dev_setup(False, B=2, n_nodes=1024, n_time=30)
    ms = np.array([0, -3, 4, 4, 9, 2, 17, 0, 5], dtype=np.int32)
    mr = np.linspace(0.5, 1.3, len(ms))
    g.iparams[0, capi.I_MON_START], g.iparams[0, capi.I_MON_COUNT] = 0, len(ms)
    g.iparams[1, capi.I_MON_START], g.iparams[1, capi.I_MON_COUNT] = 2, 5
    g.iparams[:, capi.I_KO_LO] = [100, -1]
    g.iparams[:, capi.I_KO_HI] = [900, 700]
    g.mon_step, g.mon_rebate = ms, mr
    t["iparams"] = torch.from_numpy(g.iparams).cuda()
    t["ms"], t["mr"] = torch.from_numpy(ms).cuda(), torch.from_numpy(mr).cuda()
    k_cap = capi.sm_extent(g.n_nodes, g.n_time, g.n_ranna, g.params)
    wsb = capi.plan(g.n_nodes, False, k_cap, n_time=g.n_time, B=g.B)["ws_bytes_per_scen"] * g.B
    ws = torch.empty(wsb // 8 + 1, dtype=torch.float64, device="cuda:0")
    _launch_dev(False, g, t, ws, wsb, k_cap, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = oracle_engine().backend.run_group(g)
    assert _rel(t["out"].cpu().numpy(), ref) <= 1e-10


def test_host_entry_points_are_reentrant():
    """Four threads, each pricing its own plans repeatedly through the
    host-pointer ABI (own stream, pooled allocations): every result equals
    the single-threaded run bitwise (same kernel, same inputs)."""
    rng = np.random.default_rng(21)
    plans = []
    for i in range(4):
        it = i % 2 == 0
        plans.append([random_solve(rng, 513 + 256 * i, 120, 2, it=it) for _ in range(3)])
    single = [Engine().run(p) for p in plans]
    errors = []

    def work(i):
        try:
            for _ in range(5):
                got = Engine().run(plans[i])
                for a, b in zip(got, single[i]):
                    if not np.array_equal(a, b):
                        errors.append(f"thread {i}: result differs")
        except Exception as e:  # pragma: no cover - reported below
            errors.append(f"thread {i}: {e!r}")

    threads = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads), "a thread hung"
    assert not errors, errors


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_sharded_runner_binds_the_rank_device(backend):
    """run_all_scenarios through the rank code path at world size 1 (a gloo
    or an RCCL group on 127.0.0.1; RCCL is what the 8-GPU run uses for the
    result gather): LOCAL_RANK's GPU is selected for libfdcn and the rows
    equal the plain run."""
    import torch.distributed as dist
    cfg = os.path.join(HERE, "golden", "ref_csv", "config_scenarios_space_1.csv")
    base = scenarios.runner_base_params("put", 60)
    plain = scenarios.run_all_scenarios(cfg, None, base, verbose=False)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["LOCAL_RANK"] = "0"
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    from finite_difference_amd import distributed
    gathers = []
    real_gather = distributed.gather_columns

    def counting_gather(cols):  # the shard -> gather branch runs over this group
        gathers.append(len(cols["model_price"]))
        return real_gather(cols)
    distributed.gather_columns = counting_gather
    try:
        assert distributed.bind_device() == capi.device_ordinals()[0]
        assert capi.current_device() == capi.device_ordinals()[0]
        ranked = scenarios.run_all_scenarios(cfg, None, base, verbose=False)
    finally:
        distributed.gather_columns = real_gather
        dist.destroy_process_group()
        os.environ.pop("LOCAL_RANK", None)
    assert gathers == [len(plain)], gathers
    for col in ("model_price", "model_delta", "model_gamma", "model_vega"):
        assert np.array_equal(ranked[col].to_numpy(), plain[col].to_numpy()), col
