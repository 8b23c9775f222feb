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
