"""Scenario-file wall time against the plan chunk size of the pipelined
device path (scenario_batch.CHUNK_ROWS / MAX_CHUNKS): a tuning sweep, not a
bench line.  Usage: python tools/chunk_sweep.py"""
import json
import sys
import types

sys.path.insert(0, ".")
import bench  # noqa: E402
from finite_difference_amd import scenario_batch  # noqa: E402


def main():
    for rows, mx in ((100000, 1), (4000, 2), (2667, 3), (2000, 4), (1000, 8)):
        scenario_batch.CHUNK_ROWS, scenario_batch.MAX_CHUNKS = rows, mx
        args = types.SimpleNamespace(batch=None, n_space=None, n_time=None, steps=10, warmup=3)
        import io
        import contextlib
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            bench.bench_scenario_file(args)
        d = json.loads(buf.getvalue().strip().splitlines()[-1])
        print(json.dumps({"chunk_rows": rows, "max_chunks": mx, "ms": d["value"],
                          "ms_min": d["ms_min"], "parts": d["host_parts_ms"],
                          "tail": d["march_and_epilogue_ms"]}), flush=True)


if __name__ == "__main__":
    main()
