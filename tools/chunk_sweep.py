"""Whole-file wall time against the plan chunk size of the pipelined device
paths (scenario_batch / american_batch CHUNK_ROWS, MAX_CHUNKS): a tuning
sweep, not a bench line.  Usage: python tools/chunk_sweep.py [american]"""
import json
import sys
import types

sys.path.insert(0, ".")
import bench  # noqa: E402
from finite_difference_amd import american_batch, scenario_batch  # noqa: E402


def main():
    am = len(sys.argv) > 1 and sys.argv[1] == "american"
    mod, fn = (american_batch, bench.bench_american_file) if am else \
        (scenario_batch, bench.bench_scenario_file)
    sweep = (((100000, 1), (1000, 2), (667, 3), (500, 4)) if am else
             ((100000, 1), (4000, 2), (2667, 3), (2000, 4), (1000, 8)))
    for rows, mx in sweep:
        mod.CHUNK_ROWS, mod.MAX_CHUNKS = rows, mx
        args = types.SimpleNamespace(batch=None, n_space=None, n_time=None, steps=5 if am else 10,
                                     warmup=2 if am else 3)
        import io
        import contextlib
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            fn(args)
        d = json.loads(buf.getvalue().strip().splitlines()[-1])
        print(json.dumps({"chunk_rows": rows, "max_chunks": mx, "ms": d["value"],
                          "ms_min": d["ms_min"], "parts": d["host_parts_ms"],
                          "tail": d["march_and_epilogue_ms"]}), flush=True)


if __name__ == "__main__":
    main()
