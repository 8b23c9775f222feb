"""Steady-state host profile of the whole-file runners (bench.py's
scenario_file / american_file workloads): warm up, then cProfile only the
timed calls.  Usage: python tools/host_breakdown.py scenario_file|american_file OUT"""
import cProfile
import pstats
import sys
import types

sys.path.insert(0, ".")
import bench  # noqa: E402


def main():
    wl, out = sys.argv[1], sys.argv[2]
    fn = {"scenario_file": bench.bench_scenario_file,
          "american_file": bench.bench_american_file}[wl]
    args = types.SimpleNamespace(batch=None, n_space=None, n_time=None, steps=3, warmup=3)
    fn(args)  # imports, first-call costs
    pr = cProfile.Profile()
    args.steps, args.warmup = 10, 0
    pr.enable()
    fn(args)
    pr.disable()
    with open(out, "w") as f:
        st = pstats.Stats(pr, stream=f)
        st.sort_stats("tottime").print_stats(40)
        st.sort_stats("cumulative").print_stats(50)


if __name__ == "__main__":
    main()
