#!/bin/bash
# Whole-file host-time breakdown: the two file workloads' bench lines and a
# steady-state cProfile of each (tools/host_breakdown.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04g}
mkdir -p $O
export TMPDIR=/tmp
for wl in scenario_file american_file; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || exit $?
  timeout -k 10 300 python tools/host_breakdown.py $wl $O/prof_$wl.txt > $O/prof_$wl.json 2> $O/prof_$wl.err || exit $?
done
