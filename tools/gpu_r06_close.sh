#!/bin/bash
# Round 6 closing session after the last fdcn_kernels.hip change (one gpurun
# call): the -m gpu suite and smoke, the three march throughput lines (CPU
# baseline + parity) each under rocprofv3 --kernel-trace --stats (line and
# summary from the same process), config 5's two-stream record, and the PMC
# passes behind profiles/pmc_counters.json for the three march workloads.
# Usage: bash tools/gpu_r06_close.sh TAG
set -o pipefail
TAG=${1:-r06_close}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for wl in american barrier double; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o $wl -- \
      python3 bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || exit $?
done
timeout -k 10 300 python bench.py --workload double --overlap-streams --no-cpu-baseline \
    > $O/bench_double_overlap.json 2> $O/bench_double_overlap.err || exit $?
bash tools/pmc_counters.sh ${TAG}_pmc american barrier double || exit $?
