#!/bin/bash
# Round 4, first box session: the -m gpu suite (new: multi-rank config 4,
# session destroy ordering, spot-space layouts / _dev monitor skips), smoke,
# the spot_vc bench line of the HEAD kernel with its rocprofv3 summary, and
# the spot_vc PMC passes.  Usage: bash tools/gpu_r04a.sh TAG
set -o pipefail
TAG=${1:-r04a}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 180 \
    --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload spot_vc > $O/bench_spot_vc.json 2> $O/bench_spot_vc.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_spot_vc -o spot_vc -- \
    python3 bench.py --workload spot_vc --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_spot_vc.log 2>&1 || exit $?
bash tools/pmc_counters.sh ${TAG}_pmc spot_vc || exit $?
