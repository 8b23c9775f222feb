#!/bin/bash
# Spot-space march evidence on one GPU box: the -m gpu suite, smoke(), the
# spot_vc bench line and the rocprofv3 kernel-trace summary of the same run.
# Usage: bash tools/gpu_vc.sh TAG
set -o pipefail
TAG=${1:-vc}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload spot_vc > $O/bench_spot_vc.json 2> $O/bench_spot_vc.err || exit $?
timeout -k 10 300 python bench.py --workload spot_vc --n-space 600 --n-time 600 \
    > $O/bench_spot_vc_600.json 2> $O/bench_spot_vc_600.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_spot_vc -o spot_vc -- \
    python3 bench.py --workload spot_vc --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_spot_vc.log 2>&1 || exit $?
