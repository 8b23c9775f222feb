#!/bin/bash
# Full GPU parity suite, then one bench workload without the CPU baseline.
# Usage: bash tools/gpu_tests_wl.sh TAG WORKLOAD
set -o pipefail
TAG=${1:-tw}; WL=${2:-double}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/${TAG}_${WL}.json 2> gpurun_out/${TAG}_${WL}.err
