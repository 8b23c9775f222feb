#!/bin/bash
# Forced-variant sweep of one workload (no tests).
# Usage: bash tools/gpu_sweep.sh TAG WORKLOAD "W,NPT W,NPT ..."
set -o pipefail
TAG=${1:-sw}; WL=${2:-american}; VARS=${3:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/${TAG}_${WL}.json 2> gpurun_out/${TAG}_${WL}.err || exit $?
for v in $VARS; do
  FDCN_VARIANT=$v timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/${TAG}_${WL}_${v/,/_}.json 2>> gpurun_out/${TAG}_${WL}.err || exit $?
done
