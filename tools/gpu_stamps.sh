#!/bin/bash
# Phase shares (tools/stamps.py) of each workload with a -DFDCN_STAMPS build.
# Usage: bash tools/gpu_stamps.sh TAG LIB [workloads...]
set -o pipefail
TAG=$1; LIB=$2; shift 2
WLS=${@:-american barrier double}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in $WLS; do
  FDCN_STAMPS_LIB=$LIB timeout -k 10 200 python tools/stamps.py $wl > gpurun_out/${TAG}_${wl}.json 2>&1 || exit $?
done
