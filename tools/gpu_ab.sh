#!/bin/bash
# A/B timing: each workload with the in-tree library and with build/ab/<name>.
# Usage: bash tools/gpu_ab.sh TAG NAME [workloads...]
set -o pipefail
TAG=${1:-ab}; NAME=$2; shift 2
WLS=${@:-american barrier double}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in $WLS; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/${TAG}_${wl}_A.json 2>> gpurun_out/${TAG}.err || exit $?
  FDCN_LIB=build/ab/$NAME/libfdcn.so timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/${TAG}_${wl}_B.json 2>> gpurun_out/${TAG}.err || exit $?
done
