#!/bin/bash
# A/B/C...: one workload, the in-tree library then each build/ab/<name>.
# Usage: bash tools/gpu_ab_multi.sh TAG WORKLOAD NAME...
set -o pipefail
TAG=$1; WL=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/${TAG}_base.json 2>> gpurun_out/${TAG}.err || exit $?
for n in "$@"; do
  FDCN_LIB=build/ab/$n/libfdcn.so timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/${TAG}_$n.json 2>> gpurun_out/${TAG}.err || exit $?
done
timeout -k 10 300 python bench.py --workload $WL --no-cpu-baseline > gpurun_out/${TAG}_base2.json 2>> gpurun_out/${TAG}.err || exit $?
