#!/bin/bash
# A/B/C timing: each workload with the in-tree library, then each build/ab/<name>,
# then the in-tree library again (drift check).
# Usage: bash tools/gpu_ab_n.sh TAG "name1 name2 ..." [workloads...]
set -o pipefail
TAG=${1:-abn}; NAMES=$2; shift 2
WLS=${@:-american barrier double}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in $WLS; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/${TAG}_${wl}_A.json 2>> gpurun_out/${TAG}.err || exit $?
  for n in $NAMES; do
    FDCN_LIB=build/ab/$n/libfdcn.so timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/${TAG}_${wl}_$n.json 2>> gpurun_out/${TAG}.err || exit $?
  done
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/${TAG}_${wl}_A2.json 2>> gpurun_out/${TAG}.err || exit $?
done
