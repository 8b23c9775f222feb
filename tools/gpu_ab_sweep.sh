#!/bin/bash
# A/B of libfdcn builds over batch sizes of one workload (WT = in-tree).
# Usage: bash tools/gpu_ab_sweep.sh OUT WORKLOAD "TAG ..." "B ..." [bench args]
set -o pipefail
OUT=$1; WL=$2; TAGS=$3; BS=$4; shift 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/$OUT
for B in $BS; do
  for t in $TAGS; do
    lib=""; [ "$t" != WT ] && lib="--lib ab/$t/libfdcn.so"
    timeout -k 10 200 python bench.py $lib --workload $WL --batch $B --no-cpu-baseline "$@" \
        > gpurun_out/$OUT/${t}_b$B.json 2>> gpurun_out/$OUT/ab.err || exit $?
  done
done
