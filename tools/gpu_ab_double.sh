#!/bin/bash
# A/B of libfdcn builds on the config-5 workload: WT = the in-tree library.
# Usage: bash tools/gpu_ab_double.sh OUT "TAG ..." [bench args]
set -o pipefail
OUT=$1; TAGS=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/$OUT
for rep in 1 2; do
  for t in $TAGS; do
    lib=""; [ "$t" != WT ] && lib="--lib ab/$t/libfdcn.so"
    timeout -k 10 200 python bench.py $lib --no-cpu-baseline "$@" > gpurun_out/$OUT/${t}_$rep.json 2>> gpurun_out/$OUT/ab.err || exit $?
  done
done
