#!/bin/bash
# A/B kernel timing: each TAG's ab/TAG/libfdcn.so (tools/build_ab.sh) on each
# bench workload, interleaved twice.  Usage: bash tools/gpu_ab.sh OUT "TAG ..." "WL ..." [bench args]
set -o pipefail
OUT=$1; TAGS=$2; WLS=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for wl in $WLS; do
    for t in $TAGS; do
      timeout -k 10 200 python bench.py --lib ab/$t/libfdcn.so --workload $wl --no-cpu-baseline "$@" \
          > gpurun_out/${OUT}_${wl}_${t}_${rep}.json 2>> gpurun_out/${OUT}.err || exit $?
    done
  done
done
