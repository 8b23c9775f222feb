#!/bin/bash
# IT batches on the American 2N grid (4097 nodes): one wave of 64-node chunks
# against two waves of 32.  Usage: bash tools/gpu_it4097_ab.sh TAG
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 1,64 2,32 4,16; do
    FDCN_VARIANT=$v timeout -k 10 200 python bench.py --workload american --n-space 4096 --n-time 2048 \
        --batch 2048 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/${TAG}_${v/,/_}_$rep.json 2>> gpurun_out/$TAG.err || exit $?
  done
done
