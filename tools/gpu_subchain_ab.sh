#!/bin/bash
# One chain per lane (throughput variant) vs four interleaved sub-chains (the
# single-trade flavour) on the config-2 and config-3 batches, interleaved.
# Usage: bash tools/gpu_subchain_ab.sh TAG
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in 1,32 1,32,1; do
    FDCN_VARIANT=$v timeout -k 10 200 python bench.py --workload american --no-cpu-baseline \
        --steps 10 --warmup 2 > gpurun_out/${TAG}_american_${v/,/_}_$rep.json 2>> gpurun_out/$TAG.err || exit $?
  done
  for v in 1,16 1,16,1; do
    FDCN_VARIANT=$v timeout -k 10 200 python bench.py --workload barrier --no-cpu-baseline \
        --steps 10 --warmup 2 > gpurun_out/${TAG}_barrier_${v/,/_}_$rep.json 2>> gpurun_out/$TAG.err || exit $?
  done
done
