#!/bin/bash
# Small-batch (latency) variant sweep on the GPU box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lat; mkdir -p $O
for v in 1,64 2,32 4,16 8,8; do
  FDCN_VARIANT=$v timeout -k 10 200 python bench.py --workload double --batch 1 --steps 2 --warmup 1 --no-cpu-baseline > $O/double1_$v.json 2>> $O/err.log || exit $?
done
for v in 1,32 2,16 4,8; do
  FDCN_VARIANT=$v timeout -k 10 200 python bench.py --workload american --batch 64 --steps 3 --warmup 1 --no-cpu-baseline > $O/am64_$v.json 2>> $O/err.log || exit $?
done
