#!/bin/bash
# All bench workloads on one GPU box (after the parity tests).
# Usage: bash tools/gpu_workloads.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-wl}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for wl in american barrier double; do
  timeout -k 10 400 python bench.py --workload $wl "$@" > gpurun_out/${TAG}_${wl}.json 2> gpurun_out/${TAG}_${wl}.err || exit $?
done
timeout -k 10 300 python bench.py --workload double --batch 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_double1.json 2>> gpurun_out/${TAG}_double.err || exit $?
