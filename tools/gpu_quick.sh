#!/bin/bash
# Quick GPU iteration: parity tests, bench (no CPU baseline), phase stamps.
# Usage: bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-q}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
if [ -f finite_difference_amd/_lib/libfdcn_stamps.so ]; then
  timeout -k 10 300 python tools/stamps.py american > gpurun_out/${TAG}_stamps.json 2>> gpurun_out/${TAG}_bench.err || exit $?
fi
