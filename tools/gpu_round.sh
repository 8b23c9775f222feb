#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_round.sh TAG [bench args...]
# Stops at the first crash/timeout (exit status other than 0/1 from pytest).
set -o pipefail
TAG=${1:-run}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o ${TAG} -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_prof.log 2>&1
