#!/bin/bash
# Recovery-form solve on half-chunk aggregates (config 5): the kernel parity
# tests, then A/B of ab/c5base (HEAD) against ab/c5new (working tree).
# Usage: bash tools/gpu_r04k.sh TAG
set -o pipefail
TAG=${1:-r04k}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_timed_variants.py \
    tests/test_gpu_pricers.py tests/test_gpu_fuzz.py -m gpu -x -q \
    -p no:cacheprovider --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab.sh ${TAG}_ab "${ABTAGS:-c5base c5new}" "double" --steps 10 || exit $?
