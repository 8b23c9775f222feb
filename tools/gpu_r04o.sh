#!/bin/bash
# Kernel parity tests on the working tree, then A/B of ab/* libraries.
# Usage: ABTAGS="a b" WLS="double barrier" bash tools/gpu_r04o.sh TAG
set -o pipefail
TAG=${1:-r04o}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_timed_variants.py \
    tests/test_gpu_pricers.py tests/test_gpu_fuzz.py -m gpu -x -q \
    -p no:cacheprovider --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab.sh ${TAG}_ab "$ABTAGS" "$WLS" --steps 10 || exit $?
