#!/bin/bash
# Log-space kernel changes of round 4 (split-form scan stage 0 unconditional,
# hidden scan-weight address, accumulated-tau runs walked in the prologue
# without the workspace round trip): the kernel parity tests, then A/B of
# ab/c3base (HEAD) against ab/c3new (working tree) on configs 2, 3 and 5.
# Usage: bash tools/gpu_r04f.sh TAG
set -o pipefail
TAG=${1:-r04f}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_timed_variants.py \
    tests/test_gpu_pricers.py tests/test_gpu_boundary.py tests/test_gpu_fuzz.py tests/test_spot_barrier.py \
    tests/test_spot_barrier_analytic.py -m gpu -x -q \
    -p no:cacheprovider --timeout 180 --timeout-method thread > $O/tests.log 2>&1 || exit $?
bash tools/gpu_ab.sh ${TAG}_ab "c3base c3new" "barrier american double spot_vc" --steps 10 || exit $?
