#!/bin/bash
# kRec A/B: parity of the NPT>=48 CN variants with build/ab/rec, then timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export FDCN_LIB=build/ab/rec/libfdcn.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pricers.py -m gpu -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread -k "w1n48 or w1n64 or cn_ko or config5 or barrier_golden or cn_log or config3 or runner or partial or correction" > gpurun_out/rec_tests.log 2>&1 || exit $?
unset FDCN_LIB
bash tools/gpu_ab.sh rec rec double
