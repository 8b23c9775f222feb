#!/bin/bash
# Session / whole-file runner tests, then the file workloads' host breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_session.py tests/test_gpu_multirank.py -m gpu -x -v \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
bash tools/gpu_r04g.sh ${1:-r04j}
