#!/bin/bash
# Chunked whole-file runners: the session tests, then the chunk sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_session.py tests/test_gpu_multirank.py -m gpu -x -v \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python tools/chunk_sweep.py american > $O/chunk_sweep_american.json 2> $O/sweep.err || exit $?
