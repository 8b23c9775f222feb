#!/bin/bash
# Analytic batch kernels: GPU tests, bench line, rocprof kernel stats.
set -o pipefail
TAG=${1:-an}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_analytic.py -m gpu -q -s -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload analytic > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o analytic -- \
    python bench.py --workload analytic --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
