#!/bin/bash
# Spot-space pointwise form: its GPU tests first, then the whole -m gpu
# suite, the spot_vc bench lines (1 025 x 2 000 and 601 x 600) with their
# rocprofv3 summary, and the PMC passes.  Usage: bash tools/gpu_r04b.sh TAG
set -o pipefail
TAG=${1:-r04b}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spot_barrier.py tests/test_gpu_timed_variants.py \
    -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/vc_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 \
    --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload spot_vc > $O/bench_spot_vc.json 2> $O/bench_spot_vc.err || exit $?
timeout -k 10 300 python bench.py --workload spot_vc --n-space 600 --n-time 600 \
    > $O/bench_spot_vc_600.json 2> $O/bench_spot_vc_600.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_spot_vc -o spot_vc -- \
    python3 bench.py --workload spot_vc --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_spot_vc.log 2>&1 || exit $?
bash tools/pmc_counters.sh ${TAG}_pmc spot_vc || exit $?
