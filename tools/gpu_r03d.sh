#!/bin/bash
# Session: parity of the two-pass recovery form (config-5 kernel) and its A/B
# against the previous commit's library (ab/base).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_timed_variants.py \
    tests/test_double_out.py tests/test_gpu_pricers.py tests/test_gpu_properties.py -m gpu -x -v -s \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload double --no-cpu-baseline > $O/double_new_$rep.json 2>> $O/ab.err || exit $?
  timeout -k 10 200 python bench.py --lib ab/base/libfdcn.so --workload double --no-cpu-baseline > $O/double_base_$rep.json 2>> $O/ab.err || exit $?
done
