#!/bin/bash
# The host-array rate with the caller's reused v_out buffer (bench.py
# pcie_inclusive), and the out= tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04q2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for wl in barrier american double; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > $O/pcie_$wl.json 2>> $O/err.log || exit $?
done
timeout -k 10 200 python bench.py --workload barrier --batch 5000 --no-cpu-baseline \
    > $O/pcie_barrier_b5000.json 2>> $O/err.log || exit $?
