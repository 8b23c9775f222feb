#!/bin/bash
# Parity tests, then the CN workloads with the default and forced variants.
# Usage: bash tools/gpu_variants.sh TAG "W,NPT W,NPT ..." (forced variants for config 5)
set -o pipefail
TAG=${1:-var}; VARS=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for wl in american barrier double; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/${TAG}_${wl}.json 2> gpurun_out/${TAG}_${wl}.err || exit $?
done
for v in $VARS; do
  FDCN_VARIANT=$v timeout -k 10 300 python bench.py --workload double --no-cpu-baseline > gpurun_out/${TAG}_double_${v/,/_}.json 2>> gpurun_out/${TAG}_double.err || exit $?
done
