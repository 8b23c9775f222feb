#!/bin/bash
# Single-trade latency through the facades (bench.py trade_* workloads) and a
# rocprofv3 kernel-trace summary of each.  Usage: bash tools/gpu_latency.sh TAG
set -o pipefail
TAG=${1:-lat}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in trade_cnlog trade_american trade_double; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 > gpurun_out/${TAG}_${wl}.json 2> gpurun_out/${TAG}_${wl}.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${wl}_prof -o $wl -- \
      python bench.py --workload $wl --steps 5 --warmup 1 > gpurun_out/${TAG}_${wl}_prof.log 2>&1 || exit $?
done
