#!/bin/bash
# Evidence for every bench workload on one GPU box: the bench line (with the
# CPU baseline) and a rocprofv3 kernel-trace summary of the same command.
# Usage: bash tools/gpu_profile_all.sh TAG [workloads...]
set -o pipefail
TAG=${1:-prof}; shift || true
WLS=${@:-american barrier double}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in $WLS; do
  timeout -k 10 400 python bench.py --workload $wl > gpurun_out/${TAG}_${wl}.json 2> gpurun_out/${TAG}_${wl}.err || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${wl}_prof -o $wl -- \
      python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${wl}_prof.log 2>&1 || exit $?
done
