#!/bin/bash
# Round evidence on one GPU box: full -m gpu suite, smoke(), then every bench
# workload (bench line with CPU baseline + rocprofv3 kernel-trace summary).
# Usage: bash tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
bash tools/gpu_profile_all.sh ${TAG}
