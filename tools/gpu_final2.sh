#!/bin/bash
# Round-5 closing session: PMC passes for the final kernel sources (so the
# bench lines carry traffic), then every workload's line and the rocprofv3
# summary of the same command for the three BASELINE throughput configs.
# Usage: bash tools/gpu_final2.sh TAG
set -o pipefail
TAG=${1:-final2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/pmc_counters.sh ${TAG}_pmc american barrier double spot_vc || exit $?
