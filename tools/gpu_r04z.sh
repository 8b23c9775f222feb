#!/bin/bash
# Prologue A/B (Dirichlet values evaluated once per step and lane-shifted,
# constant sides without exp): base = HEAD before, pro = working tree, pro2 =
# the shift alone; the bench lines' out_sha must match.  Then (TESTS=1) the
# -m gpu suite on the new build, or (PMC=1) the VALU counters of config 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04z}
TAGS=${TAGS:-"base pro"}
WLS=${WLS:-"barrier american double"}
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu_ab.sh ${1:-r04z}_ab "$TAGS" "$WLS" --steps 20 --warmup 5 || exit $?
mv gpurun_out/${1:-r04z}_ab_* $O/ || exit $?
if [ "${PMC:-0}" = 1 ]; then
  bash tools/pmc_counters.sh ${1:-r04z}_pmc barrier || exit $?
fi
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
      --timeout-method thread > $O/tests.log 2>&1 || exit $?
fi
