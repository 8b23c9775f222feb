#!/bin/bash
# Time a bench workload under forced kernel variants (FDCN_VARIANT="W,NPT"),
# one line per variant.  Usage: bash tools/gpu_variant_sweep.sh TAG WORKLOAD "W,NPT ..." [bench args]
set -o pipefail
TAG=$1; WL=$2; VARS=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $VARS; do
  FDCN_VARIANT=$v timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline "$@" \
      > gpurun_out/${TAG}_${WL}_${v/,/_}.json 2>> gpurun_out/${TAG}_${WL}.err || exit $?
done
