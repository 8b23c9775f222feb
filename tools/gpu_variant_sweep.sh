#!/bin/bash
# Time a bench workload under forced kernel variants (bench.py --force-variant
# "W,NPT[,FLAVOUR]", fdcn_force_variant of include/fdcn_diag.h), one line per
# variant.  Usage: bash tools/gpu_variant_sweep.sh TAG WORKLOAD "W,NPT[,F] ..." [bench args]
set -o pipefail
TAG=$1; WL=$2; VARS=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in $VARS; do
  timeout -k 10 200 python bench.py --force-variant "$v" --workload $WL --no-cpu-baseline "$@" \
      > gpurun_out/${TAG}_${WL}_${v//,/_}.json 2>> gpurun_out/${TAG}_${WL}.err || exit $?
done
