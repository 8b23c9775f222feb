#!/bin/bash
# HBM traffic per launch (FETCH_SIZE, WRITE_SIZE in separate rocprofv3 passes)
# for the given bench workloads.  Usage: bash tools/pmc_traffic.sh TAG WORKLOAD...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for wl in "$@"; do
  O=gpurun_out/${TAG}_$wl
  mkdir -p "$O"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$O/$c" -o $c -- \
        python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > "$O/$c.log" 2>&1 || exit $?
  done
done
