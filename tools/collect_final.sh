#!/bin/bash
# Copy one tools/gpu_final.sh session (gpurun_out/TAG, gpurun_out/TAG_pmc_*)
# into profiles/DEST and rebuild profiles/pmc_counters.json from its PMC
# passes.  Run it with the working tree's fdcn_kernels.hip equal to the one
# the session measured: counters_json.py keys the counters by its sha.
# Usage: bash tools/collect_final.sh TAG DEST
set -euo pipefail
TAG=$1; DEST=$2
cd "$(dirname "$0")/.."
S=gpurun_out/$TAG; D=profiles/$DEST
mkdir -p "$D/pmc"
cp "$S"/bench_*.json "$D/"
cp "$S/gpu_tests.log" "$D/gpu_tests.txt"
cp "$S/smoke.log" "$D/smoke.txt"
for wl in american barrier double spot_vc; do
  # the line of the rocprofv3 process beside its kernel-trace summary
  cp "$S/prof_$wl.json" "$D/rocprof_bench_$wl.json"
  cp "$S/prof_$wl/${wl}_kernel_stats.csv" "$D/kernel_stats_$wl.csv"
  for p in fetch grbm sq write; do
    cp "gpurun_out/${TAG}_pmc_$wl/$p/${p}_counter_collection.csv" "$D/pmc/${wl}_$p.csv"
  done
done
python tools/counters_json.py "${TAG}_pmc" american barrier double spot_vc
