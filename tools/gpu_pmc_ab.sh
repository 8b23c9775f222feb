#!/bin/bash
# SQ instruction / wait counters of each TAG's ab/TAG/libfdcn.so on each
# workload (one rocprofv3 --pmc pass each).  Usage: bash tools/gpu_pmc_ab.sh OUT "TAG ..." "WL ..."
set -o pipefail
OUT=$1; TAGS=$2; WLS=$3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for wl in $WLS; do
  for t in $TAGS; do
    O=gpurun_out/${OUT}/${wl}_${t}
    mkdir -p "$O"
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
        SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SMEM \
        --output-format csv -d "$O" -o sq -- \
        python bench.py --lib ab/$t/libfdcn.so --workload "$wl" --steps 2 --warmup 1 --no-cpu-baseline > "$O/sq.log" 2>&1 || exit $?
  done
done
