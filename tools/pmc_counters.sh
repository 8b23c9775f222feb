#!/bin/bash
# Hardware counters of the bench launches, one counter group per rocprofv3
# pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass; no trace domains
# with --pmc).  Run on the GPU box; then tools/counters_json.py TAG turns the
# CSVs into profiles/pmc_counters.json (keyed by workload and kernel source).
# Usage: bash tools/pmc_counters.sh TAG WORKLOAD...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for wl in "$@"; do
  O=gpurun_out/${TAG}_$wl
  mkdir -p "$O"
  pass() {  # name counters...
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o "$name" -- \
        python bench.py --workload "$wl" --steps 2 --warmup 1 --no-cpu-baseline \
        > "$O/$name.log" 2>&1
  }
  pass fetch FETCH_SIZE || exit $?
  pass write WRITE_SIZE || exit $?
  pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
      SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
  pass grbm GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 \
      SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 || exit $?
done
