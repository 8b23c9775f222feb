#!/bin/bash
# PMC passes for the bench kernel (GPU box).  One counter group per rocprofv3
# run (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass); no trace domains.
# Usage: bash tools/pmc.sh TAG [bench args...]
set -o pipefail
TAG=${1:-pmc}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG}
mkdir -p "$O"
timeout -k 10 120 rocprofv3 -L > "$O/counters.txt" 2>&1
echo "list rc=$?" >> "$O/counters.txt"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" --output-format csv -d "$O/$name" -o "$name" -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline "${BENCH_ARGS[@]}" \
      > "$O/$name.log" 2>&1
}
BENCH_ARGS=("$@")
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64
