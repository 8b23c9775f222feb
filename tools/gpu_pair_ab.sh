#!/bin/bash
# Paired vs one-scenario-per-wave A/B on the config-3 workload at two grid
# sizes.  Usage: bash tools/gpu_pair_ab.sh TAG
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # out lib variant bench-args...
  local out=$1 lib=$2 var=$3; shift 3
  FDCN_LIB=$lib FDCN_VARIANT=$var timeout -k 10 200 python bench.py --workload barrier \
      --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/${TAG}_$out.json 2>> gpurun_out/${TAG}.err
}
for rep in 1 2; do
  run n1024_tab16_$rep ab/tab/libfdcn.so 1,16 || exit $?
  run n1024_new16_$rep ab/pair/libfdcn.so 1,16 || exit $?
  run n1024_pair32_$rep ab/pair/libfdcn.so 1,32,2 || exit $?
  run n512_new8_$rep ab/pair/libfdcn.so 1,8 --n-space 512 || exit $?
  run n512_pair16_$rep ab/pair/libfdcn.so 1,16,2 --n-space 512 || exit $?
  run n256_new4_$rep ab/pair/libfdcn.so 1,4 --n-space 256 || exit $?
  run n256_pair8_$rep ab/pair/libfdcn.so 1,8,2 --n-space 256 || exit $?
done
