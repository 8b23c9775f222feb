#!/bin/bash
# Round 6 closing profiles (one gpurun call): rocprofv3 kernel-trace summaries
# of the four throughput lines, the torchrun line, and the spot-space NPT-32
# layout A/B (ab/r6_vc32: fdcn_vc_march<1,32> at one wave per SIMD, VGPR +
# AGPR) on a 2 049-node grid against the planner's <4,8> from the same library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_final; mkdir -p $O/vc32
export TMPDIR=/tmp
for wl in american barrier double spot_vc; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o $wl -- \
      python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_$wl.json 2> $O/prof_$wl.err || exit $?
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/bench_torchrun_n1.json 2> $O/bench_torchrun_n1.err || exit $?
L="--lib ab/r6_vc32/libfdcn.so --workload spot_vc --n-space 2048"
for rep in 1 2; do
  for v in 4,8 1,32; do
    timeout -k 10 200 python bench.py $L --force-variant $v --no-cpu-baseline \
        > $O/vc32/spot_vc_2048_${v/,/_}_$rep.json 2>> $O/vc32/ab.err || exit $?
  done
done
timeout -k 10 300 python bench.py $L --force-variant 1,32 > $O/vc32/spot_vc_2048_1_32_parity.json \
    2>> $O/vc32/ab.err || exit $?
