#!/bin/bash
# End-of-round measurement session on one GPU box: the -m gpu suite, every
# bench workload's JSON line, the throughput lines under rocprofv3
# --kernel-trace --stats (line and summary from one process), config 5's
# two-stream record, the PMC passes bench.py reads (profiles/pmc_counters.json,
# via tools/collect_final.sh) and the torchrun line.
# Usage: bash tools/gpu_final.sh TAG [PART]   PART: all (default), lines (the
# tests, smoke and every bench line) or profiles (rocprofv3 summaries, PMC
# passes, the torchrun line) -- one gpurun call each when the whole session
# would not fit one call's time limit
set -o pipefail
TAG=${1:-final}
PART=${2:-all}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$PART" != profiles ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
# the driver's smoke check (__graft_entry__.smoke, no build: the tree's .so)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_american.json 2> $O/bench_american.err || exit $?
for wl in barrier double analytic spot_vc scenario_file american_file trade_cnlog trade_american trade_double; do
  timeout -k 10 300 python bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || exit $?
done
# BASELINE config 4: one 10 000-scenario batch; the per-rank batch sizes of
# its 2/4/8-GPU shards on this one GPU
timeout -k 10 300 python bench.py --workload barrier --total 10000 > $O/bench_barrier_total.json \
    2> $O/bench_barrier_total.err || exit $?
for B in 1250 2500 5000; do
  timeout -k 10 300 python bench.py --workload barrier --batch $B --no-cpu-baseline \
      > $O/bench_barrier_b$B.json 2> $O/bench_barrier_b$B.err || exit $?
done
timeout -k 10 300 python bench.py --workload spot_vc --n-space 600 --n-time 600 \
    > $O/bench_spot_vc_600.json 2> $O/bench_spot_vc_600.err || exit $?
# config 4 with N = 2 ranks sharing this GPU over gloo (the N > 1 code path)
FDCN_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --workload barrier --total 10000 \
    --backend gloo > $O/bench_barrier_total_2ranks_gloo.json 2> $O/bench_barrier_total_2ranks_gloo.err || exit $?
fi
[ "$PART" = lines ] && exit 0
# the default bench command of each throughput config under rocprofv3: the
# line (with its CPU baselines and parity record) and the kernel-trace
# summary come from the same process
for wl in american barrier double spot_vc; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o $wl -- \
      python3 bench.py --workload $wl > $O/prof_$wl.json 2> $O/prof_$wl.err || exit $?
done
# config 5's two-stream record (a serving loop; the line stays one launch)
timeout -k 10 300 python bench.py --workload double --overlap-streams --no-cpu-baseline \
    > $O/bench_double_overlap.json 2> $O/bench_double_overlap.err || exit $?
bash tools/pmc_counters.sh ${TAG}_pmc american barrier double spot_vc || exit $?
# the launcher path the driver's scaling run uses (one rank here: one GPU)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/bench_torchrun_n1.json 2> $O/bench_torchrun_n1.err || exit $?
