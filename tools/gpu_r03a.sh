#!/bin/bash
# Round-3 first GPU session: host facts, the -m gpu suite, the default bench
# (with its parity record), config 4 as one sharded batch, and the variant
# sweep behind the choice for 1024 < B < 4096 (config-4 shards).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03a
mkdir -p $O
{ cat /sys/fs/cgroup/cpu.max; nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"; } > $O/host.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench_american.json 2> $O/bench_american.err || exit $?
for B in 1250 2500 5000; do
  for v in 1,16,0 1,16,1 2,8,0; do
    timeout -k 10 200 python bench.py --workload barrier --batch $B --force-variant $v \
        --no-cpu-baseline > $O/sweep_b${B}_${v//,/_}.json 2>> $O/sweep.err || exit $?
  done
done
timeout -k 10 300 python bench.py --workload barrier --total 10000 > $O/bench_barrier_total.json \
    2> $O/bench_barrier_total.err || exit $?
