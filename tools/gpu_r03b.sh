#!/bin/bash
# Round-3 session 2: the -m gpu suite (analytic-pricer drop-in, RCCL shard ->
# gather runner) and an A/B of the config-5 kernel (S = 4 sub-chains at
# NPT 64, ab/c5s4) plus config 5 at twice the batch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload double --no-cpu-baseline > $O/double_base_$rep.json 2>> $O/ab.err || exit $?
  timeout -k 10 200 python bench.py --lib ab/c5s4/libfdcn.so --workload double --no-cpu-baseline > $O/double_c5s4_$rep.json 2>> $O/ab.err || exit $?
done
timeout -k 10 200 python bench.py --workload double --batch 4096 --no-cpu-baseline > $O/double_b4096.json 2>> $O/ab.err || exit $?
timeout -k 10 200 python bench.py --lib ab/c5s4/libfdcn.so --workload double --batch 4096 --no-cpu-baseline > $O/double_c5s4_b4096.json 2>> $O/ab.err || exit $?
