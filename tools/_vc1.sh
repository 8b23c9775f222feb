set -o pipefail
D=gpurun_out/vc5
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spot_barrier.py tests/test_spot_barrier_analytic.py tests/test_gpu_fuzz.py -k "spot or vc or analytic" -m gpu > $D/tests.txt 2>&1 &&
for g in "1024 2000" "600 600" "4096 500"; do
  set -- $g
  timeout -k 10 300 python -u bench.py --workload spot_vc --n-space $1 --n-time $2 --steps 5 --warmup 1 --cpu-seconds 3 > $D/new_$1.json 2> $D/new_$1.err || exit 1
  timeout -k 10 300 python -u bench.py --workload spot_vc --n-space $1 --n-time $2 --steps 5 --warmup 1 --no-cpu-baseline --lib ablib/libfdcn_split.so > $D/split_$1.json 2> $D/split_$1.err || exit 1
  timeout -k 10 300 python -u bench.py --workload spot_vc --n-space $1 --n-time $2 --steps 5 --warmup 1 --no-cpu-baseline --lib ablib/libfdcn_prev.so > $D/prev_$1.json 2> $D/prev_$1.err || exit 1
done
