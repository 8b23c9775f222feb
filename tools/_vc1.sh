set -o pipefail
D=gpurun_out/vc2
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spot_barrier.py tests/test_spot_barrier_analytic.py tests/test_gpu_fuzz.py -k "spot or vc or analytic" -m gpu > $D/tests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --workload spot_vc --steps 5 --warmup 1 --cpu-seconds 8 > $D/b1025.json 2> $D/b1025.err &&
timeout -k 10 300 python -u bench.py --workload spot_vc --n-space 1023 --steps 5 --warmup 1 --cpu-seconds 4 > $D/b1024.json 2> $D/b1024.err &&
timeout -k 10 300 python -u bench.py --workload spot_vc --n-space 600 --n-time 600 --steps 5 --warmup 1 --cpu-seconds 4 > $D/b600.json 2> $D/b600.err
