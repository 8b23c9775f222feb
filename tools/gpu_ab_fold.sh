set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_timed_variants.py tests/test_gpu_pricers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03n_tests.log 2>&1 || exit $?
bash tools/gpu_ab_double.sh r03n_c3 "base WT" --workload barrier && \
bash tools/gpu_ab_double.sh r03n_c2 "base WT" --workload american && \
bash tools/gpu_ab_double.sh r03n_40 "base WT" --workload barrier --n-space 2133 --batch 4096
