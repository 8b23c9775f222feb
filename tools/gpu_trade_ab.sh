set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in s4 cur; do
    FDCN_LIB=ab/$t/libfdcn.so timeout -k 10 200 python bench.py --workload trade_american --steps 10 --warmup 2 > gpurun_out/r02t_${t}_$rep.json 2>>gpurun_out/r02t.err || exit $?
  done
done
