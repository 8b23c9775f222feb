#!/bin/bash
# Host-array copies in 8 MB pieces (copy_pieces): the pcie_inclusive rate of
# the old and new builds (bench --lib), then the -m gpu suite and the PMC
# passes of the new kernel source (bench.py keys its counters by the sha).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r04p}
mkdir -p $O
export TMPDIR=/tmp
for t in prev chunk; do
  for wl in barrier american double; do
    timeout -k 10 200 python bench.py --lib ab/$t/libfdcn.so --workload $wl --no-cpu-baseline \
        > $O/pcie_${wl}_$t.json 2>> $O/err.log || exit $?
  done
  timeout -k 10 200 python bench.py --lib ab/$t/libfdcn.so --workload barrier --batch 5000 \
      --no-cpu-baseline > $O/pcie_barrier_b5000_$t.json 2>> $O/err.log || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1 || exit $?
bash tools/pmc_counters.sh ${1:-r04p}_pmc american barrier double || exit $?
