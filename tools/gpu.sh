#!/bin/bash
# GPU-box sessions, one parametrized entry point (round 6: replaces the
# one-off tools/gpu_r0*.sh of rounds 3-5).  Run from the repo root on the box:
#
#   bash tools/gpu.sh tests TAG [pytest args...]     the -m gpu suite (or the
#                                                    files / -k given) -> gpurun_out/TAG/tests.log
#   bash tools/gpu.sh ab OUT "TAG ..." "WL ..." [bench args...]
#                                                    A/B of ab/TAG/libfdcn.so builds
#                                                    (tools/build_ab.sh; WT = the in-tree
#                                                    library) on bench workloads, interleaved
#                                                    twice -> gpurun_out/OUT/WL_TAG_REP.json
#   bash tools/gpu.sh sweep OUT WL "TAG ..." "B ..." [bench args...]
#                                                    the same A/B over batch sizes
#   bash tools/gpu.sh variants OUT WL "W,NPT[,F] ..." [bench args...]
#                                                    one line per forced kernel variant
#                                                    (bench.py --force-variant)
#   bash tools/gpu.sh pmc-ab OUT "TAG ..." "WL ..."  SQ instruction / wait counters of each
#                                                    build (one rocprofv3 --pmc pass each)
#   bash tools/gpu.sh prof TAG WL [bench args...]    rocprofv3 --kernel-trace --stats of one
#                                                    bench command -> gpurun_out/TAG/prof_WL
#   bash tools/gpu.sh final TAG                      the end-of-round session (tools/gpu_final.sh)
#
# Every GPU step runs under its own timeout and the steps are chained: the
# first failure ends the session (no retries).  When an A/B step fails, the
# build's PROVENANCE.txt (and its sources) are copied next to the outputs, so
# the record of what faulted survives the call.
set -o pipefail
CMD=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
case "$CMD" in
  tests)
    TAG=$1; shift
    mkdir -p gpurun_out/$TAG
    ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
    timeout -k 10 900 python -u -m pytest "${ARGS[@]}" -m gpu -x -v -s -p no:cacheprovider \
        --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
    rc=$?; echo "tests rc=$rc" >> gpurun_out/$TAG/tests.log; exit $rc ;;
  ab)
    OUT=$1; TAGS=$2; WLS=$3; shift 3
    mkdir -p gpurun_out/$OUT
    for rep in 1 2; do
      for wl in $WLS; do
        for t in $TAGS; do
          lib=""; [ "$t" != WT ] && lib="--lib ab/$t/libfdcn.so"
          timeout -k 10 200 python bench.py $lib --workload $wl --no-cpu-baseline "$@" \
              > gpurun_out/$OUT/${wl}_${t}_${rep}.json 2>> gpurun_out/$OUT/ab.err
          rc=$?
          if [ $rc -ne 0 ]; then
            echo "FAILED: $t $wl rep $rep rc=$rc" >> gpurun_out/$OUT/ab.err
            [ "$t" != WT ] && cp -r ab/$t/PROVENANCE.txt ab/$t/src gpurun_out/$OUT/ 2>/dev/null
            exit $rc
          fi
        done
      done
    done ;;
  sweep)
    OUT=$1; WL=$2; TAGS=$3; BS=$4; shift 4
    mkdir -p gpurun_out/$OUT
    for B in $BS; do
      for t in $TAGS; do
        lib=""; [ "$t" != WT ] && lib="--lib ab/$t/libfdcn.so"
        timeout -k 10 200 python bench.py $lib --workload $WL --batch $B --no-cpu-baseline "$@" \
            > gpurun_out/$OUT/${t}_b$B.json 2>> gpurun_out/$OUT/ab.err || exit $?
      done
    done ;;
  variants)
    OUT=$1; WL=$2; VARS=$3; shift 3
    mkdir -p gpurun_out/$OUT
    for v in $VARS; do
      timeout -k 10 200 python bench.py --force-variant "$v" --workload $WL --no-cpu-baseline "$@" \
          > gpurun_out/$OUT/${WL}_${v//,/_}.json 2>> gpurun_out/$OUT/ab.err || exit $?
    done ;;
  pmc-ab)
    OUT=$1; TAGS=$2; WLS=$3
    for wl in $WLS; do
      for t in $TAGS; do
        O=gpurun_out/$OUT/${wl}_${t}
        mkdir -p "$O"
        lib=""; [ "$t" != WT ] && lib="--lib ab/$t/libfdcn.so"
        timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
            SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SMEM \
            --output-format csv -d "$O" -o sq -- \
            python3 bench.py $lib --workload "$wl" --steps 2 --warmup 1 --no-cpu-baseline \
            > "$O/sq.log" 2>&1 || exit $?
      done
    done ;;
  prof)
    TAG=$1; WL=$2; shift 2
    mkdir -p gpurun_out/$TAG
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof_$WL \
        -o $WL -- python3 bench.py --workload $WL "$@" > gpurun_out/$TAG/prof_$WL.log 2>&1 ;;
  final)
    bash tools/gpu_final.sh "$@"; exit $? ;;
  *)
    echo "usage: tools/gpu.sh tests|ab|prof|final ..." >&2; exit 2 ;;
esac
