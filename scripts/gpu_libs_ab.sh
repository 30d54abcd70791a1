#!/bin/bash
# GPU-box: same-box A/B of several libmgr.so builds (tools/ab/libmgr_<v>.so,
# v in $LIBS, the first is the baseline), alternating processes over AB_REPS
# rounds.  Each non-baseline build first runs the parity tests in $AB_TESTS.
# AB_TOOL: cfg5 (tools/cfg5_ab.py) | kb (tools/kbench.py) | both | bench
# (bench.py $BENCH_ARGS, one JSON line per run).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=mpi_grid_redistribute_amd/libmgr.so
LIBS=${LIBS:-"prev new"}
LOG=${AB_LOG:-libs_ab.log}
first=${LIBS%% *}
for v in $LIBS; do
  [ "$v" = "$first" ] && continue
  [ -z "$AB_TESTS" ] && continue
  cp tools/ab/libmgr_$v.so $L
  timeout -k 10 400 python -u -m pytest $AB_TESTS -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_ab_$v.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_ab_$v.log; [ $rc -ne 0 ] && exit $rc
done
: > gpurun_out/$LOG
for rep in $(seq 1 ${AB_REPS:-3}); do
  for v in $LIBS; do
    cp tools/ab/libmgr_$v.so $L
    echo "lib=$v" >> gpurun_out/$LOG
    if [ "${AB_TOOL:-cfg5}" = cfg5 ] || [ "${AB_TOOL:-cfg5}" = both ]; then
      CF5_REPEAT=1 timeout -k 10 200 python tools/cfg5_ab.py >> gpurun_out/$LOG 2>&1 || exit 1
    fi
    if [ "${AB_TOOL:-cfg5}" = kb ] || [ "${AB_TOOL:-cfg5}" = both ]; then
      KB_REPEAT=1 timeout -k 10 200 python tools/kbench.py >> gpurun_out/$LOG 2>&1 || exit 1
    fi
    if [ "${AB_TOOL:-cfg5}" = bench ]; then
      timeout -k 10 200 python bench.py --no-cpu-baseline $BENCH_ARGS >> gpurun_out/$LOG 2>/dev/null || exit 1
    fi
  done
done
