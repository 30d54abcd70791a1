#!/bin/bash
# Round-4 final check A: smoke, the whole -m gpu suite, the default bench line
# (with its CPU baselines).  Stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_r4_check.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_default.log
exit $rc
