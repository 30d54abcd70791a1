#!/bin/bash
# A/B of kernel knobs on one bench line: BENCH_ARGS fixed, each argument is
# one MGR_TUNE setting ("" = defaults).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/bench_ab.log
for t in "$@"; do
  echo "### MGR_TUNE=$t" >> gpurun_out/bench_ab.log
  MGR_TUNE="$t" timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS >> gpurun_out/bench_ab.log 2>&1 || { echo "rc=$?" >> gpurun_out/bench_ab.log; exit 1; }
done
