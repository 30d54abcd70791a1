#!/bin/bash
# Several bench lines in one call: each argument is one bench argument string.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/bench_set.log
for a in "$@"; do
  echo "### $a" >> gpurun_out/bench_set.log
  timeout -k 10 300 python bench.py --no-cpu-baseline $a >> gpurun_out/bench_set.log 2>&1 || { echo "rc=$?" >> gpurun_out/bench_set.log; exit 1; }
done
