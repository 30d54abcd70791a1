#!/bin/bash
# GPU-box quick loop: selected tests ($TESTS) then a bench ($BENCH_ARGS).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_quick.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench_quick.log
