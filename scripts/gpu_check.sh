#!/bin/bash
# GPU check: smoke, then the named tests first (new this round), then
# the whole -m gpu suite.  Stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$FIRST_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST_TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_first.log 2>&1
  rc=$?; echo "pytest-first rc=$rc" >> gpurun_out/pytest_first.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "$SKIP_FULL" ]; then exit 0; fi
timeout -k 10 ${CHECK_TIMEOUT:-1000} python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 960 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
exit $rc
