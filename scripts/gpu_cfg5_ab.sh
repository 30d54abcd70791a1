#!/bin/bash
# GPU-box: config-5 kernel A/B (tools/cfg5_ab.py); CF5_VARIANTS from the caller.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$CF5_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest $CF5_TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cf5.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_cf5.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 400 python tools/cfg5_ab.py > gpurun_out/cfg5_ab.log 2>&1
echo "cfg5_ab rc=$?" >> gpurun_out/cfg5_ab.log
