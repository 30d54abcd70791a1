#!/bin/bash
# Round-4 GPU check: smoke, the whole -m gpu suite (multi-rank RCCL and the
# full-size cases included).  Stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
T=${CHECK_TESTS:-tests}
timeout -k 10 ${CHECK_TIMEOUT:-1000} python -u -m pytest $T -m gpu -x -v --durations=15 --timeout 960 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
exit $rc
