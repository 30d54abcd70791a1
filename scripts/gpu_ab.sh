#!/bin/bash
# GPU-box: the -m gpu suite, then kernel A/B (tools/kbench.py, KB_VARIANTS) and
# config 5 (tools/cfg5_ab.py, CF5_VARIANTS).  Stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --ignore=tests/test_gpu_multi.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=${KB_REPEAT:-3} timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench_ab.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench_ab.log; if [ $rc -ne 0 ]; then exit $rc; fi
CF5_REPEAT=${CF5_REPEAT:-2} timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/cfg5_ab.log 2>&1
echo "cfg5 rc=$?" >> gpurun_out/cfg5_ab.log
