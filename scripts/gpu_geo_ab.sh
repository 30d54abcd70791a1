#!/bin/bash
# GPU-box: the whole -m gpu suite, then A/B of the compile-time-geometry bin
# kernel (bin_geo) on config 2 (kbench) and config 5 (cfg5_ab).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --ignore=tests/test_gpu_multi.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=3 KB_VARIANTS='[{"bin_skip_clean": 0, "bin_geo": 0}, {"bin_skip_clean": 0}]' \
  timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench_geo.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench_geo.log; if [ $rc -ne 0 ]; then exit $rc; fi
CF5_REPEAT=2 CF5_VARIANTS='[{"bin_geo": 0}, {}]' timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/cfg5_geo.log 2>&1
echo "cfg5 rc=$?" >> gpurun_out/cfg5_geo.log
