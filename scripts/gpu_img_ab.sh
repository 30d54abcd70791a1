#!/bin/bash
# GPU-box: the -m gpu suite, then the 36-byte record pack shapes (image pack at
# 512 / 1024-row tiles, 4-byte-unit cooperative pack) next to the 32-B pack.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --ignore=tests/test_gpu_multi.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=3 KB_VARIANTS='[{"bin_skip_clean": 0}, {"rec": 36}, {"rec": 40}]' \
  timeout -k 10 400 python tools/kbench.py > gpurun_out/kbench_img.log 2>&1
echo "kbench rc=$?" >> gpurun_out/kbench_img.log
