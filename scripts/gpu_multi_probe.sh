#!/bin/bash
# GPU-box: multi-rank RCCL parity runs on one GPU (worlds given in $WORLDS).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
MGR_MULTI_TIMEOUT=${MGR_MULTI_TIMEOUT:-200} timeout -k 10 ${OUTER:-600} python -u -m pytest tests/test_gpu_multi.py -x -v -k "${WORLDS:-2}" --timeout 500 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
echo "multi rc=$?" >> gpurun_out/pytest_multi.log
