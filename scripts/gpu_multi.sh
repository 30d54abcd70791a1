#!/bin/bash
# GPU-box: multi-rank RCCL parity (tests/test_gpu_multi.py), then the whole
# -m gpu suite, then a short bench.  Stops at the first fatal step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
stop_if_fatal() { if [ $1 -ne 0 ] && [ $1 -ne 1 ]; then echo "fatal rc=$1 at $2"; exit $1; fi; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 330 --timeout-method thread ${MULTI_ARGS} > gpurun_out/pytest_multi.log 2>&1
rc=$?; echo "multi rc=$rc" >> gpurun_out/pytest_multi.log; stop_if_fatal $rc multi
if [ -n "$MULTI_ONLY" ]; then exit 0; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread --ignore=tests/test_gpu_multi.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log
