#!/bin/bash
# GPU-box round check: smoke, multi-rank RCCL parity, the -m gpu suite, the
# default bench line (with its CPU baselines).  Stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 330 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
rc=$?; echo "multi rc=$rc" >> gpurun_out/pytest_multi.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread --ignore=tests/test_gpu_multi.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_default.log
exit $rc
