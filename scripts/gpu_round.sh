#!/bin/bash
# GPU-box: full GPU test suite, then kernel A/B (interleaved repeats), then bench.
# Each step has its own time limit; stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=${KB_REPEAT:-3} KB_VARIANTS_FILE=${KB_VARIANTS_FILE:-tools/variants.json} timeout -k 10 400 python -u tools/kbench.py > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log
exit $rc
