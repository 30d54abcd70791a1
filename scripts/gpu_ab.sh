#!/bin/bash
# GPU-box kernel A/B: variant parity tests (PYTEST_K selects), then interleaved
# kbench repeats of KB_VARIANTS.  Stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-variants}" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=${KB_REPEAT:-3} timeout -k 10 500 python -u tools/kbench.py > gpurun_out/kbench_ab.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench_ab.log
exit $rc
