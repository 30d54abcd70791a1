#!/bin/bash
# GPU-box kernel A/B: parity tests of the variants first (stop on failure), then kbench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_variants.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=${KB_REPEAT:-1} KB_VARIANTS_FILE=${KB_VARIANTS_FILE:-tools/variants.json} timeout -k 10 600 python -u tools/kbench.py > gpurun_out/kbench.log 2>&1
echo "kbench rc=$?" >> gpurun_out/kbench.log
