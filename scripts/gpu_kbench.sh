#!/bin/bash
# GPU-box kernel A/B: parity tests first (stop on failure), then variants.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
KB_VARIANTS='[{}, {"bin_staged": 0}, {"pack_small": 0}, {"tile_rounds": 4}, {"tile_rounds": 8}, {"tile_rounds": 32}, {"tile_rounds": 64}]' \
  timeout -k 10 600 python tools/kbench.py > gpurun_out/kbench.log 2>&1
echo "kbench rc=$?" >> gpurun_out/kbench.log
