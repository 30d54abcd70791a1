#!/bin/bash
# tests -> kernel A/B -> PMC passes (default variant)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
KB_VARIANTS_FILE=tools/variants.json timeout -k 10 600 python tools/kbench.py > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/hbm_probe.py > gpurun_out/hbm_probe.log 2>&1
rc=$?; echo "probe rc=$rc" >> gpurun_out/hbm_probe.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$WITH_PMC" ]; then rm -rf gpurun_out/pmc; bash scripts/gpu_pmc.sh; fi
