#!/bin/bash
# GPU-box: variant parity tests, kernel A/B, then bench under each profiling mode.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
KB_REPEAT=3 KB_VARIANTS_FILE=tools/variants.json timeout -k 10 400 python -u tools/kbench.py > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench.log
if [ $rc -ne 0 ]; then exit $rc; fi
for a in "--prof report" "--prof none" "--prof report --steps 100"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a >> gpurun_out/bench_modes.log 2>&1
  rc=$?; echo "bench $a rc=$rc" >> gpurun_out/bench_modes.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
