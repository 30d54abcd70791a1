#!/bin/bash
# Round-5: the sweep destination sort -- parity first (fine tests, race
# tests, full-size config-5 step), then the config-5 A/B of the two paths in
# one build (tools/cfg5_ab.py: dst_sweep vs dst_ranked, and the product's
# dst_sort), then the config-5 bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fine.py tests/test_gpu_fullsize.py "tests/test_gpu_api.py::test_scan_race_fine_late_inclusive_word" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_sweep.log; [ $rc -ne 0 ] && exit $rc
CF5_REPEAT=3 timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/cfg5_sweep_ab.log 2>&1
rc=$?; echo "ab rc=$rc" >> gpurun_out/cfg5_sweep_ab.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config 5 --steps 30 >> gpurun_out/cfg5_sweep_bench.log 2>&1 || exit 1
done
