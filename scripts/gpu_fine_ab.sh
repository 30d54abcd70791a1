#!/bin/bash
# GPU-box: fine-sort parity (golden + oracle + variants), then fine_bench per variant.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fine.py tests/test_gpu_variants.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fine.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_fine.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/fine_ab.log
for v in '{}' '{"scan_max_chunks": 4096}' '{"scan_onepass": 0}' '{"scan_max_chunks": 512}'; do
  FB_VARIANT="$v" timeout -k 10 120 python tools/fine_bench.py >> gpurun_out/fine_ab.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc ($v)" >> gpurun_out/fine_ab.log; exit $rc; fi
done
