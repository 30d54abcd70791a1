#!/bin/bash
# Round-3 A/B on the GPU box: the fine-sort parity tests, then config-5
# (CF5_VARIANTS) and config-2 (KB_VARIANTS) kernel variants, each optional.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_gpu_fine.py} -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$CF5_VARIANTS" ]; then
  CF5_REPEAT=${CF5_REPEAT:-2} timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/ab_cfg5.log 2>&1
  rc=$?; echo "cfg5 rc=$rc" >> gpurun_out/ab_cfg5.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "$KB_VARIANTS" ]; then
  KB_REPEAT=${KB_REPEAT:-3} timeout -k 10 300 python tools/kbench.py > gpurun_out/ab_kb.log 2>&1
  rc=$?; echo "kbench rc=$rc" >> gpurun_out/ab_kb.log; if [ $rc -ne 0 ]; then exit $rc; fi
fi
