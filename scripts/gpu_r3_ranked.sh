#!/bin/bash
# Round-3: ranked fine sort rewrite -- its parity tests, the multi-rank run,
# then the config-5 A/B of the old and new ranked pack / rank_ids.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fine.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r3_fine.log 2>&1
rc=$?; echo "fine rc=$rc" >> gpurun_out/r3_fine.log; if [ $rc -ne 0 ]; then exit $rc; fi
CF5_REPEAT=${CF5_REPEAT:-2} CF5_VARIANTS=${CF5_VARIANTS:-'[{}, {"ranked_v": 2}, {"rank_orm": 0}]'} \
  timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/r3_cfg5_ab.log 2>&1
rc=$?; echo "cfg5 rc=$rc" >> gpurun_out/r3_cfg5_ab.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 330 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
rc=$?; echo "multi rc=$rc" >> gpurun_out/pytest_multi.log; exit $rc
