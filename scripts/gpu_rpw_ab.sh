#!/bin/bash
# GPU-box: variant + fine parity, then the image pack's rounds per wave (img_rpw)
# on 36/40-byte records (kbench) and config 5 (cfg5_ab).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fine.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_rpw.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_rpw.log; if [ $rc -ne 0 ]; then exit $rc; fi
#KB_REPEAT=3 KB_VARIANTS='[{"rec": 36, "img_rpw": 1}, {"rec": 36}, {"rec": 36, "img_rpw": 4}, {"rec": 24}, {"rec": 24, "img_rpw": 4}]' \
#  timeout -k 10 300 python tools/kbench.py > gpurun_out/kbench_rpw.log 2>&1
#rc=$?; echo "kbench rc=$rc" >> gpurun_out/kbench_rpw.log; if [ $rc -ne 0 ]; then exit $rc; fi
CF5_REPEAT=2 CF5_VARIANTS='[{}, {"scan_max_chunks": 2048}, {"scan_max_chunks": 4096}, {"scan_max_chunks": 4096, "scan_chunk": 1024}]' timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/cfg5_rpw.log 2>&1
echo "cfg5 rc=$?" >> gpurun_out/cfg5_rpw.log
