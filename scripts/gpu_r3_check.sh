#!/bin/bash
# Round-3 GPU check: the changed kernels' parity tests, then the bench lines
# (default = config 2, config 5, the halo line at world 1) and the config-5 A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${CHECK_TESTS:-"tests/test_gpu_fine.py tests/test_gpu_halo.py tests/test_gpu_api.py tests/test_gpu_variants.py"}
timeout -k 10 700 python -u -m pytest $T -m gpu -q -x --timeout 240 --timeout-method thread > gpurun_out/check_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/check_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
B="--steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 200 python bench.py $B > gpurun_out/check_b2.json 2> gpurun_out/check_b2.err || exit 1
timeout -k 10 200 python bench.py $B --config 5 > gpurun_out/check_b5.json 2> gpurun_out/check_b5.err || exit 1
timeout -k 10 300 python bench.py $B --exchange --config 3 --overload 0.05 > gpurun_out/check_bh.json 2> gpurun_out/check_bh.err || exit 1
if [ -n "$CF5_VARIANTS" ]; then
  CF5_REPEAT=${CF5_REPEAT:-2} timeout -k 10 300 python tools/cfg5_ab.py > gpurun_out/ab_cfg5.log 2>&1 || exit 1
fi
