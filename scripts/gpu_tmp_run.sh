cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_soa.py tests/test_gpu_fine.py tests/test_gpu_parity.py tests/test_gpu_variants.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_a.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_a.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/lines; LINES="cfg5soa:--config 5 --soa;cfg2:" REPS=2 bash scripts/gpu_lines.sh
