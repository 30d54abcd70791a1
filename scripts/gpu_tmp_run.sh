cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_onepass.py tests/test_gpu_soa.py tests/test_gpu_fine.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_a.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_a.log; [ $rc -ne 0 ] && exit $rc
LINES="cfg5soa:--config 5 --soa --steps 20 --warmup 5;cfg5:--config 5 --steps 20 --warmup 5;cfg5one:--config 5 --onepass --steps 20 --warmup 5;cfg2soa:--soa --steps 20 --warmup 5" bash scripts/gpu_lines.sh
