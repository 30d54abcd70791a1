cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_soa.py tests/test_gpu_fine.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_a.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_a.log; [ $rc -ne 0 ] && exit $rc
AB_VARIANTS='[[8,2]]' timeout -k 10 300 python tools/soa_ab.py > gpurun_out/soa_ab.json 2> gpurun_out/soa_ab.err
