#!/bin/bash
# Round-3: halo selection kernels -- their parity tests, then the halo bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/halo_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/halo_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --exchange --config 3 --overload 0.05 > gpurun_out/bh.json 2> gpurun_out/bh.err
