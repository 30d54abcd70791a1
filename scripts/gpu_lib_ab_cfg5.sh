#!/bin/bash
# GPU-box: same-box A/B of two libmgr.so builds (tools/ab/libmgr_{prev,new}.so)
# on config 5 (tools/cfg5_ab.py), alternating processes; the fine-sort parity
# tests run on the new build first.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=mpi_grid_redistribute_amd/libmgr.so
cp tools/ab/libmgr_new.so $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_fine.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_fine.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_fine.log; if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/cfg5_lib_ab.log
for rep in 1 2 3; do
  for v in prev new; do
    cp tools/ab/libmgr_$v.so $L
    echo "lib=$v" >> gpurun_out/cfg5_lib_ab.log
    CF5_REPEAT=1 timeout -k 10 200 python tools/cfg5_ab.py >> gpurun_out/cfg5_lib_ab.log 2>&1 || exit 1
  done
done
cp tools/ab/libmgr_new.so $L
