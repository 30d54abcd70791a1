#!/bin/bash
# GPU-box: same-box A/B of two libmgr.so builds (tools/ab/libmgr_{prev,new}.so),
# alternating processes: config 5 (tools/cfg5_ab.py) and config 2
# (tools/kbench.py), AB_REPS rounds.  The new build is restored at the end.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=mpi_grid_redistribute_amd/libmgr.so
: > gpurun_out/lib_ab.log
for rep in $(seq 1 ${AB_REPS:-3}); do
  for v in prev new; do
    cp tools/ab/libmgr_$v.so $L
    echo "lib=$v" >> gpurun_out/lib_ab.log
    CF5_REPEAT=1 timeout -k 10 200 python tools/cfg5_ab.py >> gpurun_out/lib_ab.log 2>&1 || exit 1
    KB_REPEAT=1 timeout -k 10 200 python tools/kbench.py >> gpurun_out/lib_ab.log 2>&1 || exit 1
  done
done
cp tools/ab/libmgr_new.so $L
