#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of one bench line with tools/ab/libmgr_$LIB.so
# (gpurun_out/pmc_$LIB_<counter>/), e.g. LIB=nt BENCH_ARGS="--exchange ...".
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cp tools/ab/libmgr_$LIB.so mpi_grid_redistribute_amd/libmgr.so
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_${LIB}_$c -o pmc \
    -- python3 $R/bench.py --no-cpu-baseline --prof none $BENCH_ARGS --steps 3 --warmup 1 > $R/gpurun_out/pmc_${LIB}_$c.log 2>&1 || exit 1
done
