#!/bin/bash
# GPU-box: bench.py on the BASELINE configs that run on one GPU: 2, 4, 5 local;
# 3, 4, 5 through the RCCL exchange path at world size 1.  CFGS overrides the list.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
LOG=gpurun_out/bench_configs.log
: > $LOG
IFS=';' read -ra RUNS <<< "${CFGS:---config 2;--config 4;--config 5;--exchange --config 3;--exchange --config 4;--exchange --config 5}"
for a in "${RUNS[@]}"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $a >> $LOG 2> gpurun_out/bench_configs.err
  rc=$?; echo "bench $a rc=$rc" >> $LOG
  if [ $rc -ne 0 ]; then cat gpurun_out/bench_configs.err >> $LOG; exit $rc; fi
done
