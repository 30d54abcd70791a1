#!/bin/bash
# Round-5 final check: smoke + the whole -m gpu suite (gpu_r5_check.sh), the
# default bench line with its CPU baselines (as the driver runs it), then
# every bench line untraced three times (gpurun_out/r5_lines.log).  Stops at
# the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/gpu_r5_check.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_default.log
if [ $rc -ne 0 ]; then exit $rc; fi
L=gpurun_out/r5_lines.log
: > $L
for rep in 1 2 3; do
  for args in "" "--config 4" "--config 5" "--exchange --config 3" "--exchange --config 3 --overload 0.05"; do
    echo "args=$args" >> $L
    timeout -k 10 200 python bench.py --no-cpu-baseline $args --steps 30 --warmup 10 >> $L 2>/dev/null || exit 1
  done
done
