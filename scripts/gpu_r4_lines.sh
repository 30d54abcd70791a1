#!/bin/bash
# Round-4: every bench line untraced, three times each (the numbers README /
# DESIGN quote beside the rocprofv3-traced ones), into gpurun_out/r4_lines.log.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/r4_lines.log
: > $L
for rep in 1 2 3; do
  for args in "" "--config 4" "--config 5" "--exchange --config 3" "--exchange --config 3 --overload 0.05"; do
    echo "args=$args" >> $L
    timeout -k 10 200 python bench.py --no-cpu-baseline $args --steps 30 --warmup 10 >> $L 2>/dev/null || exit 1
  done
done
