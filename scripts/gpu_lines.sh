#!/bin/bash
# Bench lines on one box, untraced, then a rocprofv3 kernel-trace of each:
#   LINES="name:args;name:args" bash scripts/gpu_lines.sh
# Each line: python bench.py <args> --no-cpu-baseline -> gpurun_out/lines/<name>.json,
# then (TRACE=1) rocprofv3 --kernel-trace --stats -> gpurun_out/lines/<name>_trace/.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lines
export TMPDIR=/tmp
IFS=';' read -ra L <<< "$LINES"
for item in "${L[@]}"; do
  name="${item%%:*}"; args="${item#*:}"
  for rep in $(seq 1 ${REPS:-1}); do
    timeout -k 10 240 python bench.py $args --no-cpu-baseline > gpurun_out/lines/${name}_r${rep}.json 2> gpurun_out/lines/${name}_r${rep}.err
    rc=$?; echo "$name rep $rep rc=$rc" >> gpurun_out/lines/status.txt; [ $rc -ne 0 ] && exit $rc
  done
  if [ -n "$TRACE" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lines/${name}_trace -o run -- python3 bench.py $args --no-cpu-baseline > gpurun_out/lines/${name}_traced.json 2> gpurun_out/lines/${name}_traced.err
    rc=$?; echo "$name traced rc=$rc" >> gpurun_out/lines/status.txt; [ $rc -ne 0 ] && exit $rc
  fi
done
exit 0
