#!/bin/bash
# Config-5 line under the scan's chunking hooks (same build): the fine scan
# (512 bins x 16384 tiles) with fewer/more chunks per bin and shorter chunks.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/scan_chunks_ab.log
: > $L
for rep in 1 2; do
  for h in '{}' '{"scan_max_chunks": 512}' '{"scan_max_chunks": 256}' '{"scan_max_chunks": 2048}'; do
    echo "hooks=$h" >> $L
    BENCH_HOOKS="$h" timeout -k 10 200 python tools/bench_hooks.py --no-cpu-baseline --config 5 --steps 30 --warmup 10 >> $L 2>/dev/null || exit 1
  done
done
