#!/bin/bash
# Kernel + copy trace of the config-3 halo bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_halo -o run -- python3 bench.py --no-cpu-baseline --exchange --config 3 --overload 0.05 --steps 10 --warmup 3 > gpurun_out/prof_halo.log 2>&1
echo "rc=$?" >> gpurun_out/prof_halo.log
