#!/bin/bash
# GPU-box: full GPU tests, then the halo bench (config 3, overload 0.05) under
# rocprofv3 kernel stats.  Stops at the first failing step.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/hprof
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hprof -o halo \
  -- python3 $R/bench.py --exchange --config 3 --overload 0.05 --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/hprof.log 2>&1
rc=$?; echo "prof rc=$rc" >> $R/gpurun_out/hprof.log
exit $rc
