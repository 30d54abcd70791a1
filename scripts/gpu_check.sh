#!/bin/bash
# GPU-box check: smoke -> parity tests -> bench -> rocprofv3 kernel trace.
# Stops at the first step that faults, aborts or times out.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
stop_if_fatal() { if [ $1 -ne 0 ] && [ $1 -ne 1 ]; then echo "fatal rc=$1 at $2"; exit $1; fi; }
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=20 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log; stop_if_fatal $rc bench
if [ -n "$SKIP_PROF" ]; then exit 0; fi
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench \
  -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
echo "prof rc=$?" >> $R/gpurun_out/prof.log
