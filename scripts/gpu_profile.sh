#!/bin/bash
# Round profile: bench (default), rocprofv3 kernel-trace --stats of the same
# command, and separate --pmc passes (FETCH_SIZE / WRITE_SIZE) for HBM bytes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/profile
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/profile/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/profile/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profile -o trace \
  -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/profile/trace.log 2>&1
rc=$?; echo "trace rc=$rc" >> $R/gpurun_out/profile/trace.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/profile -o pmc_$c \
    -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 > $R/gpurun_out/profile/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc" >> $R/gpurun_out/profile/pmc_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
