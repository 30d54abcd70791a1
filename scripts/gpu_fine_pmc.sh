#!/bin/bash
# GPU-box: fine-cell sort timing (tools/fine_bench.py) and rocprofv3 PMC passes
# (FETCH_SIZE, WRITE_SIZE) over it.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fine
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python tools/fine_bench.py > gpurun_out/fine/bench.log 2>&1
rc=$?; echo "fine_bench rc=$rc" >> gpurun_out/fine/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  FB_ITERS=3 timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/fine -o pmc_$c \
    -- python3 $R/tools/fine_bench.py > $R/gpurun_out/fine/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc" >> $R/gpurun_out/fine/pmc_$c.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
