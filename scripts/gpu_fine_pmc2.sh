#!/bin/bash
# GPU-box: fine-cell sort PMC passes (HBM bytes; SQ wait/issue split) for the
# fine pack variants ($FB_VARIANT).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fine2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  FB_ITERS=3 timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/fine2/${TAG:-x}_p$i -o pmc \
    -- python3 $R/tools/fine_bench.py > $R/gpurun_out/fine2/${TAG:-x}_p$i.log 2>&1
  rc=$?; echo "pmc $c rc=$rc" >> $R/gpurun_out/fine2/${TAG:-x}_p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
