#!/bin/bash
# rocprofv3 PMC passes (one counter group per pass, no tracing domains) on the
# kernel A/B bench (default variant), plus the counter list.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters.txt 2>&1
echo "list rc=$?" >> $R/gpurun_out/pmc/counters.txt
export KB_ITERS=3
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc -o pass$i \
    -- python3 $R/tools/kbench.py > $R/gpurun_out/pmc/pass$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc ($grp)" >> $R/gpurun_out/pmc/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
