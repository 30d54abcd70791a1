#!/bin/bash
# rocprofv3 SQ/TA PMC passes over the halo bench line (one
# counter group per pass, no tracing domains): what bounds the selections.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmch
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM TA_BUSY_avr TA_TA_BUSY_max" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmch -o pass$i \
    -- python3 $R/bench.py --no-cpu-baseline --prof none --exchange --config 3 --overload 0.05 --steps 3 --warmup 1 > $R/gpurun_out/pmch/pass$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc ($grp)" >> $R/gpurun_out/pmch/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
