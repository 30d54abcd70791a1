#!/bin/bash
# rocprofv3 PMC passes over one bench line (one counter group per pass, no
# tracing domains): SQ/TA groups (what bounds each kernel) and FETCH/WRITE
# (HBM traffic).  OUT=<name> BENCH_ARGS="--config 5 --soa" [PASSES="sq hbm"]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_$OUT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
groups=()
case " ${PASSES:-sq hbm} " in *" sq "*)
  groups+=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
  groups+=("SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM TA_BUSY_avr TA_TA_BUSY_max")
  groups+=("SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT");;
esac
case " ${PASSES:-sq hbm} " in *" hbm "*) groups+=("FETCH_SIZE") groups+=("WRITE_SIZE");; esac
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_$OUT -o pass$i \
    -- python3 $R/bench.py --no-cpu-baseline --prof none $BENCH_ARGS --steps 3 --warmup 1 > $R/gpurun_out/pmc_$OUT/pass$i.log 2>&1
  rc=$?; echo "pass$i rc=$rc ($grp)" >> $R/gpurun_out/pmc_$OUT/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
