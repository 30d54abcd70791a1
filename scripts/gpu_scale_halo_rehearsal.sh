#!/bin/bash
# GPU-box rehearsal of the N>1 halo bench line (config 3 + overload 0.05) on ONE GPU, ranks
# sharing GPU 0 over RCCL's socket transport (times are not xGMI times).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/scale_halo
export MGR_BENCH_SHARED_GPU=1
P=29700
for N in 2 4; do
  P=$((P+1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $P bench.py --gpus $N --steps 5 --warmup 2 \
    --config 3 --overload 0.05 --particles 8000000 > gpurun_out/scale_halo/n${N}.log 2>&1
  rc=$?; echo "n=$N rc=$rc" >> gpurun_out/scale_halo/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
