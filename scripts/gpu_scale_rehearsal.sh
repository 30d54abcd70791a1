#!/bin/bash
# GPU-box rehearsal of the driver's N>1 bench launch on ONE GPU: every rank
# binds GPU 0 (MGR_BENCH_SHARED_GPU=1, RCCL socket transport between ranks),
# configs 3/4/5 at N = 2 and 4, reduced particle counts.  Numbers are not
# xGMI numbers; the point is that every N>1 code path runs to its JSON line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/scale
export MGR_BENCH_SHARED_GPU=1
env | grep '^NCCL_' > gpurun_out/scale/nccl_env.txt || true
P=29600
for N in 2 4; do
  for cfg in 3 4 5; do
    P=$((P+1))
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $P bench.py --gpus $N --steps 5 --warmup 2 \
      --config $cfg --particles 8000000 > gpurun_out/scale/n${N}_cfg${cfg}.log 2>&1
    rc=$?; echo "n=$N cfg=$cfg rc=$rc" >> gpurun_out/scale/summary.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
    # the self-checking keys of the line (rccl: version/nranks/transport; exchange_ab: both timings)
    python - gpurun_out/scale/n${N}_cfg${cfg}.log >> gpurun_out/scale/summary.txt <<'PYEOF' || exit 1
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
rec = json.loads(line)
print("  ms_per_step", rec["ms_per_step"], "value", rec["value"])
print("  rccl", json.dumps(rec["rccl"]))
print("  exchange_ab", json.dumps(rec["exchange_ab"]))
PYEOF
  done
done
ls -la /tmp/mgr_bench_rccl.* > gpurun_out/scale/left_rccl_logs.txt 2>&1 || true
