cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rccldbg
export MGR_BENCH_SHARED_GPU=1
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,P2P,SHM,NET timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29650 bench.py --gpus 2 --steps 3 --warmup 1 --config 3 --particles 2000000 > gpurun_out/rccldbg/explicit.log 2>&1 || exit 1
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=ALL timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 2 --steps 3 --warmup 1 --config 3 --particles 2000000 > gpurun_out/rccldbg/all.log 2>&1 || exit 1
