cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/scale
export MGR_BENCH_SHARED_GPU=1
timeout -k 10 400 python bench.py --gpus 2 --particles 8000000 --steps 10 --warmup 3 --launch-timeout 300 > gpurun_out/scale/bare_n2.json 2> gpurun_out/scale/bare_n2.err
echo "n2 rc=$?" >> gpurun_out/scale/status.txt
timeout -k 10 400 python bench.py --gpus 4 --particles 4000000 --steps 10 --warmup 3 --launch-timeout 300 > gpurun_out/scale/bare_n4.json 2> gpurun_out/scale/bare_n4.err
echo "n4 rc=$?" >> gpurun_out/scale/status.txt
timeout -k 10 400 python bench.py --gpus 2 --config 5 --soa --particles 4000000 --steps 10 --warmup 3 --launch-timeout 300 > gpurun_out/scale/bare_n2_cfg5soa.json 2> gpurun_out/scale/bare_n2_cfg5soa.err
echo "n2 cfg5soa rc=$?" >> gpurun_out/scale/status.txt
