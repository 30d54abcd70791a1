cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
FIRST_TESTS="tests/test_gpu_soa.py tests/test_gpu_onepass.py" bash scripts/gpu_check.sh || exit 1
LINES="cfg2:--steps 30 --warmup 10;cfg5:--config 5 --steps 30 --warmup 10;cfg5classic:--config 5 --classic --steps 30 --warmup 10;cfg5soa:--config 5 --soa --steps 30 --warmup 10;cfg2soa:--soa --steps 30 --warmup 10" bash scripts/gpu_lines.sh
