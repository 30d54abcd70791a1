#!/bin/bash
# Round-5: the halo's stream selection kernel -- halo parity first (both
# kernels), then the one-rank halo bench line, stream vs list kernel, same
# build, alternating processes.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_variants.py -k "halo" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_msel.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_msel.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/msel_ab.log
for rep in 1 2 3; do
  for h in '{}' '{"msel_lists": 1}'; do
    echo "hooks=$h" >> gpurun_out/msel_ab.log
    BENCH_HOOKS="$h" timeout -k 10 300 python tools/bench_hooks.py --no-cpu-baseline --exchange --config 3 --overload 0.05 --steps 20 --warmup 5 >> gpurun_out/msel_ab.log 2>/dev/null || exit 1
  done
done
