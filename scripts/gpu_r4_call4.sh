# Round-4 A/B: single-flush-site selection pack (halo line), two f32 slabs in
# flight in the bin kernel and the two-half ranked pack (config 5), each with
# its parity tests first.
LIBS="cur msel3" AB_TESTS="tests/test_gpu_halo.py" AB_REPS=3 AB_TOOL=bench AB_LOG=ab_msel3.log BENCH_ARGS="--steps 20 --warmup 5 --exchange --config 3 --overload 0.05" bash scripts/gpu_libs_ab.sh || exit $?
LIBS="cur bind2 half" AB_TESTS="tests/test_gpu_fine.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py" AB_REPS=3 AB_TOOL=cfg5 AB_LOG=ab_bind2.log bash scripts/gpu_libs_ab.sh
