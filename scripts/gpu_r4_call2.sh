bash scripts/gpu_r4_check.sh || exit $?
LIBS="base seq noscat dpp" AB_TESTS= AB_REPS=2 AB_TOOL=cfg5 AB_LOG=ab_cfg5.log bash scripts/gpu_libs_ab.sh || exit $?
LIBS="base msel dpp" AB_TESTS= AB_REPS=2 AB_TOOL=bench AB_LOG=ab_halo.log BENCH_ARGS="--steps 20 --warmup 5 --exchange --config 3 --overload 0.05" bash scripts/gpu_libs_ab.sh
