# Round-4 A/B: direct-scatter ranked pack (d4, d2) vs the image pack (cur) on
# config 5 with the fine-sort parity tests; msel_pack ablations on the halo line.
LIBS="cur d4 d2" AB_TESTS="tests/test_gpu_fine.py tests/test_gpu_fullsize.py" AB_REPS=3 AB_TOOL=cfg5 AB_LOG=ab_direct.log bash scripts/gpu_libs_ab.sh || exit $?
LIBS="cur mnocopy mnostore mnoload" AB_TESTS= AB_REPS=2 AB_TOOL=bench AB_LOG=ab_msel.log BENCH_ARGS="--steps 20 --warmup 5 --exchange --config 3 --overload 0.05" bash scripts/gpu_libs_ab.sh
