#!/bin/bash
# A round's evidence: rocprofv3 kernel-trace stats of every bench line, and
# FETCH_SIZE / WRITE_SIZE PMC passes (one counter per run) of each line, into
# gpurun_out/$PROF (default r6prof; tools/round_profiles.py assembles them).
PROF=${PROF:-r6prof}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$PROF
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprof args..., -- bench args
  local name=$1; shift
  timeout -k 10 240 "$@" > $R/gpurun_out/$PROF/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc" >> $R/gpurun_out/$PROF/summary.txt
  return $rc
}
LINESET=${LINESET:-"cfg2:: cfg4::--config 4 cfg5::--config 5 cfg5classic::--config 5 --classic cfg5soa::--config 5 --soa cfg2soa::--soa cfg3x::--exchange --config 3 halo::--exchange --config 3 --overload 0.05"}
IFS='|' read -ra CFGS <<< "$(echo "$LINESET" | sed -E 's/ (cfg[0-9a-z]*::|halo::)/|\1/g')"
for cfg in "${CFGS[@]}"; do
  name=${cfg%%::*}; args=${cfg#*::}
  run ${name}_trace rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$PROF/${name}_trace -o run \
    -- python3 $R/bench.py --no-cpu-baseline $args --steps 20 --warmup 5 || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    run ${name}_${c} rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/$PROF/${name}_${c} -o pmc \
      -- python3 $R/bench.py --no-cpu-baseline --prof none $args --steps 3 --warmup 1 || exit 1
  done
done
