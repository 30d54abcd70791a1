#!/bin/bash
# GPU-box: same-box A/B of source trees.  Each tools/ab/trees/<v>/ overlays
# files (relative paths) on a copy of this tree in /tmp/tree_<v>; the bench
# ($BENCH_ARGS) runs in each, alternating, $AB_REPS rounds, into $AB_LOG.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
LOG=gpurun_out/${AB_LOG:-tree_ab.log}
: > $LOG
for v in $TREES; do
  rm -rf /tmp/tree_$v && mkdir -p /tmp/tree_$v
  tar --exclude=./gpurun_out --exclude=./tools/ab -cf - . | tar -xf - -C /tmp/tree_$v
  cp -r tools/ab/trees/$v/. /tmp/tree_$v/
done
for rep in $(seq 1 ${AB_REPS:-3}); do
  for v in $TREES; do
    echo "lib=$v" >> $LOG
    (cd /tmp/tree_$v && timeout -k 10 200 python bench.py --no-cpu-baseline $BENCH_ARGS) >> $LOG 2>/dev/null || exit 1
  done
done
