#!/bin/bash
# Run-to-run spread of the gather/scatter-heavy lines (halo, config 5): five
# runs each with torch's default caching allocator, then five with
# expandable segments (virtual-memory-mapped allocations).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=gpurun_out/alloc_variance.log
: > $L
for conf in default expandable; do
  for rep in 1 2 3 4 5; do
    for args in "--config 5" "--exchange --config 3 --overload 0.05"; do
      echo "conf=$conf args=$args" >> $L
      if [ $conf = expandable ]; then
        PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 200 python bench.py --no-cpu-baseline $args --steps 30 --warmup 10 >> $L 2>/dev/null || exit 1
      else
        timeout -k 10 200 python bench.py --no-cpu-baseline $args --steps 30 --warmup 10 >> $L 2>/dev/null || exit 1
      fi
    done
  done
done
