#!/bin/bash
# GPU-box: fine-sort (512-cell pack) breakdown -- FB_VARIANTS is a list of
# tuning dicts, each timed by tools/fine_bench.py in its own process.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/fine_diag.log
python3 -c 'import json,os; [print(json.dumps(v)) for v in json.loads(os.environ["FB_VARIANTS"])]' > /tmp/fb_variants.txt || exit 1
for rep in 1 2; do
  while read -r v; do
    FB_VARIANT="$v" timeout -k 10 120 python -u tools/fine_bench.py >> gpurun_out/fine_diag.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "fine_bench rc=$rc ($v)" >> gpurun_out/fine_diag.log; exit $rc; fi
  done < /tmp/fb_variants.txt
done
