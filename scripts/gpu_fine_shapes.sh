#!/bin/bash
# GPU-box: full GPU tests, then the fine-cell sort at several cell counts for
# the shipped default and each FB_VARIANTS entry (tools/fine_bench.py).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/fine_shapes.log
python3 -c 'import json,os; [print(json.dumps(v)) for v in json.loads(os.environ["FB_VARIANTS"])]' > /tmp/fb_variants.txt || exit 1
for fine in "[8, 8, 8]" "[4, 5, 6]" "[8, 8, 16]" "[4, 4, 8]"; do
  while read -r v; do
    FB_FINE="$fine" FB_VARIANT="$v" timeout -k 10 120 python -u tools/fine_bench.py >> gpurun_out/fine_shapes.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "fine_bench rc=$rc ($fine $v)" >> gpurun_out/fine_shapes.log; exit $rc; fi
  done < /tmp/fb_variants.txt
done
