#!/bin/bash
# GPU-box: fine-sort parity tests, then fine_bench A/B of the pack variants ($VARIANTS).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fine.py tests/test_gpu_parity.py tests/test_gpu_variants.py -k "fine or many or partition" -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fine.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_fine.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in "${VARIANTS[@]:-{\}}"; do :; done
done
python - <<'PY' >> gpurun_out/fine_ab2.log 2>&1
import json, os, subprocess
vs = json.loads(os.environ.get("VARIANTS_JSON", "[{}]"))
for rep in range(2):
    for v in vs:
        r = subprocess.run(["timeout", "-k", "10", "120", "python", "tools/fine_bench.py"],
                           env=dict(os.environ, FB_VARIANT=json.dumps(v)), capture_output=True, text=True)
        print(r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:], flush=True)
        if r.returncode:
            raise SystemExit(r.returncode)
PY
