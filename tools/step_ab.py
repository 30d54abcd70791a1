"""Step-level A/B of tuning knobs on BASELINE config 2 (bin + scan + pack of
2^26 uniform particles, 2x2x2): the whole step's time, so effects a kernel
has on the NEXT kernel (dirty lines it leaves in L2/MALL) show up, which the
per-kernel A/B (kbench.py) cannot see.  Interleaved repeats, median ms/step.
Usage: python tools/step_ab.py '[{"xcd_pack": 0}, {"xcd_bin": 1}]'"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402

variants = [{}] + json.loads(sys.argv[1] if len(sys.argv) > 1 else "[]")
steps, reps = 50, int(os.environ.get("AB_REPEAT", "5"))
n = 1 << 26
part = mgr.GridPartitioner([2, 2, 2], [1.0, 1.0, 1.0])
pos, rec = mgr.synth_uniform(n, seed=20261015, gid0=0)
flat = rec.reshape(-1)
_lib.tune("bin_skip_clean", 0)
res = {i: [] for i in range(len(variants))}
for rep in range(reps):
    for i, v in enumerate(variants):
        for k, x in v.items():
            _lib.tune(k, x)
        for _ in range(5):
            part.partition_device(flat, 32, pos)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            part.partition_device(flat, 32, pos)
        torch.cuda.synchronize()
        res[i].append((time.perf_counter() - t0) / steps * 1e3)
        for k in v:
            _lib.tune(k, {"xcd_bin": 0, "xcd_pack": 1, "bin_waves": 0}.get(k, 0))
    print("rep", rep, [round(res[i][-1], 4) for i in res], flush=True)
for i, v in enumerate(variants):
    r = sorted(res[i])
    print(json.dumps({"variant": v, "median_ms": r[len(r) // 2], "all": [round(x, 4) for x in res[i]]}))
