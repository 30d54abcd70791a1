#!/usr/bin/env python3
"""Time GridPartitioner.partition_device on BASELINE config-5 rows (64M 36-byte
records, f32 positions viewed in the records, 2x2x2) with and without the
source-side fine cells (fine_cells=[8,8,8]), per kernel (HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402

N = int(os.environ.get("PB_N", 1 << 26))
ITERS = int(os.environ.get("PB_ITERS", 10))


def run(fine):
    rec, pos = mgr.synth_wide(N, seed=3)
    P = mgr.GridPartitioner([2, 2, 2], [1.0] * 3)
    flat = rec.reshape(-1)
    for _ in range(2):
        P.partition_device(flat, 36, pos, fine_cells=fine)
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        P.partition_device(flat, 36, pos, fine_cells=fine)
    b.record()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    out = {"n": N, "fine": fine, "variant": json.loads(os.environ.get("PB_VARIANT", "{}")),
           "ms": a.elapsed_time(b) / ITERS}
    for k in _lib.PROFILE_KERNELS:
        ms, cnt = _lib.profile_read(k)
        if cnt:
            out[k] = round(ms / cnt, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for k, v in json.loads(os.environ.get("PB_VARIANT", "{}")).items():
        _lib.tune(k, v)
    run(None)
    run([8, 8, 8])
