#!/usr/bin/env python3
"""Time the destination-side fine-cell sort (BASELINE config 5 shape, one
GPU's share: 64M 36-byte records [pos f32x3, vel f32x3, mass f32, id i64]
inside rank 0's cell of a 2x2x2 grid, fine cells 8x8x8) with the per-kernel
HIP-event profiler."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402

N = int(os.environ.get("FB_N", 1 << 26))
ITERS = int(os.environ.get("FB_ITERS", 10))
FINE = json.loads(os.environ.get("FB_FINE", "[8, 8, 8]"))


def main():
    for k, v in json.loads(os.environ.get("FB_VARIANT", "{}")).items():
        _lib.tune(k, v)
    R = mgr.MPIGridRedistributor(None, [1, 1, 1], [0.5, 0.5, 0.5])  # rank 0's cell of 2x2x2
    g = torch.Generator(device="cuda").manual_seed(5)
    rec = torch.empty((N, 36), dtype=torch.uint8, device="cuda")
    f = rec.view(torch.float32)  # (N, 9)
    f[:, :3] = torch.rand((N, 3), generator=g, device="cuda") * 0.5
    f[:, 3:7] = torch.randn((N, 4), generator=g, device="cuda")
    ids = rec.view(torch.int32)  # id i64 at bytes 28..35: low and high words
    ids[:, 7] = torch.arange(N, device="cuda", dtype=torch.int32)
    ids[:, 8] = 0
    pos = f[:, :3]
    for _ in range(2):
        R.fine_cell_sort(rec, pos, FINE)
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        R.fine_cell_sort(rec, pos, FINE)
    b.record()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    out = {"n": N, "fine": FINE, "variant": json.loads(os.environ.get("FB_VARIANT", "{}")),
           "ms_per_sort": a.elapsed_time(b) / ITERS}
    for k in ("bin_count", "scan", "pack"):
        ms, cnt = _lib.profile_read(k)
        if cnt:
            out[k] = round(ms / cnt, 4)
    if "pack" in out:
        out["pack_GBps"] = round((2 * 36 + 2) * N / (out["pack"] / 1e3) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
