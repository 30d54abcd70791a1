#!/usr/bin/env python3
"""Config-5 kernel A/B (GPU): per-kernel HIP-event times of the source-side
partition of 64M 36-byte records with and without the fine-cell side field,
the one-pass partition (mgr_partition_onepass) and the destination-side
fine sort, for test-hook variants
(CF5_VARIANTS, JSON list, include/mgr_instrument.h; CF5_REPEAT interleaved
repeats).  Library builds are compared by scripts/gpu_libs_ab.sh."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402

N = int(os.environ.get("CF5_N", 1 << 26))
ITERS = int(os.environ.get("CF5_ITERS", 10))
KERNELS = ("bin_count", "bin_fine", "scan", "pack", "count_ids", "pack_fine", "pack_narrow",
           "onepass")


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(ITERS):
        fn()
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        fn()
    b.record()
    torch.cuda.synchronize()
    out = {"ms": round(a.elapsed_time(b) / ITERS, 4)}
    for k in KERNELS:
        ms, cnt = _lib.profile_read(k)
        if cnt:
            out[k] = round(ms / cnt * (cnt / ITERS), 4)   # per call of fn
    return out


def main():
    variants = json.loads(os.environ.get("CF5_VARIANTS", "[{}]"))
    repeat = int(os.environ.get("CF5_REPEAT", 1))
    rec, pos = mgr.synth_wide(N, seed=5)
    recv, rpos = mgr.synth_wide(N, seed=6, hi=0.5)
    part = mgr.GridPartitioner([2, 2, 2], [1.0] * 3)
    R1 = mgr.MPIGridRedistributor(None, [1, 1, 1], [0.5] * 3)
    _, fids, _ = mgr.GridPartitioner([1, 1, 1], [0.5] * 3).partition_device(
        recv.reshape(-1), 36, rpos, fine_cells=[8, 8, 8])
    fids = fids.clone()
    flat = rec.reshape(-1)
    for _ in range(repeat):
        for v in variants:
            for k, x in v.items():
                _lib.test_hook(k, x)
            res = {"variant": v,
                   "src_plain": timed(lambda: part.partition_device(flat, 36, pos)),
                   "src_fine": timed(lambda: part.partition_device(flat, 36, pos, fine_cells=[8, 8, 8])),
                   "src_onepass": timed(lambda: part.partition_onepass_device(
                       flat, 36, pos, fine_cells=[8, 8, 8])),
                   "src_onepass_plain": timed(lambda: part.partition_onepass_device(flat, 36, pos)),
                   "dst_sort": timed(lambda: R1.fine_cell_sort(recv, rpos, [8, 8, 8], fine_ids=fids))}
            print(json.dumps(res), flush=True)
            for k in v:
                _lib.test_hook(k, _lib.HOOK_DEFAULTS[k])


if __name__ == "__main__":
    main()
