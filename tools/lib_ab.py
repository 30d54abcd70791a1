#!/usr/bin/env python3
"""Same-box A/B of two builds of libmgr.so (e.g. the round-1 library against
the current one) on the 1-GPU local stage, through the C ABI calls both
builds share (mgr_plan_create, mgr_partition_by_position, the profiler).
usage: python tools/lib_ab.py LIB [LIB ...]   (env AB_ITERS, AB_N)"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402  (inputs only)

N = int(os.environ.get("AB_N", 1 << 26))
ITERS = int(os.environ.get("AB_ITERS", 10))
P = ctypes.c_void_p


def bench(lib, pos, rec, rb, nbins=8, topo=(2, 2, 2)):
    L = ctypes.CDLL(lib)
    t = np.array(topo, dtype=np.int64)
    box = np.ones(3)
    h = P()
    assert L.mgr_plan_create(3, t.ctypes.data_as(P), box.ctypes.data_as(P), 2, nbins,
                             ctypes.byref(h)) == 0
    n = pos.shape[0]
    L.mgr_tile_rows.restype = ctypes.c_int
    L.mgr_workspace_bytes.restype = ctypes.c_int64
    tr = L.mgr_tile_rows(ctypes.c_int64(rb), nbins)
    ws = torch.empty(L.mgr_workspace_bytes(ctypes.c_int64(n), nbins, tr), dtype=torch.uint8,
                     device="cuda")
    dest = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = torch.empty(n * rb, dtype=torch.uint8, device="cuda")
    cnt = torch.empty(nbins, dtype=torch.int64, device="cuda")
    code = 1 if pos.dtype == torch.float32 else 2
    s = P(torch.cuda.current_stream().cuda_stream)
    L.mgr_tune(b"bin_skip_clean", ctypes.c_int64(0 if code == 2 else 1))

    def go():
        rc = L.mgr_partition_by_position(h, P(pos.data_ptr()), code, ctypes.c_int64(n),
                                         ctypes.c_int64(pos.stride(0)), 1, P(rec.data_ptr()),
                                         ctypes.c_int64(rb), P(out.data_ptr()),
                                         P(dest.data_ptr()), P(cnt.data_ptr()), tr,
                                         P(ws.data_ptr()), s)
        assert rc == 0
    for _ in range(3):
        go()
    torch.cuda.synchronize()
    L.mgr_profile_reset()
    L.mgr_profile_enable(1)
    for _ in range(ITERS):
        go()
    torch.cuda.synchronize()
    L.mgr_profile_enable(0)
    res = {}
    for k in ("bin_count", "scan", "pack"):
        ms, c = ctypes.c_double(), ctypes.c_int64()
        L.mgr_profile_read(k.encode(), ctypes.byref(ms), ctypes.byref(c))
        res[k] = round(ms.value / max(c.value, 1), 4)
    return res


def main():
    pos2, rec2 = mgr.synth_uniform(N, seed=1)
    rec5, pos5 = mgr.synth_wide(N, seed=3)
    for rep in range(int(os.environ.get("AB_REPEAT", 3))):
        for lib in sys.argv[1:]:
            r2 = bench(lib, pos2, rec2.reshape(-1), 32)
            r5 = bench(lib, pos5, rec5.reshape(-1), 36)
            print(json.dumps({"lib": os.path.basename(lib), "cfg2": r2, "cfg5_part": r5}),
                  flush=True)


if __name__ == "__main__":
    main()
