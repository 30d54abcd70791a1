"""Builder's probe: a one-bin stable pack (the one-rank redistribution's
identity copy, pack_coop through GridPartitioner([1,1,1])) against torch's
device-to-device copy of the same 125M x 32-byte rows.  Prints JSON (ms and
TB/s of the 2 x 4 GB moved; the pack also reads 125 MB of destination bytes)."""
import json
import time

import torch

import mpi_grid_redistribute_amd as mgr
from mpi_grid_redistribute_amd import _lib


def timeit(f, k=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3


def main():
    n = 125_000_000
    pos, rec = mgr.synth_uniform(n, seed=20261015, gid0=0)
    flat = rec.reshape(-1).view(torch.uint8)
    dst = torch.empty_like(flat)
    part = mgr.GridPartitioner([1, 1, 1], [1.0, 1.0, 1.0])
    _lib.load().mgr_profile_enable(1)
    res = {}
    for rep in range(3):
        _lib.load().mgr_profile_reset()
        step_ms = timeit(lambda: part.partition_device(flat, 32, pos))
        ms, cnt = _lib.profile_read("pack")
        res.setdefault("pack_kernel_ms", []).append(ms / max(cnt, 1))
        res.setdefault("partition_step_ms", []).append(step_ms)
        res.setdefault("torch_copy_ms", []).append(timeit(lambda: dst.copy_(flat)))
    gb = 2 * n * 32 / 1e9
    res["copy_TBps"] = [gb / m for m in res["torch_copy_ms"]]
    res["pack_TBps_rows_only"] = [gb / m for m in res["pack_kernel_ms"]]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
