#!/usr/bin/env python3
"""Selection-pack microbenchmark (the halo's send selection, redist.py:271-275):
n rows, a fraction `frac` selected (2-bin partition, bin 1 dropped), one pack of
`rb`-byte rows per variant; per-kernel HIP-event times."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_grid_redistribute_amd import _lib  # noqa: E402
from mpi_grid_redistribute_amd.halo import DeviceSelect  # noqa: E402

N = int(os.environ.get("SB_N", 125_000_000))
FRAC = float(os.environ.get("SB_FRAC", 0.1))


def run(rb, variant, iters=10):
    for k, v in variant.items():
        _lib.tune(k, v)
    g = torch.Generator(device="cuda").manual_seed(1)
    flags = (torch.rand(N, generator=g, device="cuda") < FRAC).to(torch.int16)
    src = torch.randint(0, 256, (N * rb,), dtype=torch.uint8, device="cuda")
    sel = DeviceSelect(torch.device("cuda"))
    h, cnt = sel.select(flags, N, 1, rb)
    c = int(cnt.item())
    dst = torch.empty(max(c * rb, 1), dtype=torch.uint8, device="cuda")
    for _ in range(2):
        sel.pack(h, src, rb, dst)
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(iters):
        sel.pack(h, src, rb, dst)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    ms, k = _lib.profile_read("pack")
    ok = True
    if rb % 4 == 0:   # spot check: selected rows in order
        idx = torch.nonzero(flags != 0).flatten()[:1000]
        exp = src.view(-1, rb)[idx]
        ok = bool(torch.equal(dst.view(-1, rb)[:len(idx)], exp))
    for k2 in variant:
        _lib.tune(k2, {"pack_sel": 1, "pack_img": 1, "pack_compact": 1}[k2])
    return {"rb": rb, "variant": variant, "selected": c, "pack_ms": round(ms / k, 4), "ok": ok}


if __name__ == "__main__":
    for rb in (32, 24, 36):
        for v in ({}, {"pack_compact": 0}):
            print(json.dumps(run(rb, v)), flush=True)
