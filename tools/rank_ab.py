#!/usr/bin/env python3
"""rank_ids microbenchmark (GPU): mgr_rank_ids over RK_N uniform u16 ids in
[0, RK_BINS) (config 5's destination fine cells: 512), the 4096-row ranked
tiles, timed with HIP events over RK_ITERS launches; checks the slots against
a torch stable sort on the first tile.  Prints one JSON line.  Run under
rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS for the conflicts."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_grid_redistribute_amd import _lib  # noqa: E402
from mpi_grid_redistribute_amd.redistributor import _scratch  # noqa: E402

N = int(os.environ.get("RK_N", 1 << 26))
NB = int(os.environ.get("RK_BINS", 512))
ITERS = int(os.environ.get("RK_ITERS", 20))


def main():
    g = torch.Generator(device="cuda").manual_seed(5)
    ids = torch.randint(0, NB, (N,), device="cuda", generator=g, dtype=torch.int32).to(torch.int16)
    tr = int(_lib.load().mgr_ranked_tile_rows(36, NB))
    tile_rows, ws, _ = _scratch(N, NB, 36, torch.device("cuda"), dest=False, tile_rows=tr)
    T = (N + tile_rows - 1) // tile_rows
    ranks = torch.empty(N + 8, dtype=torch.int16, device="cuda")
    ts = torch.empty(T * NB * 4, dtype=torch.int16, device="cuda")
    s = _lib.stream_handle()

    def run():
        _lib.call("mgr_rank_ids", _lib.ptr(ids), N, NB, tile_rows, _lib.ptr(ranks), _lib.ptr(ts),
                  None, _lib.ptr(ws), s)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        run()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / ITERS
    # first tile: slot = position of the row in the tile's stable sort by id
    t0 = ids[:tile_rows].to(torch.int64)
    order = torch.sort(t0, stable=True).indices
    want = torch.empty_like(order)
    want[order] = torch.arange(tile_rows, device="cuda")
    ok = bool(torch.equal(ranks[:tile_rows].to(torch.int64) & 0xFFFF, want))
    print(json.dumps({"n": N, "bins": NB, "tile_rows": tile_rows, "ms": round(ms, 4),
                      "GBps_alg": round(N * 4 / ms / 1e6, 1), "first_tile_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
