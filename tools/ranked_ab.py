#!/usr/bin/env python3
"""Ranked-pack occupancy A/B (GPU): config 5's destination-side fine-cell sort
of 64M 36-byte records (8x8x8 cells) with
  * t4096_cu1 -- 4096-row tiles, one 1024-thread workgroup per CU (the product),
  * t2048_cu1 -- 2048-row tiles, one per CU,
  * t2048_cu2 -- 2048-row tiles, two per CU (hook ranked_per_cu; <= 64 VGPRs),
alternating, each timed by the library's HIP events (count_ids / scan /
pack_fine per call) and end to end; every variant's output must equal the
product's.  Prints one JSON line.
Record of a round-6 A/B (profiles/round6/ranked_ab.json: two per CU took the
pack from 1.02 to 1.49 ms); the ranked_per_cu hook and its kernel instance
were removed with the result, so t2048_cu2 now needs them put back."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402

N = int(os.environ.get("AB_N", 1 << 26))
ITERS = int(os.environ.get("AB_ITERS", 10))
VARIANTS = {"t4096_cu1": (0, 1), "t2048_cu1": (2048, 1), "t2048_cu2": (2048, 2)}


def main():
    R1 = mgr.MPIGridRedistributor(None, [1, 1, 1], [0.5] * 3)
    drec, dpos = mgr.synth_wide(N, seed=2, hi=0.5)
    out, ref = {}, None
    for rep in range(2):
        for label, (rows, per_cu) in VARIANTS.items():
            _lib.test_hook("rank_rows", rows)
            _lib.test_hook("ranked_per_cu", per_cu)
            fn = lambda: R1.fine_cell_sort(drec, dpos, [8, 8, 8])  # noqa: E731
            res = fn()
            torch.cuda.synchronize()
            got = res[0] if isinstance(res, tuple) else res
            if ref is None:
                ref = got.clone()
            same = bool(torch.equal(ref, got))
            del res, got
            _lib.profile_enable(True)
            _lib.profile_reset()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(ITERS):
                fn()
            b.record()
            torch.cuda.synchronize()
            rec = {"call_ms": round(a.elapsed_time(b) / ITERS, 4), "equal_to_product": same}
            for k in ("count_ids", "scan", "pack_fine"):
                ms, cnt = _lib.profile_read(k)
                if cnt:
                    rec[k] = round(ms / cnt, 4)
            _lib.profile_enable(False)
            out.setdefault(label, []).append(rec)
    _lib.test_hook("rank_rows", 0)
    _lib.test_hook("ranked_per_cu", 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
