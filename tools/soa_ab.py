#!/usr/bin/env python3
"""SoA pack A/B (GPU): the same config-5 rows (64M: pos f32 x3, vel f32 x3,
mass f32, id i64 + the u16 fine id) partitioned into 8 destinations by
  * fields  -- ONE mgr_pack_fields launch for every field (the product path),
  * perfield -- one mgr_pack launch per field (each re-reads the destinations),
  * aos     -- the same bytes as one 36-byte record array (mgr_pack_ids),
  * copy    -- torch's device copy of the four arrays (a practical ceiling),
each timed with HIP events over ITERS launches after a warm-up, on one shared
binning/scan.  Also the destination-side ranked pack of every field (one
launch per field, mgr_pack_ranked) against the 36-byte record's.
Prints one JSON line."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402
from mpi_grid_redistribute_amd.redistributor import _i64s, _ptrs, _scratch  # noqa: E402

N = int(os.environ.get("AB_N", 1 << 26))
ITERS = int(os.environ.get("AB_ITERS", 10))


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / ITERS, 4)


def main():
    cfg2 = os.environ.get("AB_FIELDS", "cfg5") == "cfg2"   # config 2's f64 positions + ids
    if cfg2:
        rpos, rec = mgr.synth_uniform(N, seed=1)
        soa = (rpos.contiguous(), rec[:, 24:32].contiguous().view(torch.int64).reshape(-1))
        rbs, arb = [24, 8], 32
    else:
        soa = mgr.synth_wide_soa(N, seed=1)
        rec, rpos = mgr.synth_wide(N, seed=1)
        rbs, arb = [12, 12, 4, 8], 36
    flats = [t.reshape(-1).view(torch.uint8) for t in soa]
    P = mgr.GridPartitioner([2, 2, 2], [1.0] * 3)
    fplan = P._fine_plan([8, 8, 8])
    s = _lib.stream_handle()
    out = {}
    variants = json.loads(os.environ.get("AB_VARIANTS", '[[0, 0], [8, 2], [16, 2], [8, 3], [8, 1]]'))
    for rounds, img in variants:
        label = f"rounds{rounds}_kernel{img}"
        _lib.test_hook("tile_rounds", rounds)
        _lib.test_hook("fields_kernel", img)
        tr, ws, dest = _scratch(N, 8, 36, torch.device("cuda"))
        counts = torch.empty(8, dtype=torch.int64, device="cuda")
        fid = torch.empty(N, dtype=torch.int16, device="cuda")
        fido = torch.empty(N, dtype=torch.int16, device="cuda")
        if cfg2:
            _lib.call("mgr_bin_count", P._plan.h, _lib.ptr(soa[0]), _lib.MGR_F64, N, 3, 1,
                      _lib.ptr(dest), tr, _lib.ptr(ws), s)
        else:
            _lib.call("mgr_bin_count_fine", P._plan.h, fplan.h, _lib.ptr(soa[0]), _lib.MGR_F32, N,
                      3, 1, _lib.ptr(dest), _lib.ptr(fid), tr, _lib.ptr(ws), s)
        _lib.call("mgr_scan", N, 8, tr, _lib.ptr(ws), _lib.ptr(counts), s)
        outs = [torch.empty(N * b, dtype=torch.uint8, device="cuda") for b in rbs]
        o36 = torch.empty(N * arb, dtype=torch.uint8, device="cuda")

        side = (None, None) if cfg2 else (_lib.ptr(fid), _lib.ptr(fido))

        def fields():
            _lib.call("mgr_pack_fields", len(rbs), _ptrs([f.data_ptr() for f in flats]), _i64s(rbs),
                      N, _lib.ptr(dest), 8, -1, tr, _lib.ptr(ws),
                      _ptrs([o.data_ptr() for o in outs]), -1, None, side[0], side[1], None, 0, -1, s)

        def perfield():
            for i, (f, b, o) in enumerate(zip(flats, rbs, outs)):
                if i == 0 and not cfg2:
                    _lib.call("mgr_pack_ids", _lib.ptr(f), b, N, _lib.ptr(dest), 8, -1, tr,
                              _lib.ptr(ws), _lib.ptr(o), -1, None, _lib.ptr(fid), _lib.ptr(fido),
                              None, s)
                else:
                    _lib.call("mgr_pack", _lib.ptr(f), b, N, _lib.ptr(dest), 8, -1, tr,
                              _lib.ptr(ws), _lib.ptr(o), -1, None, s)

        def aos():
            if cfg2:
                _lib.call("mgr_pack", _lib.ptr(rec), arb, N, _lib.ptr(dest), 8, -1, tr,
                          _lib.ptr(ws), _lib.ptr(o36), -1, None, s)
            else:
                _lib.call("mgr_pack_ids", _lib.ptr(rec), arb, N, _lib.ptr(dest), 8, -1, tr,
                          _lib.ptr(ws), _lib.ptr(o36), -1, None, side[0], side[1], None, s)

        def copy():
            for f, o in zip(flats, outs):
                o.copy_(f)

        out[label] = {"tile_rows": tr, "fields": timed(fields), "aos": timed(aos)}
        if rounds == 0 and not img:
            out[label]["perfield"] = timed(perfield)
            out[label]["copy"] = timed(copy)
        # check: the multi-field pack == the per-field packs
        fields()
        ref = [o.clone() for o in outs]
        perfield()
        out[label]["fields_equal_perfield"] = all(torch.equal(a, b) for a, b in zip(ref, outs))
        del outs, o36
    _lib.test_hook("tile_rounds", 0)
    _lib.test_hook("fields_kernel", 0)
    if cfg2:
        print(json.dumps(out), flush=True)
        return
    # destination side: ranked pack per field vs the 36-byte record
    ids = fido[:N]
    R1 = mgr.MPIGridRedistributor(None, [1, 1, 1], [0.5] * 3)
    dst_soa = mgr.synth_wide_soa(N, seed=2, hi=0.5)
    drec, dpos = mgr.synth_wide(N, seed=2, hi=0.5)
    out["dest_sort_soa"] = timed(lambda: R1.fine_cell_sort(dst_soa, dst_soa[0], [8, 8, 8],
                                                           fine_ids=ids))
    out["dest_sort_aos"] = timed(lambda: R1.fine_cell_sort(drec, dpos, [8, 8, 8], fine_ids=ids))
    # the dest sort's kernels (library HIP events): a ranked pack launch per
    # field against the 36-byte record's one
    for label, fn in (("soa", lambda: R1.fine_cell_sort(dst_soa, dst_soa[0], [8, 8, 8],
                                                       fine_ids=ids)),
                      ("aos", lambda: R1.fine_cell_sort(drec, dpos, [8, 8, 8], fine_ids=ids))):
        fn()
        torch.cuda.synchronize()
        _lib.profile_enable(True)
        _lib.profile_reset()
        for _ in range(ITERS):
            fn()
        torch.cuda.synchronize()
        rec_k = {}
        for k in ("count_ids", "scan", "pack_fine"):
            ms, cnt = _lib.profile_read(k)
            if cnt:
                rec_k[k] = {"ms_per_call": round(ms / ITERS, 4), "launches_per_call": cnt / ITERS}
        _lib.profile_enable(False)
        out[f"dest_kernels_{label}"] = rec_k
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
