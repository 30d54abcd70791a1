"""Helpers to read the golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
from __future__ import annotations

import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def redist_cases():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "redist_*.npz")))


def halo_cases():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "halo_p*.npz")))


def halo_direct_cases():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "halo_direct_*.npz")))


def soa_cases():
    """SoA fixtures of the position path (make_golden.py make_soa)."""
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "soa_p*.npz")))


def soa_inputs(f, size, as_torch=False):
    """Per-rank (fields, position) of a soa_* fixture: numpy copies, or GPU
    torch tensors; the field at ``pos_field`` is the position array itself
    (the same object / tensor, so its wrapped values travel)."""
    nf, pf = int(f["nfields"]), int(f["pos_field"])
    fields, pos = [], []
    for r in range(size):
        p = f[f"r{r}_pos_in"].copy()
        fl = [p if i == pf else f[f"r{r}_f{i}_in"].copy() for i in range(nf)]
        if as_torch:
            import torch
            tp = torch.from_numpy(p).cuda()
            tl = []
            for i, x in enumerate(fl):
                if i == pf:
                    tl.append(tp)
                    continue
                if x.dtype.names:
                    x = x.view(np.uint8).reshape(len(x), -1)
                tl.append(torch.from_numpy(np.ascontiguousarray(x)).cuda())
            fl, p = tl, tp
        fields.append(fl)
        pos.append(p)
    return fields, pos


def fixture_inputs(f, case, size, as_torch):
    """Per-rank (data, position) inputs of a redist_* fixture: numpy copies, or
    GPU torch tensors with the same aliasing (position = data, or a view of
    the records' pos field)."""
    pos = [p.copy() for p in per_rank(f, "pos_in", size)]
    if bool(f["alias"]):
        data = pos
    elif "view" in case:
        data = [d.copy() for d in per_rank(f, "data", size)]
        pos = [d["pos"] for d in data]
    else:
        data = [d.copy() for d in per_rank(f, "data", size)]
    if not as_torch:
        return data, pos
    import torch
    tdata, tpos = [], []
    for r in range(size):
        if bool(f["alias"]):
            t = torch.from_numpy(pos[r]).cuda()
            tdata.append(t)
            tpos.append(t)
        elif "view" in case:
            raw = torch.from_numpy(data[r].view(np.uint8).reshape(len(data[r]), -1)).cuda()
            tdata.append(raw)
            tpos.append(raw.view(torch.float32)[:, :3])
        else:
            d = data[r]
            if d.dtype.names:
                d = d.view(np.uint8).reshape(len(d), -1)
            tdata.append(torch.from_numpy(np.ascontiguousarray(d)).cuda())
            tpos.append(torch.from_numpy(pos[r]).cuda())
    return tdata, tpos


def bin_edge_keys(f):
    return sorted({k[: k.rindex("_pos_in")] for k in f.keys() if k.endswith("_pos_in")})


def per_rank(f, key, size):
    return [f[f"r{r}_{key}"] for r in range(size)]


def same_bytes(a, b):
    """Bit-exact comparison (NaN-safe): dtype, shape and raw bytes."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and a.tobytes() == b.tobytes()


def diff_report(a, b, limit=8):
    """First differing elements of two same-shape arrays, as hex bit patterns."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return f"shape/dtype {a.shape} {a.dtype} vs {b.shape} {b.dtype}"
    ua = a.view(np.uint8).reshape(len(a), -1) if a.ndim else a.view(np.uint8)
    ub = b.view(np.uint8).reshape(len(b), -1) if b.ndim else b.view(np.uint8)
    rows = np.nonzero((ua != ub).any(axis=1))[0]
    out = [f"{len(rows)} differing rows"]
    for r in rows[:limit]:
        out.append(f"row {r}: {a[r]!r} [{ua[r].tobytes().hex()}] vs {b[r]!r} "
                   f"[{ub[r].tobytes().hex()}]")
    return "\n".join(out)
