#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Run in the survey container only (needs /root/reference, never on the GPU
box):   python tests/golden/make_golden.py [all|redist|halo|fine|dtypes|dtype_edges|soa]

How the reference is run (SURVEY.md §8c recipe; nothing is copied):
  * stub ``mpi4py`` / ``mpi4py.MPI`` modules are placed in ``sys.modules``
    (mpi4py is not installed here);
  * ``np.int = int`` and ``np.product = np.prod`` restore the two numpy<1.24
    aliases the reference uses (S14);
  * ``MPLBACKEND=Agg``;
  * ``/root/reference/redist.py`` is loaded read-only with importlib;
  * ranks run as threads on a fake communicator whose ``alltoall`` is a
    barrier-synchronised slot exchange returning a list indexed by source rank
    (mpi4py lowercase semantics, redist.py:199).

Each fixture is an .npz of inputs and the reference's outputs (data only):
per-rank positions before/after the call (the reference mutates them in place,
S1), the cell ids, and the per-rank redistributed data.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

# the reference is imported read-only: no bytecode cache is written next to
# /root/reference/redist.py (nothing under /root/reference is created)
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

REF_PATH = "/root/reference/redist.py"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(OUT_DIR))
from fake_mpi import run_ranks  # noqa: E402  (threaded mpi4py stand-in)


def load_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    mpi4py = types.ModuleType("mpi4py")
    mpi = types.ModuleType("mpi4py.MPI")
    mpi.COMM_WORLD = None
    mpi4py.MPI = mpi
    sys.modules["mpi4py"] = mpi4py
    sys.modules["mpi4py.MPI"] = mpi
    np.int = int  # noqa: S14 shim
    np.product = np.prod
    spec = importlib.util.spec_from_file_location("redist_reference", REF_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class SingleComm:
    """Rank 0 of a ``size``-rank world; binning needs no transport."""

    def __init__(self, size):
        self.size = size

    def Get_rank(self):
        return 0

    def Get_size(self):
        return self.size


def edge_values(L, rng):
    L = float(L)
    v = [0.0, -0.0, L, 2 * L, -L, -2 * L, np.nextafter(L, 0), np.nextafter(L, 2 * L),
         np.nextafter(0.0, 1.0), -np.nextafter(0.0, 1.0), 1e-300, -1e-300, 1e-10, -1e-10,
         0.49999999999999994 * L, 0.5 * L, 0.25 * L, -0.25 * L, -0.75 * L, 2.6 * L,
         L / 3, 2 * L / 3, 1e20, -1e20, 1e300, -1e300, np.nan, np.inf, -np.inf, 6 * L - 1e-9]
    v = np.array(v, dtype=np.float64)
    u = rng.uniform(-6 * L, 6 * L, 200)
    w = rng.uniform(0, L, 200)
    return np.concatenate([v, u, w])


def make_bin_edges(ref, rng):
    """Single-rank binning of edge values (S1-S3, S9-S11) over several (L, n)."""
    out = {}
    combos = [(1.0, 2), (1.0, 3), (0.3, 3), (62.5, 2), (1000.0, 3), (7.0, 3), (10.0, 7),
              (1e-3, 5), (3, 4)]  # (3, 4): integer box (S11a)
    for ci, (L, n) in enumerate(combos):
        vals = edge_values(L, rng)
        for mode in ("f64", "f32_boxf64", "f32_boxf32", "f64_nonperiodic", "f32_nonperiodic"):
            if isinstance(L, int) and mode == "f32_boxf32":
                continue
            pos_dtype = np.float64 if mode.startswith("f64") else np.float32
            periodic = not mode.endswith("nonperiodic")
            if mode == "f32_boxf32":
                box = np.array([L], dtype=np.float32)
            elif isinstance(L, int):
                box = [L]
            else:
                box = [L]
            with np.errstate(all="ignore"):
                pos = vals.astype(pos_dtype).reshape(-1, 1)
            pos_in = pos.copy()

            R = ref.MPIGridRedistributor(SingleComm(n), [n], box)
            p2 = pos.copy()
            with np.errstate(all="ignore"):
                idx = R.get_cell_indexes_from_position(p2, periodic=periodic)
                cell = R.get_cell_number_from_position(pos, periodic=periodic)
            key = f"c{ci}_{mode}"
            out[key + "_L"] = np.asarray(box)
            out[key + "_n"] = np.int64(n)
            out[key + "_pos_in"] = pos_in
            out[key + "_pos_out"] = pos
            out[key + "_idx"] = idx
            out[key + "_cell"] = cell
    np.savez_compressed(os.path.join(OUT_DIR, "bin_edges.npz"), **out)
    return len(out)


def rec32(pos, gid0):
    rec = np.zeros(len(pos), dtype=[("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])
    rec["x"], rec["y"], rec["z"] = pos[:, 0], pos[:, 1], pos[:, 2]
    rec["id"] = np.arange(gid0, gid0 + len(pos))
    return rec


def rec36(pos, rng, gid0):
    dt = np.dtype([("pos", "f4", 3), ("vel", "f4", 3), ("mass", "f4"), ("id", "i8")])
    assert dt.itemsize == 36
    rec = np.zeros(len(pos), dtype=dt)
    rec["pos"] = pos
    rec["vel"] = rng.normal(size=(len(pos), 3)).astype(np.float32)
    rec["mass"] = rng.uniform(1, 2, len(pos)).astype(np.float32)
    rec["id"] = np.arange(gid0, gid0 + len(pos))
    return rec


def positions(rng, n, dim, box, frac_out=0.05, dtype=np.float64):
    box = np.asarray(box, dtype=np.float64)
    p = rng.uniform(0, 1, (n, dim)) * box
    k = rng.random(n) < frac_out
    p[k] = rng.uniform(-2, 3, (int(k.sum()), dim)) * box
    return p.astype(dtype)


CASES = [
    # name, topology, box, size, dim, pos dtype, payload kind, periodic, alias
    ("p8_f64_rec32", [2, 2, 2], [1.0, 1.0, 1.0], 8, 3, np.float64, "rec32", True, False),
    ("p1_f64_rec32", [1, 1, 1], [1.0, 1.0, 1.0], 1, 3, np.float64, "rec32", True, False),
    ("p2_f32_rec36", [2, 1, 1], [1.0, 1.0, 1.0], 2, 3, np.float32, "rec36", True, False),
    ("p4_2d_intbox_mat", [2, 2], [10, 10], 4, 2, np.float64, "mat3", True, False),
    ("p27_333_ids", [3, 3, 3], [0.3, 62.5, 7.0], 27, 3, np.float64, "ids", True, False),
    ("p9_421_rec32", [4, 2, 1], [4.0, 2.0, 1.0], 9, 3, np.float64, "rec32", True, False),
    ("p4_f32box_rec36", [2, 2, 1], np.array([1.0, 2.0, 1.0], np.float32), 4, 3, np.float32,
     "rec36", True, False),
    ("p8_nonperiodic_rec32", [2, 2, 2], [1.0, 1.0, 1.0], 8, 3, np.float64, "rec32", False, False),
    ("p4_2d_alias", [2, 2], [10.0, 10.0], 4, 2, np.float64, "alias", True, False),
    ("p6_321_f32_mat", [3, 2, 1], [3.0, 2.0, 1.5], 6, 3, np.float32, "mat_i32", True, False),
    # Cfg5 shape: position is the strided f32 (N,3) view of a 36 B record (S9)
    ("p8_rec36_view", [2, 2, 2], [1.0, 1.0, 1.0], 8, 3, np.float32, "rec36_view", True, False),
]


def make_redistribute(ref, rng):
    n_files = 0
    for name, topo, box, size, dim, pdt, kind, periodic, _ in CASES:
        n_per = rng.integers(50, 400, size)
        pos_in, data_in = [], []
        gid = 0
        for r in range(size):
            p = positions(rng, int(n_per[r]), dim, box, dtype=pdt)
            if kind == "rec32":
                d = rec32(p.astype(np.float64), gid)
            elif kind in ("rec36", "rec36_view"):
                d = rec36(p, rng, gid)
            elif kind == "mat3":
                d = rng.normal(size=(len(p), 3))
            elif kind == "ids":
                d = np.arange(gid, gid + len(p), dtype=np.int64)
            elif kind == "mat_i32":
                d = rng.integers(-1000, 1000, (len(p), 5)).astype(np.int32)
            elif kind == "alias":
                d = None
            gid += len(p)
            pos_in.append(p)
            data_in.append(d)

        pos_work = [p.copy() for p in pos_in]
        data_work = [pos_work[r] if kind == "alias" else data_in[r] for r in range(size)]
        if kind == "rec36_view":
            data_work = [d.copy() for d in data_in]
            pos_work = [d["pos"] for d in data_work]
        cell_pos = [p.copy() for p in pos_in]

        def fn(comm, r):
            R = ref.MPIGridRedistributor(comm, topo, box)
            with np.errstate(all="ignore"):
                cell = R.get_cell_number_from_position(cell_pos[r], periodic=periodic)
                out = R.redistribute_by_position(data_work[r], pos_work[r], periodic=periodic)
            return cell, out

        res = run_ranks(size, fn)
        f = {"topology": np.asarray(topo, dtype=np.int64), "box": np.asarray(box),
             "size": np.int64(size), "periodic": np.bool_(periodic),
             "alias": np.bool_(kind == "alias")}
        for r in range(size):
            f[f"r{r}_pos_in"] = pos_in[r]
            f[f"r{r}_pos_out"] = pos_work[r]
            if kind != "alias":
                f[f"r{r}_data"] = data_in[r]
            f[f"r{r}_cell"] = res[r][0]
            f[f"r{r}_out"] = res[r][1]
        np.savez_compressed(os.path.join(OUT_DIR, f"redist_{name}.npz"), **f)
        n_files += 1

    # redistribute_by_cell_number with caller ids incl. out-of-range (S6)
    size = 5
    ids_in, data_in = [], []
    for r in range(size):
        n = int(rng.integers(30, 300))
        ids_in.append(rng.integers(-2, size + 3, n).astype(np.int64))
        data_in.append(rng.normal(size=(n, 3)).astype(np.float32))

    def fn2(comm, r):
        R = ref.MPIGridRedistributor(comm, [size], [1.0])
        return R.redistribute_by_cell_number(data_in[r], ids_in[r])

    res = run_ranks(size, fn2)
    f = {"size": np.int64(size)}
    for r in range(size):
        f[f"r{r}_ids"] = ids_in[r]
        f[f"r{r}_data"] = data_in[r]
        f[f"r{r}_out"] = res[r]
    np.savez_compressed(os.path.join(OUT_DIR, "cellnum_p5_f32mat.npz"), **f)
    n_files += 1

    # constructor geometry (redist.py:16-61) for a few topologies
    g = {}
    for i, (topo, box, size) in enumerate([([2, 2, 2], [1.0, 1.0, 1.0], 8),
                                           ([3, 3, 3], [0.3, 62.5, 7.0], 27),
                                           ([4, 2, 1], [4.0, 2.0, 1.0], 9),
                                           ([2.0, 2.0], [10, 40], 4), ([5], [2.5], 5)]):
        def fn3(comm, r, topo=topo, box=box):
            R = ref.MPIGridRedistributor(comm, topo, box)
            return (R.cell_index_offset.copy(), R.cell_length.copy(), R.rank_cell_index.copy(),
                    R.rank_cell_limits.copy(),
                    R.get_indexes_from_cell_number(np.arange(int(np.prod(topo)))),
                    R.get_cell_number_from_indexes(
                        np.array([[-1] * len(topo), [3] * len(topo), [0] * len(topo)]),
                        periodic=False))
        res = run_ranks(size, fn3)
        for r in range(size):
            for j, nm in enumerate(("offset", "cell_length", "rank_cell_index",
                                    "rank_cell_limits", "indexes_from_cell", "cellnum_nonper")):
                g[f"g{i}_r{r}_{nm}"] = res[r][j]
        g[f"g{i}_topology"] = np.asarray(topo)
        g[f"g{i}_box"] = np.asarray(box)
        g[f"g{i}_size"] = np.int64(size)
    np.savez_compressed(os.path.join(OUT_DIR, "geometry.npz"), **g)
    return n_files + 1


HALO_CASES = [
    # name, topology, box, dim, pos dtype, payload kind, overload_lengths
    ("p8_f64_rec32", [2, 2, 2], [1.0, 1.0, 1.0], 3, np.float64, "rec32", [0.1, 0.1, 0.1]),
    ("p4_2d_mat", [4, 1], [4.0, 1.0], 2, np.float64, "mat3", [0.3, 0.2]),
    ("p2_f32_rec36", [2, 1, 1], [1.0, 1.0, 1.0], 3, np.float32, "rec36", [0.05, 0.1, 0.2]),
    ("p27_333_ids", [3, 3, 3], [0.3, 62.5, 7.0], 3, np.float64, "ids", [0.05, 10.0, 3.0]),
    ("p8_wide", [2, 2, 2], [1.0, 1.0, 1.0], 3, np.float64, "rec32", [0.6, 0.3, 0.55]),
    ("p1_self", [1, 1, 1], [1.0, 1.0, 1.0], 3, np.float64, "rec32", [0.2, 0.1, 0.3]),
    ("p6_321_i32", [3, 2, 1], [3.0, 2.0, 1.5], 3, np.float32, "mat_i32", [0.2, 0.4, 0.1]),
]


def make_halo(ref, rng):
    """redistribute_by_position(..., overload_lengths=ol) (redist.py:161-166,
    :202-309, periodic); plus direct exchange_overload_by_position calls with
    periodic=False (the :287 flag quirk)."""
    n_files = 0
    for name, topo, box, dim, pdt, kind, ol in HALO_CASES:
        size = int(np.prod(topo))
        n_per = rng.integers(40, 300, size)
        pos_in, data_in = [], []
        gid = 0
        for r in range(size):
            p = positions(rng, int(n_per[r]), dim, box, dtype=pdt)
            if kind == "rec32":
                d = rec32(p.astype(np.float64), gid)
            elif kind == "rec36":
                d = rec36(p, rng, gid)
            elif kind == "mat3":
                d = rng.normal(size=(len(p), 3))
            elif kind == "ids":
                d = np.arange(gid, gid + len(p), dtype=np.int64)
            elif kind == "mat_i32":
                d = rng.integers(-1000, 1000, (len(p), 5)).astype(np.int32)
            gid += len(p)
            pos_in.append(p)
            data_in.append(d)
        pos_work = [p.copy() for p in pos_in]

        def fn(comm, r):
            R = ref.MPIGridRedistributor(comm, topo, box)
            with np.errstate(all="ignore"):
                return R.redistribute_by_position(data_in[r], pos_work[r], overload_lengths=ol)

        res = run_ranks(size, fn)
        f = {"topology": np.asarray(topo, dtype=np.int64), "box": np.asarray(box),
             "size": np.int64(size), "overload": np.asarray(ol, dtype=np.float64)}
        for r in range(size):
            f[f"r{r}_pos_in"] = pos_in[r]
            f[f"r{r}_pos_out"] = pos_work[r]
            f[f"r{r}_data"] = data_in[r]
            f[f"r{r}_out"] = res[r]
        np.savez_compressed(os.path.join(OUT_DIR, f"halo_{name}.npz"), **f)
        n_files += 1

    # direct calls, periodic=False: neighbours across the box edge get nothing,
    # and the left send uses the right neighbour's flag (redist.py:287)
    for name, topo, box, ol in [("p6_321_nonperiodic", [3, 2, 1], [3.0, 2.0, 1.5], [0.4, 0.3, 0.2]),
                                ("p8_nonperiodic", [2, 2, 2], [1.0, 1.0, 1.0], [0.2, 0.2, 0.2])]:
        size = int(np.prod(topo))
        pos_l, data_l = [], []

        def fn0(comm, r):
            R = ref.MPIGridRedistributor(comm, topo, box)
            return R.rank_cell_limits.copy()

        lims = run_ranks(size, fn0)
        for r in range(size):
            n = int(rng.integers(30, 200))
            lo, hi = lims[r][:, 0], lims[r][:, 1]
            p = lo + rng.random((n, len(topo))) * (hi - lo)
            pos_l.append(p)
            data_l.append(rng.normal(size=(n, 2)))

        def fn1(comm, r):
            R = ref.MPIGridRedistributor(comm, topo, box)
            return R.exchange_overload_by_position(data_l[r], pos_l[r], ol, periodic=False)

        res = run_ranks(size, fn1)
        f = {"topology": np.asarray(topo, dtype=np.int64), "box": np.asarray(box),
             "size": np.int64(size), "overload": np.asarray(ol, dtype=np.float64)}
        for r in range(size):
            f[f"r{r}_pos"] = pos_l[r]
            f[f"r{r}_data"] = data_l[r]
            f[f"r{r}_out"] = res[r]
        np.savez_compressed(os.path.join(OUT_DIR, f"halo_direct_{name}.npz"), **f)
        n_files += 1
    return n_files


def _ref_fine_ids(ref, topo, fine, box, pos):
    """Fine cell ids from the REFERENCE's binning at the global topology
    topo*fine (get_cell_number_from_position, redist.py:87-90, periodic=False:
    positions are already wrapped; the index wrap of :90 still applies), then
    decomposed and reduced to the index inside the rank's cell."""
    glob = [int(t) * int(f) for t, f in zip(topo, fine)]
    R = ref.MPIGridRedistributor(SingleComm(int(np.prod(glob))), glob, box)
    with np.errstate(all="ignore"):
        cell = R.get_cell_number_from_position(pos.copy(), periodic=False)
    fid = np.zeros(len(pos), dtype=np.int64)
    for d in range(len(glob)):
        k = (cell // R.cell_index_offset[d]) % glob[d]
        fid = fid * int(fine[d]) + k % int(fine[d])
    return fid


def make_fine(ref, rng):
    """SURVEY §8d Cfg5 oracle: the reference output followed by a stable
    argsort of the fine id (the reference has no fine sort of its own)."""
    n_files = 0
    # Cfg5 shape: the 2x2x2 redistribution of 36-byte records (f32 positions
    # as a view of the record), fine cells 8x8x8 inside each rank's cell
    f = np.load(os.path.join(OUT_DIR, "redist_p8_rec36_view.npz"), allow_pickle=False)
    size, topo, box, fine = int(f["size"]), f["topology"], f["box"], [8, 8, 8]
    g = {"topology": np.asarray(topo), "box": np.asarray(box), "size": np.int64(size),
         "fine": np.asarray(fine, dtype=np.int64)}
    for r in range(size):
        data = f[f"r{r}_out"]
        fid = _ref_fine_ids(ref, topo, fine, box, data["pos"])
        g[f"r{r}_data"] = data
        g[f"r{r}_fine_id"] = fid
        g[f"r{r}_sorted"] = data[np.argsort(fid, kind="stable")]
    np.savez_compressed(os.path.join(OUT_DIR, "fine_p8_rec36_888.npz"), **g)
    n_files += 1
    # non-power-of-two fine grid, f64 positions with the rows' own ids, 3x2x1
    size, topo, box, fine = 6, [3, 2, 1], [3.0, 2.0, 1.5], [4, 5, 6]

    def fn0(comm, r):
        return ref.MPIGridRedistributor(comm, topo, box).rank_cell_limits.copy()

    lims = run_ranks(size, fn0)
    g = {"topology": np.asarray(topo), "box": np.asarray(box), "size": np.int64(size),
         "fine": np.asarray(fine, dtype=np.int64)}
    for r in range(size):
        n = int(rng.integers(500, 3000))
        lo, hi = lims[r][:, 0], lims[r][:, 1]
        pos = lo + rng.random((n, 3)) * (hi - lo)
        pos[:5] = lo  # cell faces
        fid = _ref_fine_ids(ref, topo, fine, box, pos)
        data = np.arange(n, dtype=np.int64) + 100_000 * r
        g[f"r{r}_pos"] = pos
        g[f"r{r}_data"] = data
        g[f"r{r}_fine_id"] = fid
        g[f"r{r}_sorted"] = data[np.argsort(fid, kind="stable")]
    np.savez_compressed(os.path.join(OUT_DIR, "fine_p6_321_456.npz"), **g)
    return n_files + 1


BOX_KINDS = {  # how the caller spells box_length -> np.array(box_length) (redist.py:46)
    "f64": lambda L: [float(L)], "int": lambda L: [int(L)],
    "f32": lambda L: np.array([L], np.float32), "f16": lambda L: np.array([L], np.float16),
    "i8": lambda L: np.array([L], np.int8), "i16": lambda L: np.array([L], np.int16),
    "i32": lambda L: np.array([L], np.int32), "u32": lambda L: np.array([L], np.uint32),
    "u64": lambda L: np.array([L], np.uint64), "u8": lambda L: np.array([L], np.uint8),
    "b1": lambda L: np.array([bool(L)]),
}


def int_edge_values(L, rng, dt):
    if dt == np.bool_:
        return np.concatenate([np.array([False, True]), rng.random(40) < 0.5])
    info = np.iinfo(dt)
    L = int(L)
    v = [0, -1, 1, L - 1, L, L + 1, -L, -L + 1, 2 * L, -2 * L, 6 * L - 1, -6 * L + 1,
         info.min, info.max, info.min + 1, info.max - 1, 12345, -12345]
    if dt == np.int64:
        v += [2 ** 53 + 1, -(2 ** 53 + 1), 2 ** 62, -(2 ** 62), 2 ** 31, -(2 ** 31) - 1]
    v = [x for x in v if info.min <= x <= info.max]
    u = rng.integers(max(-6 * L, int(info.min)), min(6 * L, int(info.max)) + 1, 64)
    w = rng.integers(info.min, info.max, 32, dtype=dt, endpoint=True)
    return np.concatenate([np.array(v, dtype=dt), u.astype(dt), w])


def f16_edge_values(L, rng):
    h = np.float16(L)
    v = np.array([0.0, -0.0, h, 2 * h, -h, -2 * h, 0.5 * h, 0.25 * h, -0.25 * h, -0.75 * h,
                  2.6 * h, 65504.0, -65504.0, np.inf, -np.inf, np.nan, 1e-7, -1e-7,
                  6.0e-8, -6.0e-8, 1000.0, -1000.0], dtype=np.float16)
    near = np.array([np.nextafter(h, np.float16(0)), np.nextafter(h, np.float16(np.inf)),
                     np.nextafter(np.float16(0), np.float16(1))], dtype=np.float16)
    bits = np.array([0x7c01, 0xfc01, 0x7e00, 0xfe00, 0x7d55, 0x0001, 0x8001, 0x03ff, 0x0400],
                    dtype=np.uint16).view(np.float16)
    rnd = rng.integers(0, 1 << 16, 96).astype(np.uint16).view(np.float16)
    u = rng.uniform(-6 * float(L), 6 * float(L), 64).astype(np.float16)
    w = rng.uniform(0, float(L), 32).astype(np.float16)
    return np.concatenate([v, near, bits, rnd, u, w])


def make_bin_dtypes(ref, rng):
    """Single-rank binning of int32 / int64 / float16 positions -- and of
    float32 positions against the narrow boxes that keep numpy's arithmetic
    in float32 -- across box dtypes (numpy 2.2.6 promotion of :68-69)."""
    out = {}
    combos = [(10, 3), (7, 2), (64, 4), (100, 7), (1, 1), (2.5, 2), (0.3, 3), (1000.0, 5)]
    plan = {"i32": (np.int32, list(BOX_KINDS)), "i64": (np.int64, list(BOX_KINDS)),
            "f16": (np.float16, list(BOX_KINDS)),
            "f32": (np.float32, ["f16", "i8", "i16", "i32", "u32", "u64", "u8", "b1"]),
            "i8": (np.int8, list(BOX_KINDS)), "i16": (np.int16, list(BOX_KINDS)),
            "u8": (np.uint8, list(BOX_KINDS)), "u16": (np.uint16, list(BOX_KINDS)),
            "u32": (np.uint32, list(BOX_KINDS)), "u64": (np.uint64, list(BOX_KINDS)),
            "b1": (np.bool_, list(BOX_KINDS))}
    for ci, (L, n) in enumerate(combos):
        integral = float(L) == int(L)
        for pname, (pdt, boxes) in plan.items():
            for bk in boxes:
                if bk not in ("f64", "f32", "f16") and not integral:
                    continue
                if bk == "i8" and L > 127 or bk == "u8" and L > 255 or bk == "b1" and L != 1:
                    continue
                for periodic in (True, False):
                    box = BOX_KINDS[bk](L)
                    with np.errstate(all="ignore"):
                        if np.dtype(pdt).kind in "iub":
                            vals = int_edge_values(L, rng, pdt)
                        elif pdt == np.float16:
                            vals = f16_edge_values(L, rng)
                        else:
                            vals = edge_values(float(np.asarray(box, dtype=np.float64)[0]),
                                               rng).astype(np.float32)
                    pos = vals.reshape(-1, 1)
                    pos_in = pos.copy()
                    R = ref.MPIGridRedistributor(SingleComm(n), [n], box)
                    p2 = pos.copy()
                    with np.errstate(all="ignore"):
                        idx = R.get_cell_indexes_from_position(p2, periodic=periodic)
                        cell = R.get_cell_number_from_position(pos, periodic=periodic)
                    key = f"c{ci}_{pname}_box{bk}" + ("" if periodic else "_nonperiodic")
                    out[key + "_L"] = np.asarray(box)
                    out[key + "_n"] = np.int64(n)
                    out[key + "_pos_in"] = pos_in
                    out[key + "_pos_out"] = pos
                    out[key + "_idx"] = idx
                    out[key + "_cell"] = cell
    np.savez_compressed(os.path.join(OUT_DIR, "bin_dtypes.npz"), **out)
    return len(out)


def make_bin_dtype_edges(ref, rng):
    """Degenerate boxes for every non-float64 position dtype: float boxes 0,
    negative and +-inf (the float wrap gives NaN / out-of-range values that
    numpy's x86 casts write back into integer columns: cvttsd2si's INT_MIN,
    then the low bits), integer boxes 0 and negative (x % 0 == 0; floor-mod
    by a negative divisor), a float16 box 0 -- single-rank binning, n = 3."""
    out = {}
    boxes = {"f64_zero": [0.0], "f64_neg": [-2.5], "f64_inf": [np.inf], "f64_ninf": [-np.inf],
             "f32_inf": np.array([np.inf], np.float32), "int_zero": [0], "int_neg": [-3],
             "f16_zero": np.array([0.0], np.float16)}
    pdts = {"i8": np.int8, "i16": np.int16, "i32": np.int32, "i64": np.int64, "u8": np.uint8,
            "u16": np.uint16, "u32": np.uint32, "u64": np.uint64, "b1": np.bool_,
            "f16": np.float16, "f32": np.float32}
    n = 3
    for pname, pdt in pdts.items():
        for bname, box in boxes.items():
            for periodic in (True, False):
                with np.errstate(all="ignore"):
                    if np.dtype(pdt).kind in "iub":
                        vals = int_edge_values(3, rng, pdt)
                    elif pdt == np.float16:
                        vals = f16_edge_values(3.0, rng)
                    else:
                        vals = edge_values(3.0, rng).astype(np.float32)
                pos = vals.reshape(-1, 1)
                pos_in = pos.copy()
                R = ref.MPIGridRedistributor(SingleComm(n), [n], box)
                p2 = pos.copy()
                with np.errstate(all="ignore"):
                    idx = R.get_cell_indexes_from_position(p2, periodic=periodic)
                    cell = R.get_cell_number_from_position(pos, periodic=periodic)
                key = f"e_{pname}_box{bname}" + ("" if periodic else "_nonperiodic")
                out[key + "_L"] = np.asarray(box)
                out[key + "_n"] = np.int64(n)
                out[key + "_pos_in"] = pos_in
                out[key + "_pos_out"] = pos
                out[key + "_idx"] = idx
                out[key + "_cell"] = cell
    np.savez_compressed(os.path.join(OUT_DIR, "bin_dtype_edges.npz"), **out)
    return len(out)


DTYPE_CASES = [
    # name, topology, box, pos dtype, position range (in box units)
    ("p4_2d_i32pos_intbox", [2, 2], [100, 60], np.int32, (-1.5, 2.5)),
    ("p8_f16pos", [2, 2, 2], [1.0, 1.0, 1.0], np.float16, (-0.5, 1.5)),
    ("p2_i64pos_floatbox", [2, 1, 1], [2.5, 3.0, 1.5], np.int64, (-3.0, 4.0)),
    ("p4_f16pos_f16box", [2, 2, 1], np.array([1.0, 2.0, 1.0], np.float16), np.float16,
     (-0.3, 1.3)),
    ("p6_321_i64pos_intbox", [3, 2, 1], [30, 20, 10], np.int64, (-2.0, 3.0)),
    ("p2_u16pos_intbox", [2, 1, 1], [60, 30, 20], np.uint16, (0.0, 3.0)),
    ("p4_i8pos_f16box", [2, 2, 1], np.array([40.0, 20.0, 10.0], np.float16), np.int8, (-2.0, 3.0)),
]


def _dtype_positions(rng, n, box, pdt, lo_hi):
    b = np.asarray(box, dtype=np.float64)
    p = rng.uniform(lo_hi[0], lo_hi[1], (n, len(b))) * b
    if np.issubdtype(pdt, np.integer):
        p = np.floor(p * (1 if b.min() >= 10 else 4))   # integer grid positions
        info = np.iinfo(pdt)
        p = np.clip(p, info.min, info.max)
    return p.astype(pdt)


def make_dtypes(ref, rng):
    """Per-rank redistribution (and one halo case) of int32 / int64 / float16
    positions through the reference: the in-place wrap's cast back to the
    column (redist.py:68) and the binning of the stored values (:69)."""
    n_files = make_bin_dtypes(ref, rng) and 1
    for name, topo, box, pdt, lo_hi in DTYPE_CASES:
        size = int(np.prod(topo))
        pos_in, data_in = [], []
        gid = 0
        for r in range(size):
            n = int(rng.integers(50, 400))
            pos_in.append(_dtype_positions(rng, n, box, pdt, lo_hi))
            data_in.append(np.arange(gid, gid + n, dtype=np.int64))
            gid += n
        pos_work = [p.copy() for p in pos_in]
        cell_pos = [p.copy() for p in pos_in]

        def fn(comm, r):
            R = ref.MPIGridRedistributor(comm, topo, box)
            with np.errstate(all="ignore"):
                cell = R.get_cell_number_from_position(cell_pos[r])
                out = R.redistribute_by_position(data_in[r], pos_work[r])
            return cell, out

        res = run_ranks(size, fn)
        f = {"topology": np.asarray(topo, dtype=np.int64), "box": np.asarray(box),
             "size": np.int64(size), "periodic": np.bool_(True), "alias": np.bool_(False)}
        for r in range(size):
            f[f"r{r}_pos_in"] = pos_in[r]
            f[f"r{r}_pos_out"] = pos_work[r]
            f[f"r{r}_data"] = data_in[r]
            f[f"r{r}_cell"] = res[r][0]
            f[f"r{r}_out"] = res[r][1]
        np.savez_compressed(os.path.join(OUT_DIR, f"redist_{name}.npz"), **f)
        n_files += 1
    # halo with int32 positions: the float64 comparisons of :271-276
    topo, box, ol = [2, 2, 1], [100, 100, 10], [6.5, 12.0, 1.0]
    size = 4
    pos_in, data_in = [], []
    for r in range(size):
        n = int(rng.integers(60, 300))
        pos_in.append(_dtype_positions(rng, n, box, np.int32, (-0.2, 1.2)))
        data_in.append(rng.normal(size=(n, 2)))
    pos_work = [p.copy() for p in pos_in]

    def fnh(comm, r):
        R = ref.MPIGridRedistributor(comm, topo, box)
        with np.errstate(all="ignore"):
            return R.redistribute_by_position(data_in[r], pos_work[r], overload_lengths=ol)

    res = run_ranks(size, fnh)
    f = {"topology": np.asarray(topo, dtype=np.int64), "box": np.asarray(box),
         "size": np.int64(size), "overload": np.asarray(ol, dtype=np.float64)}
    for r in range(size):
        f[f"r{r}_pos_in"] = pos_in[r]
        f[f"r{r}_pos_out"] = pos_work[r]
        f[f"r{r}_data"] = data_in[r]
        f[f"r{r}_out"] = res[r]
    np.savez_compressed(os.path.join(OUT_DIR, "halo_p4_i32pos.npz"), **f)
    return n_files + 1


SOA_CASES = [
    # name, topology, box, pos dtype, periodic, fields (pos = the position
    # array itself moves as field 0), empty ranks
    ("p8_cfg5_soa", [2, 2, 2], [1.0, 1.0, 1.0], np.float32, True,
     ["pos", "vel_f32x3", "mass_f32", "id_i64"], ()),
    ("p4_f64_two_fields_empty", [2, 2, 1], [1.0, 2.0, 1.0], np.float64, True,
     ["id_i64", "mat_f64x3"], (2,)),
    ("p6_321_nonperiodic_mixed", [3, 2, 1], [3.0, 2.0, 1.5], np.float64, False,
     ["pos", "vel_f32x3", "id_i32", "flag_u8", "tri_i16x3", "rec32"], ()),
    ("p2_f32_intbox_three", [2, 1, 1], [4, 2, 2], np.float32, True,
     ["mass_f32", "pos", "id_i64"], (1,)),
]


def soa_field(kind, pos, rng, gid0):
    n = len(pos)
    if kind == "pos":
        return pos
    if kind == "vel_f32x3":
        return rng.normal(size=(n, 3)).astype(np.float32)
    if kind == "mass_f32":
        return rng.uniform(1, 2, n).astype(np.float32)
    if kind == "id_i64":
        return np.arange(gid0, gid0 + n, dtype=np.int64)
    if kind == "id_i32":
        return np.arange(gid0, gid0 + n, dtype=np.int32)
    if kind == "mat_f64x3":
        return rng.normal(size=(n, 3))
    if kind == "flag_u8":
        return rng.integers(0, 256, n).astype(np.uint8)
    if kind == "tri_i16x3":
        return rng.integers(-30000, 30000, (n, 3)).astype(np.int16)
    if kind == "rec32":
        return rec32(pos.astype(np.float64), gid0)
    raise ValueError(kind)


def make_soa(ref, rng):
    """SoA payloads -- several arrays sharing axis 0 -- through the
    REFERENCE's own multi-field pattern (redist.py:157-164): the destinations
    are binned ONCE from the positions (get_cell_number_from_position, which
    wraps them in place, :157), then every field is redistributed with that
    same rank_to_send (redistribute_by_cell_number, :160 for data, :164 for
    position).  A field named "pos" is the position array itself (its
    wrapped values travel).  Plus a caller-ids case (:169-200, out-of-range
    ids dropped) with three fields."""
    n_files = 0
    for name, topo, box, pdt, periodic, kinds, empty in SOA_CASES:
        size = int(np.prod(topo))
        pos_in, fields_in = [], []
        gid = 0
        for r in range(size):
            n = 0 if r in empty else int(rng.integers(60, 400))
            p = positions(rng, n, len(topo), box, dtype=pdt)
            pos_in.append(p)
            fields_in.append([soa_field(k, p, rng, gid) for k in kinds])
            gid += n
        pos_work = [p.copy() for p in pos_in]
        work = [[pos_work[r] if k == "pos" else f for k, f in zip(kinds, fields_in[r])]
                for r in range(size)]

        def fn(comm, r):
            R = ref.MPIGridRedistributor(comm, topo, box)
            with np.errstate(all="ignore"):
                rank_to_send = R.get_cell_number_from_position(pos_work[r], periodic=periodic)
                return rank_to_send, [R.redistribute_by_cell_number(f, rank_to_send)
                                      for f in work[r]]

        res = run_ranks(size, fn)
        f = {"topology": np.asarray(topo, dtype=np.int64), "box": np.asarray(box),
             "size": np.int64(size), "periodic": np.bool_(periodic),
             "nfields": np.int64(len(kinds)),
             "pos_field": np.int64(kinds.index("pos") if "pos" in kinds else -1)}
        for r in range(size):
            f[f"r{r}_pos_in"] = pos_in[r]
            f[f"r{r}_pos_out"] = pos_work[r]
            f[f"r{r}_cell"] = res[r][0]
            for i in range(len(kinds)):
                f[f"r{r}_f{i}_in"] = fields_in[r][i] if kinds[i] != "pos" else pos_in[r]
                f[f"r{r}_f{i}_out"] = res[r][1][i]
        np.savez_compressed(os.path.join(OUT_DIR, f"soa_{name}.npz"), **f)
        n_files += 1

    # caller ids (redistribute_by_cell_number), three fields, ids out of range
    size = 5
    ids_in, fields_in = [], []
    for r in range(size):
        n = 0 if r == 3 else int(rng.integers(30, 300))
        ids_in.append(rng.integers(-2, size + 3, n).astype(np.int64))
        fields_in.append([rng.normal(size=(n, 3)).astype(np.float32),
                          np.arange(n, dtype=np.int64) + 1000 * r,
                          rng.integers(0, 1 << 16, n).astype(np.uint16)])

    def fn2(comm, r):
        R = ref.MPIGridRedistributor(comm, [size], [1.0])
        return [R.redistribute_by_cell_number(x, ids_in[r]) for x in fields_in[r]]

    res = run_ranks(size, fn2)
    f = {"size": np.int64(size), "nfields": np.int64(3)}
    for r in range(size):
        f[f"r{r}_ids"] = ids_in[r]
        for i in range(3):
            f[f"r{r}_f{i}_in"] = fields_in[r][i]
            f[f"r{r}_f{i}_out"] = res[r][i]
    np.savez_compressed(os.path.join(OUT_DIR, "soa_cellnum_p5_three.npz"), **f)
    return n_files + 1


def main():
    ref = load_reference()
    only = sys.argv[1] if len(sys.argv) > 1 else "all"
    if only in ("all", "dtypes"):
        d = make_dtypes(ref, np.random.default_rng(20261018))
        print(f"position-dtype fixtures: {d}")
    if only in ("all", "redist"):
        rng = np.random.default_rng(20261015)
        a = make_bin_edges(ref, rng)
        b = make_redistribute(ref, rng)
        print(f"bin_edges arrays: {a}; redistribute fixtures: {b}")
    if only in ("all", "halo"):
        c = make_halo(ref, np.random.default_rng(20261016))
        print(f"halo fixtures: {c}")
    if only in ("all", "fine"):
        e = make_fine(ref, np.random.default_rng(20261017))
        print(f"fine-cell fixtures: {e}")
    if only in ("all", "dtype_edges"):
        k = make_bin_dtype_edges(ref, np.random.default_rng(20261020))
        print(f"degenerate-box dtype arrays: {k}")
    if only in ("all", "soa"):
        g = make_soa(ref, np.random.default_rng(20261019))
        print(f"SoA fixtures: {g}")


if __name__ == "__main__":
    main()
