"""Pin the CPU oracle (NumPy + C restatements) against the reference's own outputs.

The fixtures were produced by running /root/reference/redist.py itself
(tests/golden/make_golden.py); these tests run anywhere (no reference, no GPU).
"""
import os

import numpy as np
import pytest

from oracle import c_oracle
from oracle import redist_oracle as ro
from tests import golden_io as G


# bin_edges: float32/float64 positions; bin_dtypes: int32/int64/float16
# positions (and float32 against narrow boxes) over every box dtype
@pytest.fixture(scope="module", params=["bin_edges.npz", "bin_dtypes.npz", "bin_dtype_edges.npz"])
def edges(request):
    return G.load(request.param)


def _box_for(f, key):
    return f[key + "_L"]


def test_bin_edges_numpy(edges):
    for key in G.bin_edge_keys(edges):
        n = int(edges[key + "_n"])
        box = _box_for(edges, key)
        periodic = not key.endswith("nonperiodic")
        geo = ro.Geometry([n], box, n)
        pos = edges[key + "_pos_in"].copy()
        p2 = pos.copy()
        with np.errstate(all="ignore"):
            idx = ro.cell_indexes_from_position(geo, p2, periodic)
            cell = ro.cell_number_from_position(geo, pos, periodic)
        assert G.same_bytes(pos, edges[key + "_pos_out"]), key
        assert np.array_equal(idx, edges[key + "_idx"]), key
        assert np.array_equal(cell, edges[key + "_cell"]), key


def test_bin_edges_c(edges):
    for key in G.bin_edge_keys(edges):
        n = int(edges[key + "_n"])
        box = _box_for(edges, key)
        periodic = not key.endswith("nonperiodic")
        pos = edges[key + "_pos_in"].copy()
        cell, idx = c_oracle.bin_positions(pos, [n], box, periodic=periodic, want_idx=True)
        assert G.same_bytes(pos, edges[key + "_pos_out"]), key
        assert np.array_equal(idx, edges[key + "_idx"]), key
        assert np.array_equal(cell, edges[key + "_cell"]), key


@pytest.mark.parametrize("case", G.redist_cases())
def test_redistribute_numpy(case):
    f = G.load(case)
    size = int(f["size"])
    topo, box, periodic = f["topology"], f["box"], bool(f["periodic"])
    pos = [p.copy() for p in G.per_rank(f, "pos_in", size)]
    if bool(f["alias"]):
        data = pos
    elif f["r0_data"].dtype.names and "pos" in f["r0_data"].dtype.names and "view" in case:
        data = [d.copy() for d in G.per_rank(f, "data", size)]
        pos = [d["pos"] for d in data]
    else:
        data = G.per_rank(f, "data", size)
    outs = ro.redistribute_by_position_all_ranks(topo, box, size, data, pos, periodic)
    for r in range(size):
        assert G.same_bytes(pos[r], f[f"r{r}_pos_out"]), (case, r)
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)


@pytest.mark.parametrize("case", G.redist_cases())
def test_redistribute_c(case):
    """C binning + C stable partition + source-ordered concat == reference."""
    f = G.load(case)
    size = int(f["size"])
    topo, box, periodic = f["topology"], f["box"], bool(f["periodic"])
    sends = []
    for r in range(size):
        pin = f[f"r{r}_pos_in"].copy()
        cell = c_oracle.bin_positions(pin, topo, box, periodic=periodic)
        assert G.same_bytes(pin, f[f"r{r}_pos_out"]), (case, r)
        assert np.array_equal(cell, f[f"r{r}_cell"]), (case, r)
        if bool(f["alias"]):
            data = pin
        elif "view" in case:
            data = f[f"r{r}_data"].copy()
            data["pos"] = pin
        else:
            data = f[f"r{r}_data"]
        part, off = c_oracle.partition(data, cell, size)
        sends.append([part[off[d]:off[d + 1]] for d in range(size)])
    for r in range(size):
        out = np.concatenate([sends[s][r] for s in range(size)])
        assert G.same_bytes(out, f[f"r{r}_out"]), (case, r)


def test_cell_number_redistribute():
    f = G.load("cellnum_p5_f32mat.npz")
    size = int(f["size"])
    outs = ro.redistribute_by_cell_number_all_ranks(size, G.per_rank(f, "data", size),
                                                    G.per_rank(f, "ids", size))
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"])


@pytest.mark.parametrize("case", G.soa_cases())
def test_soa_redistribute_numpy(case):
    """The multi-field (SoA) restatement == the reference's :157-164 pattern
    run on every field (make_golden.py make_soa)."""
    f = G.load(case)
    size = int(f["size"])
    fields, pos = G.soa_inputs(f, size)
    outs = ro.redistribute_fields_by_position_all_ranks(f["topology"], f["box"], size, fields,
                                                        pos, bool(f["periodic"]))
    for r in range(size):
        assert G.same_bytes(pos[r], f[f"r{r}_pos_out"]), (case, r)
        for i in range(int(f["nfields"])):
            assert G.same_bytes(outs[r][i], f[f"r{r}_f{i}_out"]), (case, r, i)


@pytest.mark.parametrize("case", G.soa_cases())
def test_soa_redistribute_c(case):
    """C binning once, C stable partition of every field, source-ordered
    concat == the reference's per-field outputs."""
    f = G.load(case)
    size = int(f["size"])
    nf, pf = int(f["nfields"]), int(f["pos_field"])
    sends = []
    for r in range(size):
        pin = f[f"r{r}_pos_in"].copy()
        cell = c_oracle.bin_positions(pin, f["topology"], f["box"], periodic=bool(f["periodic"]))
        assert G.same_bytes(pin, f[f"r{r}_pos_out"]), (case, r)
        assert np.array_equal(cell, f[f"r{r}_cell"]), (case, r)
        per = []
        for i in range(nf):
            part, off = c_oracle.partition(pin if i == pf else f[f"r{r}_f{i}_in"], cell, size)
            per.append([part[off[d]:off[d + 1]] for d in range(size)])
        sends.append(per)
    for r in range(size):
        for i in range(nf):
            out = np.concatenate([sends[s][i][r] for s in range(size)])
            assert G.same_bytes(out, f[f"r{r}_f{i}_out"]), (case, r, i)


def test_soa_cell_number():
    f = G.load("soa_cellnum_p5_three.npz")
    size, nf = int(f["size"]), int(f["nfields"])
    fields = [[f[f"r{r}_f{i}_in"] for i in range(nf)] for r in range(size)]
    outs = ro.redistribute_fields_by_cell_number_all_ranks(size, fields,
                                                           G.per_rank(f, "ids", size))
    for r in range(size):
        for i in range(nf):
            assert G.same_bytes(outs[r][i], f[f"r{r}_f{i}_out"]), (r, i)


def test_geometry():
    g = G.load("geometry.npz")
    i = 0
    while f"g{i}_size" in g:
        size = int(g[f"g{i}_size"])
        for r in range(size):
            geo = ro.Geometry(g[f"g{i}_topology"], g[f"g{i}_box"], size, r)
            assert np.array_equal(geo.cell_index_offset, g[f"g{i}_r{r}_offset"])
            assert G.same_bytes(geo.cell_length, g[f"g{i}_r{r}_cell_length"])
            assert np.array_equal(geo.rank_cell_index, g[f"g{i}_r{r}_rank_cell_index"])
            assert G.same_bytes(geo.rank_cell_limits, g[f"g{i}_r{r}_rank_cell_limits"])
            ncell = int(np.prod(geo.grid_topology))
            assert np.array_equal(ro.indexes_from_cell_number(geo, np.arange(ncell)),
                                  g[f"g{i}_r{r}_indexes_from_cell"])
            probe = np.array([[-1] * geo.dim, [3] * geo.dim, [0] * geo.dim])
            assert np.array_equal(ro.cell_number_from_indexes(geo, probe, periodic=False),
                                  g[f"g{i}_r{r}_cellnum_nonper"])
        i += 1
    assert i == 5


def test_synth_numpy_matches_c():
    p_np = ro.synth_uniform(20261015, 12345, 1000, 3, 1.0)
    p_c, ids = c_oracle.synth_uniform(20261015, 12345, 1000, 3, 1.0)
    assert G.same_bytes(p_np, p_c)
    assert np.array_equal(ids, np.arange(12345, 13345))
    assert p_np.min() >= 0 and p_np.max() < 1


def test_partition_matches_masks():
    rng = np.random.default_rng(1)
    data = rng.integers(0, 1 << 30, (5000, 3)).astype(np.int64)
    dest = rng.integers(-1, 9, 5000)
    out, off = c_oracle.partition(data, dest, 8)
    ref = np.concatenate(ro.stable_split(data, dest, 8))
    assert G.same_bytes(out, ref)
    out2, off2 = ro.stable_partition(data, dest, 8)
    assert G.same_bytes(out2, ref) and np.array_equal(off, off2)


# ------------------------------------------------- overload / halo (f1)
def _halo_cases():
    import glob
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(G.GOLDEN, "halo_*.npz")))


@pytest.mark.parametrize("case", _halo_cases())
def test_oracle_halo_matches_reference(case):
    """exchange_overload_by_position (redist.py:202-309) restated for all
    ranks at once, against the reference's own outputs."""
    f = G.load(case)
    size = int(f["size"])
    topo, box, ol = f["topology"], f["box"], list(f["overload"])
    data = G.per_rank(f, "data", size)
    if case.startswith("halo_direct_"):
        exp = ro.exchange_overload_all_ranks(topo, box, size, data, G.per_rank(f, "pos", size), ol,
                                             periodic=False)
    else:
        pos = [p.copy() for p in G.per_rank(f, "pos_in", size)]
        exp = ro.redistribute_by_position_overload_all_ranks(topo, box, size, data, pos, ol)
        for r in range(size):
            assert G.same_bytes(pos[r], f[f"r{r}_pos_out"]), (case, r)
    for r in range(size):
        assert G.same_bytes(exp[r], f[f"r{r}_out"]), (case, r)


# ------------------------------------------------- fine cells (f4, Cfg5)
@pytest.mark.parametrize("case", ["fine_p8_rec36_888.npz", "fine_p6_321_456.npz"])
def test_oracle_fine_cells_match_reference_binning(case):
    """Fine ids from the reference's own binning at topology*fine, and the
    stable argsort (SURVEY §8d Cfg5 oracle)."""
    f = G.load(case)
    size = int(f["size"])
    nfine = int(np.prod(f["fine"]))
    for r in range(size):
        d = f[f"r{r}_data"]
        pos = np.ascontiguousarray(d["pos"]) if d.dtype.names else f[f"r{r}_pos"]
        fid = ro.fine_cell_ids(f["topology"], f["fine"], f["box"], pos)
        assert np.array_equal(fid, f[f"r{r}_fine_id"]), (case, r)
        out, off = ro.fine_cell_sort(d, fid, nfine)
        assert G.same_bytes(out, f[f"r{r}_sorted"]), (case, r)
        assert off[-1] == len(d) and np.all(np.diff(off) == np.bincount(fid, minlength=nfine))


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("topo", [[2, 2, 2], [3, 1, 5], [7]])
def test_local_partition_omp_matches_serial(threads, topo):
    """The threaded host restatement (bench cpu_baseline_c) equals the serial
    C oracle: same wrapped positions, offsets and row order."""
    rng = np.random.default_rng(threads * 10 + len(topo))
    n = 20_011
    dim = len(topo)
    pos = rng.uniform(-1.5, 2.5, (n, dim))
    data = rng.integers(0, 256, (n, 20 if threads != 3 else 32), dtype=np.uint8)
    p1, p2 = pos.copy(), pos.copy()
    cell = c_oracle.bin_positions(p1, topo, [1.0] * dim)
    exp, exp_off = c_oracle.partition(data, cell, int(np.prod(topo)))
    got, off = c_oracle.local_partition_omp(p2, data, topo, [1.0] * dim, threads=threads)
    assert p1.tobytes() == p2.tobytes()
    assert np.array_equal(off, exp_off)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("boxdt", __import__("tests.dtype_cases", fromlist=["x"]).ALL_DTYPES,
                         ids=lambda d: np.dtype(d).name)
def test_c_oracle_every_dtype_pair_matches_numpy(boxdt):
    """All 12 x 12 (position, box) dtype pairs, 5k rows each: the C
    restatement (the GPU tests' large-N checker) equals the NumPy one, which
    runs the reference's own numpy expressions (redist.py:63-90, :328-329) --
    beyond the pairs the reference-run fixtures hold."""
    from tests.dtype_cases import ALL_DTYPES, dtype_case
    for dt in ALL_DTYPES:
        topo, box, pos = dtype_case(dt, boxdt, 5000)
        geo = ro.Geometry(topo, box, 30)
        for periodic in (True, False):
            p_np, p_c = pos.copy(), pos.copy()
            with np.errstate(all="ignore"):
                cell_np = ro.cell_number_from_position(geo, p_np, periodic)
            cell_c = c_oracle.bin_positions(p_c, topo, box, periodic=periodic)
            name = (np.dtype(dt).name, np.dtype(boxdt).name, periodic)
            assert G.same_bytes(p_c, p_np), name
            assert np.array_equal(cell_c, cell_np), name
