"""GPU parity of the destination-side fine-cell sort (SURVEY §8d config 5,
§8f f4): mgr_plan_create_fine + mgr_bin_count + mgr_scan + mgr_pack, bit-exact
against the reference's binning at topology*fine plus a stable argsort
(tests/golden/fine_*.npz) and the C oracle at larger sizes."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import redist_oracle as ro
from tests import golden_io as G
from tests.fake_mpi import run_ranks

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import MPIGridRedistributor, _lib  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _redistributors(f):
    size = int(f["size"])
    return run_ranks(size, lambda comm, r: MPIGridRedistributor(comm, f["topology"], f["box"]))


@pytest.mark.parametrize("as_torch", [False, True])
def test_fine_golden_rec36_view(as_torch):
    """Cfg5 layout: 36-byte records, positions = the f32 view of the record."""
    f = G.load("fine_p8_rec36_888.npz")
    Rs = _redistributors(f)
    nfine = int(np.prod(f["fine"]))
    for r, R in enumerate(Rs):
        d = f[f"r{r}_data"].copy()
        if as_torch:
            raw = torch.from_numpy(d.view(np.uint8).reshape(len(d), 36)).cuda()
            out, off = R.fine_cell_sort(raw, raw.view(torch.float32)[:, :3], f["fine"])
            got = out.cpu().numpy().reshape(-1).view(d.dtype)
            off = off.cpu().numpy()
        else:
            got, off = R.fine_cell_sort(d, d["pos"], f["fine"])
        assert G.same_bytes(got, f[f"r{r}_sorted"]), r
        assert G.same_bytes(d, f[f"r{r}_data"]), r          # input untouched
        assert np.array_equal(np.diff(off), np.bincount(f[f"r{r}_fine_id"], minlength=nfine))


def test_fine_golden_456_with_positions():
    f = G.load("fine_p6_321_456.npz")
    Rs = _redistributors(f)
    for r, R in enumerate(Rs):
        pos = f[f"r{r}_pos"]
        got, gpos, off = R.fine_cell_sort(f[f"r{r}_data"], pos, f["fine"], return_positions=True)
        assert G.same_bytes(got, f[f"r{r}_sorted"]), r
        order = np.argsort(f[f"r{r}_fine_id"], kind="stable")
        assert G.same_bytes(gpos, pos[order]), r


@pytest.mark.parametrize("fine", [[8, 8, 8], [16, 16, 16], [2, 3, 4], [1, 1, 64]])
def test_fine_large_vs_c_oracle(fine):
    """1M rows of one rank's cell (2x2x2 grid, rank 5), 36-byte records."""
    rng = np.random.default_rng(sum(fine))
    topo, box = [2, 2, 2], [1.0, 1.0, 1.0]
    R = run_ranks(8, lambda comm, r: MPIGridRedistributor(comm, topo, box) if r == 5 else None)[5]
    n = 1_000_003
    lo, hi = R.rank_cell_limits[:, 0], R.rank_cell_limits[:, 1]
    dt = np.dtype([("pos", "f4", 3), ("vel", "f4", 3), ("mass", "f4"), ("id", "i8")])
    rec = np.zeros(n, dtype=dt)
    rec["pos"] = (lo + rng.random((n, 3)) * (hi - lo)).astype(np.float32)
    rec["id"] = np.arange(n)
    glob = [t * k for t, k in zip(topo, fine)]
    pos = np.ascontiguousarray(rec["pos"])
    _, idx = c_oracle.bin_positions(pos.copy(), glob, box, periodic=False, want_idx=True)
    k = ro.periodic_wrap(idx, np.array(glob)) % np.array(fine)
    fid = (k[:, 0] * fine[1] + k[:, 1]) * fine[2] + k[:, 2]
    exp, exp_off = c_oracle.partition(rec, fid, int(np.prod(fine)))
    t = torch.from_numpy(rec.view(np.uint8).reshape(n, 36).copy()).cuda()
    out, off = R.fine_cell_sort(t, t.view(torch.float32)[:, :3], fine)
    assert np.array_equal(off.cpu().numpy(), exp_off)
    assert out.cpu().numpy().tobytes() == exp.tobytes()


def test_fine_after_redistribution_golden():
    """redistribute_by_position then fine_cell_sort == the Cfg5 pipeline on
    the reference's own redistribution fixture."""
    f = G.load("redist_p8_rec36_view.npz")
    fine = G.load("fine_p8_rec36_888.npz")
    size = int(f["size"])
    data = [d.copy() for d in G.per_rank(f, "data", size)]

    def fn(comm, r):
        R = MPIGridRedistributor(comm, f["topology"], f["box"])
        local = R.redistribute_by_position(data[r], data[r]["pos"])
        return R.fine_cell_sort(local, local["pos"], [8, 8, 8])[0]

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], fine[f"r{r}_sorted"]), r


# ------------------------------------------- fine cells binned at the source
def test_fused_fine_redistribution_golden():
    """redistribute_by_position(..., fine_cells) -- fine cells computed by the
    source's bin kernel, exchanged as a 2-byte field, rows sorted by them at
    the destination -- == redistribution then fine_cell_sort, on the
    reference's own fixtures (the Cfg5 pipeline)."""
    f = G.load("redist_p8_rec36_view.npz")
    fine = G.load("fine_p8_rec36_888.npz")
    size = int(f["size"])
    data = [d.copy() for d in G.per_rank(f, "data", size)]

    def fn(comm, r):
        R = MPIGridRedistributor(comm, f["topology"], f["box"])
        return R.redistribute_by_position(data[r], data[r]["pos"], fine_cells=[8, 8, 8])

    outs = run_ranks(size, fn)
    for r in range(size):
        got, off = outs[r]
        assert G.same_bytes(got, fine[f"r{r}_sorted"]), r
        assert np.array_equal(np.diff(off), np.bincount(fine[f"r{r}_fine_id"], minlength=512)), r
        assert G.same_bytes(data[r]["pos"], f[f"r{r}_pos_out"]), r   # wrapped in place


@pytest.mark.parametrize("fine", [[8, 8, 8], [4, 4, 4], [2, 3, 4], [16, 16, 16], [1, 1, 64]])
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_fused_fine_vs_oracle(fine, dt):
    """Four threaded ranks (2x2x1), out-of-box positions (the wrap), f64 and
    f32 positions, <= 256 fine cells (1-byte destination array) and up to 4096,
    with return_positions: bit-exact against the oracle's redistribution +
    fine_cell_ids + stable sort."""
    rng = np.random.default_rng(sum(fine) * 3 + (dt == np.float32))
    size, topo, box = 4, [2, 2, 1], [1.0, 1.0, 1.0]
    pos = [rng.uniform(-0.3, 1.3, (int(rng.integers(20_000, 60_000)), 3)).astype(dt)
           for _ in range(size)]
    data = [np.arange(len(p), dtype=np.int64) * 8 + r for r, p in enumerate(pos)]
    pos_o = [p.copy() for p in pos]
    loc = ro.redistribute_by_position_all_ranks(topo, box, size, data, pos_o)
    geos = [ro.Geometry(topo, box, size, r) for r in range(size)]
    lpos = ro.redistribute_by_cell_number_all_ranks(
        size, pos_o, [ro.cell_number_from_position(g, p.copy()) for g, p in zip(geos, pos_o)])
    nf = int(np.prod(fine))

    def fn(comm, r):
        R = MPIGridRedistributor(comm, topo, box)
        return R.redistribute_by_position(data[r], pos[r], fine_cells=fine, return_positions=True)

    outs = run_ranks(size, fn)
    for r in range(size):
        fid = ro.fine_cell_ids(topo, fine, box, lpos[r])
        exp, exp_off = ro.fine_cell_sort(loc[r], fid, nf)
        got, gpos, off = outs[r]
        assert G.same_bytes(got, exp), r
        assert np.array_equal(off, exp_off), r
        assert G.same_bytes(gpos, lpos[r][np.argsort(fid, kind="stable")]), r
        assert G.same_bytes(pos[r], pos_o[r]), r


def test_partition_fine_ids_then_sort():
    """The 1-GPU Cfg5 step's device API: GridPartitioner.partition_device(...,
    fine_cells) partitions the rows and their fine cells; fine_cell_sort(...,
    fine_ids=) of a destination's segment == fine_cell_sort binning again."""
    n = 1 << 20
    rec, pos = mgr.synth_wide(n, seed=9)
    P = mgr.GridPartitioner([2, 2, 2], [1.0] * 3)
    out, fids, counts = P.partition_device(rec.reshape(-1), 36, pos, fine_cells=[8, 8, 8])
    out2, counts2 = mgr.GridPartitioner([2, 2, 2], [1.0] * 3).partition_device(
        rec.reshape(-1).clone(), 36, pos.clone())
    assert torch.equal(counts, counts2) and torch.equal(out[: n * 36], out2[: n * 36])
    c = counts.cpu().numpy()
    starts = np.concatenate([[0], np.cumsum(c)])
    R = run_ranks(8, lambda comm, r: MPIGridRedistributor(comm, [2, 2, 2], [1.0] * 3))
    for cell in (0, 5):
        seg = out[starts[cell] * 36: starts[cell + 1] * 36].reshape(-1, 36)
        a, oa = R[cell].fine_cell_sort(seg, seg.view(torch.float32)[:, :3], [8, 8, 8],
                                       fine_ids=fids[starts[cell]: starts[cell + 1]])
        b, ob = R[cell].fine_cell_sort(seg, seg.view(torch.float32)[:, :3], [8, 8, 8])
        assert torch.equal(a, b) and torch.equal(oa, ob)


@pytest.mark.parametrize("rank_rows", [0, 2048, 4096])
@pytest.mark.parametrize("row_bytes", [4, 12, 36, 40, 64])
def test_ranked_sort_tile_sizes(rank_rows, row_bytes):
    """mgr_rank_ids + mgr_pack_ranked on both tile sizes (4096 where the LDS
    image fits, 2048 otherwise and on request), a ragged last tile, a hot
    cell and empty cells: the stable sort of the rows by their ids."""
    rng = np.random.default_rng(row_bytes * 13 + rank_rows)
    n = 300_001 + row_bytes
    ids = rng.integers(0, 512, n).astype(np.uint16)
    ids[rng.random(n) < 0.3] = 77            # a hot cell
    ids[(ids >= 400) & (ids < 420)] = 5      # empty cells
    data = rng.integers(0, 256, (n, row_bytes), dtype=np.uint8)
    exp = data[np.argsort(ids, kind="stable")]
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    pos = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
    _lib.test_hook("rank_rows", rank_rows)
    try:
        got, off = R.fine_cell_sort(torch.from_numpy(data).cuda(), pos, [8, 8, 8],
                                    fine_ids=torch.from_numpy(ids.view(np.int16)).cuda())
    finally:
        _lib.test_hook("rank_rows", 0)
    assert np.array_equal(got.cpu().numpy(), exp)
    assert np.array_equal(np.diff(off.cpu().numpy()), np.bincount(ids, minlength=512))


@pytest.mark.parametrize("row_bytes", [36, 6])   # ranked path / count + generic pack
def test_fine_ids_out_of_range(row_bytes):
    """ids of another fine grid (>= nbins): host ids raise before anything
    runs; device ids are clamped by the kernels (no out-of-range table
    access) and the call reports -1 counts; host results raise."""
    n = 50_000
    rng = np.random.default_rng(row_bytes)
    ids = rng.integers(0, 64, n).astype(np.uint16)
    ids[777] = 64                                   # one id past 4x4x4 = 64 cells
    data = rng.integers(0, 256, (n, row_bytes), dtype=np.uint8)
    pos = np.zeros((n, 3), dtype=np.float32)
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    with pytest.raises(ValueError):
        R.fine_cell_sort(data, pos, [4, 4, 4], fine_ids=ids)
    with pytest.raises(ValueError):
        R.fine_cell_sort(data, pos, [4, 4, 4], fine_ids=np.full(n, -1, dtype=np.int32))
    tid = torch.from_numpy(ids.view(np.int16)).cuda()
    out, off = R.fine_cell_sort(torch.from_numpy(data).cuda(), torch.from_numpy(pos).cuda(),
                                [4, 4, 4], fine_ids=tid)
    torch.cuda.synchronize()
    assert (torch.diff(off) == -1).all()            # counts poisoned, like a failed scan
    # in range again: the same redistributor sorts correctly (no stale flag)
    ids[777] = 3
    got, off = R.fine_cell_sort(torch.from_numpy(data).cuda(), torch.from_numpy(pos).cuda(),
                                [4, 4, 4], fine_ids=torch.from_numpy(ids.view(np.int16)).cuda())
    assert np.array_equal(got.cpu().numpy(), data[np.argsort(ids, kind="stable")])
    assert np.array_equal(np.diff(off.cpu().numpy()), np.bincount(ids, minlength=64))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 63, 4095, 4097, 8193])
@pytest.mark.parametrize("row_bytes", [4, 36])
def test_ranked_sort_small_and_ragged(n, row_bytes):
    """The ranked sort at tiny and tile-edge sizes (the unit-streamed pack
    reads the slots of row pairs: no read before row 0 or past row n - 1)."""
    rng = np.random.default_rng(n * 7 + row_bytes)
    ids = rng.integers(0, 512, n).astype(np.uint16)
    data = rng.integers(0, 256, (n, row_bytes), dtype=np.uint8)
    exp = data[np.argsort(ids, kind="stable")]
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    pos = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
    got, off = R.fine_cell_sort(torch.from_numpy(data).cuda(), pos, [8, 8, 8],
                                fine_ids=torch.from_numpy(ids.view(np.int16)).cuda())
    assert np.array_equal(got.cpu().numpy(), exp)
    assert np.array_equal(np.diff(off.cpu().numpy()), np.bincount(ids, minlength=512))
