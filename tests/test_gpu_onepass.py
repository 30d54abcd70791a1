"""GPU parity of the one-pass source partition (mgr_partition_onepass,
GridPartitioner.partition_lists / partition_onepass_device): records that
hold their own positions binned, ranked and scattered in ONE read, the output
being the reference's send_buff list (redist.py:195-198: send_buff[i] =
data[rank_to_send == i], order kept).  Bit-exact against the C oracle's
binning + stable partition (and the reference-made fixtures), including the
in-place wrap (S1), non-periodic input, fine cells, partial tiles, the
generic row sizes, a bin that outgrows its region (the classic redo, which
must not wrap twice) and a failed look-back."""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import redist_oracle as ro
from tests import golden_io as G

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import GridPartitioner, _lib  # noqa: E402

REC36 = np.dtype([("pos", "f4", 3), ("vel", "f4", 3), ("mass", "f4"), ("id", "i8")])
REC32 = np.dtype([("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _rec36(n, rng, lo=-0.3, hi=1.3):
    rec = np.zeros(n, dtype=REC36)
    rec["pos"] = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    rec["vel"] = rng.normal(size=(n, 3)).astype(np.float32)
    rec["mass"] = rng.uniform(1, 2, n).astype(np.float32)
    rec["id"] = np.arange(n)
    return rec


def _rec32(n, rng, lo=-0.3, hi=1.3):
    rec = np.zeros(n, dtype=REC32)
    p = rng.uniform(lo, hi, (n, 3))
    rec["x"], rec["y"], rec["z"] = p[:, 0], p[:, 1], p[:, 2]
    rec["id"] = np.arange(n)
    return rec


def _pos_view(rec):
    return rec["pos"] if rec.dtype == REC36 else rec.view(np.float64).reshape(len(rec), 4)[:, :3]


def _expect(rec, topo, box, periodic=True):
    """C oracle: wrap + bin the records' own positions (in place, on a copy),
    then the stable split per destination."""
    r = rec.copy()
    pos = np.ascontiguousarray(_pos_view(r))
    cell = c_oracle.bin_positions(pos, topo, box, periodic=periodic)
    if r.dtype == REC36:
        r["pos"] = pos
    else:
        r["x"], r["y"], r["z"] = pos[:, 0], pos[:, 1], pos[:, 2]
    nb = int(np.prod(topo))
    part, off = c_oracle.partition(r, cell, nb)
    return r, [part[off[b]:off[b + 1]] for b in range(nb)]


@pytest.mark.parametrize("n", [1, 1023, 1024, 1025, 300_007])
@pytest.mark.parametrize("kind", ["rec36", "rec32"])
@pytest.mark.parametrize("as_torch", [False, True])
def test_lists_vs_c_oracle(n, kind, as_torch):
    rng = np.random.default_rng(n + len(kind))
    rec = (_rec36 if kind == "rec36" else _rec32)(n, rng)
    topo, box = [2, 2, 2], [1.0] * 3
    wrapped, exp = _expect(rec, topo, box)
    P = GridPartitioner(topo, box)
    if as_torch:
        raw = torch.from_numpy(rec.view(np.uint8).reshape(n, -1).copy()).cuda()
        pos = raw.view(torch.float32)[:, :3] if kind == "rec36" else raw.view(torch.float64)[:, :3]
        got = P.partition_lists(raw, pos)
        for b in range(8):
            assert np.array_equal(got[b].cpu().numpy().reshape(-1),
                                  exp[b].view(np.uint8).reshape(-1)), b
        assert np.array_equal(raw.cpu().numpy().reshape(-1), wrapped.view(np.uint8)), "wrap"
    else:
        r = rec.copy()
        got = P.partition_lists(r, _pos_view(r))
        for b in range(8):
            assert G.same_bytes(got[b], exp[b]), b
        assert G.same_bytes(r, wrapped), "in-place wrap of the caller's records"


@pytest.mark.parametrize("topo", [[1, 1, 1], [3, 3, 3], [4, 4, 4], [2, 3, 5]])
def test_lists_bins_and_nonperiodic(topo):
    rng = np.random.default_rng(sum(topo))
    n = 200_003
    rec = _rec36(n, rng, 0.0, 1.0)
    box = [1.0, 2.0, 0.5]
    rec["pos"] *= np.array(box, np.float32)
    for periodic in (True, False):
        wrapped, exp = _expect(rec, topo, box, periodic)
        r = rec.copy()
        got = GridPartitioner(topo, box).partition_lists(r, r["pos"], periodic=periodic)
        for b in range(int(np.prod(topo))):
            assert G.same_bytes(got[b], exp[b]), (periodic, b)
        assert G.same_bytes(r, wrapped), periodic


def test_lists_fine_cells_match_fine_binning():
    """Fine cells beside the rows == the reference-pinned fine binning of the
    partitioned positions (tests/golden/fine_*.npz path)."""
    rng = np.random.default_rng(3)
    n = 500_001
    rec = _rec36(n, rng)
    topo, box, fine = [2, 2, 2], [1.0] * 3, [8, 8, 8]
    _, exp = _expect(rec, topo, box)
    r = rec.copy()
    got, fids = GridPartitioner(topo, box).partition_lists(r, r["pos"], fine_cells=fine)
    for b in range(8):
        assert G.same_bytes(got[b], exp[b]), b
        want = ro.fine_cell_ids(topo, fine, box, np.ascontiguousarray(exp[b]["pos"]))
        assert np.array_equal(fids[b].astype(np.int64), want), b


def test_lists_fixture_rec36_view():
    """The reference's own config-5-shaped redistribution (redist_p8_rec36_view):
    rank r's send_buff list, concatenated over ranks in source order, is the
    fixture's output (S7)."""
    f = G.load("redist_p8_rec36_view.npz")
    size = int(f["size"])
    sends = []
    for r in range(size):
        d = f[f"r{r}_data"].copy()
        sends.append(GridPartitioner(f["topology"], f["box"]).partition_lists(d, d["pos"]))
        assert G.same_bytes(d["pos"], f[f"r{r}_pos_out"]), r
    for r in range(size):
        assert G.same_bytes(np.concatenate([sends[s][r] for s in range(size)]), f[f"r{r}_out"]), r


def test_generic_row_sizes():
    """Rows the one-pass kernel moves with its generic gather (20 and 44 bytes,
    f32 positions at an offset) and 8-byte rows."""
    rng = np.random.default_rng(9)
    n = 100_003
    for rb, off in ((20, 8), (44, 4), (12, 0)):
        raw = rng.integers(0, 255, (n, rb)).astype(np.uint8)
        pos = rng.uniform(-0.2, 1.2, (n, 3)).astype(np.float32)
        raw[:, off:off + 12] = pos.view(np.uint8).reshape(n, 12)
        t = torch.from_numpy(raw.copy()).cuda()
        tp = torch.as_strided(t.view(torch.float32), (n, 3), (rb // 4, 1), off // 4)
        got = GridPartitioner([2, 2, 2], [1.0] * 3).partition_lists(t, tp)
        p2 = pos.copy()
        cell = c_oracle.bin_positions(p2, [2, 2, 2], [1.0] * 3)
        exp_raw = raw.copy()
        exp_raw[:, off:off + 12] = p2.view(np.uint8).reshape(n, 12)
        part, eoff = c_oracle.partition(exp_raw, cell, 8)
        for b in range(8):
            assert np.array_equal(got[b].cpu().numpy(), part[eoff[b]:eoff[b + 1]]), (rb, b)
        assert np.array_equal(t.cpu().numpy(), exp_raw), rb


def test_overflow_redoes_without_wrapping_twice():
    """Clustered rows: one bin holds 90 % -- it outgrows its region, the
    partition is redone by the classic path, which re-bins the stored
    positions (periodic = 0): exact, and the caller's positions equal ONE
    wrap (a second wrap of x + L - L can change bits again, S1)."""
    rng = np.random.default_rng(4)
    n = 400_000
    rec = _rec32(n, rng, -0.5, 1.5)
    hot = rng.random(n) < 0.9
    for c in ("x", "y", "z"):
        rec[c][hot] = rng.uniform(-1.0, -0.5, int(hot.sum()))   # wraps into [0, 0.5)
    wrapped, exp = _expect(rec, [2, 2, 2], [1.0] * 3)
    r = rec.copy()
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    got = P.partition_lists(r, _pos_view(r))
    for b in range(8):
        assert G.same_bytes(got[b], exp[b]), b
    assert G.same_bytes(r, wrapped)


def test_device_counts_above_cap_flag_overflow():
    n = 50_000
    rec, pos = mgr.synth_wide(n, seed=1)
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    out, fo, counts, cap = P.partition_onepass_device(rec.reshape(-1), 36, pos, cap_rows=100)
    c = counts.cpu().numpy()
    assert cap == 100 and (c > cap).all() and c.sum() == n


def test_failed_lookback_reports_minus_one():
    """Bounded look-back polls that give up at once (scan_spins = -1): every
    tile after the first publishes a poisoned prefix, the counts read -1 and
    the partition_lists caller raises -- never a hang, never wrong rows."""
    n = 100_000
    rec, pos = mgr.synth_wide(n, seed=2)
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    _lib.test_hook("scan_spins", -1)
    try:
        _, _, counts, _ = P.partition_onepass_device(rec.reshape(-1), 36, pos)
        c = counts.cpu().numpy()
    finally:
        _lib.test_hook("scan_spins", 1 << 24)
    assert (c == -1).all(), c
    _, _, counts, _ = P.partition_onepass_device(rec.reshape(-1), 36, pos)
    assert counts.sum().item() == n


def test_unsupported_shapes_take_the_classic_path():
    """2-D grids, f16 positions and positions outside the records are not the
    one-pass kernel's: partition_lists still returns the send_buff list."""
    rng = np.random.default_rng(6)
    n = 5000
    data = rng.normal(size=(n, 3))
    pos = rng.uniform(-1, 2, (n, 2))
    exp_pos = pos.copy()
    cell = c_oracle.bin_positions(exp_pos, [2, 3], [1.0, 1.0])
    part, off = c_oracle.partition(data, cell, 6)
    got = GridPartitioner([2, 3], [1.0, 1.0]).partition_lists(data, pos)
    for b in range(6):
        assert np.array_equal(got[b], part[off[b]:off[b + 1]])
    assert np.array_equal(pos, exp_pos)
