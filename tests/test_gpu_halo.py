"""GPU parity of the overload (halo) exchange (redist.py:161-166, :202-309):
face flags from the binning kernel (mgr_bin_count_halo) or mgr_halo_flags,
multi-selections (mgr_msel_count, mgr_scan, mgr_msel_pack) and the
transport's grouped point-to-point batches, bit-exact against the reference's own
outputs (tests/golden/halo_*.npz) and the NumPy oracle on larger inputs."""
import numpy as np
import pytest
import torch

from oracle import redist_oracle as ro
from tests import golden_io as G
from tests.fake_mpi import run_ranks

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import MPIGridRedistributor  # noqa: E402

CASES = ["halo_p8_f64_rec32.npz", "halo_p4_2d_mat.npz", "halo_p2_f32_rec36.npz",
         "halo_p27_333_ids.npz", "halo_p8_wide.npz", "halo_p1_self.npz", "halo_p6_321_i32.npz"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("as_torch", [False, True])
@pytest.mark.parametrize("case", CASES)
def test_halo_golden(case, as_torch):
    f = G.load(case)
    size = int(f["size"])
    topo, box, ol = f["topology"], f["box"], list(f["overload"])
    data = [d.copy() for d in G.per_rank(f, "data", size)]
    pos = [p.copy() for p in G.per_rank(f, "pos_in", size)]
    if as_torch:
        data = [torch.from_numpy(d.view(np.uint8).reshape(len(d), -1) if d.dtype.names else d)
                .cuda() for d in data]
        pos = [torch.from_numpy(p).cuda() for p in pos]

    def fn(comm, r):
        out = MPIGridRedistributor(comm if size > 1 else None, topo, box).redistribute_by_position(
            data[r], pos[r], overload_lengths=ol)
        torch.cuda.synchronize()
        return out

    outs = run_ranks(size, fn)
    for r in range(size):
        exp = f[f"r{r}_out"]
        if as_torch:
            got = outs[r].cpu().numpy()
            assert got.tobytes() == np.ascontiguousarray(exp).tobytes(), (case, r)
            assert G.same_bytes(pos[r].cpu().numpy(), f[f"r{r}_pos_out"]), (case, r)
        else:
            assert G.same_bytes(outs[r], exp), (case, r)
            assert G.same_bytes(pos[r], f[f"r{r}_pos_out"]), (case, r)


@pytest.mark.parametrize("case", ["halo_direct_p6_321_nonperiodic.npz",
                                  "halo_direct_p8_nonperiodic.npz"])
def test_halo_direct_nonperiodic_golden(case):
    """exchange_overload_by_position(periodic=False): the :287 flag quirk."""
    f = G.load(case)
    size = int(f["size"])
    topo, box, ol = f["topology"], f["box"], list(f["overload"])

    def fn(comm, r):
        return MPIGridRedistributor(comm, topo, box).exchange_overload_by_position(
            f[f"r{r}_data"], f[f"r{r}_pos"], ol, periodic=False)

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)


def test_halo_large_vs_oracle_with_positions():
    """8 ranks x ~60k particles, 32-byte records, f64 positions; also checks
    return_positions (local + overload positions, same selections)."""
    rng = np.random.default_rng(31)
    size, topo, box, ol = 8, [2, 2, 2], [1.0, 1.0, 1.0], [0.07, 0.12, 0.05]
    pos = [rng.uniform(-0.1, 1.1, (int(rng.integers(40_000, 80_000)), 3)) for _ in range(size)]
    data = []
    for r, p in enumerate(pos):
        rec = np.zeros(len(p), dtype=[("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])
        rec["id"] = np.arange(len(p)) + 1_000_000 * r
        data.append(rec)
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_overload_all_ranks(topo, box, size, data, pos_o, ol)

    def fn(comm, r):
        return MPIGridRedistributor(comm, topo, box).redistribute_by_position(
            data[r], pos[r], overload_lengths=ol, return_positions=True)

    outs = run_ranks(size, fn)
    for r in range(size):
        got, gpos = outs[r]
        assert G.same_bytes(got, exp[r]), r
        assert G.same_bytes(pos[r], pos_o[r]), r
        assert len(gpos) == len(got)
        # the positions travel with the rows: local rows' positions equal the
        # wrapped coordinates (records hold the unwrapped input here, so check
        # the id -> position map against the wrapped inputs)
        src_rank = got["id"] // 1_000_000
        src_idx = got["id"] % 1_000_000
        want = np.stack([pos_o[s][i] for s, i in zip(src_rank, src_idx)]) if len(got) else gpos
        assert G.same_bytes(gpos, want), r


def test_halo_rccl_single_rank():
    """RcclComm at world size 1: neighbours are the rank itself (mgr_group_p2p
    self copies), periodic self-images without a shift."""
    from mpi_grid_redistribute_amd import RcclComm
    f = G.load("halo_p1_self.npz")
    comm = RcclComm(RcclComm.unique_id(), 1, 0)
    try:
        pos = f["r0_pos_in"].copy()
        out = MPIGridRedistributor(comm, f["topology"], f["box"]).redistribute_by_position(
            f["r0_data"], pos, overload_lengths=list(f["overload"]))
        assert G.same_bytes(out, f["r0_out"])
        assert G.same_bytes(pos, f["r0_pos_out"])
    finally:
        comm.close()



@pytest.mark.parametrize("clustered", [False, True])
def test_halo_in_place_and_overflow(clustered):
    """The halo rows are appended in place after the redistributed rows while
    they fit the spare capacity halo_capacity() reserves (uniform estimate);
    particles packed against the cell faces outgrow it and take the
    concatenating path.  Both against the oracle, with return_positions."""
    from mpi_grid_redistribute_amd.halo import halo_capacity
    rng = np.random.default_rng(77 + clustered)
    size, topo, box, ol = 4, [2, 2, 1], [1.0, 1.0, 1.0], [0.1, 0.1, 0.05]
    pos = []
    for r in range(size):
        p = rng.uniform(0.0, 1.0, (30_000 + 1000 * r, 3))
        if clustered:   # most rows within ol of the x = 0.5 / y = 0.5 faces
            k = rng.random(len(p)) < 0.85
            p[k, 0] = 0.5 + rng.uniform(-0.09, 0.09, int(k.sum()))
            p[k, 1] = 0.5 + rng.uniform(-0.09, 0.09, int(k.sum()))
        pos.append(p)
    data = [np.arange(len(p), dtype=np.int64) + 1_000_000 * r for r, p in enumerate(pos)]
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_overload_all_ranks(topo, box, size, data, pos_o, ol)

    def fn(comm, r):
        R = MPIGridRedistributor(comm, topo, box)
        out = R.redistribute_by_position(data[r], pos[r], overload_lengths=ol,
                                         return_positions=True)
        return out, R

    outs = run_ranks(size, fn)
    fits = []
    for r in range(size):
        (got, gpos), R = outs[r]
        assert G.same_bytes(got, exp[r]), r
        assert len(gpos) == len(got)
        src_rank, src_idx = got // 1_000_000, got % 1_000_000
        want = np.stack([pos_o[s][i] for s, i in zip(src_rank, src_idx)])
        assert G.same_bytes(gpos, want), r
        own = sum(int(np.sum(ro.cell_number_from_position(
            ro.Geometry(topo, box, size, s), pos_o[s].copy()) == r)) for s in range(size))
        fits.append(len(got) - own <= halo_capacity(R, own, ol))
    assert all(fits) if not clustered else not any(fits)


@pytest.mark.parametrize("rb,offset", [(32, 0), (24, 0), (12, 0), (36, 0), (6, 0), (3, 0),
                                       (64, 0), (100, 0), (200, 8), (7, 1)])
@pytest.mark.parametrize("n,nsets", [(1, 2), (4095, 6), (4097, 1), (300001, 6), (1 << 18, 16)])
def test_msel_pack(n, nsets, rb, offset):
    """mgr_msel_count + mgr_scan + mgr_msel_pack: set k = rows with flag bit
    bits[k], every set's rows in order, set after set (the halo's local sends
    of every dimension and direction, redist.py:271-275) -- the <= 64-byte
    kernel and the wide/unaligned one."""
    from mpi_grid_redistribute_amd.halo import DeviceSelect
    rng = np.random.default_rng(n + 7 * rb + nsets)
    flags = rng.integers(0, 1 << 16, n).astype(np.uint16) & rng.integers(0, 1 << 16, n).astype(np.uint16)
    flags[rng.random(n) < 0.5] = 0
    bits = list(rng.permutation(16)[:nsets])
    a = rng.integers(0, 256, (n, rb), dtype=np.uint8)
    sel = DeviceSelect(torch.device("cuda"))
    fl = torch.from_numpy(flags.view(np.int16)).cuda()
    h, cnt = sel.msel(fl, n, bits, "_t")
    src = torch.zeros(n * rb + offset, dtype=torch.uint8, device="cuda")
    src[offset:].copy_(torch.from_numpy(a.reshape(-1)))
    want = [a[(flags >> b) & 1 == 1] for b in bits]
    tot = sum(len(w) for w in want)
    dst = torch.full((tot * rb + offset + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    starts = np.concatenate([[0], np.cumsum([len(w_) for w_ in want])])
    sel.msel_pack(h, src[offset:], rb, [dst[offset + starts[k] * rb:] for k in range(nsets)])
    torch.cuda.synchronize()
    assert cnt.cpu().tolist() == [len(w) for w in want]
    out = dst.cpu().numpy()
    exp = np.concatenate(want).reshape(-1) if tot else np.zeros(0, np.uint8)
    np.testing.assert_array_equal(out[offset:offset + tot * rb], exp)
    assert (out[:offset] == 0xAB).all() and (out[offset + tot * rb:] == 0xAB).all()


@pytest.mark.parametrize("rec_bytes", [100, 7])
def test_halo_wide_rows_vs_oracle(rec_bytes):
    """Payload rows wider than 64 bytes (and odd-sized ones) through the
    fused halo path: 4 ranks, f32 positions."""
    rng = np.random.default_rng(rec_bytes)
    size, topo, box, ol = 4, [2, 1, 2], [2.0, 1.0, 1.0], [0.2, 0.3, 0.1]
    pos = [rng.uniform(0.0, 1.0, (20_000 + 500 * r, 3)).astype(np.float32) * np.float32([2, 1, 1])
           for r in range(size)]
    data = [rng.integers(0, 256, (len(p), rec_bytes), dtype=np.uint8) for p in pos]
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_overload_all_ranks(topo, box, size, data, pos_o, ol)

    def fn(comm, r):
        out = MPIGridRedistributor(comm, topo, box).redistribute_by_position(
            data[r], pos[r], overload_lengths=ol)
        torch.cuda.synchronize()
        return out

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], exp[r]), r


def test_msel_pack_scattered_destinations():
    """mgr_msel_pack writes set k to dsts[k] wherever it lies (here in
    reverse order with gaps) and skips sets whose destination is None."""
    from mpi_grid_redistribute_amd.halo import DeviceSelect
    rng = np.random.default_rng(5)
    n, rb, bits = 70_001, 24, [0, 1, 2, 3]
    flags = rng.integers(0, 16, n).astype(np.uint16)
    a = rng.integers(0, 256, (n, rb), dtype=np.uint8)
    sel = DeviceSelect(torch.device("cuda"))
    h, cnt = sel.msel(torch.from_numpy(flags.view(np.int16)).cuda(), n, bits, "_s")
    want = [a[(flags >> b) & 1 == 1] for b in bits]
    gap = 3
    sizes = [len(w_) * rb for w_ in want]
    buf = torch.full((sum(sizes) + gap * rb * 5,), 0x77, dtype=torch.uint8, device="cuda")
    src = torch.from_numpy(a.reshape(-1)).cuda()
    place, o = {}, gap * rb
    for k in (3, 2, 0):          # set 1 skipped
        place[k] = o
        o += sizes[k] + gap * rb
    sel.msel_pack(h, src, rb, [buf[place[k]:] if k in place else None for k in range(4)])
    out = buf.cpu().numpy()
    for k in (3, 2, 0):
        np.testing.assert_array_equal(out[place[k]:place[k] + sizes[k]], want[k].reshape(-1))
    mask = np.ones(len(out), bool)
    for k in (3, 2, 0):
        mask[place[k]:place[k] + sizes[k]] = False
    assert (out[mask] == 0x77).all()


def test_halo_overload_beyond_cell_length():
    """overload_lengths larger than the cell (every row is within reach of
    both faces): 8 ranks x ~40k rows against the oracle -- the reserved
    capacity stays bounded and the result exact."""
    rng = np.random.default_rng(41)
    size, topo, box, ol = 8, [2, 2, 2], [1.0, 1.0, 1.0], [0.7, 2.0, 0.55]
    pos = [rng.uniform(0.0, 1.0, (int(rng.integers(30_000, 50_000)), 3)) for _ in range(size)]
    data = [np.arange(len(p), dtype=np.int64) + 1_000_000 * r for r, p in enumerate(pos)]
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_overload_all_ranks(topo, box, size, data, pos_o, ol)

    def fn(comm, r):
        out = MPIGridRedistributor(comm, topo, box).redistribute_by_position(
            data[r], pos[r], overload_lengths=ol)
        torch.cuda.synchronize()
        return out

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], exp[r]), r


@pytest.mark.parametrize("dim", [1, 2, 3])
@pytest.mark.parametrize("n", [4097, 300_001])
def test_msel_masks_self_pieces(dim, n):
    """Selections by flag MASK (a row is in set k when its flags hold every
    bit of masks[k]): the 3^dim - 1 face / edge / corner pieces of the
    one-rank halo, up to 26 sets, every set's rows in order, set after set."""
    from mpi_grid_redistribute_amd.halo import DeviceSelect, self_halo_pieces
    rng = np.random.default_rng(n + dim)
    flags = np.zeros(n, dtype=np.uint16)
    for b in range(2 * dim):   # each face ~15 % of the rows, left/right exclusive
        flags |= ((rng.random(n) < 0.15).astype(np.uint16) << b)
    for d in range(dim):
        both = ((flags >> (2 * d)) & 3) == 3
        flags[both] &= np.uint16(~(1 << (2 * d + 1)) & 0xFFFF)
    masks = self_halo_pieces(dim)
    assert len(masks) == 3 ** dim - 1
    rb = 36
    a = rng.integers(0, 256, (n, rb), dtype=np.uint8)
    sel = DeviceSelect(torch.device("cuda"))
    fl = torch.from_numpy(flags.view(np.int16)).cuda()
    h, cnt = sel.msel_masks(fl, n, masks, "_t")
    want = [a[(flags & m) == m] for m in masks]
    tot = sum(len(w) for w in want)
    dst = torch.full((tot * rb + 64,), 0xAB, dtype=torch.uint8, device="cuda")
    starts = np.concatenate([[0], np.cumsum([len(w_) for w_ in want])])
    src = torch.from_numpy(a.reshape(-1)).cuda()
    sel.msel_pack_fields(h, [src], [rb], [[dst[starts[k] * rb:starts[k + 1] * rb]
                                           if len(want[k]) else None for k in range(len(masks))]])
    torch.cuda.synchronize()
    assert cnt.cpu().tolist() == [len(w) for w in want]
    out = dst.cpu().numpy()
    np.testing.assert_array_equal(out[:tot * rb], np.concatenate(want).reshape(-1))
    assert (out[tot * rb:] == 0xAB).all()


def test_one_rank_halo_vs_oracle():
    """The one-rank halo (every neighbour is this rank: one selection pass,
    one multi-set pack) against the oracle, f64 and f32 positions, with and
    without returned positions."""
    rng = np.random.default_rng(5)
    for dt, rp in ((np.float64, False), (np.float32, True)):
        n = 250_000
        pos = rng.uniform(-0.2, 1.2, (n, 3)).astype(dt)
        data = np.zeros(n, dtype=[("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])
        data["id"] = np.arange(n)
        ol = [0.05, 0.08, 0.03]
        pos_o = pos.copy()
        exp = ro.redistribute_by_position_overload_all_ranks([1, 1, 1], [1.0] * 3, 1, [data],
                                                             [pos_o], ol)[0]
        R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
        out = R.redistribute_by_position(data, pos, overload_lengths=ol, return_positions=rp)
        if rp:
            out, opos = out
            ids = out["id"]
            assert np.array_equal(opos.view(np.uint8), pos_o[ids % n].view(np.uint8))
        assert out.tobytes() == exp.tobytes()


@pytest.mark.parametrize("case", ["f64", "f32_positions", "corner_overflow", "torch"])
def test_halo_one_rank_vs_oracle(case):
    """One rank (1x1x1 grid): the rows stay in order and the halo is the
    rank's own periodic images (one selection pass over the received flags,
    one multi-set pack) against the oracle, with the wrapped positions
    returned; 'corner_overflow' puts every row into all 7 corner-region
    pieces, beyond the reserved capacity."""
    rng = np.random.default_rng(len(case))
    n, box, ol = 200_003, [1.0, 1.0, 1.0], [0.06, 0.1, 0.04]
    pos = rng.uniform(-0.2, 1.2, (n, 3))
    if case == "corner_overflow":
        pos = rng.uniform(0.0, 0.03, (n, 3))
    if case == "f32_positions":
        pos = pos.astype(np.float32)
    data = np.arange(n, dtype=np.int64) * 3 + 1
    pos_o = pos.copy()
    exp = ro.redistribute_by_position_overload_all_ranks([1, 1, 1], box, 1, [data],
                                                         [pos_o], ol)[0]
    R = MPIGridRedistributor(None, [1, 1, 1], box)
    if case == "torch":
        d, p = torch.from_numpy(data).cuda(), torch.from_numpy(pos).cuda()
    else:
        d, p = data, pos
    out, opos = R.redistribute_by_position(d, p, overload_lengths=ol, return_positions=True)
    torch.cuda.synchronize()
    if case == "torch":
        out, opos, p = out.cpu().numpy(), opos.cpu().numpy(), p.cpu().numpy()
    assert np.array_equal(out, exp)
    # positions travel with the rows: every output row's position is its source row's
    want = pos_o[(out - 1) // 3]
    assert np.array_equal(np.asarray(opos).view(np.uint8), want.view(np.uint8))
    assert np.array_equal(np.asarray(p).view(np.uint8), pos_o.view(np.uint8))   # wrapped in place


@pytest.mark.parametrize("dim,rec", [(1, 8), (2, 36), (3, 7), (3, 100)])
def test_one_rank_halo_dims_vs_oracle(dim, rec):
    """One rank in 1, 2 and 3 dimensions with odd and wide records (the
    selection pack's byte, 4-byte and row-by-row copies), against the oracle,
    positions returned."""
    rng = np.random.default_rng(dim * 100 + rec)
    n = 150_001
    topo, box = [1] * dim, [1.0] * dim
    ol = [0.05, 0.11, 0.07][:dim]
    pos = rng.uniform(-0.3, 1.3, (n, dim))
    data = rng.integers(0, 256, (n, rec), dtype=np.uint8)
    pos_o = pos.copy()
    exp = ro.redistribute_by_position_overload_all_ranks(topo, box, 1, [data], [pos_o], ol)[0]
    R = MPIGridRedistributor(None, topo, box)
    out, opos = R.redistribute_by_position(data, pos, overload_lengths=ol, return_positions=True)
    assert G.same_bytes(out, exp)
    assert G.same_bytes(pos, pos_o)
    assert len(opos) == len(out)
