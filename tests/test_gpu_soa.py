"""GPU parity of SoA (multi-field) redistribution: a payload given as several
arrays sharing axis 0 -- e.g. (pos, vel, mass, ids) -- moved with ONE
binning, one scan, one count exchange and one pack launch (mgr_pack_fields,
the multi-field kernel), bit-exact against

  * the reference's own multi-field pattern, run by make_golden.py make_soa:
    destinations binned once (redist.py:157), every field redistributed with
    them (:160, :164; redistribute_by_cell_number per field);
  * the C oracle's per-field stable partition at larger sizes, including the
    field shapes the multi-field kernel leaves to the per-field packs
    (rows that are not 4-byte multiples, unaligned views, many fields).
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import redist_oracle as ro
from tests import golden_io as G
from tests.fake_mpi import run_ranks

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import GridPartitioner, MPIGridRedistributor, _lib  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _bytes(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().contiguous().numpy().view(np.uint8).reshape(-1)
    return np.ascontiguousarray(x).view(np.uint8).reshape(-1)


@pytest.mark.parametrize("as_torch", [False, True])
@pytest.mark.parametrize("case", G.soa_cases())
def test_soa_golden_threads(case, as_torch):
    f = G.load(case)
    size, nf = int(f["size"]), int(f["nfields"])
    fields, pos = G.soa_inputs(f, size, as_torch)

    def fn(comm, r):
        R = MPIGridRedistributor(comm, f["topology"], f["box"])
        out = R.redistribute_by_position(tuple(fields[r]), pos[r], periodic=bool(f["periodic"]))
        torch.cuda.synchronize()
        return out

    outs = run_ranks(size, fn)
    for r in range(size):
        assert isinstance(outs[r], tuple) and len(outs[r]) == nf
        assert np.array_equal(_bytes(pos[r]), _bytes(f[f"r{r}_pos_out"])), (case, r)
        for i in range(nf):
            exp = f[f"r{r}_f{i}_out"]
            if as_torch:
                assert np.array_equal(_bytes(outs[r][i]), _bytes(exp)), (case, r, i)
            else:
                assert G.same_bytes(outs[r][i], exp), (case, r, i, G.diff_report(outs[r][i], exp))


@pytest.mark.parametrize("as_torch", [False, True])
def test_soa_cell_number_golden(as_torch):
    f = G.load("soa_cellnum_p5_three.npz")
    size, nf = int(f["size"]), int(f["nfields"])

    def fn(comm, r):
        fl = [f[f"r{r}_f{i}_in"] for i in range(nf)]
        ids = f[f"r{r}_ids"]
        if as_torch:
            fl = [torch.from_numpy(x.copy()).cuda() for x in fl]
            ids = torch.from_numpy(ids.copy()).cuda()
        return MPIGridRedistributor(comm, [size], [1.0]).redistribute_by_cell_number(fl, ids)

    outs = run_ranks(size, fn)
    for r in range(size):
        for i in range(nf):
            assert np.array_equal(_bytes(outs[r][i]), _bytes(f[f"r{r}_f{i}_out"])), (r, i)


def _soa(n, r, rng, lo=-0.5, hi=1.5):
    """Config 5's fields as four arrays: pos f32 x3, vel f32 x3, mass f32, id i64."""
    pos = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    vel = rng.normal(size=(n, 3)).astype(np.float32)
    mass = rng.uniform(1, 2, n).astype(np.float32)
    ids = np.arange(n, dtype=np.int64) + 1_000_000 * r
    return [pos, vel, mass, ids]


@pytest.mark.parametrize("return_positions", [False, True])
def test_soa_random_threads(return_positions):
    """4 ranks, skewed sizes with an empty rank; position = field 0."""
    rng = np.random.default_rng(61)
    size, topo, box = 4, [2, 2, 1], [1.0, 1.0, 1.0]
    sizes = [20_000, 0, 3_000, 45_000]
    fields = [_soa(n, r, rng) for r, n in enumerate(sizes)]
    ofields = [[x.copy() for x in fl] for fl in fields]
    exp = ro.redistribute_fields_by_position_all_ranks(topo, box, size, ofields,
                                                       [fl[0] for fl in ofields])

    def fn(comm, r):
        return MPIGridRedistributor(comm, topo, box).redistribute_by_position(
            tuple(fields[r]), fields[r][0], return_positions=return_positions)

    outs = run_ranks(size, fn)
    for r in range(size):
        got = outs[r][0] if return_positions else outs[r]
        for i in range(4):
            assert G.same_bytes(got[i], exp[r][i]), (r, i)
        if return_positions:
            assert G.same_bytes(outs[r][1], exp[r][0]), r   # the wrapped positions
        assert G.same_bytes(fields[r][0], ofields[r][0]), r


def test_soa_fine_cells_threads():
    """SoA + fine_cells (config 5 as four arrays): the fine cells binned at the
    source travel as a side field, every field sorted by them."""
    rng = np.random.default_rng(62)
    size, topo, box, fine = 2, [2, 1, 1], [1.0, 1.0, 1.0], [8, 8, 8]
    sizes = [30_000, 7_000]
    fields = [_soa(n, r, rng) for r, n in enumerate(sizes)]
    ofields = [[x.copy() for x in fl] for fl in fields]
    loc = ro.redistribute_fields_by_position_all_ranks(topo, box, size, ofields,
                                                       [fl[0] for fl in ofields])

    def fn(comm, r):
        t = [torch.from_numpy(x).cuda() for x in fields[r]]
        return MPIGridRedistributor(comm, topo, box).redistribute_by_position(
            t, t[0], fine_cells=fine, return_positions=True)

    outs = run_ranks(size, fn)
    for r in range(size):
        fid = ro.fine_cell_ids(topo, fine, box, loc[r][0])
        order = np.argsort(fid, kind="stable")
        got, gpos, off = outs[r]
        for i in range(4):
            assert np.array_equal(_bytes(got[i]), _bytes(loc[r][i][order])), (r, i)
        assert np.array_equal(_bytes(gpos), _bytes(loc[r][0][order])), r
        assert np.array_equal(np.diff(off.cpu().numpy()),
                              np.bincount(fid, minlength=int(np.prod(fine)))), r


def _field_set(kind, n, rng):
    """Field shapes: the multi-field kernel's (4-byte-multiple rows) and the
    per-field packs' (other widths, unaligned starts)."""
    if kind == "cfg5":
        return [rng.integers(0, 2**31, (n, 3)).astype(np.float32),
                rng.normal(size=(n, 3)).astype(np.float32),
                rng.normal(size=n).astype(np.float32), np.arange(n, dtype=np.int64)]
    if kind == "wide":       # 16-byte multiples and a 64-byte row
        return [rng.normal(size=(n, 2)), rng.normal(size=(n, 8)),
                rng.integers(0, 9, (n, 4)).astype(np.int32)]
    if kind == "narrow":     # 1-, 2-, 6-byte rows: per-field packs
        return [rng.integers(0, 255, n).astype(np.uint8), rng.normal(size=n).astype(np.float32),
                rng.integers(0, 999, (n, 3)).astype(np.int16),
                rng.integers(0, 99, n).astype(np.int16)]
    if kind == "many":       # 10 fields: more than one multi-field launch
        return [rng.integers(0, 1 << 30, (n, 1 + i % 4)).astype(np.int32) for i in range(10)]
    if kind == "big":        # rows too wide for one launch's LDS together
        return [rng.integers(0, 1 << 30, (n, 32)).astype(np.int32) for _ in range(4)]
    if kind == "pos_id":     # configs 2-4 as arrays: f64 positions + i64 ids
        return [rng.normal(size=(n, 3)), np.arange(n, dtype=np.int64)]
    if kind == "unaligned":  # a 12-byte field starting 4 bytes into its buffer
        base = rng.integers(0, 1 << 30, (n * 3 + 1,)).astype(np.int32)
        return [base, rng.normal(size=(n, 3)).astype(np.float32)]
    raise ValueError(kind)


@pytest.mark.parametrize("kernel", [1, 2, 3])
@pytest.mark.parametrize("kind", ["cfg5", "wide", "narrow", "many", "big", "unaligned", "pos_id"])
@pytest.mark.parametrize("topo", [[2, 2, 2], [4, 4, 4], [2, 3, 1], [1]])
def test_partition_fields_vs_c_oracle(kind, topo, kernel):
    """GridPartitioner.partition_by_position with a tuple payload == the C
    oracle's partition of every field by the same destinations -- through the
    per-wave LDS-image, the tile-image and the cooperative multi-field kernels
    (test hook fields_kernel; each where it takes the fields)."""
    _lib.test_hook("fields_kernel", kernel)
    try:
        _partition_fields_case(kind, topo)
    finally:
        _lib.test_hook("fields_kernel", 0)


def _partition_fields_case(kind, topo):
    rng = np.random.default_rng(len(kind) * 7 + sum(topo))
    n = 300_007
    dim = len(topo)
    box = [1.0] * dim
    fl = _field_set(kind, n, rng)
    pos = rng.uniform(-0.3, 1.3, (n, dim))
    tf = [torch.from_numpy(x).cuda() for x in fl]
    if kind == "unaligned":
        tf[0] = tf[0][1:].view(n, 3)        # storage offset 4 bytes
        fl[0] = fl[0][1:].reshape(n, 3)
    pin = pos.copy()
    cell = c_oracle.bin_positions(pin, topo, box)
    P = GridPartitioner(topo, box)
    got, off = P.partition_by_position(tuple(tf), torch.from_numpy(pos).cuda())
    for i, x in enumerate(fl):
        exp, eoff = c_oracle.partition(x, cell, int(np.prod(topo)))
        assert np.array_equal(_bytes(got[i]), _bytes(exp)), (kind, i)
        assert np.array_equal(off.cpu().numpy(), eoff), kind


@pytest.mark.parametrize("tile_rounds", [2, 4, 16, 32])
def test_pack_fields_tile_shapes(tile_rounds):
    """The multi-field kernel on other tile shapes (test hook tile_rounds: 128 ..
    2048-row tiles, 1 .. 16 waves), a partial last tile."""
    rng = np.random.default_rng(tile_rounds)
    n = 100_003
    fl = _field_set("cfg5", n, rng)
    pos = rng.uniform(0, 1, (n, 3))
    cell = c_oracle.bin_positions(pos.copy(), [2, 2, 2], [1.0] * 3)
    _lib.test_hook("tile_rounds", tile_rounds)
    try:
        P = GridPartitioner([2, 2, 2], [1.0] * 3)
        got, _ = P.partition_by_position(tuple(torch.from_numpy(x).cuda() for x in fl),
                                         torch.from_numpy(pos).cuda())
    finally:
        _lib.test_hook("tile_rounds", 0)
    for i, x in enumerate(fl):
        exp, _ = c_oracle.partition(x, cell, 8)
        assert np.array_equal(_bytes(got[i]), _bytes(exp)), i


@pytest.mark.parametrize("kind", ["cfg5", "wide", "narrow", "many", "big", "pos_id",
                                  "cfg5_3", "pair"])
@pytest.mark.parametrize("nfine", [[8, 8, 8], [4, 4, 4], [3, 5, 7]])
def test_fine_sort_fields_vs_stable_sort(kind, nfine):
    """MPIGridRedistributor.fine_cell_sort of a SoA payload by given fine ids
    == numpy's stable argsort of the ids applied to every field (one rank +
    scan, the ranked pack per field; the generic pack for rows it does not
    take), with a partial last tile."""
    rng = np.random.default_rng(len(kind) * 11 + sum(nfine))
    n = 250_007
    base = "cfg5" if kind in ("cfg5_3", "pair") else kind
    fl = _field_set(base, n, rng)
    if kind == "cfg5_3":
        fl = fl[:3]             # pos, vel, mass: the (3, 3, 1) signature
    elif kind == "pair":
        fl = [fl[2], fl[2].copy()]   # two 4-byte fields: (1, 1)
    nb = int(np.prod(nfine))
    ids = rng.integers(0, nb, n).astype(np.uint16)
    order = np.argsort(ids, kind="stable")
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    t = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in fl]
    pos = torch.zeros((n, 3), dtype=torch.float32, device="cuda")
    got, off = R.fine_cell_sort(t, pos, nfine, fine_ids=torch.from_numpy(ids.view(np.int16)).cuda())
    assert np.array_equal(np.diff(off.cpu().numpy()), np.bincount(ids, minlength=nb))
    for i, x in enumerate(fl):
        assert np.array_equal(_bytes(got[i]), _bytes(np.ascontiguousarray(x)[order])), (kind, i)


def test_partition_fields_device_cfg5_fine():
    """The bench's SoA config-5 source step (partition_fields_device with
    fine cells): every field partitioned, the fine ids beside them, equal to
    the single-record path's fine ids."""
    rng = np.random.default_rng(71)
    n = (1 << 20) + 37     # a partial last round: the side ids of its few rows
    fl = _field_set("cfg5", n, rng)
    fl[0] = rng.uniform(0, 1, (n, 3)).astype(np.float32)
    cell = c_oracle.bin_positions(fl[0].copy(), [2, 2, 2], [1.0] * 3)
    tf = [torch.from_numpy(x.copy()).cuda() for x in fl]
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    outs, fids, counts = P.partition_fields_device(
        [t.reshape(-1).view(torch.uint8) for t in tf], [12, 12, 4, 8], tf[0],
        fine_cells=[8, 8, 8])
    torch.cuda.synchronize()
    for i, x in enumerate(fl):
        exp, eoff = c_oracle.partition(x, cell, 8)
        assert np.array_equal(_bytes(outs[i]), _bytes(exp)), i
    assert np.array_equal(counts.cpu().numpy(), np.diff(eoff))
    # fine ids: the fine binning of the partitioned positions (topology * 8)
    fid = ro.fine_cell_ids([2, 2, 2], [8, 8, 8], [1.0] * 3,
                           c_oracle.partition(fl[0], cell, 8)[0])
    assert np.array_equal(fids.cpu().numpy().view(np.uint16).astype(np.int64), fid)


def test_pack_fields_scan_failure_writes_nothing():
    """A failed scan makes the multi-field pack write nothing, like every pack:
    forced deterministically (scan chunk 0 publishes its prefix poisoned, test
    hook scan_poison_chunk), so the outputs keep their sentinel bytes and the
    counts read -1."""
    n = 1 << 22
    rng = np.random.default_rng(5)
    fl = [torch.from_numpy(x).cuda() for x in _field_set("cfg5", n, rng)]
    flats = [t.reshape(-1).view(torch.uint8) for t in fl]
    pos = torch.from_numpy(rng.uniform(0, 1, (n, 3))).cuda()
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    outs, counts = P.partition_fields_device(flats, [12, 12, 4, 8], pos.clone())
    torch.cuda.synchronize()
    assert (counts.cpu().numpy() >= 0).all()
    for o in outs:
        o.fill_(0xAB)
    hooks = dict(scan_poison_chunk=0)
    for k, v in hooks.items():
        _lib.test_hook(k, v)
    try:
        outs, counts = P.partition_fields_device(flats, [12, 12, 4, 8], pos.clone())
        c = counts.cpu().numpy()
    finally:
        for k in hooks:
            _lib.test_hook(k, _lib.HOOK_DEFAULTS[k])
    assert (c == -1).all(), c
    for o in outs:
        assert bool((o == 0xAB).all()), "a pack wrote after a failed scan"


def test_soa_errors():
    R = run_ranks(2, lambda comm, r: MPIGridRedistributor(comm, [2, 1, 1], [1.0] * 3))[0]
    p = np.zeros((10, 3))
    with pytest.raises(ValueError):
        R.redistribute_by_position((np.zeros(10), np.zeros(9)), p)
    with pytest.raises(ValueError):
        R.redistribute_by_position((), p)
    with pytest.raises(NotImplementedError):
        R.redistribute_by_position((np.zeros(10), np.zeros(10)), p, overload_lengths=[0.1] * 3)
