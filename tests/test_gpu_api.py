"""The rest of the drop-in boundary on the GPU: the module function
``mpi_grid_redistribute`` (redist.py:11-13, intended behaviour -- the
reference's raises AttributeError, S13), ``stack_position`` (:311-312) and the
intended ``unstack_position`` (:314-318), the scan's failure path (a look-back
that gives up must surface as an error, never as wrong offsets), and scratch
reuse across calls (no per-call device allocation after warm-up)."""
import numpy as np
import pytest
import torch

from oracle import redist_oracle as ro
from tests import golden_io as G
from tests.fake_mpi import run_ranks

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import (GridPartitioner, MPIGridRedistributor,  # noqa: E402
                                       mpi_grid_redistribute)
from mpi_grid_redistribute_amd import _lib  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("case", ["redist_p8_f64_rec32.npz", "redist_p4_2d_alias.npz",
                                  "redist_p8_nonperiodic_rec32.npz"])
def test_module_function_golden(case):
    """mpi_grid_redistribute(data, pos, grid_topology, box_lengths, comm) on
    threaded ranks = the reference's redistribute_by_position outputs."""
    f = G.load(case)
    size = int(f["size"])
    data, pos = G.fixture_inputs(f, case, size, as_torch=False)

    def fn(comm, r):
        return mpi_grid_redistribute(data[r], pos[r], f["topology"], f["box"], comm,
                                     periodic=bool(f["periodic"]))

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), r
        assert G.same_bytes(pos[r], f[f"r{r}_pos_out"]), r


def test_module_function_overload_vs_oracle():
    """... with overload_lengths (the halo rows follow, redist.py:161-166) and
    periodic=False binning, against the oracle's intended-behaviour restatement."""
    rng = np.random.default_rng(41)
    size, topo, box, ol = 4, [2, 2, 1], [1.0, 1.0, 1.0], [0.1, 0.05, 0.2]
    pos = [rng.uniform(-0.3, 1.3, (int(rng.integers(2000, 6000)), 3)) for _ in range(size)]
    data = [np.arange(len(p), dtype=np.int64) * 10 + r for r, p in enumerate(pos)]
    pos_o = [p.copy() for p in pos]
    exp = ro.mpi_grid_redistribute_all_ranks(data, pos_o, topo, box, size,
                                             overload_lengths=ol, periodic=False)

    def fn(comm, r):
        return mpi_grid_redistribute(data[r], pos[r], topo, box, comm, overload_lengths=ol,
                                     periodic=False)

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], exp[r]), r
        assert G.same_bytes(pos[r], pos_o[r]), r


def test_module_function_single_rank_torch():
    rng = np.random.default_rng(3)
    pos = rng.uniform(-1, 2, (50_000, 3))
    data = np.arange(50_000, dtype=np.float64)
    pos_o = pos.copy()
    exp = ro.mpi_grid_redistribute_all_ranks([data], [pos_o], [1, 1, 1], [1.0] * 3, 1)[0]
    tpos = torch.from_numpy(pos).cuda()
    out = mpi_grid_redistribute(torch.from_numpy(data).cuda(), tpos, [1, 1, 1], [1.0] * 3, None)
    assert out.is_cuda
    assert G.same_bytes(out.cpu().numpy(), exp)
    assert G.same_bytes(tpos.cpu().numpy(), pos_o)


@pytest.mark.parametrize("dim", [1, 2, 3])
def test_stack_unstack_position(dim):
    rng = np.random.default_rng(dim)
    cols = [rng.uniform(0, 1, 1000) for _ in range(dim)]
    R = MPIGridRedistributor(None, [1] * dim, [1.0] * dim)
    got = R.stack_position(cols)
    exp = ro.stack_position(cols)
    assert G.same_bytes(got, exp)
    tcols = [torch.from_numpy(c).cuda() for c in cols]
    tgot = R.stack_position(tcols)
    assert tgot.is_cuda and G.same_bytes(tgot.cpu().numpy(), exp)
    back = R.unstack_position(got)
    ref = ro.unstack_position(exp, dim)
    assert len(back) == dim and all(G.same_bytes(a, b) for a, b in zip(back, ref))
    tback = R.unstack_position(tgot)
    assert all(G.same_bytes(a.cpu().numpy(), b) for a, b in zip(tback, ref))
    # the stacked array feeds redistribute_by_position like any (N, d) position
    p2 = got.copy()
    out = R.redistribute_by_position(np.arange(1000), p2)
    assert np.array_equal(out, np.arange(1000))


def test_scan_failure_is_loud():
    """A look-back that gives up (test hook scan_spins = -1) must not yield wrong
    offsets: the counts come back -1, the pack writes nothing, and the API
    raises at its count read."""
    n = 1 << 20
    pos, rec = mgr.synth_uniform(n, seed=5)
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    _lib.test_hook("scan_spins", -1)
    try:
        out, counts = P.partition_device(rec.reshape(-1), 32, pos)
        out.fill_(0xAB)
        out, counts = P.partition_device(rec.reshape(-1), 32, pos)
        torch.cuda.synchronize()
        assert (counts.cpu().numpy() == -1).all()
        assert bool((out == 0xAB).all())                  # nothing was written
        with pytest.raises(_lib.MgrError, match="scan failed"):
            P.partition_by_position(rec.cpu().numpy(), pos.cpu().numpy())
    finally:
        _lib.test_hook("scan_spins", 1 << 24)
    out, counts = P.partition_device(rec.reshape(-1), 32, pos)
    assert (counts.cpu().numpy() > 0).all()


class _Hooks:
    """Set test hooks for a block, back to the shipped defaults after it."""

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        for k, v in self.kw.items():
            _lib.test_hook(k, v)

    def __exit__(self, *exc):
        for k in self.kw:
            _lib.test_hook(k, _lib.HOOK_DEFAULTS[k])


# ~2000 x s_sleep(127) = several ms: far longer than the rest of the scan
_LATE = 2000


@pytest.mark.parametrize("bin_", [0, 5])
def test_scan_race_cfg2_late_inclusive_word(bin_):
    """The round-4 scan race, forced (scan_delay_bin): in the 8-bin config-2
    scan (2^26 rows, 512-row tiles, 64 chunks per bin) the chunk that ends bin
    b counts itself done several ms before it stores its inclusive word --
    the order relaxed atomics on two words allow.  The last chunk polls the
    bin-end words, so counts and the whole partition stay exact against the
    C oracle (redist.py:195-198 counts).  With one look at those words
    (scan_end_spins = 0: the pre-fix reader) the same interleaving shows up as
    a failed scan: the test does produce the race."""
    from oracle import c_oracle
    n = 1 << 26
    pos0, _ = mgr.synth_uniform(n, seed=20261015)
    pos_h = pos0.cpu().numpy()
    cell = c_oracle.bin_positions(pos_h.copy(), [2, 2, 2], [1.0] * 3)
    exp, exp_off = c_oracle.partition(np.arange(n, dtype=np.int64), cell, 8)
    ids = torch.arange(n, dtype=torch.int64, device="cuda").view(torch.uint8)
    P = GridPartitioner([2, 2, 2], [1.0] * 3)
    with _Hooks(scan_delay_bin=bin_, scan_delay_sleeps=_LATE):
        out, counts = P.partition_device(ids, 8, pos0.clone())
        torch.cuda.synchronize()
        assert np.array_equal(counts.cpu().numpy(), np.diff(exp_off))
        assert np.array_equal(out[: 8 * n].view(torch.int64).cpu().numpy(), exp)
    with _Hooks(scan_delay_bin=bin_, scan_delay_sleeps=_LATE, scan_end_spins=0):
        out, counts = P.partition_device(ids, 8, pos0.clone())
        c = counts.cpu().numpy()
    assert c[bin_] == -1 and c[bin_ + 1] == -1, c      # the late word was seen
    out, counts = P.partition_device(ids, 8, pos0.clone())   # defaults again
    assert np.array_equal(counts.cpu().numpy(), np.diff(exp_off))


@pytest.mark.parametrize("bin_", [0, 300])
def test_scan_race_fine_late_inclusive_word(bin_):
    """The same forced race in the config-5 destination scan: 512 fine cells x
    16384 ranked tiles (2^26 ids, 2 chunks per bin, 8192 counts per chunk):
    counts and the stable sort exact against numpy's stable argsort."""
    from mpi_grid_redistribute_amd.redistributor import _IdField, _sort_by_ids
    n, nb = 1 << 26, 512
    rng = np.random.default_rng(bin_)
    ids_h = rng.integers(0, nb, n).astype(np.uint16)
    ids = torch.from_numpy(ids_h.view(np.int16)).cuda()
    rows = _IdField(torch.arange(n, dtype=torch.int32, device="cuda").view(torch.uint8))
    rows.row_bytes = 4
    order = np.argsort(ids_h, kind="stable").astype(np.int32)
    cnt = np.bincount(ids_h, minlength=nb)
    dev = torch.device("cuda", torch.cuda.current_device())
    with _Hooks(scan_delay_bin=bin_, scan_delay_sleeps=_LATE):
        outs, counts = _sort_by_ids([rows], ids, n, nb, dev, check_ids=False)
        torch.cuda.synchronize()
        assert np.array_equal(counts.cpu().numpy(), cnt)
        assert np.array_equal(outs[0][: 4 * n].view(torch.int32).cpu().numpy(), order)
    with _Hooks(scan_delay_bin=bin_, scan_delay_sleeps=_LATE, scan_end_spins=0):
        _, counts = _sort_by_ids([rows], ids, n, nb, dev, check_ids=False)
        c = counts.cpu().numpy()
    assert c[bin_] == -1 and c[bin_ + 1] == -1


def test_single_rank_scan_failure_raises():
    pos, rec = mgr.synth_uniform(1 << 20, seed=6)
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    _lib.test_hook("scan_spins", -1)
    try:
        with pytest.raises(_lib.MgrError, match="scan failed"):
            R.redistribute_by_cell_number(rec, torch.zeros(1 << 20, dtype=torch.int64,
                                                           device="cuda"))
    finally:
        _lib.test_hook("scan_spins", 1 << 24)


@pytest.mark.parametrize("n", [1, 1 << 22])
def test_single_rank_position_scan_failure_raises(n):
    """One rank keeping every row: the pack is launched without a count read
    (the output holds n rows); the counts, read behind the pack, still raise.
    The failure is forced deterministically: scan chunk 0 publishes its
    prefix poisoned (test hook scan_poison_chunk), every prefix built on it
    carries the bit, the scan reports -1 counts and the pack writes nothing
    -- on the first call, with one chunk or many."""
    pos, rec = mgr.synth_uniform(n, seed=7)
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    with _Hooks(scan_poison_chunk=0):
        with pytest.raises(_lib.MgrError, match="scan failed"):
            R.redistribute_by_position(rec, pos.clone())
    out = R.redistribute_by_position(rec, pos.clone())
    assert torch.equal(out, rec)


def test_halo_scan_failure_raises():
    """The halo's selection scans (mgr_msel_count + mgr_scan) failing: the -1
    counts are checked at the halo's first host sync and raise, instead of
    turning into negative slices and mismatched messages."""
    rng = np.random.default_rng(8)
    n = 200_000
    pos = rng.random((n, 3))
    data = np.arange(n)
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    _lib.test_hook("scan_spins", -1)
    try:
        with pytest.raises(_lib.MgrError, match="scan failed"):
            R.exchange_overload_by_position(data, pos, [0.1, 0.1, 0.1])
    finally:
        _lib.test_hook("scan_spins", 1 << 24)
    out = R.exchange_overload_by_position(data, pos, [0.1, 0.1, 0.1])
    assert len(out) > 0


@pytest.mark.parametrize("ol", [0.1, 0.45])
def test_one_rank_halo_deferred_count_check_raises(ol):
    """One rank with overload_lengths: the redistribution's counts are not
    read back (all rows stay) -- a failed scan must still raise, at the
    halo's host read."""
    rng = np.random.default_rng(9)
    n = 200_000
    pos = rng.random((n, 3))
    data = np.arange(n)
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    ol = [ol] * 3
    _lib.test_hook("scan_spins", -1)
    try:
        with pytest.raises(_lib.MgrError, match="scan failed"):
            R.redistribute_by_position(data, pos.copy(), overload_lengths=ol)
    finally:
        _lib.test_hook("scan_spins", 1 << 24)
    out = R.redistribute_by_position(data, pos.copy(), overload_lengths=ol)
    assert len(out) > n


def test_no_device_allocation_after_warmup():
    """Skewed inputs of changing size on repeated calls: after warm-up the
    redistributor reuses its scratch (workspace, destination bytes, send
    buffers) and the caching allocator serves the fresh outputs -- no new
    device segment (hipMalloc) per call."""
    from mpi_grid_redistribute_amd.redistributor import Scratch
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    assert isinstance(R._scratch, Scratch)
    base = 1 << 22
    inputs = []
    for k in range(6):
        n = base - 10_000 * k
        pos, rec = mgr.synth_clustered(n, seed=k)
        inputs.append((pos, rec))
    for pos, rec in inputs[:2]:
        R.redistribute_by_position(rec, pos)
    torch.cuda.synchronize()
    seg0 = torch.cuda.memory_stats()["segment.all.allocated"]
    for pos, rec in inputs[2:]:
        out = R.redistribute_by_position(rec, pos)
        del out
    torch.cuda.synchronize()
    assert torch.cuda.memory_stats()["segment.all.allocated"] == seg0


def test_scratch_per_stream_capped():
    """Calls on many streams keep at most Scratch.MAX_STREAMS sets of scratch
    buffers (the least recently used stream is waited for and its set freed),
    and every call's result stays correct."""
    R = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    R2 = MPIGridRedistributor(None, [1, 1, 1], [1.0] * 3)
    n = 200_003
    pos, rec = mgr.synth_uniform(n, seed=77)
    want = R2.redistribute_by_position(rec.clone(), pos.clone())
    streams = [torch.cuda.Stream() for _ in range(R._scratch.MAX_STREAMS + 3)]
    outs = []
    for st in streams:
        with torch.cuda.stream(st):
            outs.append(R.redistribute_by_position(rec.clone(), pos.clone()))
        assert len(R._scratch.streams) <= R._scratch.MAX_STREAMS
        assert len({k[1] for k in R._scratch.bufs}) <= R._scratch.MAX_STREAMS
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, want)


@pytest.mark.parametrize("rb", [1, 2, 3, 12, 32, 36])
@pytest.mark.parametrize("n", [1, 15, 4097, 100_003])
def test_one_bin_pack_is_the_input(rb, n):
    """One bin, nothing dropped (a rank keeping its rows): the stable pack is
    the array itself, fine cells carried beside the rows, from a 16-byte
    aligned and from a misaligned source (the pack's unit width follows the
    alignment)."""
    rng = np.random.default_rng(n * 7 + rb)
    P = GridPartitioner([1, 1, 1], [1.0] * 3)
    pos = torch.from_numpy(rng.random((n, 3))).cuda()
    raw = torch.from_numpy(rng.integers(0, 256, n * rb + 16, dtype=np.uint8)).cuda()
    for off in (0, 1):   # 16-byte aligned source, then a misaligned one
        data = raw[off: off + n * rb]
        out, counts = P.partition_device(data, rb, pos.clone())
        assert int(counts[0]) == n
        assert torch.equal(out[: n * rb], data)
    out, fids, counts = P.partition_device(raw[: n * rb], rb, pos.clone(), fine_cells=[4, 4, 4])
    exp_f = ((pos.cpu().numpy() * 4).astype(np.int64) % 4) @ np.array([16, 4, 1])
    assert torch.equal(out[: n * rb], raw[: n * rb])
    assert np.array_equal(fids.cpu().numpy().astype(np.int64), exp_f)
