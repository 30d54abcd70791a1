"""GPU parity of every path the test hooks force (include/mgr_instrument.h
mgr_test_hook) and of the per-plan write-back option.

The shipped defaults are covered by test_gpu_parity.py; here each fallback
the product reaches on other inputs (unstaged bin slabs, run-time geometry,
the generic pack, the image pack's narrow rows), every tile shape and scan
chunking, and the unconditional position write-back must give the same bytes
on the same inputs: the C oracle on seeded inputs, and the reference's own
golden fixtures.
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from tests import golden_io as G
from tests.fake_mpi import run_ranks

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import GridPartitioner, MPIGridRedistributor, _lib  # noqa: E402

VARIANTS = [
    {"tile_rounds": 1},
    {"tile_rounds": 8},
    {"tile_rounds": 16},
    {"tile_rounds": 32},   # 2048-row tiles: the coop pack's largest
    {"tile_rounds": 64},   # 4096-row tiles: coop / image packs refuse -> generic pack
    {"bin_generic": 1},
    {"bin_generic": 1, "write_back": "all"},
    {"write_back": "all"},
    {"bin_unstaged": 1},
    {"bin_unstaged": 1, "write_back": "all", "tile_rounds": 1},
    {"pack_generic": 1},
    {"pack_generic": 1, "tile_rounds": 1},
    {"scan_chunk": 256, "tile_rounds": 1},
    {"scan_chunk": 4096},
    {"scan_chunk": 65536},
    {"scan_max_chunks": 4096},
    {"scan_max_chunks": 8, "scan_chunk": 256},
    {"pack_img_all": 1},
    {"pack_img_all": 1, "tile_rounds": 16},
]


@pytest.fixture(params=VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def variant(request):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    for k, v in request.param.items():
        if k != "write_back":
            _lib.test_hook(k, v)
    yield request.param
    for k, v in _lib.HOOK_DEFAULTS.items():
        _lib.test_hook(k, v)


def _wb(obj, variant):
    obj.set_write_back(variant.get("write_back", "changed"))
    return obj


@pytest.mark.parametrize("topo,row_bytes", [([2, 2, 2], 32), ([2, 2, 2], 36), ([7], 8),
                                            ([4, 4, 4], 12), ([3, 3, 3], 64), ([2], 4),
                                            ([8, 8, 8], 36), ([5, 6, 10], 24), ([9, 9, 9], 36)])
def test_partition_variant_vs_c_oracle(variant, topo, row_bytes):
    rng = np.random.default_rng(row_bytes * 7 + len(topo))
    n = 70_001 + row_bytes
    dim = len(topo)
    box = [1.0] * dim
    pos = rng.uniform(0.0, 1.0, (n, dim))
    # a few out-of-box rows: some 64-row slabs are dirty, most are clean
    k = rng.integers(0, n, 300)
    pos[k] = rng.uniform(-1.0, 2.0, (300, dim))
    data = rng.integers(0, 256, (n, row_bytes), dtype=np.uint8)
    exp_pos = pos.copy()
    cell = c_oracle.bin_positions(exp_pos, topo, box)
    nb = int(np.prod(topo))
    exp, exp_off = c_oracle.partition(data, cell, nb)
    P = _wb(GridPartitioner(topo, box), variant)
    tpos = torch.from_numpy(pos).cuda()
    out, off = P.partition_by_position(torch.from_numpy(data).cuda(), tpos)
    assert G.same_bytes(tpos.cpu().numpy(), exp_pos)
    assert np.array_equal(off.cpu().numpy(), exp_off)
    assert np.array_equal(out.cpu().numpy(), exp)


@pytest.mark.parametrize("case", ["redist_p8_f64_rec32.npz", "redist_p8_rec36_view.npz",
                                  "redist_p27_333_ids.npz", "redist_p2_f32_rec36.npz"])
def test_golden_variant(variant, case):
    f = G.load(case)
    size = int(f["size"])
    topo, box, periodic = f["topology"], f["box"], bool(f["periodic"])
    pos = [p.copy() for p in G.per_rank(f, "pos_in", size)]
    if bool(f["alias"]):
        data = pos
    elif "view" in case:
        data = [d.copy() for d in G.per_rank(f, "data", size)]
        pos = [d["pos"] for d in data]
    else:
        data = [d.copy() for d in G.per_rank(f, "data", size)]

    def fn(comm, r):
        return _wb(MPIGridRedistributor(comm, topo, box), variant).redistribute_by_position(
            data[r], pos[r], periodic=periodic)

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(pos[r], f[f"r{r}_pos_out"]), (case, r)
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)


def test_cellnum_drop_variant(variant):
    f = G.load("cellnum_p5_f32mat.npz")
    size = int(f["size"])

    def fn(comm, r):
        return MPIGridRedistributor(comm, [size], [1.0]).redistribute_by_cell_number(
            f[f"r{r}_data"], f[f"r{r}_ids"])

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), r


@pytest.mark.parametrize("row_bytes", [12, 20, 24, 28, 36, 40, 44, 52, 56, 60])
@pytest.mark.parametrize("topo", [[2, 2, 2], [4, 4, 4], [7], [1]])
def test_image_pack_row_sizes(row_bytes, topo):
    """pack_img (16-byte image pack) for every row size it takes, ragged n,
    1..64 bins, against the C oracle."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    _lib.test_hook("pack_img_all", 1)     # every row size the image pack takes
    try:
        rng = np.random.default_rng(row_bytes * 31 + len(topo))
        n = 50_003 + 7 * row_bytes
        dim = len(topo)
        pos = rng.uniform(-0.5, 1.5, (n, dim))
        data = rng.integers(0, 256, (n, row_bytes), dtype=np.uint8)
        exp_pos = pos.copy()
        cell = c_oracle.bin_positions(exp_pos, topo, [1.0] * dim)
        exp, exp_off = c_oracle.partition(data, cell, int(np.prod(topo)))
        P = GridPartitioner(topo, [1.0] * dim)
        out, off = P.partition_by_position(torch.from_numpy(data).cuda(),
                                           torch.from_numpy(pos).cuda())
        assert np.array_equal(off.cpu().numpy(), exp_off)
        assert np.array_equal(out.cpu().numpy(), exp)
    finally:
        _lib.test_hook("pack_img_all", 0)


@pytest.mark.parametrize("case", ["halo_p8_f64_rec32.npz", "halo_p2_f32_rec36.npz",
                                  "halo_p27_333_ids.npz"])
def test_halo_variant(variant, case):
    """The overload exchange (selection packs: compaction, coop, image) under
    every variant, against the reference's own outputs."""
    f = G.load(case)
    size = int(f["size"])
    topo, box, ol = f["topology"], f["box"], list(f["overload"])
    data = [d.copy() for d in G.per_rank(f, "data", size)]
    pos = [p.copy() for p in G.per_rank(f, "pos_in", size)]

    def fn(comm, r):
        R = _wb(MPIGridRedistributor(comm if size > 1 else None, topo, box), variant)
        return R.redistribute_by_position(data[r], pos[r], overload_lengths=ol)

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)


@pytest.mark.parametrize("row_bytes", [4, 7, 12, 32, 36, 72])
def test_one_rank_cell_number_drops(row_bytes):
    """One rank, ids outside [0, 1) dropped (S6): the 2-bin selection with a
    drop bin through the coop / image packs (the selection variant that loads
    only kept rows) and the generic pack for > 64-byte rows."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from oracle import redist_oracle as ro
    rng = np.random.default_rng(row_bytes)
    n = 90_001
    data = rng.integers(0, 256, (n, row_bytes), dtype=np.uint8)
    ids = rng.integers(-1, 3, n)                     # -1, 1, 2 dropped; 0 kept
    exp = ro.redistribute_by_cell_number_all_ranks(1, [data], [ids])[0]
    got = MPIGridRedistributor(None, [1], [1.0]).redistribute_by_cell_number(data, ids)
    assert np.array_equal(got, exp)
