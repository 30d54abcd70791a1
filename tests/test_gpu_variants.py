"""GPU parity of every kernel variant the tuning knobs select (mgr_tune).

The shipped defaults are covered by test_gpu_parity.py; here each non-default
variant (XCD-contiguous tile order, unconditional position write-back, tile
shapes, scan chunking, the generic pack) must give the same bytes on the same inputs: the C
oracle on seeded inputs, and the reference's own golden fixtures.
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

DEFAULTS = {"xcd_pack": 16, "xcd_bin": 0, "bin_skip_clean": 1, "bin_waves": 0, "pack_coop": 1,
            "many_rows": 0, "bin_staged": 1, "tile_rounds": 0,
            "pack_many": 1, "scan_chunk": 2048, "pack_img": 1, "many_super": 1,
            "scan_max_chunks": 1024, "pack_sel": 1, "pack_compact": 1, "bin_geo": 1, "rank_rows": 0,
            "img_rpw": 2, "ranked_walk": 0,
            "rank_orm": 1}
VARIANTS = [
    {"img_rpw": 1},
    {"img_rpw": 1, "tile_rounds": 1},
    {"img_rpw": 2, "tile_rounds": 16, "pack_sel": 0},
    {"bin_geo": 0},
    {"bin_geo": 0, "bin_skip_clean": 0},
    {"xcd_pack": 1, "xcd_bin": 1},
    {"bin_skip_clean": 0},
    {"tile_rounds": 8},
    {"bin_waves": 16, "xcd_pack": 1},
    {"bin_waves": 8, "bin_skip_clean": 0},
    {"bin_waves": 2},
    {"bin_skip_clean": 0, "bin_staged": 0},
    {"bin_waves": 1, "xcd_bin": 1},
    {"xcd_pack": 0},
    {"pack_coop": 0},
    {"pack_coop": 0, "xcd_pack": 0},
    {"pack_many": 0},
    {"xcd_pack": 4},
    {"xcd_pack": 64, "tile_rounds": 1},
    {"tile_rounds": 1},
    {"scan_chunk": 256, "tile_rounds": 1},
    {"scan_chunk": 4096},
    {"pack_img": 0},
    {"pack_sel": 0},
    {"pack_compact": 0},
    {"many_super": 4},
    {"scan_max_chunks": 4096},
    {"scan_max_chunks": 8, "scan_chunk": 256},
    {"many_super": 16, "xcd_pack": 0},
    {"pack_img": 1, "tile_rounds": 16},
    {"pack_img": 1, "xcd_pack": 0, "tile_rounds": 1},
    {"scan_chunk": 65536},
    {"many_rows": 4096},
    {"many_rows": 2048, "many_super": 2},
    {"many_rows": 1024},
    {"many_rows": 1024, "many_super": 4},
]


@pytest.fixture(params=VARIANTS, ids=lambda v: ",".join(f"{k}={x}" for k, x in v.items()))
def variant(request):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    for k, v in request.param.items():
        _lib.tune(k, v)
    yield request.param
    for k, v in DEFAULTS.items():
        _lib.tune(k, v)


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
    P = GridPartitioner(topo, box)
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
        return MPIGridRedistributor(comm, topo, box).redistribute_by_position(
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


@pytest.mark.parametrize("img_rpw", [1, 2])
@pytest.mark.parametrize("row_bytes", [12, 20, 24, 28, 36, 40, 44, 52, 56, 60])
@pytest.mark.parametrize("topo", [[2, 2, 2], [4, 4, 4], [7], [1]])
def test_image_pack_row_sizes(row_bytes, topo, img_rpw):
    """pack_img (16-byte image pack) for every row size it takes, ragged n,
    1..64 bins, against the C oracle."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    _lib.tune("pack_img", 2)     # every row size the image pack takes
    _lib.tune("img_rpw", img_rpw)
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
        _lib.tune("pack_img", DEFAULTS["pack_img"])
        _lib.tune("img_rpw", DEFAULTS["img_rpw"])


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
        return MPIGridRedistributor(comm if size > 1 else None, topo, box).redistribute_by_position(
            data[r], pos[r], overload_lengths=ol)

    outs = run_ranks(size, fn)
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)
