"""Full-size parity of the bench's own config-5 step:
the exact work ``bench.py --config 5`` times per step, at its size -- 64M
36-byte records partitioned into the 2x2x2 grid with their 8x8x8 fine cells
(GridPartitioner.partition_device(..., fine_cells=)) and the destination-side
fine-cell sort of 64M received rows (MPIGridRedistributor.fine_cell_sort(...,
fine_ids=)) -- bit-exact against the C oracle (wrap + bin + stable partition,
redist.py:63-90, :195-198) plus the fine-cell restatement
(oracle/redist_oracle.fine_cell_ids) and a stable partition by fine cell.

Configs 3 and 4 at full size (125M rows per rank over RCCL) are the
``fullsize`` set of tests/rccl_worker.py (tests/test_gpu_multi.py).
"""
import numpy as np
import pytest
import torch

from oracle import c_oracle
from oracle import redist_oracle as ro

pytestmark = pytest.mark.gpu

mgr = pytest.importorskip("mpi_grid_redistribute_amd")
from mpi_grid_redistribute_amd import GridPartitioner, MPIGridRedistributor  # noqa: E402

SEED = 20261015          # bench.py's seed
N = 1 << 26              # bench.py config 5 at one GPU (512M / 8)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _fine_ids(pos_f32, topo, fine, box):
    """oracle fine cell of every row (global fine grid topo * fine, index
    wrap, k % fine, row-major), through the C oracle's binning at N rows."""
    glob = [t * k for t, k in zip(topo, fine)]
    _, idx = c_oracle.bin_positions(pos_f32.copy(), glob, box, periodic=False, want_idx=True)
    k = ro.periodic_wrap(idx, np.array(glob)) % np.array(fine)
    del idx
    return (k[:, 0] * fine[1] + k[:, 1]) * fine[2] + k[:, 2]


def test_cfg5_bench_step_full_size():
    topo, box, fine = [2, 2, 2], [1.0, 1.0, 1.0], [8, 8, 8]
    # ---- source side: 64M records into the 2x2x2 grid, fine cells alongside
    rec, pos = mgr.synth_wide(N, seed=SEED, gid0=0)
    rec_h = rec.cpu().numpy()                                   # (N, 36) uint8, input
    part = GridPartitioner(topo, box)
    out, fids, counts = part.partition_device(rec.reshape(-1), 36, pos, fine_cells=fine)
    torch.cuda.synchronize()
    p_h = np.ascontiguousarray(rec_h.view(np.float32)[:, :3])
    cell = c_oracle.bin_positions(p_h, topo, box)               # wraps p_h in place (S1, S9)
    exp_rec = rec_h.copy()
    exp_rec.view(np.float32)[:, :3] = p_h                        # the in-place wrap of the view
    del rec_h
    assert np.array_equal(rec.cpu().numpy(), exp_rec), "wrapped positions in the records"
    exp, exp_off = c_oracle.partition(exp_rec, cell, 8)
    assert np.array_equal(counts.cpu().numpy(), np.diff(exp_off)), "source counts"
    assert np.array_equal(out[: N * 36].cpu().numpy().reshape(N, 36), exp), "source partition"
    del exp
    fid = _fine_ids(p_h, topo, fine, box).astype(np.uint16)
    exp_fid, _ = c_oracle.partition(fid, cell, 8)
    assert np.array_equal(fids.cpu().numpy().view(np.uint16), exp_fid), "fine ids at the source"
    del exp_rec, p_h, cell, fid, exp_fid, out, fids, rec, pos

    # ---- destination side: 64M rows received in one cell, sorted by fine cell
    recv, rpos = mgr.synth_wide(N, seed=SEED + 1, gid0=0, hi=0.5)
    R1 = MPIGridRedistributor(None, [1, 1, 1], [0.5, 0.5, 0.5])
    _, recv_fids, _ = GridPartitioner([1, 1, 1], [0.5] * 3).partition_device(
        recv.reshape(-1), 36, rpos, fine_cells=fine)
    recv_fids = recv_fids.clone()
    sorted_, off = R1.fine_cell_sort(recv, rpos, fine, fine_ids=recv_fids)
    torch.cuda.synchronize()
    recv_h = recv.cpu().numpy()
    rp = np.ascontiguousarray(recv_h.view(np.float32)[:, :3])
    fid = _fine_ids(rp, [1, 1, 1], fine, [0.5] * 3)
    assert np.array_equal(recv_fids.cpu().numpy().view(np.uint16), fid.astype(np.uint16)), \
        "fine ids of the received rows"
    exp, exp_off = c_oracle.partition(recv_h, fid, 512)
    assert np.array_equal(off.cpu().numpy(), exp_off), "fine offsets"
    assert np.array_equal(sorted_.cpu().numpy().reshape(N, 36), exp), "fine-sorted rows"
