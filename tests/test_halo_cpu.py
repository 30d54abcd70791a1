"""Overload (halo) exchange host logic on CPU (no GPU): neighbour ranks,
selection order (local rows, then earlier dimensions' received rows), the
two send/receive steps per dimension, buffer growth concat(buffer, from_a,
from_b) and the periodic=False flag quirk -- through the same
``halo.exchange_overload`` the GPU path uses, with the selections done by a
NumPy stand-in instead of the HIP kernels.  Checked against the reference's
own outputs (tests/golden/halo_*.npz).

* world_size 2 and 4 with torch.distributed ``gloo`` (TorchDistComm.sendrecv);
* 6-27 threaded ranks on the mpi4py-style fake comm (MpiHostComm.sendrecv).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpi_grid_redistribute_amd import _lib
from mpi_grid_redistribute_amd.comm import MpiHostComm, TorchDistComm
from mpi_grid_redistribute_amd.halo import exchange_overload
from oracle import redist_oracle as ro
from tests import golden_io as G
from tests.fake_mpi import run_ranks


class GeoRank:
    """The host geometry the halo orchestration reads from an
    MPIGridRedistributor (redist.py:16-61, :73-85)."""

    def __init__(self, topo, box, size, rank):
        g = ro.Geometry(topo, box, size, rank)
        self._g = g
        self.dim = g.dim
        self.grid_topology = g.grid_topology
        self.rank_cell_index = g.rank_cell_index
        self.rank_cell_limits = g.rank_cell_limits

    def get_cell_number_from_indexes_host(self, idx, periodic=True):
        return ro.cell_number_from_indexes(self._g, idx, periodic=periodic)


class CpuSelect:
    """NumPy stand-in for halo.DeviceSelect (mgr_halo_flags / mgr_select_count
    / mgr_scan / mgr_pack)."""

    def flags(self, pos_flat, n, ncols, code, dim, hi, lo):
        dt = np.float32 if code == _lib.MGR_F32 else np.float64
        p = pos_flat.numpy().view(dt).reshape(n, ncols).astype(np.float64)
        f = np.zeros(n, dtype=np.uint16)
        for d in range(dim):
            f |= (p[:, d] > hi[d]).astype(np.uint16) << (2 * d)
            f |= (p[:, d] < lo[d]).astype(np.uint16) << (2 * d + 1)
        return torch.from_numpy(f.view(np.int16))

    def select(self, flags, n, mask, max_row_bytes):
        idx = np.nonzero(flags.numpy().view(np.uint16)[:n] & mask)[0]
        return (idx,), torch.tensor([len(idx)], dtype=torch.int64)

    def pack(self, handle, src_flat, row_bytes, dst_flat):
        idx = handle[0]
        rows = src_flat.numpy().reshape(-1, row_bytes)[idx].reshape(-1)
        dst_flat[: rows.size].copy_(torch.from_numpy(rows.copy()))

    def pack2(self, handle, src1, rb1, dst1, src2, rb2, dst2):
        self.pack(handle, src1, rb1, dst1)
        self.pack(handle, src2, rb2, dst2)


def _flat(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy())


def local_inputs(f, case):
    """Per-rank local rows + positions for the halo step: for the
    redistribute fixtures, the main redistribution done by the oracle."""
    size = int(f["size"])
    topo, box = f["topology"], f["box"]
    data = G.per_rank(f, "data", size)
    if case.startswith("halo_direct_"):
        return data, G.per_rank(f, "pos", size), False
    pos = [p.copy() for p in G.per_rank(f, "pos_in", size)]
    dest = [ro.cell_number_from_position(ro.Geometry(topo, box, size, r), pos[r])
            for r in range(size)]
    local = ro.redistribute_by_cell_number_all_ranks(size, data, dest)
    local_pos = ro.redistribute_by_cell_number_all_ranks(size, pos, dest)
    return local, local_pos, True


def run_rank(f, case, transport, r, spare=None):
    """``spare``: None = the overload gets a store of its own; else the local
    rows sit at the head of a store with ``spare`` free rows after them (the
    layout redistribute_by_position hands over) and the halo appends there."""
    size = int(f["size"])
    data, pos, periodic = local_inputs(f, case)
    R = GeoRank(f["topology"], f["box"], size, r)
    d, p = data[r], pos[r]
    code = _lib.MGR_F32 if p.dtype == np.float32 else _lib.MGR_F64
    rbd = d.dtype.itemsize * int(np.prod(d.shape[1:], dtype=np.int64))
    rbp = p.dtype.itemsize * p.shape[1]
    n = len(d)
    d_flat, p_flat, arena = _flat(d), _flat(p), None
    if spare is not None:
        st_d = torch.full(((n + spare) * rbd,), 0xA5, dtype=torch.uint8)
        st_p = torch.full(((n + spare) * rbp,), 0x5A, dtype=torch.uint8)
        st_d[: n * rbd].copy_(d_flat)
        st_p[: n * rbp].copy_(p_flat)
        d_flat, p_flat, arena = st_d[: n * rbd], st_p[: n * rbp], (st_d, st_p, n, spare)
    ov_d, ov_p, m, in_arena = exchange_overload(R, transport, d_flat, rbd, p_flat, p.shape[1],
                                                code, n, list(f["overload"]), periodic=periodic,
                                                sel=CpuSelect(), arena=arena)
    if spare is not None:
        assert in_arena == (m <= spare), (m, spare, in_arena)
        assert torch.equal(st_d[: n * rbd], _flat(d)), "the local rows were overwritten"
        if in_arena and periodic:
            whole = st_d[: (n + m) * rbd].numpy().view(d.dtype).reshape((n + m,) + d.shape[1:])
            assert np.array_equal(st_p[n * rbp:(n + m) * rbp].numpy(), ov_p.numpy())
            return whole
    ov = ov_d.numpy().view(d.dtype).reshape((m,) + d.shape[1:])
    return np.concatenate([d, ov]) if periodic else ov


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, size, port, case):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        f = G.load(case)
        got = run_rank(f, case, TorchDistComm(), rank)
        assert G.same_bytes(got, f[f"r{rank}_out"]), (case, rank)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["halo_p2_f32_rec36.npz", "halo_p4_2d_mat.npz"])
def test_gloo_halo(case):
    size = int(G.load(case)["size"])
    mp.spawn(_gloo_worker, args=(size, _free_port(), case), nprocs=size, join=True)


@pytest.mark.parametrize("case", ["halo_p8_f64_rec32.npz", "halo_p8_wide.npz",
                                  "halo_p27_333_ids.npz", "halo_p6_321_i32.npz",
                                  "halo_p1_self.npz", "halo_direct_p6_321_nonperiodic.npz",
                                  "halo_direct_p8_nonperiodic.npz"])
def test_threaded_halo(case):
    f = G.load(case)
    size = int(f["size"])
    outs = run_ranks(size, lambda comm, r: run_rank(f, case, MpiHostComm(comm), r)
                     if size > 1 else run_rank(f, case, _SelfT(), r))
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)


@pytest.mark.parametrize("spare", [0, 3, 40, 10**6])
@pytest.mark.parametrize("case", ["halo_p8_f64_rec32.npz", "halo_p1_self.npz",
                                  "halo_direct_p8_nonperiodic.npz"])
def test_threaded_halo_in_place(case, spare):
    """The halo rows appended in place after the local rows (the arena that
    redistribute_by_position passes), fitting or outgrowing the spare rows."""
    f = G.load(case)
    size = int(f["size"])
    outs = run_ranks(size, lambda comm, r: run_rank(f, case, MpiHostComm(comm), r, spare)
                     if size > 1 else run_rank(f, case, _SelfT(), r, spare))
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r, spare)


class _SelfT:
    rank, size = 0, 1

    def sendrecv(self, send, dest, recv, source):
        recv.copy_(send)
