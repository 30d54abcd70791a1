"""Overload (halo) exchange host logic on CPU (no GPU): neighbour ranks,
selection order (local rows, then earlier dimensions' received rows), the
two send/receive steps per dimension, buffer growth concat(buffer, from_a,
from_b) and the periodic=False flag quirk -- through the same
``halo.exchange_overload`` the GPU path uses, with the selections done by a
NumPy stand-in instead of the HIP kernels.  Checked against the reference's
own outputs (tests/golden/halo_*.npz).

* world_size 2 and 4 with torch.distributed ``gloo`` (TorchDistComm.p2p);
* 6-27 threaded ranks on the mpi4py-style fake comm (MpiHostComm.p2p).
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
        self.cell_length = np.asarray(box, dtype=np.float64) / np.asarray(topo)

    def get_cell_number_from_indexes_host(self, idx, periodic=True):
        return ro.cell_number_from_indexes(self._g, idx, periodic=periodic)


_POS_NP = {_lib.MGR_F16: np.dtype(np.float16), _lib.MGR_F32: np.dtype(np.float32),
           _lib.MGR_F64: np.dtype(np.float64), _lib.MGR_I32: np.dtype(np.int32),
           _lib.MGR_I64: np.dtype(np.int64)}


class CpuSelect:
    """NumPy stand-in for halo.DeviceSelect (mgr_halo_flags / mgr_msel_count
    / mgr_scan / mgr_msel_pack)."""

    def _buf(self, name, nbytes):
        return torch.empty(max(int(nbytes), 1), dtype=torch.uint8)

    def flags(self, pos_flat, n, ncols, code, dim, hi, lo):
        dt = _POS_NP[code]
        p = pos_flat.numpy().view(dt).reshape(n, ncols).astype(np.float64)
        f = np.zeros(n, dtype=np.uint16)
        for d in range(dim):
            f |= (p[:, d] > hi[d]).astype(np.uint16) << (2 * d)
            f |= (p[:, d] < lo[d]).astype(np.uint16) << (2 * d + 1)
        return torch.from_numpy(f.view(np.int16))

    def msel(self, flags, n, bits, tag):
        return self.msel_masks(flags, n, [1 << int(b) for b in bits], tag)

    def msel_masks(self, flags, n, masks, tag):
        fl = flags.numpy().view(np.uint16)[:n]
        sets = [np.nonzero((fl & m) == m)[0] for m in masks]
        return sets, torch.tensor([len(s) for s in sets], dtype=torch.int64)

    def msel_pack(self, handle, src_flat, row_bytes, dsts):
        src = src_flat.numpy()
        rows = src[: (len(src) // row_bytes) * row_bytes].reshape(-1, row_bytes)
        for idx, d in zip(handle, dsts):
            if d is not None and len(idx):
                d[: len(idx) * row_bytes].copy_(torch.from_numpy(rows[idx].reshape(-1).copy()))

    def msel_pack_fields(self, handle, srcs, row_bytes, dsts, rows_out=0):
        for src, rb, d in zip(srcs, row_bytes, dsts):
            self.msel_pack(handle, src, rb, [t if t0 is not None else None
                                             for t, t0 in zip(d, dsts[0])])

    def msel_pack_placed(self, handle, srcs, row_bytes, dsts, cap_rows):
        """Sets back to back from dsts[f]; rows at or beyond cap_rows dropped."""
        for src, rb, d in zip(srcs, row_bytes, dsts):
            s = src.numpy()
            rows = s[: (len(s) // rb) * rb].reshape(-1, rb)
            idx = np.concatenate(list(handle))[:cap_rows] if len(handle) else np.zeros(0, int)
            if len(idx):
                d[: len(idx) * rb].copy_(torch.from_numpy(rows[idx].reshape(-1).copy()))

    def to_host(self, tensors):
        return [t.numpy().copy() for t in tensors]

    def to_host_start(self, tensors):
        return self.to_host(tensors)

    @staticmethod
    def to_host_wait(read):
        return read


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


def run_rank(f, case, transport, r, spare=None, carry_pos=True):
    """``spare``: None = the overload gets a store of its own; else the local
    rows sit at the head of a store with ``spare`` free rows after them (the
    layout redistribute_by_position hands over) and the halo appends there."""
    size = int(f["size"])
    data, pos, periodic = local_inputs(f, case)
    R = GeoRank(f["topology"], f["box"], size, r)
    d, p = data[r], pos[r]
    code = {v: k for k, v in _POS_NP.items()}[p.dtype]
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
    flags = None
    if not carry_pos:   # flags computed up front, positions not carried
        from mpi_grid_redistribute_amd.halo import thresholds
        hi, lo = thresholds(R, list(f["overload"]))
        flags = CpuSelect().flags(p_flat, n, p.shape[1], code, R.dim, hi, lo)
        p_flat = None
        if arena is not None:
            arena = (arena[0], None, n, spare)
    ov_d, ov_p, m, in_arena = exchange_overload(R, transport, d_flat, rbd, p_flat, p.shape[1],
                                                code, n, list(f["overload"]), periodic=periodic,
                                                sel=CpuSelect(), arena=arena, flags=flags)
    assert (ov_p is None) == (not carry_pos)
    if spare is not None:
        assert in_arena == (m <= spare), (m, spare, in_arena)
        assert torch.equal(st_d[: n * rbd], _flat(d)), "the local rows were overwritten"
        if in_arena and periodic:
            whole = st_d[: (n + m) * rbd].numpy().view(d.dtype).reshape((n + m,) + d.shape[1:])
            if carry_pos:
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
@pytest.mark.parametrize("carry_pos", [True, False])
def test_threaded_halo(case, carry_pos):
    f = G.load(case)
    size = int(f["size"])
    outs = run_ranks(size, lambda comm, r: run_rank(f, case, MpiHostComm(comm), r,
                                                    carry_pos=carry_pos)
                     if size > 1 else run_rank(f, case, _SelfT(), r, carry_pos=carry_pos))
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r)


@pytest.mark.parametrize("spare", [0, 3, 40, 10**6])
@pytest.mark.parametrize("case", ["halo_p8_f64_rec32.npz", "halo_p1_self.npz",
                                  "halo_direct_p8_nonperiodic.npz"])
@pytest.mark.parametrize("carry_pos", [True, False])
def test_threaded_halo_in_place(case, spare, carry_pos):
    """The halo rows appended in place after the local rows (the arena that
    redistribute_by_position passes), fitting or outgrowing the spare rows."""
    f = G.load(case)
    size = int(f["size"])
    outs = run_ranks(size, lambda comm, r: run_rank(f, case, MpiHostComm(comm), r, spare,
                                                    carry_pos)
                     if size > 1 else run_rank(f, case, _SelfT(), r, spare, carry_pos))
    for r in range(size):
        assert G.same_bytes(outs[r], f[f"r{r}_out"]), (case, r, spare)


def _SelfT():
    from mpi_grid_redistribute_amd.comm import SelfComm
    return SelfComm()


def test_halo_capacity_clamped():
    """halo_capacity caps the overload length at the cell length (the
    exchange reaches the immediate neighbours only): ol >> cl reserves at
    most (3^dim - 1) * m * 1.25 + 4096 rows, not a polynomial blow-up."""
    from mpi_grid_redistribute_amd.halo import halo_capacity
    R = GeoRank([2, 2, 2], [1.0, 1.0, 1.0], 8, 0)
    m = 1_000_000
    big = halo_capacity(R, m, [1.5, 3.0, 10.0])
    assert big == halo_capacity(R, m, [0.5, 0.5, 0.5])
    assert big <= int((3 ** 3 - 1) * m * 1.25) + 4096
    assert halo_capacity(R, m, [0.0, 0.0, 0.0]) == 4096
    small = halo_capacity(R, m, [0.05, 0.05, 0.05])
    assert int(m * ((1.2 ** 3) - 1)) < small < big


@pytest.mark.parametrize("case", ["halo_p8_f64_rec32.npz", "halo_p27_333_ids.npz",
                                  "halo_direct_p6_321_nonperiodic.npz"])
def test_threaded_halo_traffic(case):
    """xGMI accounting of the halo's messages (Transport.traffic): what rank r
    counts as sent to p is what p counts as received from r, nothing is
    counted to self, and the bytes are the rows each rank actually received
    (the halo store grew by them) times the fields' row bytes."""
    f = G.load(case)
    size = int(f["size"])

    def fn(comm, r):
        t = MpiHostComm(comm)
        t.reset_traffic()
        out = run_rank(f, case, t, r, carry_pos=True)
        return out, t.traffic

    res = run_ranks(size, fn)
    send = np.array([tr.send for _, tr in res])
    recv = np.array([tr.recv for _, tr in res])
    assert np.array_equal(send, recv.T)
    assert not np.diag(send).any() and not np.diag(recv).any()
    if case.startswith("halo_direct_"):
        return   # a grid extent of 1: rows of that dimension never leave the rank
    local, local_pos, _ = local_inputs(f, case)
    dim = len(f["topology"])
    for r in range(size):
        d, lp = local[r], local_pos[r]
        m = len(res[r][0]) - len(d)                       # halo rows received
        rb = d.dtype.itemsize * int(np.prod(d.shape[1:], dtype=np.int64)) \
            + lp.dtype.itemsize * lp.shape[1] + 2          # data + positions + face flags
        extra = int(recv[r].sum()) - m * rb                # the 8-byte count messages
        assert extra % 8 == 0 and 0 < extra <= 8 * 4 * dim, (r, extra)


@pytest.mark.parametrize("fail_tag", ["_local", "_ghost"])
def test_halo_failed_selection_raises(fail_tag):
    """A selection scan that failed on one rank (-1 counts) -- of its local
    rows, or of the rows received in an earlier dimension -- makes every rank
    raise: the failure travels as a bit in the count messages (sizes stay
    consistent, every message still matches) and the ranks agree once at the
    end of the exchange."""
    from mpi_grid_redistribute_amd._lib import MgrError

    class FailingSelect(CpuSelect):
        def msel(self, flags, n, bits, tag):
            sets, counts = super().msel(flags, n, bits, tag)
            if tag == fail_tag:
                counts = torch.full_like(counts, -1)
            return sets, counts

    f = G.load("halo_p8_f64_rec32.npz")
    size = int(f["size"])

    def fn(comm, r):
        data, pos, periodic = local_inputs(f, "halo_p8_f64_rec32.npz")
        R = GeoRank(f["topology"], f["box"], size, r)
        d, p = data[r], pos[r]
        sel = FailingSelect() if r == 3 else CpuSelect()
        with pytest.raises(MgrError, match="scan failed"):
            exchange_overload(R, MpiHostComm(comm), _flat(d), d.dtype.itemsize, _flat(p),
                              p.shape[1], _lib.MGR_F64, len(d), list(f["overload"]),
                              periodic=periodic, sel=sel)
        return True

    assert all(run_ranks(size, fn))
