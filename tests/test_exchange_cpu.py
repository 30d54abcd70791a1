"""Multi-rank host logic on CPU (no GPU): count exchange, send/receive
layout, source-rank ordering (S7), self-segment redirect, empty ranks,
dropped ids -- through the same ``exchange()`` the GPU path uses, with the
pack done by the C oracle instead of the HIP kernel.

* world_size 2 and 3 with torch.distributed ``gloo`` (TorchDistComm);
* 4 threaded ranks on the mpi4py-style fake comm (MpiHostComm, redirect on).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpi_grid_redistribute_amd.comm import MpiHostComm, TorchDistComm
from mpi_grid_redistribute_amd.exchange import exchange
from oracle import c_oracle
from oracle import redist_oracle as ro
from tests.fake_mpi import run_ranks

BOX = [1.0, 1.0, 1.0]


def make_rank_inputs(size, seed=42, empty_rank=None):
    rng = np.random.default_rng(seed)
    pos, data = [], []
    for r in range(size):
        n = 0 if r == empty_rank else int(rng.integers(100, 3000))
        pos.append(rng.uniform(-0.5, 1.5, (n, 3)))
        rec = np.zeros(n, dtype=[("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])
        rec["id"] = np.arange(n) + 100_000 * r
        data.append(rec)
    return pos, data


def oracle_pack(data, dest, size, rb):
    """C-oracle stand-in for mgr_pack: returns pack(field, send, redirect, out)."""
    part, off = c_oracle.partition(data, dest, size)
    raw = part.view(np.uint8).reshape(-1)

    def pack(f, snd, redirect_bin, redirect_out):
        for b in range(size):
            seg = torch.from_numpy(raw[off[b] * rb: off[b + 1] * rb].copy())
            if b == redirect_bin:
                redirect_out[: seg.numel()].copy_(seg)
            elif seg.numel():
                snd[off[b] * rb: off[b + 1] * rb].copy_(seg)

    counts = torch.from_numpy(np.diff(off).astype(np.int64))
    return pack, counts


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, size, port, empty_rank, drop, topo):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        pos, data = make_rank_inputs(size, empty_rank=empty_rank)
        rb = data[0].dtype.itemsize
        if drop:  # redistribute_by_cell_number: ids incl. out-of-range (S6)
            ids = [np.random.default_rng(100 + r).integers(-1, size + 1, len(data[r]))
                   for r in range(size)]
            expect = ro.redistribute_by_cell_number_all_ranks(size, data, ids)[rank]
            dest = ids[rank]
        else:
            expect = ro.redistribute_by_position_all_ranks(
                topo, BOX, size, data, [p.copy() for p in pos])[rank]
            geo = ro.Geometry(topo, BOX, size, rank)
            dest = ro.cell_number_from_position(geo, pos[rank].copy())
        pack, counts = oracle_pack(data[rank], dest, size, rb)
        comm = TorchDistComm()
        assert comm.Get_rank() == rank and comm.Get_size() == size
        outs, lay = exchange(comm, [rb], counts, rank, "cpu", pack)
        got = outs[0][: lay.total_recv * rb].numpy().view(data[0].dtype)
        assert lay.total_recv == len(expect)
        assert got.tobytes() == expect.tobytes()
        comm.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,empty_rank,drop", [(2, None, False), (2, 1, False), (3, 0, False),
                                                  (3, None, True)])
def test_gloo_exchange(size, empty_rank, drop):
    topo = [2, 1, 1] if size == 2 else [3, 1, 1]
    mp.spawn(_gloo_worker, args=(size, _free_port(), empty_rank, drop, topo), nprocs=size,
             join=True)


def test_threaded_mpi_host_comm_redirect():
    size = 4
    topo = [2, 2, 1]
    pos, data = make_rank_inputs(size, seed=7, empty_rank=2)
    expect = ro.redistribute_by_position_all_ranks(topo, BOX, size, data,
                                                   [p.copy() for p in pos])
    rb = data[0].dtype.itemsize

    def fn(comm, r):
        geo = ro.Geometry(topo, BOX, size, r)
        dest = ro.cell_number_from_position(geo, pos[r].copy())
        pack, counts = oracle_pack(data[r], dest, size, rb)
        t = MpiHostComm(comm)
        assert t.skips_self
        outs, lay = exchange(t, [rb], counts, r, "cpu", pack)
        return outs[0][: lay.total_recv * rb].numpy().copy()

    outs = run_ranks(size, fn)
    for r in range(size):
        assert outs[r].tobytes() == expect[r].tobytes(), r
