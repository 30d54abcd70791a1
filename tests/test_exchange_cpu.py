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

from mpi_grid_redistribute_amd.comm import MpiHostComm, TorchDistComm, Transport
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

    def pack(f, snd, redirect_bin, out, out_offset):
        redirect_out = out[out_offset:] if out is not None else None
        # mgr_pack semantics: the redirect bin goes to redirect_out from row 0,
        # the bins after it close its gap in the send buffer
        for b in range(size):
            seg = torch.from_numpy(raw[off[b] * rb: off[b + 1] * rb].copy())
            if b == redirect_bin:
                redirect_out[: seg.numel()].copy_(seg)
            elif seg.numel():
                o = off[b]
                if 0 <= redirect_bin < b:
                    o -= off[redirect_bin + 1] - off[redirect_bin]
                snd[o * rb: o * rb + seg.numel()].copy_(seg)

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


def chunked_oracle_pack(data, dest, size, rb, nchunks):
    """Stand-in for mgr_pack_tiles: the rows split into nchunks row ranges
    (the tile chunks); chunk c's rows of every bin go to their final places
    -- bin-major, stable, the redirect bin straight into the output.
    Returns (chunk_offsets() -> [nchunks+1][size], pack_chunk, counts)."""
    n = len(data)
    raw = np.ascontiguousarray(data).view(np.uint8).reshape(n, rb)
    bounds = [n * c // nchunks for c in range(nchunks + 1)]
    counts = np.bincount(dest, minlength=size).astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)])
    off = np.array([[starts[b] + int(np.sum(dest[:bounds[c]] == b)) for b in range(size)]
                    for c in range(nchunks + 1)], dtype=np.int64)

    def pack_chunk(c, sends, outs, redirect_bin, offs):
        for b in range(size):
            rows = np.nonzero(dest[bounds[c]:bounds[c + 1]] == b)[0] + bounds[c]
            if not len(rows):
                continue
            seg = torch.from_numpy(raw[rows].reshape(-1).copy())
            o = off[c][b] - starts[b]          # rows of bin b in earlier chunks
            if b == redirect_bin:
                outs[0][offs[0] + o * rb: offs[0] + (o + len(rows)) * rb].copy_(seg)
            else:
                g = starts[b] - (counts[redirect_bin] if 0 <= redirect_bin < b else 0) + o
                sends[0][g * rb:(g + len(rows)) * rb].copy_(seg)

    return (lambda: off), pack_chunk, torch.from_numpy(counts)


def _gloo_pipelined_worker(rank, size, port, empty_rank, nchunks):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from mpi_grid_redistribute_amd.exchange import exchange_pipelined
        topo = [size, 1, 1]
        pos, data = make_rank_inputs(size, seed=31 + size, empty_rank=empty_rank)
        rb = data[0].dtype.itemsize
        expect = ro.redistribute_by_position_all_ranks(topo, BOX, size, data,
                                                       [p.copy() for p in pos])[rank]
        dest = ro.cell_number_from_position(ro.Geometry(topo, BOX, size, rank), pos[rank].copy())
        offs_fn, pack_chunk, counts = chunked_oracle_pack(data[rank], dest, size, rb, nchunks)
        comm = TorchDistComm()
        comm.reset_traffic()
        outs, lay = exchange_pipelined(comm, [rb], counts, rank, "cpu", offs_fn, pack_chunk,
                                       nchunks)
        got = outs[0][: lay.total_recv * rb].numpy()
        assert got.tobytes() == np.ascontiguousarray(expect).view(np.uint8).tobytes()
        sent = sum(int(counts[p]) * rb for p in range(size) if p != rank)
        assert comm.traffic.send.sum() == sent + 8 * (size - 1) * (1 + nchunks)
        comm.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,empty_rank,nchunks", [(2, None, 3), (3, 1, 2), (3, None, 5)])
def test_gloo_pipelined_exchange(size, empty_rank, nchunks):
    """The pipelined exchange (pack in chunks, each chunk's pieces sent while
    the next is packed) gives exchange()'s bytes: gloo ranks, the oracle's
    stable partition as the chunked pack, empty ranks, more chunks than rows
    of some bins."""
    mp.spawn(_gloo_pipelined_worker, args=(size, _free_port(), empty_rank, nchunks), nprocs=size,
             join=True)


# ------------------------------------------------ the RCCL schedule (host)
class _SimWorld:
    """Shared state of the simulated RCCL group: per (src, dst) FIFO of the
    bytes each send carried, in issue order (RCCL matches a pair's sends and
    receives inside one group in order)."""

    def __init__(self, size):
        import threading
        self.size = size
        self.barrier = threading.Barrier(size)
        self.slots = [None] * size
        self.mail = {}
        self.lock = threading.Lock()


class SimRcclComm(Transport):
    """RcclComm's host side (counts all-to-all, the arrays it hands to
    mgr_exchange_rows: comm.row_exchange_arrays) with the device transfers
    replaced by executing mgr_exchange_schedule's operation list on host
    buffers.  Lets the CPU suite run exchange() exactly as the GPU path does,
    skip_self included."""

    skips_self = True

    def __init__(self, world, rank):
        self.world, self.rank, self.size = world, rank, world.size

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.size

    def exchange_counts(self, send_counts):
        w = self.world
        s = send_counts.detach().cpu().numpy().astype(np.int64)
        w.slots[self.rank] = s.copy()
        w.barrier.wait()
        r = np.array([w.slots[src][self.rank] for src in range(self.size)], dtype=np.int64)
        w.barrier.wait()
        return s, r

    def exchange_rows(self, sends, outs, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets):
        from mpi_grid_redistribute_amd import _lib
        from mpi_grid_redistribute_amd.comm import row_exchange_arrays
        rb, sc, so, rc, ro_, skip = row_exchange_arrays(self.size, row_bytes, send_counts,
                                                        send_offsets, recv_counts, recv_offsets)
        lib = _lib.load()
        n = lib.mgr_exchange_schedule(self.rank, self.size, len(sends), rb, sc, so, rc, ro_, skip,
                                      None, 0)
        assert n >= 0, lib.mgr_last_error()
        ops = (_lib.XOp * max(n, 1))()
        lib.mgr_exchange_schedule(self.rank, self.size, len(sends), rb, sc, so, rc, ro_, skip,
                                  ops, n)
        ops = ops[:n]
        self.sched = [(o.kind, o.peer, o.bytes) for o in ops]
        assert all(o.kind != _lib.MGR_XOP_COPY for o in ops)      # skip_self: no self copy
        assert all(o.peer != self.rank for o in ops)
        w = self.world
        with w.lock:
            for o in ops:
                if o.kind == _lib.MGR_XOP_SEND:
                    buf = sends[o.field].numpy()
                    assert o.src_offset + o.bytes <= buf.size            # inside the send buffer
                    w.mail.setdefault((self.rank, o.peer), []).append(
                        (o.field, buf[o.src_offset:o.src_offset + o.bytes].copy()))
        w.barrier.wait()
        for o in ops:
            if o.kind == _lib.MGR_XOP_RECV:
                with w.lock:
                    field, data = w.mail[(o.peer, self.rank)].pop(0)
                assert field == o.field and data.size == o.bytes
                out = outs[o.field].numpy()
                assert o.dst_offset + o.bytes <= out.size
                out[o.dst_offset:o.dst_offset + o.bytes] = data
        w.barrier.wait()
        with w.lock:   # every send was received
            assert all(not v for v in w.mail.values()), "unmatched send"


@pytest.mark.parametrize("size,empty_rank,drop", [(2, None, False), (4, 2, False), (8, 0, False),
                                                  (8, None, True), (3, 1, True)])
def test_rccl_schedule_exchange(size, empty_rank, drop):
    """exchange() over the exact RCCL operation list (mgr_exchange_schedule, the
    list mgr_exchange_rows issues) with RcclComm's arrays and the self-segment
    redirect, two fields, against the oracle: every send matches a receive of
    the same size in order, every receive lands at its source-ordered offset."""
    topo = {2: [2, 1, 1], 3: [3, 1, 1], 4: [2, 2, 1], 8: [2, 2, 2]}[size]
    pos, data = make_rank_inputs(size, seed=size * 10 + 3, empty_rank=empty_rank)
    rb = data[0].dtype.itemsize
    if drop:
        ids = [np.random.default_rng(200 + r).integers(-1, size + 1, len(data[r]))
               for r in range(size)]
        expect = ro.redistribute_by_cell_number_all_ranks(size, data, ids)
    else:
        expect = ro.redistribute_by_position_all_ranks(topo, BOX, size, data,
                                                       [p.copy() for p in pos])
    world = _SimWorld(size)

    def fn(comm, r):
        if drop:
            dest = ids[r]
        else:
            dest = ro.cell_number_from_position(ro.Geometry(topo, BOX, size, r), pos[r].copy())
        pack0, counts = oracle_pack(data[r], dest, size, rb)
        ids2 = (np.arange(len(data[r]), dtype=np.int32) + 7 * r).view(np.uint8).reshape(-1, 4)
        pack1, _ = oracle_pack(ids2, dest, size, 4)

        def pack(f, snd, redirect_bin, out, out_offset):
            (pack0 if f == 0 else pack1)(f, snd, redirect_bin, out, out_offset)

        t = SimRcclComm(world, r)
        t.reset_traffic()
        outs, lay = exchange(t, [rb, 4], counts, r, "cpu", pack)
        assert lay.total_send == int(counts.sum()) - int(counts[r])   # no self rows in the buffer
        # xGMI accounting: the bytes RCCL moves per peer and direction (the
        # operation list) + one int64 count each way per peer, both fields
        from mpi_grid_redistribute_amd import _lib
        want_s, want_r = np.zeros(size, np.int64), np.zeros(size, np.int64)
        for kind, peer, nbytes in t.sched:
            (want_s if kind == _lib.MGR_XOP_SEND else want_r)[peer] += nbytes
        for p in range(size):
            if p != r:
                want_s[p] += 8
                want_r[p] += 8
        assert t.traffic.send.tolist() == want_s.tolist()
        assert t.traffic.recv.tolist() == want_r.tolist()
        assert t.traffic.send[r] == 0 and t.traffic.recv[r] == 0   # the self rows never travel
        return outs[0][: lay.total_recv * rb].numpy().copy(), outs[1][: lay.total_recv * 4].numpy()

    outs = run_ranks(size, fn)
    for r in range(size):
        assert outs[r][0].tobytes() == expect[r].tobytes(), r
        # the second field followed the same rows
        assert len(outs[r][1]) // 4 == len(expect[r])


def test_rccl_schedule_order_and_self_copy():
    """Ring order (to = rank+j, from = rank-j), fields inside a peer, and the
    self-segment copy when the transport does not skip it."""
    from mpi_grid_redistribute_amd import _lib
    sc, rc = [3, 0, 5, 1], [2, 4, 0, 6]
    so, ro_ = [0, 3, 3, 8], [0, 2, 6, 6]
    ops = _lib.exchange_schedule(1, 4, [32, 24], sc, so, rc, ro_, skip_self=False)
    S, R, C = _lib.MGR_XOP_SEND, _lib.MGR_XOP_RECV, _lib.MGR_XOP_COPY
    assert ops == [
        (S, 2, 0, 3 * 32, -1, 5 * 32), (R, 0, 0, -1, 0, 2 * 32),
        (S, 2, 1, 3 * 24, -1, 5 * 24), (R, 0, 1, -1, 0, 2 * 24),
        (S, 3, 0, 8 * 32, -1, 1 * 32), (R, 3, 0, -1, 6 * 32, 6 * 32),
        (S, 3, 1, 8 * 24, -1, 1 * 24), (R, 3, 1, -1, 6 * 24, 6 * 24),
        (S, 0, 0, 0, -1, 3 * 32),
        (S, 0, 1, 0, -1, 3 * 24),
    ]   # rank 1: no self rows (sc[1] == 0) -> no copy; nothing from rank 2
    ops = _lib.exchange_schedule(0, 2, [8], [2, 3], [0, 2], [2, 1], [0, 2], skip_self=False)
    assert ops[-1] == (C, 0, 0, 0, 0, 16)
    with pytest.raises(_lib.MgrError):
        _lib.exchange_schedule(0, 2, [8], [-1, 3], [0, 0], [0, 1], [0, 0])


def _gloo_pipelined_bad_worker(rank, size, port, bad_rank):
    """One rank's chunk offsets do not add up to its counts: it sends -2
    totals in the one count message, so EVERY rank raises there (none is left
    waiting inside a row message), naming the inconsistent chunks -- not a
    timed-out look-back (-1)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from mpi_grid_redistribute_amd._lib import MgrError
        from mpi_grid_redistribute_amd.exchange import exchange_pipelined
        topo = [size, 1, 1]
        pos, data = make_rank_inputs(size, seed=77)
        rb = data[0].dtype.itemsize
        dest = ro.cell_number_from_position(ro.Geometry(topo, BOX, size, rank), pos[rank].copy())
        offs_fn, pack_chunk, counts = chunked_oracle_pack(data[rank], dest, size, rb, 3)
        if rank == bad_rank:
            good = offs_fn()
            bad = good.copy()
            bad[1, 0] += 1                     # chunk 0 / chunk 1 boundary off by one row
            bad[3, 1] -= 1                     # and the totals no longer add up
            offs_fn = lambda: bad  # noqa: E731
        comm = TorchDistComm()
        with pytest.raises(MgrError, match="chunk counts do not add up") as e:
            exchange_pipelined(comm, [rb], counts, rank, "cpu", offs_fn, pack_chunk, 3)
        assert "look-back" not in str(e.value)
        comm.barrier()                          # every rank got here: nobody hangs
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,bad_rank", [(2, 1), (3, 0)])
def test_gloo_pipelined_failure_agreed(size, bad_rank):
    mp.spawn(_gloo_pipelined_bad_worker, args=(size, _free_port(), bad_rank), nprocs=size,
             join=True)


def test_check_counts_names_the_cause():
    from mpi_grid_redistribute_amd._lib import MgrError
    from mpi_grid_redistribute_amd.exchange import check_counts
    check_counts([1, 2], [0, 3])
    with pytest.raises(MgrError, match="look-back timed out") as e:
        check_counts([-1, -1], [2, 3])
    assert "chunk counts" not in str(e.value)
    with pytest.raises(MgrError, match="chunk counts do not add up") as e:
        check_counts([4, 5], [2, -2])
    assert "look-back" not in str(e.value)
    with pytest.raises(MgrError, match="look-back.*; pipelined"):
        check_counts([-1, 5], [-2, 3])


def test_count_skew_hand_built():
    """the count matrix's max/mean (exchange.count_skew)
    on a hand-built skewed layout: 4 sources x 4 destinations, destination 2
    receives most rows."""
    from mpi_grid_redistribute_amd.exchange import count_skew
    c = np.array([[10, 0, 90, 0],
                  [5, 5, 80, 10],
                  [0, 0, 100, 0],
                  [25, 15, 50, 10]])
    s = count_skew(c)
    recv = c.sum(axis=0)                          # 40, 20, 320, 20 -> mean 100
    assert s["recv_max"] == 320 and s["recv_min"] == 20
    assert s["recv_mean"] == 100.0 and s["recv_max_over_mean"] == 3.2
    assert s["entry_max"] == 100 and s["entry_max_over_mean"] == 100 / c.mean()
    assert s["sources"] == 4 and s["destinations"] == 4 and s["total_rows"] == recv.sum()
    # one GPU: a 1 x D row of virtual destinations; balanced -> 1.0
    assert count_skew([7, 7, 7, 7])["recv_max_over_mean"] == 1.0
    assert count_skew(np.zeros((2, 3), dtype=np.int64))["recv_max_over_mean"] is None
    with pytest.raises(ValueError):
        count_skew([[1, -1]])                     # a failed scan's -1 counts


def test_bench_xgmi_report_names_its_path():
    """bench.py's xGMI figures say which exchange produced them."""
    import bench
    traffic = {"send_bytes": 1e9, "recv_bytes": 2e9, "send_peers": 2, "recv_peers": 1}
    exch = {"avg_ms": 1.0, "launches": 4, "steps": 2}   # 2 ms of RCCL groups per step
    r = bench.xgmi_report(traffic, exch, None, 1, 4)
    assert r["path"].startswith("pipelined, 4 chunks")
    assert r["ms_per_step"] == 2.0
    assert abs(r["send"]["achieved"] - 500.0) < 1e-9 and r["send"]["peers"] == 2
    assert abs(r["recv"]["achieved"] - 1000.0) < 1e-9
    assert bench.xgmi_report(traffic, exch, None, 1, 1)["path"].startswith("one message")


def test_bench_halo_pack_bytes_by_world():
    """The halo line's pack carries the 2-byte flag field only between ranks
    (one rank reads the binning's flags in place)."""
    import bench
    assert bench.row_bytes_per_kernel(3, True, world=1)["pack"] == 65
    assert bench.row_bytes_per_kernel(3, True, world=2)["pack"] == 69
    assert bench.row_bytes_per_kernel(3, False)["pack"] == 65


def test_bench_scaling_record_schema():
    """The N > 1 record checks itself: RCCL versions, library, ranks as RCCL
    counts them, transports from RCCL's connection lines, and the one-message
    exchange timed beside the pipelined one."""
    import bench
    env = {}
    path = bench.rccl_log_env(env)
    assert env["NCCL_DEBUG"] == "INFO" and env["NCCL_DEBUG_FILE"] == path
    assert bench.rccl_log_env({"NCCL_DEBUG": "INFO"}) is None      # the caller's INFO wins
    low = {"NCCL_DEBUG": "VERSION"}                                  # a preset low level: raised
    assert bench.rccl_log_env(low) == low["NCCL_DEBUG_FILE"] and low["NCCL_DEBUG"] == "INFO"
    log = ("host:1:2 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC/read\n"
           "host:1:2 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC\n"
           "host:1:2 [0] NCCL INFO Channel 00/1 : 1[0] -> 0[0] [send] via NET/Socket/0\n"
           "host:1:2 [0] NCCL INFO comm 0x1 rank 0 nRanks 2\n")
    assert bench.rccl_transports(log) == ["NET/Socket", "P2P/IPC"]
    info = {"version_compiled": 22707, "version_runtime": 22606, "nranks": 8,
            "library": "/x/librccl.so"}
    r = bench.rccl_block(info, ["P2P/IPC"], 8)
    assert set(r) == {"version_compiled", "version_runtime", "library", "nranks", "nranks_ok",
                      "transports"}
    assert r["nranks_ok"] and not bench.rccl_block(info, [], 4)["nranks_ok"]
    assert bench.rccl_block({"error": "x"}, ["NET/Socket"], 2) == {"error": "x",
                                                                   "transports": ["NET/Socket"]}
    ab = bench.exchange_ab_block(2.0, 4, 3.0, 10)
    assert set(ab) == {"pipelined_ms_per_step", "chunks", "one_message_ms_per_step",
                       "one_message_steps", "pipelined_speedup", "in_timed_region"}
    assert ab["pipelined_speedup"] == 1.5 and ab["in_timed_region"] is False


def test_rccl_runtime_version_is_the_loaded_library():
    """mgr_rccl_version reports the headers libmgr.so was built with and the
    RCCL this process loaded (torch's bundled one once torch is imported);
    mgr_comm_create accepts only a runtime of the same major version, >= 2.18."""
    import ctypes
    from mpi_grid_redistribute_amd import _lib
    from mpi_grid_redistribute_amd.comm import loaded_rccl_path
    compiled, runtime = _lib.rccl_version()
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "include", "mgr.h")).read()
    assert "mgr_rccl_version" in hdr
    # the version code of the rccl.h libmgr.so was built against (csrc/Makefile:
    # $(ROCM)/include), parsed from that header rather than hard-coded
    import re
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    with open(os.path.join(rocm, "include", "rccl", "rccl.h")) as fh:
        txt = fh.read()
    ver = {k: int(re.search(rf"#define NCCL_{k}\s+(\d+)", txt).group(1))
           for k in ("MAJOR", "MINOR", "PATCH")}
    want = ver["MAJOR"] * 10000 + ver["MINOR"] * 100 + ver["PATCH"]
    assert compiled == want, (compiled, want)
    path = loaded_rccl_path()
    assert path is not None
    v = ctypes.c_int(0)
    assert ctypes.CDLL(path).ncclGetVersion(ctypes.byref(v)) == 0
    assert runtime == v.value
    assert runtime // 10000 == compiled // 10000 and runtime >= 21800


def test_bench_cpu_baseline_record():
    """bench.py's cpu_baseline object (the contract's keys), on a tiny sample:
    the oracle's 8-process numpy restatement of redist.py:157-199."""
    import bench
    r = bench.cpu_baseline(n_per_rank=4096)
    assert set(r) == {"value", "unit", "cores", "kind", "sample", "stat", "spread"}
    assert r["stat"] == "median" and r["spread"][0] <= r["value"] <= r["spread"][1]
    assert r["value"] > 0 and r["unit"] == "particles/s" and r["kind"] == "port"
    assert r["cores"] >= 1 and "4096 uniform particles" in r["sample"]
