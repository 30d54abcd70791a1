"""Communicators: the ``comm`` object ``MPIGridRedistributor`` is built on.

The reference takes an mpi4py communicator and uses ``Get_rank`` /
``Get_size`` (redist.py:41-42) and the pickle-based lowercase ``alltoall``
(redist.py:199).  Here a communicator is a *transport* with two exchange
steps of the redistribution:

  exchange_counts(send_counts)   -> the count row all-to-all (host copies)
  exchange_rows(...)             -> the packed segments, landing in the
                                    output at source-ordered offsets (S7)

Implementations
  RcclComm       the product path: one process per GPU, a native RCCL
                 communicator owned by libmgr.so (grouped ncclSend/ncclRecv
                 over xGMI); created from torch.distributed or a unique id.
  SelfComm       a single rank (size 1): no transport at all.
  MpiHostComm    wraps any mpi4py-style comm (``alltoall(list)``): device
                 segments are staged through host memory.  Lets a reference
                 user keep mpi4py; slow, correctness only.
  TorchDistComm  torch.distributed all_to_all_single (gloo on CPU tensors
                 for the multi-process host-logic tests; works on nccl too).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib


_HALO_TAG = 0  # redist.py:290-299 uses tag 0 for every halo message


def excl_cumsum(counts):
    out = np.zeros(len(counts), dtype=np.int64)
    if len(counts) > 1:
        np.cumsum(counts[:-1], out=out[1:])
    return out


def row_exchange_arrays(size, row_bytes, send_counts, send_offsets, recv_counts, recv_offsets):
    """The host arrays RcclComm hands to mgr_exchange_rows / mgr_exchange_schedule
    after the field pointers: (row_bytes[nf], send_counts, send_offsets,
    recv_counts, recv_offsets, skip_self=1) -- the pack already wrote the self
    segment into the output (exchange.py)."""
    I64 = ctypes.c_int64
    arr = lambda a: (I64 * size)(*[int(x) for x in a])  # noqa: E731
    return ((I64 * len(row_bytes))(*[int(x) for x in row_bytes]), arr(send_counts),
            arr(send_offsets), arr(recv_counts), arr(recv_offsets), 1)


class Traffic:
    """Bytes one rank moved to and received from OTHER ranks (its xGMI traffic):
    per peer and direction, from the exchange's real layout -- every field's
    rows (side fields included), the count messages and the halo's
    point-to-point messages.  Messages to self never leave the GPU and are
    not counted."""

    def __init__(self, size, rank):
        self.rank = int(rank)
        self.send = np.zeros(int(size), dtype=np.int64)
        self.recv = np.zeros(int(size), dtype=np.int64)

    def add(self, kind, peer, nbytes):
        peer, nbytes = int(peer), int(nbytes)
        if peer == self.rank or nbytes <= 0:
            return
        (self.send if kind == "send" else self.recv)[peer] += nbytes

    def add_rows(self, row_bytes, send_counts, recv_counts):
        """One row exchange: send_counts[p] / recv_counts[p] rows of every
        field (row_bytes[f] bytes each) to / from peer p."""
        rb = int(sum(int(x) for x in row_bytes))
        for p in range(len(self.send)):
            self.add("send", p, int(send_counts[p]) * rb)
            self.add("recv", p, int(recv_counts[p]) * rb)

    def as_dict(self):
        return {"send_bytes": int(self.send.sum()), "recv_bytes": int(self.recv.sum()),
                "send_peers": int((self.send > 0).sum()), "recv_peers": int((self.recv > 0).sum()),
                "send_per_peer": self.send.tolist(), "recv_per_peer": self.recv.tolist()}


class Transport:
    """Interface.  ``skips_self`` True means the transport never touches the
    self segment, so the pack may write it straight into the output.
    ``traffic`` accumulates the off-rank bytes since the last
    ``reset_traffic()`` (MPIGridRedistributor resets it per call)."""

    rank = 0
    size = 1
    skips_self = True
    traffic = None

    def reset_traffic(self):
        self.traffic = Traffic(self.size, self.rank)
        return self.traffic

    def note(self, kind, peer, nbytes):
        if self.traffic is None:
            self.reset_traffic()
        self.traffic.add(kind, peer, nbytes)

    def note_rows(self, row_bytes, send_counts, recv_counts):
        if self.traffic is None:
            self.reset_traffic()
        self.traffic.add_rows(row_bytes, send_counts, recv_counts)

    def note_p2p(self, ops):
        for k, p, t in ops:
            self.note(k, p, t.numel())

    def Get_rank(self):  # mpi4py duck type (redist.py:41)
        return self.rank

    def Get_size(self):  # redist.py:42
        return self.size

    def exchange_counts(self, send_counts):
        """send_counts: int64 tensor [size] (device or host).
        Returns (send_counts_host, recv_counts_host) as int64 numpy arrays."""
        raise NotImplementedError

    def exchange_count_rows(self, send):
        """send: int64 tensor [size][w] (device or host), row p for peer p.
        Returns (send_host, recv_host) int64 numpy [size][w], recv row s from
        peer s -- one message per peer and one host sync (the pipelined
        exchange's totals + per-chunk counts)."""
        raise NotImplementedError

    def exchange_rows(self, sends, outs, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets):
        """sends/outs: per-field uint8 tensors; counts/offsets in rows (host)."""
        raise NotImplementedError

    def p2p(self, ops):
        """One batch of the halo exchange's point-to-point messages
        (redist.py:289-303): ``ops`` = [("send" | "recv", peer, flat uint8
        tensor), ...] in posting order; a pair of ranks' sends and receives
        match in that order (each rank posts step 1 -- send right, receive
        from the left -- before step 2).  Receive tensors are pre-sized."""
        raise NotImplementedError

    def barrier(self):
        pass

    def any_failed(self, failed):
        """Global agreement on a local failure flag (True if any rank failed):
        lets every rank raise together where a failure would otherwise reach
        only some peers (the halo's neighbour-only count messages)."""
        return bool(failed)


def _self_pairs(ops, rank):
    """The k-th non-empty send to ``rank`` feeds its k-th non-empty receive."""
    sends = [t for k, p, t in ops if k == "send" and p == rank and t.numel()]
    recvs = [t for k, p, t in ops if k == "recv" and p == rank and t.numel()]
    if len(sends) != len(recvs):
        raise RuntimeError(f"{len(sends)} messages to self, {len(recvs)} receives from self")
    for snd, rcv in zip(sends, recvs):
        if snd.numel() != rcv.numel():
            raise RuntimeError(f"self message of {snd.numel()} bytes into {rcv.numel()}")
        rcv.copy_(snd)


class SelfComm(Transport):
    """One rank, one GPU (or N virtual destinations on one GPU)."""

    def p2p(self, ops):
        assert all(p == 0 for _, p, _ in ops)
        _self_pairs(ops, 0)

    def exchange_counts(self, send_counts):
        s = send_counts.detach().to("cpu").numpy().astype(np.int64)
        return s, s.copy()

    def exchange_count_rows(self, send):
        s = send.detach().to("cpu").numpy().astype(np.int64)
        return s, s.copy()

    def exchange_rows(self, sends, outs, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets):
        return  # the pack wrote the self segment into the output


def loaded_rccl_path():
    """Path of the librccl mapped into this process (/proc/self/maps), or None."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if len(line.split()) >= 6 else ""
                if os.path.basename(p).startswith("librccl.so"):
                    return p
    except OSError:
        pass
    return None


class RcclComm(Transport):
    """Native RCCL communicator (libmgr.so ``mgr_comm_*``), one process per GPU.

    ``RcclComm.from_torch_distributed()`` makes the unique id on rank 0 and
    broadcasts it over the default torch.distributed group (any backend).
    """

    skips_self = True

    def __init__(self, unique_id: bytes, size: int, rank: int, device=None):
        _lib.require_gpu()
        if device is not None:
            torch.cuda.set_device(device)
        assert len(unique_id) == _lib.UNIQUE_ID_BYTES
        self.size, self.rank = int(size), int(rank)
        buf = ctypes.create_string_buffer(unique_id, _lib.UNIQUE_ID_BYTES)
        h = ctypes.c_void_p()
        _lib.call("mgr_comm_create", buf, self.size, self.rank, ctypes.byref(h))
        self._h = h
        self._pinned = torch.empty(2 * self.size, dtype=torch.int64, pin_memory=True)

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(_lib.UNIQUE_ID_BYTES)
        _lib.call("mgr_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def from_torch_distributed(cls, group=None):
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(obj[0], size, rank)

    def rccl_info(self):
        """What RCCL runs this communicator: the version codes libmgr.so was
        built with and the library loaded in this process (in a torch process
        torch's bundled RCCL; mgr_comm_create refused an incompatible one),
        that library's path, and the ranks RCCL itself counts (ncclCommCount)
        -- the first things to check on a scaling record."""
        compiled, runtime = _lib.rccl_version()
        count = _lib.load().mgr_comm_count(self._h)
        if count < 0:
            _lib.check(count, "mgr_comm_count")
        return {"version_compiled": compiled, "version_runtime": runtime,
                "nranks": int(count), "library": loaded_rccl_path()}

    def close(self):
        if getattr(self, "_h", None):
            _lib.call("mgr_comm_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def exchange_counts(self, send_counts):
        stream = _lib.stream_handle()
        recv = torch.empty_like(send_counts)
        _lib.call("mgr_exchange_counts", self._h, _lib.ptr(send_counts), _lib.ptr(recv), stream)
        P = self.size
        self._pinned[:P].copy_(send_counts, non_blocking=True)
        self._pinned[P:2 * P].copy_(recv, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        host = self._pinned[:2 * P].numpy().copy()
        return host[:P], host[P:]

    def exchange_count_rows(self, send):
        send = send.contiguous()
        P, w = self.size, int(send.shape[1])
        recv = torch.empty_like(send)
        _lib.call("mgr_exchange_count_rows", self._h, _lib.ptr(send), _lib.ptr(recv), w,
                  _lib.stream_handle())
        if self._pinned.numel() < 2 * P * w:
            self._pinned = torch.empty(2 * P * w, dtype=torch.int64, pin_memory=True)
        self._pinned[: P * w].copy_(send.reshape(-1), non_blocking=True)
        self._pinned[P * w: 2 * P * w].copy_(recv.reshape(-1), non_blocking=True)
        torch.cuda.current_stream().synchronize()
        host = self._pinned[: 2 * P * w].numpy().copy()
        return host[: P * w].reshape(P, w), host[P * w:].reshape(P, w)

    def exchange_rows(self, sends, outs, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets):
        nf = len(sends)
        P = ctypes.c_void_p * nf
        sp = P(*[s.data_ptr() for s in sends])
        rp = P(*[o.data_ptr() for o in outs])
        _lib.call("mgr_exchange_rows", self._h, nf, sp, rp,
                  *row_exchange_arrays(self.size, row_bytes, send_counts, send_offsets,
                                       recv_counts, recv_offsets),
                  _lib.stream_handle())

    def p2p(self, ops):
        """One RCCL group (mgr_group_p2p); messages to self are device copies."""
        n = len(ops)
        if not n:
            return
        kinds = (ctypes.c_int * n)(*[_lib.MGR_XOP_SEND if k == "send" else _lib.MGR_XOP_RECV
                                     for k, _, _ in ops])
        peers = (ctypes.c_int * n)(*[int(p) for _, p, _ in ops])
        bufs = (ctypes.c_void_p * n)(*[t.data_ptr() if t.numel() else 0 for _, _, t in ops])
        nbytes = (ctypes.c_int64 * n)(*[t.numel() for _, _, t in ops])
        _lib.call("mgr_group_p2p", self._h, n, kinds, peers, bufs, nbytes, _lib.stream_handle())

    def allreduce_max(self, values):
        t = torch.as_tensor(values, dtype=torch.float64, device="cuda").reshape(-1)
        out = torch.empty_like(t)
        _lib.call("mgr_comm_allreduce_max_f64", self._h, _lib.ptr(t), _lib.ptr(out), t.numel(),
                  _lib.stream_handle())
        return out.cpu().numpy()

    def barrier(self):
        self.allreduce_max([0.0])

    def any_failed(self, failed):
        if self.size == 1:
            return bool(failed)
        return bool(self.allreduce_max([1.0 if failed else 0.0])[0] > 0)


class MpiHostComm(Transport):
    """Any mpi4py-like communicator: counts and rows move with its lowercase
    ``alltoall`` (list indexed by destination -> list indexed by source,
    redist.py:199), staged through host memory."""

    skips_self = True

    def __init__(self, comm):
        self.comm = comm
        self.rank, self.size = comm.Get_rank(), comm.Get_size()

    def exchange_counts(self, send_counts):
        s = send_counts.detach().to("cpu").numpy().astype(np.int64)
        r = self.comm.alltoall([int(x) for x in s])
        return s, np.asarray(r, dtype=np.int64)

    def exchange_count_rows(self, send):
        s = send.detach().to("cpu").numpy().astype(np.int64)
        r = self.comm.alltoall([[int(x) for x in row] for row in s])
        return s, np.asarray(r, dtype=np.int64).reshape(s.shape)

    def exchange_rows(self, sends, outs, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets):
        for f, (snd, out) in enumerate(zip(sends, outs)):
            rb = row_bytes[f]
            host = snd.detach().to("cpu").numpy() if snd.numel() else np.zeros(0, np.uint8)
            lst = []
            for p in range(self.size):
                if p == self.rank:
                    lst.append(np.zeros(0, np.uint8))
                else:
                    a = send_offsets[p] * rb
                    lst.append(host[a:a + send_counts[p] * rb].copy())
            got = self.comm.alltoall(lst)
            for s in range(self.size):
                if s == self.rank or recv_counts[s] == 0:
                    continue
                a = recv_offsets[s] * rb
                out[a:a + recv_counts[s] * rb].copy_(torch.from_numpy(np.ascontiguousarray(got[s])),
                                                     non_blocking=False)

    def p2p(self, ops):
        """Host-staged isend/irecv (tag 0, as redist.py:290-299): every
        non-empty send posted first, then every receive waited in order."""
        _self_pairs(ops, self.rank)
        reqs = [self.comm.isend(t.detach().cpu().numpy(), dest=int(p), tag=_HALO_TAG)
                for k, p, t in ops if k == "send" and p != self.rank and t.numel()]
        for k, p, t in ops:
            if k != "recv" or p == self.rank or not t.numel():
                continue
            got = np.ascontiguousarray(self.comm.irecv(source=int(p), tag=_HALO_TAG).wait(),
                                       dtype=np.uint8).reshape(-1)
            if got.size != t.numel():
                raise RuntimeError(f"halo message from rank {p}: {got.size} bytes, "
                                   f"expected {t.numel()}")
            t.copy_(torch.from_numpy(got))
        for r in reqs:
            r.wait()

    def barrier(self):
        self.comm.alltoall([0] * self.size)

    def any_failed(self, failed):
        return any(bool(x) for x in self.comm.alltoall([bool(failed)] * self.size))


class TorchDistComm(Transport):
    """torch.distributed all_to_all_single (gloo for CPU tests, nccl on GPUs).
    The self segment travels with the collective, so the pack does not
    redirect it (``skips_self`` False)."""

    skips_self = False

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.rank, self.size = dist.get_rank(group), dist.get_world_size(group)

    def exchange_counts(self, send_counts):
        recv = torch.empty_like(send_counts)
        self.dist.all_to_all_single(recv, send_counts.contiguous(), group=self.group)
        return (send_counts.detach().cpu().numpy().astype(np.int64),
                recv.detach().cpu().numpy().astype(np.int64))

    def exchange_count_rows(self, send):
        send = send.contiguous()
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv.view(-1), send.view(-1), group=self.group)
        return (send.detach().cpu().numpy().astype(np.int64),
                recv.detach().cpu().numpy().astype(np.int64))

    def exchange_rows(self, sends, outs, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets):
        for f, (snd, out) in enumerate(zip(sends, outs)):
            rb = row_bytes[f]
            in_split = [int(c) * rb for c in send_counts]
            out_split = [int(c) * rb for c in recv_counts]
            # the packed send buffer is bin-major from row 0, so split sizes are enough
            nsend = int(sum(in_split))
            self.dist.all_to_all_single(out[: int(sum(out_split))], snd[:nsend].contiguous(),
                                        output_split_sizes=out_split, input_split_sizes=in_split,
                                        group=self.group)

    def p2p(self, ops):
        _self_pairs(ops, self.rank)
        reqs = []
        for k, p, t in ops:
            if p == self.rank or not t.numel():
                continue
            if k == "send":
                reqs.append(self.dist.isend(t.contiguous(), self._global(p), group=self.group))
            else:
                reqs.append(self.dist.irecv(t, self._global(p), group=self.group))
        for r in reqs:
            r.wait()

    def _global(self, r):
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def barrier(self):
        self.dist.barrier(group=self.group)

    def any_failed(self, failed):
        t = torch.tensor([1 if failed else 0], dtype=torch.int64)
        if self.dist.get_backend(self.group) == "nccl":
            t = t.cuda()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return bool(t.item())


def as_transport(comm):
    """Accept our transports, any mpi4py-like comm, or None (single rank)."""
    if comm is None:
        return SelfComm()
    if isinstance(comm, Transport):
        return comm
    if hasattr(comm, "alltoall") and hasattr(comm, "Get_rank") and hasattr(comm, "Get_size"):
        if comm.Get_size() == 1:
            return SelfComm()
        return MpiHostComm(comm)
    raise TypeError(f"unsupported communicator {type(comm)!r}: pass an RcclComm, SelfComm, "
                    "TorchDistComm or an mpi4py-style comm")
