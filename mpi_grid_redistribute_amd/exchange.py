"""Exchange orchestration shared by every transport (redist.py:199).

After the local stage has produced the per-destination row counts, one
redistribution does:
  1. count exchange    -> how many rows arrive from each source (host copy);
  2. layout            -> send offsets (bin-major packed buffer without the
                          self segment) and receive offsets in source-rank
                          order (S7), output size;
  3. pack (callback)   -> fills the send buffers; when the transport leaves
                          the self segment alone it is written straight into
                          the output at its source-ordered slot;
  4. row exchange      -> peers' segments land in place: no unpack pass.
Steps 1, 2 and 4 are device-agnostic (CPU tensors + gloo in the tests).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import MgrError
from .comm import excl_cumsum


@dataclass
class ExchangeLayout:
    send_counts: np.ndarray
    recv_counts: np.ndarray
    send_offsets: np.ndarray
    recv_offsets: np.ndarray
    total_recv: int
    total_send: int
    redirect_self: bool


# count-message sentinels: a scan whose look-back gave up reports -1 counts
# (mgr_kernels.hip scan_onepass_kernel); the pipelined exchange sends -2 when
# a rank's per-chunk counts do not add up to its scanned totals
SCAN_FAILED, CHUNKS_INCONSISTENT = -1, -2


def check_counts(send_counts, recv_counts):
    """A failure on this rank or a peer arrives as a negative count, so every
    rank raises together instead of one rank leaving the others inside the
    exchange; the message names the cause (-1: a look-back timed out, -2:
    chunk counts that do not add up to the totals -- a wrong bin total)."""
    sc, rc = np.asarray(send_counts), np.asarray(recv_counts)
    if (sc >= 0).all() and (rc >= 0).all():
        return
    causes = []
    if (sc == SCAN_FAILED).any() or (rc == SCAN_FAILED).any():
        causes.append("device scan failed (a look-back timed out on this rank or a peer)")
    if (sc == CHUNKS_INCONSISTENT).any() or (rc == CHUNKS_INCONSISTENT).any():
        causes.append("pipelined exchange: chunk counts do not add up to the scanned totals "
                      "on this rank or a peer (inconsistent scan offsets)")
    if not causes:
        causes.append("negative counts")
    raise MgrError("; ".join(causes) + f": send counts {list(sc)}, receive counts {list(rc)}")


def count_skew(matrix):
    """Load imbalance of a redistribution from its count matrix ``C[s][d]`` =
    rows source ``s`` sends destination ``d`` (the counts redist.py:199's
    alltoall moves; SURVEY §8d config 4: skewed Alltoallv counts).
    ``recv_max_over_mean`` = the most rows any destination receives over the
    mean per destination (1.0 = balanced; the slowest rank's exchange and
    unpack scale with it); ``entry_max_over_mean`` = the largest single
    message over the mean message.  A 1 x D matrix is one GPU's partition into
    D virtual destinations."""
    c = np.asarray(matrix, dtype=np.int64)
    if c.ndim == 1:
        c = c.reshape(1, -1)
    if c.ndim != 2 or c.size == 0:
        raise ValueError("count matrix must be [sources][destinations]")
    if (c < 0).any():
        raise ValueError("negative counts (a failed scan)")
    recv = c.sum(axis=0)
    rmean = float(recv.mean())
    emean = float(c.mean())
    return {"sources": int(c.shape[0]), "destinations": int(c.shape[1]),
            "total_rows": int(c.sum()), "recv_max": int(recv.max()), "recv_min": int(recv.min()),
            "recv_mean": rmean,
            "recv_max_over_mean": float(recv.max()) / rmean if rmean > 0 else None,
            "entry_max": int(c.max()),
            "entry_max_over_mean": float(c.max()) / emean if emean > 0 else None}


def host_read_start(tensors):
    """Start one device->host read of several small int64 tensors: enqueued
    now on the current stream (into pinned memory, behind the work already
    launched and ahead of what is launched next); host_read_wait waits for
    this read alone, so kernels launched in between keep the GPU busy while
    the host works on the result."""
    flat = (torch.cat([t.reshape(-1) for t in tensors]) if len(tensors) > 1
            else tensors[0].reshape(-1))
    sizes = [t.numel() for t in tensors]
    if flat.device.type != "cuda":
        return flat.numpy(), None, sizes
    host = torch.empty(flat.numel(), dtype=flat.dtype, pin_memory=True)
    host.copy_(flat, non_blocking=True)
    done = torch.cuda.Event()
    done.record()
    return host, done, sizes


def host_read_wait(read):
    """The arrays of a host_read_start, once its copy is done."""
    host, done, sizes = read
    if done is not None:
        done.synchronize()
        host = host.numpy()
    out, o = [], 0
    for k in sizes:
        out.append(host[o:o + k].copy())
        o += k
    return out


def plan_layout(send_counts, recv_counts, rank, redirect_self):
    """Send/receive offsets in rows.  Receives in source-rank order (S7).
    With ``redirect_self`` the self segment never enters the send buffer
    (mgr_pack writes it straight into the output and closes the gap), so
    the send offsets skip it and the buffer holds only the rows that travel."""
    sc = np.asarray(send_counts, dtype=np.int64)
    rc = np.asarray(recv_counts, dtype=np.int64)
    travel = sc.copy()
    if redirect_self:
        travel[rank] = 0
    return ExchangeLayout(send_counts=sc, recv_counts=rc, send_offsets=excl_cumsum(travel),
                          recv_offsets=excl_cumsum(rc), total_recv=int(rc.sum()),
                          total_send=int(travel.sum()), redirect_self=bool(redirect_self))


def exchange(transport, row_bytes, bin_counts, rank, device, pack, extra_rows=None,
             scratch=None, pack_all=None, known_rows=None):
    """Run steps 1-4.  ``bin_counts``: int64 tensor [size] of rows per
    destination (on ``device``).  ``pack(field, send, redirect_bin, out,
    out_offset)`` packs field ``field`` (the redirect bin's rows into ``out``
    from byte ``out_offset``).  ``extra_rows(total_recv)``: spare
    rows to allocate after the received ones (the halo appends there).
    ``scratch(name, nbytes)``: a reusable device buffer (the send buffers),
    else fresh allocations.  ``pack_all(sends, outs, redirect_bin,
    out_offsets)``, when given, packs every field in one call instead (fields
    moved by one kernel, e.g. rows with their fine cells).  Returns (outs, layout); outs are new flat uint8
    tensors of (total_recv + extra) * row_bytes[f] bytes (>= 1 byte).
    ``known_rows``: on one rank whose rows all stay, their number -- the
    counts are not read back (no host sync) and the CALLER checks
    ``bin_counts`` with its next host read (check_counts)."""
    if known_rows is not None and transport.size == 1 and bin_counts.numel() == 1:
        sc = rc = np.array([int(known_rows)], dtype=np.int64)
    else:
        sc, rc = transport.exchange_counts(bin_counts)
        for p in range(len(sc)):   # the count row: one int64 each way per peer
            transport.note("send", p, 8)
            transport.note("recv", p, 8)
        check_counts(sc, rc)
    lay = plan_layout(sc, rc, rank, transport.skips_self)
    extra = int(extra_rows(lay.total_recv)) if extra_rows is not None else 0
    outs, sends = [], []
    for f, rb in enumerate(row_bytes):
        # the output is returned to the caller: always a new array (redist.py:199)
        out = torch.empty(max((lay.total_recv + extra) * rb, 1), dtype=torch.uint8, device=device)
        nbytes = max(lay.total_send * rb, 1)
        snd = (scratch(f"send{f}", nbytes) if scratch is not None
               else torch.empty(nbytes, dtype=torch.uint8, device=device))
        outs.append(out)
        sends.append(snd)
    redirect = rank if lay.redirect_self else -1
    offs = [int(lay.recv_offsets[rank]) * rb if lay.redirect_self else 0 for rb in row_bytes]
    if pack_all is not None:
        pack_all(sends, outs, redirect, offs)
    else:
        for f in range(len(row_bytes)):
            pack(f, sends[f], redirect, outs[f] if lay.redirect_self else None, offs[f])
    transport.exchange_rows(sends, outs, list(row_bytes), sc, lay.send_offsets, rc,
                            lay.recv_offsets)
    transport.note_rows(row_bytes, sc, rc)
    return outs, lay


_COMM_STREAMS = OrderedDict()
_COMM_STREAMS_MAX = 16


def _comm_stream(device):
    """The side stream the pipelined exchange posts its row messages on: one
    per (device, compute stream) for the process, not one per call -- calls on
    different compute streams (the Scratch sets of redistributor.py) get
    different comm streams, so neither queues behind the other's messages.
    The cache is bounded (least recently used out beyond _COMM_STREAMS_MAX
    keys): a caller cycling through short-lived compute streams does not grow
    it, and a stale entry for a reused raw handle only means a shared comm
    stream -- every use is ordered by wait_stream on both sides."""
    d = torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(idx).cuda_stream)
    st = _COMM_STREAMS.pop(key, None)
    if st is None:
        st = torch.cuda.Stream(device=idx)
    _COMM_STREAMS[key] = st                      # most recently used last
    while len(_COMM_STREAMS) > _COMM_STREAMS_MAX:
        _COMM_STREAMS.popitem(last=False)
    return st


def exchange_pipelined(transport, row_bytes, bin_counts, rank, device, chunk_offsets, pack_chunk,
                       nchunks, extra_rows=None, scratch=None):
    """exchange() with the pack and the row transfers overlapped: the tiles are
    packed in ``nchunks`` consecutive chunks, and as soon as chunk c is packed
    its rows travel -- every bin's rows of one chunk of tiles are a
    contiguous piece of that bin's segment, so chunk c of peer p is one
    message -- while chunk c + 1 is being packed (the messages run on a
    stream of their own, ordered after chunk c's pack by an event).

    ``chunk_offsets()`` -> int64 [nchunks + 1][size] (device tensor, or host
    array in the CPU tests): the first row of every bin at each chunk boundary
    in the packed (bin-major) layout, i.e. the scan's offsets at the boundary
    tiles (mgr_tile_offsets), read without a host sync.
    ``pack_chunk(c, sends, outs, redirect_bin, out_offsets)`` packs chunk c of
    every field (the self rows straight into the output, as exchange()'s
    pack).  One count message per peer carries [total, chunk 0, ..., chunk
    k-1] (k + 1 int64 each way, one group, ONE host sync per call), so every
    receive is posted with its exact size.  A rank whose scan failed sends
    -1 totals, one whose chunk counts do not add up to its totals -2: every
    rank then raises at the same point, before any row message is posted,
    naming the cause (check_counts).  Output
    bytes and order are exactly exchange()'s (receives in source-rank order,
    S7)."""
    size = transport.size
    k = int(nchunks)
    counts = torch.as_tensor(bin_counts).to(torch.int64).reshape(-1)
    dev = counts.device
    off = torch.as_tensor(chunk_offsets()).to(device=dev, dtype=torch.int64).reshape(k + 1, size)
    cs_d = off[1:] - off[:-1]                                  # [chunk][peer] rows sent
    ok = (cs_d.sum(dim=0) == counts).all()
    msg = torch.empty((size, k + 1), dtype=torch.int64, device=dev)
    # a failed scan keeps its -1; otherwise inconsistent chunks send -2
    bad = torch.where(counts < 0, counts, torch.full_like(counts, CHUNKS_INCONSISTENT))
    msg[:, 0] = torch.where(ok, counts, bad)
    msg[:, 1:] = cs_d.t()
    sh, rh = transport.exchange_count_rows(msg)
    for p in range(size):   # [total, k chunk counts] each way per peer
        transport.note("send", p, 8 * (k + 1))
        transport.note("recv", p, 8 * (k + 1))
    sc, rc = sh[:, 0].copy(), rh[:, 0].copy()
    check_counts(sc, rc)       # a -1 from any rank (failed scan, bad chunks): all raise
    cs = np.ascontiguousarray(sh[:, 1:].T)                     # [chunk][peer] rows sent
    cr = np.ascontiguousarray(rh[:, 1:])                       # [peer][chunk] rows received
    cr[rank] = cs[:, rank]
    if not np.array_equal(cr.sum(axis=1), rc):   # a peer's message is self-consistent
        raise MgrError(f"peers' chunk counts {cr.sum(axis=1)} do not add up to {rc}")
    # the self rows always go straight into the output (the pack's redirect),
    # whatever the transport: only the other peers' pieces travel
    lay = plan_layout(sc, rc, rank, True)
    extra = int(extra_rows(lay.total_recv)) if extra_rows is not None else 0
    outs, sends = [], []
    for f, rb in enumerate(row_bytes):
        outs.append(torch.empty(max((lay.total_recv + extra) * rb, 1), dtype=torch.uint8,
                                device=device))
        nbytes = max(lay.total_send * rb, 1)
        sends.append(scratch(f"send{f}", nbytes) if scratch is not None
                     else torch.empty(nbytes, dtype=torch.uint8, device=device))
    redirect = rank
    offs = [int(lay.recv_offsets[rank]) * rb for rb in row_bytes]
    gpu = isinstance(device, torch.device) and device.type == "cuda" or str(device).startswith("cuda")
    compute = torch.cuda.current_stream() if gpu else None
    comm = _comm_stream(device) if gpu else None
    sent_c = np.zeros(size, dtype=np.int64)     # rows of each peer's segment already sent
    recv_at = np.zeros(size, dtype=np.int64)    # rows of each source already received
    for c in range(nchunks):
        pack_chunk(c, sends, outs, redirect, offs)
        ops = []
        for j in range(1, size):
            to, frm = (rank + j) % size, (rank - j) % size
            for f, rb in enumerate(row_bytes):
                if cs[c, to]:
                    a = int(lay.send_offsets[to] + sent_c[to]) * rb
                    ops.append(("send", to, sends[f][a:a + int(cs[c, to]) * rb]))
                if cr[frm, c]:
                    a = int(lay.recv_offsets[frm] + recv_at[frm]) * rb
                    ops.append(("recv", frm, outs[f][a:a + int(cr[frm, c]) * rb]))
        for j in range(1, size):
            sent_c[(rank + j) % size] += cs[c, (rank + j) % size]
            recv_at[(rank - j) % size] += cr[(rank - j) % size, c]
        if not ops:
            continue
        if comm is not None:
            comm.wait_stream(compute)              # chunk c is packed
            with torch.cuda.stream(comm):
                transport.p2p(ops)
        else:
            transport.p2p(ops)
    if comm is not None:
        compute.wait_stream(comm)
        for t in outs + sends:
            t.record_stream(comm)
    transport.note_rows(row_bytes, sc, rc)
    return outs, lay
