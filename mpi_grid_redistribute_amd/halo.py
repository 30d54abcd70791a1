"""Overload (halo) exchange -- ``exchange_overload_by_position`` (redist.py:202-309).

After the main redistribution every rank holds the rows of its own cell.  The
halo exchange adds, dimension by dimension, copies of the neighbours' rows
that lie within ``overload_lengths[d]`` of the shared face:

  for d in 0..dim-1 (redist.py:246):
      a / b = right / left neighbour cell (periodic wrap, :248-255)
      to_a  = rows with pos[:, d] > limits[d,1] - ol[d]   (local, then buffer)
      to_b  = rows with pos[:, d] < limits[d,0] + ol[d]
      step 1: send to_a -> a, receive from_b <- b         (:289-295)
      step 2: send to_b -> b, receive from_a <- a         (:298-303)
      buffer = concat(buffer, from_a, from_b)             (:305-306)

Data and positions travel with the same selections (the reference sends
them as two passes, :264); rows received in earlier dimensions are forwarded
in later ones, which fills the edge/corner regions.  Kept reference quirks:
positions are not shifted across the periodic boundary; with
``periodic=False`` the left send uses the right neighbour's flag (:287);
``redistribute_by_position`` never forwards ``periodic`` (:165).

On the GPU a dimension costs one pass over the new rows' flags, four
selection counts + scans, the packs of the selected rows into contiguous
send buffers (HIP kernels, libmgr.so) and two point-to-point steps over the
transport (RCCL ncclSend/ncclRecv for ``RcclComm``); the local rows' flags
for every dimension come from ONE pass over the local positions
(``mgr_halo_flags``).  Host syncs: two per dimension (selection counts,
received counts) -- the reference blocks on every message too.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def neighbours(R, d, periodic):
    """Right/left neighbour ranks of R's cell in dimension d and whether each
    side sends (redist.py:248-267, quirk :287 -- the left send's flag is the
    right neighbour's)."""
    ea = np.zeros(R.dim, dtype=np.int64)
    ea[d] = 1
    ia, ib = R.rank_cell_index + ea, R.rank_cell_index - ea
    a = int(R.get_cell_number_from_indexes_host(np.array([ia]))[0])
    b = int(R.get_cell_number_from_indexes_host(np.array([ib]))[0])
    if periodic:
        keep_a = keep_b = True
    else:
        keep_a = bool(R.get_cell_number_from_indexes_host(np.array([ia]), periodic=False)[0] == a)
        keep_b = keep_a
    return a, b, keep_a, keep_b


def thresholds(R, overload_lengths):
    """hi[d] = limits[d,1] - ol[d], lo[d] = limits[d,0] + ol[d], in float64
    with numpy's scalar promotion (redist.py:271-276)."""
    ol = overload_lengths
    hi = np.array([np.float64(R.rank_cell_limits[d, 1] - ol[d]) for d in range(R.dim)])
    lo = np.array([np.float64(R.rank_cell_limits[d, 0] + ol[d]) for d in range(R.dim)])
    return hi, lo


SELECT_TILE_ROWS = 4096


def halo_capacity(R, m, overload_lengths):
    """Spare rows to reserve after a rank's m redistributed rows for its halo:
    the uniform-density estimate m * (prod(1 + 2 ol/len) - 1), x1.25, + 4096.
    A halo that outgrows it still works (exchange_overload then moves to its
    own store and the caller concatenates)."""
    cl = np.asarray(R.cell_length, dtype=np.float64)
    ol = np.maximum(np.asarray(overload_lengths, dtype=np.float64), 0.0)
    frac = float(np.prod(1.0 + 2.0 * ol / cl) - 1.0)
    return int(m * frac * 1.25) + 4096


class DeviceSelect:
    """Selections on the GPU: flags (mgr_halo_flags), per-mask 2-bin
    partition counts (mgr_select_count + mgr_scan) and stable packs."""

    def __init__(self, dev):
        self.dev = dev

    def flags(self, pos_flat, n, ncols, code, dim, hi, lo):
        f = torch.empty(max(n, 1), dtype=torch.int16, device=self.dev)
        h = np.ascontiguousarray(hi, dtype=np.float64)
        l_ = np.ascontiguousarray(lo, dtype=np.float64)
        _lib.call("mgr_halo_flags", _lib.ptr(pos_flat), code, n, ncols, dim,
                  h.ctypes.data_as(ctypes.c_void_p), l_.ctypes.data_as(ctypes.c_void_p),
                  _lib.ptr(f), _lib.stream_handle())
        return f

    def select(self, flags, n, mask, max_row_bytes):
        """-> (handle, count tensor [1] on the device)."""
        lib = _lib.load()
        # long tiles: the selection pack is a wave-per-tile compaction
        # (mgr_pack with 2 bins, bin 1 dropped), whose cost is per tile
        tile_rows = SELECT_TILE_ROWS
        ws = torch.empty(int(lib.mgr_workspace_bytes(int(n), 2, tile_rows)), dtype=torch.uint8,
                         device=self.dev)
        dest = torch.empty(max(n, 1), dtype=torch.uint8, device=self.dev)
        counts = torch.empty(2, dtype=torch.int64, device=self.dev)
        s = _lib.stream_handle()
        _lib.call("mgr_select_count", _lib.ptr(flags), n, int(mask), _lib.ptr(dest), tile_rows,
                  _lib.ptr(ws), s)
        _lib.call("mgr_scan", n, 2, tile_rows, _lib.ptr(ws), _lib.ptr(counts), s)
        return (n, dest, ws, tile_rows), counts[:1]

    def pack(self, handle, src_flat, row_bytes, dst_flat):
        n, dest, ws, tile_rows = handle
        _lib.call("mgr_pack", _lib.ptr(src_flat), row_bytes, n, _lib.ptr(dest), 2, 1, tile_rows,
                  _lib.ptr(ws), _lib.ptr(dst_flat), -1, None, _lib.stream_handle())

    def pack2(self, handle, src1, rb1, dst1, src2, rb2, dst2):
        """Both fields of the selection in one pass (mgr_select_pack2)."""
        n, dest, ws, tile_rows = handle
        _lib.call("mgr_select_pack2", _lib.ptr(src1), rb1, _lib.ptr(dst1), _lib.ptr(src2), rb2,
                  _lib.ptr(dst2), n, _lib.ptr(dest), tile_rows, _lib.ptr(ws),
                  _lib.stream_handle())


def exchange_overload(R, transport, data_flat, rbd, pos_flat, ncols, pos_code, n,
                      overload_lengths, periodic=True, sel=None, arena=None):
    """Overload rows of rank R (redist.py:202-309).  ``data_flat``/``pos_flat``:
    flat uint8 tensors of this rank's n rows (payload rows of ``rbd`` bytes;
    positions (n, ncols) float32/float64 rows, ncols >= dim).  The overload
    buffer only grows at its end (concat(buffer, from_a, from_b), :305), so
    its rows live in an append-only store: ``arena`` = (data store, position
    store, first row, spare rows), e.g. the free tail of the redistribution's
    output, is used while the rows fit; beyond it the rows move once to a
    store of their own with headroom.  Returns (overload data flat, overload
    positions flat, rows, whether they stayed in the arena)."""
    dim = R.dim
    assert len(overload_lengths) == dim, \
        "Overload lengths must be the same length as the dimensions"  # redist.py:245
    dev = data_flat.device
    sel = sel or DeviceSelect(dev)
    isz = 4 if pos_code == _lib.MGR_F32 else 8
    rbp = ncols * isz
    hi, lo = thresholds(R, overload_lengths)
    seg_local = (sel.flags(pos_flat, n, ncols, pos_code, dim, hi, lo), n, data_flat, pos_flat)
    if arena is not None:
        st_d, st_p, base, cap = arena
    else:
        st_d = st_p = None
        base, cap = 0, 0
    in_arena = arena is not None
    m = 0
    for d in range(dim):
        a, b, keep_a, keep_b = neighbours(R, d, periodic)
        segs = [seg_local]
        if m:
            ov_d = st_d[base * rbd:(base + m) * rbd]
            ov_p = st_p[base * rbp:(base + m) * rbp]
            segs.append((sel.flags(ov_p, m, ncols, pos_code, dim, hi, lo), m, ov_d, ov_p))
        sends = []
        for mask, keep in ((1 << (2 * d), keep_a), (1 << (2 * d + 1), keep_b)):
            picks = [sel.select(f, k, mask, max(rbd, rbp)) + (dd, pp)
                     for f, k, dd, pp in segs if k > 0] if keep else []
            sends.append(picks)
        flat_counts = [p[1] for picks in sends for p in picks]
        host = torch.cat(flat_counts).cpu().tolist() if flat_counts else []
        cnt = [host[: len(sends[0])], host[len(sends[0]):]]
        bufs = []
        for picks, cs in zip(sends, cnt):
            tot = int(sum(cs))
            bd = torch.empty(max(tot * rbd, 1), dtype=torch.uint8, device=dev)
            bp = torch.empty(max(tot * rbp, 1), dtype=torch.uint8, device=dev)
            o = 0
            for (h, _, dd, pp), c in zip(picks, cs):
                if c:
                    # two selection packs: the fused one (sel.pack2) measured
                    # no faster (sparse rows cost a line each either way)
                    sel.pack(h, dd, rbd, bd[o * rbd:])
                    sel.pack(h, pp, rbp, bp[o * rbp:])
                o += c
            bufs.append((tot, bd[: tot * rbd], bp[: tot * rbp]))
        # row counts first (8-byte messages), both steps, then one host sync
        n_a, n_b = bufs[0][0], bufs[1][0]
        cs = torch.tensor([n_a, n_b], dtype=torch.int64, device=dev)
        cr = torch.zeros(2, dtype=torch.int64, device=dev)
        transport.sendrecv(cs[0:1].view(torch.uint8), a, cr[0:1].view(torch.uint8), b)  # :289-295
        transport.sendrecv(cs[1:2].view(torch.uint8), b, cr[1:2].view(torch.uint8), a)  # :298-303
        r_from_b, r_from_a = (int(x) for x in cr.cpu().tolist())
        new_m = m + r_from_a + r_from_b
        if st_d is None or new_m > cap:
            # outgrew the store: a store of its own with headroom, rows so far moved once
            ncap = max(2 * new_m, 1024)
            nd = torch.empty(ncap * rbd, dtype=torch.uint8, device=dev)
            npb = torch.empty(ncap * rbp, dtype=torch.uint8, device=dev)
            if m:
                nd[: m * rbd].copy_(st_d[base * rbd:(base + m) * rbd])
                npb[: m * rbp].copy_(st_p[base * rbp:(base + m) * rbp])
            st_d, st_p, base, cap, in_arena = nd, npb, 0, ncap, False
        # concat(buffer, from_a, from_b) (redist.py:305): appended in place
        od, op = st_d[base * rbd:], st_p[base * rbp:]
        ia, ib = m, m + r_from_a
        transport.sendrecv(bufs[0][1], a, od[ib * rbd:(ib + r_from_b) * rbd], b)
        transport.sendrecv(bufs[0][2], a, op[ib * rbp:(ib + r_from_b) * rbp], b)
        transport.sendrecv(bufs[1][1], b, od[ia * rbd:(ia + r_from_a) * rbd], a)
        transport.sendrecv(bufs[1][2], b, op[ia * rbp:(ia + r_from_a) * rbp], a)
        m = new_m
    if not m:
        empty = torch.empty(0, dtype=torch.uint8, device=dev)
        return empty, empty, 0, in_arena
    return st_d[base * rbd:(base + m) * rbd], st_p[base * rbp:(base + m) * rbp], m, in_arena
