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

On the GPU every row carries 16 face-flag bits (bit 2d: coordinate d beyond
the right threshold, bit 2d+1: below the left one).  Through
``redistribute_by_position`` the binning kernel computes them against the
limits of the cell the row lands in (mgr_bin_count_halo) and they travel
with the row; called directly, one pass over the local positions computes
them (mgr_halo_flags).  They stay valid on every rank a row is forwarded to:
a neighbour's cell differs from the sender's only in the dimension of the
exchange, whose bits are not read again.

  1. the local rows' 2*dim selections counted in ONE pass (mgr_msel_count,
     mgr_scan); one group exchanges the counts with the neighbours; one host
     sync reads them;
  2. the local sends of every dimension whose neighbours are other ranks
     (and of dimension 0) are packed in one pass (mgr_msel_pack_fields:
     data, positions when carried, flags), each set straight to its place;
  3. per dimension d: the received rows so far (the buffer) are selected the
     same way (2 sets) -- a small set; from d = 1 their counts travel as an
     8-byte message and one host sync reads them; then ONE group moves, in
     the reference's order (step 1, then step 2), the local piece and the
     buffer piece of every field to each neighbour, the receives landing
     appended to the buffer in place.  A dimension whose neighbours are this
     rank itself (a grid extent of 1) sends nothing: its pieces are packed
     straight into the buffer where the receives would land.
Host syncs: 1 + (dim - 1) per exchange.  The buffer is an append-only store:
redistribute_by_position hands over the spare rows of its output, so the
final concatenate(data, overload) (:166) costs nothing while the halo fits;
when the positions are not returned they are not carried at all (the flags
already hold everything the selections read).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .exchange import check_counts, host_read_start, host_read_wait


def _p2p(transport, ops):
    """One batch of point-to-point messages, its off-rank bytes counted in
    the transport's traffic."""
    transport.note_p2p(ops)
    transport.p2p(ops)


# The multi-rank halo's count messages carry a failure bit beside the size: a
# selection scan that gave up (-1 counts) is announced as size 0 with the bit
# set, so every message of the exchange keeps consistent sizes on both sides
# (nobody waits for a message that will not come), and the ranks agree on the
# failure ONCE, after the last message, instead of after every count exchange.
_FAIL = 1 << 62


def _encode_counts(c):
    """Device int64 counts -> message words: size (>= 0), plus _FAIL on every
    word when any count is negative (a failed scan poisons all of them)."""
    bad = (c < 0).any()
    return torch.where(bad, torch.full_like(c, _FAIL), c.clamp(min=0))


def _decode(words):
    w = np.asarray(words, dtype=np.int64)
    return w & (_FAIL - 1), bool((w >> 62).any())


def _agree_counts(transport, sent, received):
    """check_counts on every rank at once: a -1 count (a selection scan that
    gave up) reaches only the neighbours of the failed rank, so the ranks
    agree on the flag first and all raise, none left waiting in a message."""
    failed = (np.asarray(sent) < 0).any() or (np.asarray(received) < 0).any()
    if transport.any_failed(failed):
        check_counts(sent, received)
        check_counts([-1], [])     # a peer failed: raise here too


def self_halo_pieces(dim):
    """The overload rows of a rank that is its own neighbour in every
    dimension (one rank; periodic), as pieces in store order: piece = the
    local rows whose flags hold every bit of its mask, in row order.  The
    reference's loop (redist.py:246-306) on sets of local rows: per dimension
    to_a = local rows beyond the right face, then the buffer's; to_b the same
    at the left face; the rank receives its own to_a as from_b and its own
    to_b as from_a, and buffer = concat(buffer, from_a, from_b) (:305-306).
    3^dim - 1 pieces: the faces, edges and corners of the halo."""
    buf = []
    for d in range(dim):
        a, b = 1 << (2 * d), 1 << (2 * d + 1)
        to_a = [a] + [m | a for m in buf]
        to_b = [b] + [m | b for m in buf]
        buf = buf + to_b + to_a
    return buf


def _self_halo(transport, sel, srcs, rbs, flags, n, dim, carry_pos, arena, dev, pending=()):
    """exchange_overload when every neighbour is this rank: all pieces are
    known from the local rows' flags, so one selection pass counts them all
    and one multi-set pack writes every row straight to each of its pieces
    in the store -- the local rows are read once, not once per dimension,
    and nothing is staged or received."""
    pieces = self_halo_pieces(dim)
    h, cnt = sel.msel_masks(flags, n, pieces, "_self")
    F = len(rbs)
    placed = arena is not None and arena[3] > 0
    # the one host read is enqueued BEFORE the placed pack and waited for on
    # its own event: the host finishes this call (and launches the caller's
    # next work) while the pack runs, instead of idling the GPU after it
    read = sel.to_host_start([cnt] + list(pending))
    if placed:   # into the arena before the sizes are known: no gap at the sync
        ast = [arena[0]] + ([arena[1]] if carry_pos else [])
        sel.msel_pack_placed(h, srcs, rbs, [ast[f][arena[2] * rbs[f]:] for f in range(F)],
                             arena[3])
    got = sel.to_host_wait(read)                          # the one host sync
    counts = got[0]
    for c in got[1:]:   # the redistribution's deferred count check
        check_counts(c, [])
    _agree_counts(transport, counts, [])
    total = int(counts.sum())
    if placed and total <= arena[3]:
        _lib.alg_add("halo_pack", 2 * n + 2 * total * sum(rbs))
        if not total:
            empty = torch.empty(0, dtype=torch.uint8, device=dev)
            return empty, (empty if carry_pos else None), 0, True
        b = arena[2]
        out = [ast[f][b * rbs[f]:(b + total) * rbs[f]] for f in range(F)]
        return out[0], (out[1] if carry_pos else None), total, True
    if arena is not None and total <= arena[3]:
        st, base, in_arena = [arena[0]] + ([arena[1]] if carry_pos else []), arena[2], True
    else:
        st = [torch.empty(max(total, 1) * rb, dtype=torch.uint8, device=dev) for rb in rbs]
        base, in_arena = 0, False
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    dsts = [[st[f][(base + int(offs[k])) * rbs[f]:(base + int(offs[k + 1])) * rbs[f]]
             if counts[k] else None for k in range(len(pieces))] for f in range(F)]
    if total:
        sel.msel_pack_fields(h, srcs, rbs, dsts, total)
    if not total:
        empty = torch.empty(0, dtype=torch.uint8, device=dev)
        return empty, (empty if carry_pos else None), 0, in_arena
    out = [st[f][base * rbs[f]:(base + total) * rbs[f]] for f in range(F)]
    return out[0], (out[1] if carry_pos else None), total, in_arena


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
    the uniform-density estimate m * (prod(1 + 2 ol/len) - 1), x1.25, + 4096,
    with ol capped at the cell length (the exchange reaches the immediate
    neighbours only, so each factor is at most 3) and the whole at
    (3^dim - 1) * m.  A halo that outgrows it still works (exchange_overload
    then moves to its own store and the caller concatenates)."""
    cl = np.asarray(R.cell_length, dtype=np.float64)
    ol = np.minimum(np.maximum(np.asarray(overload_lengths, dtype=np.float64), 0.0), cl)
    with np.errstate(invalid="ignore", divide="ignore"):
        frac = float(np.prod(1.0 + 2.0 * np.where(cl > 0, ol / cl, 1.0)) - 1.0)
    frac = min(frac, 3.0 ** len(cl) - 1.0)
    return int(m * frac * 1.25) + 4096


class DeviceSelect:
    """Selections on the GPU: face flags (mgr_halo_flags) and multi-set
    selections (mgr_msel_count + mgr_scan + mgr_msel_pack)."""

    def __init__(self, dev, scratch=None):
        self.dev = dev
        self.scratch = scratch

    def _buf(self, name, nbytes):
        if self.scratch is not None:
            return self.scratch.get(name, nbytes)
        return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self.dev)

    def flags(self, pos_flat, n, ncols, code, dim, hi, lo):
        f = torch.empty(max(n, 1), dtype=torch.int16, device=self.dev)
        h = np.ascontiguousarray(hi, dtype=np.float64)
        l_ = np.ascontiguousarray(lo, dtype=np.float64)
        _lib.call("mgr_halo_flags", _lib.ptr(pos_flat), code, n, ncols, dim,
                  h.ctypes.data_as(ctypes.c_void_p), l_.ctypes.data_as(ctypes.c_void_p),
                  _lib.ptr(f), _lib.stream_handle())
        return f

    def msel(self, flags, n, bits, tag):
        """Counts of the sets {rows with flag bit bits[k]} -> (handle, device
        int64 counts [len(bits)])."""
        return self.msel_masks(flags, n, [1 << int(b) for b in bits], tag)

    def msel_masks(self, flags, n, masks, tag):
        """Counts of the sets {rows whose flags hold every bit of masks[k]}."""
        lib = _lib.load()
        tile_rows = SELECT_TILE_ROWS
        k = len(masks)
        ws = self._buf("msel_ws" + tag, int(lib.mgr_workspace_bytes(int(n), k, tile_rows)))
        counts = torch.empty(k, dtype=torch.int64, device=self.dev)
        cb = (ctypes.c_int * k)(*[int(m) for m in masks])
        s = _lib.stream_handle()
        _lib.call("mgr_msel_count", _lib.ptr(flags), n, k, cb, tile_rows, _lib.ptr(ws), s)
        _lib.alg_add("halo", 2 * n)                        # the flags, read once
        _lib.call("mgr_scan", n, k, tile_rows, _lib.ptr(ws), _lib.ptr(counts), s)
        return (n, flags, cb, k, ws, tile_rows), counts

    def msel_pack(self, handle, src_flat, row_bytes, dsts):
        """One field's selected rows: set k's rows, in row order, to dsts[k]
        (a flat uint8 tensor, or None: set k not written)."""
        n, flags, cb, k, ws, tile_rows = handle
        ptrs = (ctypes.c_void_p * k)(*[None if t is None else _lib.ptr(t) for t in dsts])
        _lib.call("mgr_msel_pack", _lib.ptr(src_flat), row_bytes, n, _lib.ptr(flags), k, cb,
                  tile_rows, _lib.ptr(ws), ptrs, _lib.stream_handle())

    def msel_pack_fields(self, handle, srcs, row_bytes, dsts, rows_out=0):
        """Several fields of the same rows in one pass: dsts[f][k] as in
        msel_pack (field 0's None entries decide which sets are written).
        ``rows_out``: the rows the written sets hold (byte accounting)."""
        n, flags, cb, k, ws, tile_rows = handle
        _lib.alg_add("halo_pack", 2 * n + 2 * rows_out * sum(row_bytes))
        nf = len(srcs)
        sp = (ctypes.c_void_p * nf)(*[_lib.ptr(t) for t in srcs])
        rb = (ctypes.c_int64 * nf)(*row_bytes)
        dp = (ctypes.c_void_p * (nf * k))(*[None if t is None else _lib.ptr(t)
                                             for row in dsts for t in row])
        _lib.call("mgr_msel_pack_fields", nf, sp, rb, n, _lib.ptr(flags), k, cb, tile_rows,
                  _lib.ptr(ws), dp, _lib.stream_handle())

    def msel_pack_placed(self, handle, srcs, row_bytes, dsts, cap_rows):
        """msel_pack_fields with the sets back to back from dsts[f] at the
        scan's set starts, rows beyond cap_rows not written: launched before
        the set sizes are known on the host."""
        n, flags, cb, k, ws, tile_rows = handle
        nf = len(srcs)
        sp = (ctypes.c_void_p * nf)(*[_lib.ptr(t) for t in srcs])
        rb = (ctypes.c_int64 * nf)(*row_bytes)
        dp = (ctypes.c_void_p * nf)(*[_lib.ptr(t) for t in dsts])
        _lib.call("mgr_msel_pack_placed", nf, sp, rb, n, _lib.ptr(flags), k, cb, tile_rows,
                  _lib.ptr(ws), dp, int(cap_rows), _lib.stream_handle())

    def to_host(self, tensors):
        """One device->host read of several small int64 tensors (one sync)."""
        return self.to_host_wait(self.to_host_start(tensors))

    @staticmethod
    def to_host_start(tensors):
        return host_read_start(tensors)

    @staticmethod
    def to_host_wait(read):
        return host_read_wait(read)


def exchange_overload(R, transport, data_flat, rbd, pos_flat, ncols, pos_code, n,
                      overload_lengths, periodic=True, sel=None, arena=None, flags=None,
                      pending=()):
    """Overload rows of rank R (redist.py:202-309).  ``data_flat``: flat uint8
    tensor of this rank's n payload rows of ``rbd`` bytes; ``pos_flat``: their
    positions (n, ncols) rows of any position dtype (ncols >= dim), or None when the
    positions are not wanted back and ``flags`` is given.  ``flags``: the
    rows' face flags (int16 [n]) when the binning computed them, else one pass
    computes them from the positions here.  The overload buffer only grows at
    its end (concat(buffer, from_a, from_b), :305), so its rows live in an
    append-only store: ``arena`` = (data store, position store or None, first
    row, spare rows), e.g. the free tail of the redistribution's output, is
    used while the rows fit; beyond it the rows move once to a store of their
    own with headroom.  Returns (overload data flat, overload positions flat
    or None, rows, whether they stayed in the arena).  ``pending``: device
    count tensors of the caller whose check (check_counts) rides on this
    exchange's first host read."""
    dim = R.dim
    assert len(overload_lengths) == dim, \
        "Overload lengths must be the same length as the dimensions"  # redist.py:245
    dev = data_flat.device
    sel = sel or DeviceSelect(dev)
    carry_pos = pos_flat is not None
    if flags is None:
        hi, lo = thresholds(R, overload_lengths)
        flags = sel.flags(pos_flat, n, ncols, pos_code, dim, hi, lo)
    flags_flat = flags.reshape(-1).view(torch.uint8)[: 2 * n]
    isz = _lib.POS_ITEMSIZE[pos_code]
    srcs = [data_flat] + ([pos_flat] if carry_pos else []) + [flags_flat]
    rbs = [rbd] + ([ncols * isz] if carry_pos else []) + [2]
    F, FL = len(rbs), len(rbs) - 1                        # fields; the flags field
    me = transport.rank
    nb = [neighbours(R, d, periodic) for d in range(dim)]
    selfd = [a == me and b == me for a, b, _, _ in nb]
    if dim <= 3 and all(selfd) and all(ka and kb for _, _, ka, kb in nb):
        return _self_halo(transport, sel, srcs[:F - 1], rbs[:F - 1], flags, n, dim, carry_pos,
                          arena, dev, pending)
    for c in pending:   # (the general path reads them here)
        check_counts(c.cpu().numpy(), [])

    # 1. the local rows' counts of every dimension's two selections, one pass
    S = 2 * dim
    lh, lcount = sel.msel(flags, n, list(range(S)), "_local")
    # 2. local counts to the neighbours (step 1 then step 2 of every dimension)
    send_l = torch.zeros(S, dtype=torch.int64, device=dev)
    send_l.copy_(_encode_counts(lcount))
    for d, (a, b, keep_a, keep_b) in enumerate(nb):
        if not keep_a:
            send_l[2 * d].zero_()
        if not keep_b:
            send_l[2 * d + 1].zero_()
    recv_l = torch.zeros(S, dtype=torch.int64, device=dev)   # [from_b, from_a] per dimension
    ops = []
    for d, (a, b, _, _) in enumerate(nb):
        ops += [("send", a, send_l[2 * d:2 * d + 1].view(torch.uint8)),
                ("recv", b, recv_l[2 * d:2 * d + 1].view(torch.uint8)),
                ("send", b, send_l[2 * d + 1:2 * d + 2].view(torch.uint8)),
                ("recv", a, recv_l[2 * d + 1:2 * d + 2].view(torch.uint8))]
    _p2p(transport, ops)
    ls, rl = sel.to_host([send_l, recv_l])                   # host sync 1
    # a failed selection scan (here, or at a neighbour through its messages)
    # travels as the failure bit; sizes stay consistent, the ranks agree at
    # the end of the exchange
    ls, f1 = _decode(ls)
    rl, f2 = _decode(rl)
    failed = f1 or f2

    # the append-only overload store: data (+ positions) + flags
    st = [None] * F
    base, cap, in_arena = 0, 0, False
    if arena is not None:
        st[0] = arena[0]
        if carry_pos:
            st[1] = arena[1]
        base, cap, in_arena = arena[2], arena[3], True
        st[FL] = torch.empty(max(cap, 1) * 2, dtype=torch.uint8, device=dev)
    fbase = [base] * (F - 1) + [0]                           # the flags store is our own
    m = 0

    def store(f, row0=0, rows=None):
        o = (fbase[f] + row0) * rbs[f]
        return st[f][o:] if rows is None else st[f][o:o + rows * rbs[f]]

    def ensure(new_m):
        nonlocal st, fbase, cap, in_arena
        if st[0] is not None and new_m <= cap:
            return
        # outgrew the store: a store of its own with headroom, rows so far moved once
        ncap = max(2 * new_m, 1024)
        nst = [torch.empty(ncap * rb, dtype=torch.uint8, device=dev) for rb in rbs]
        for f in range(F):
            if m:
                nst[f][: m * rbs[f]].copy_(store(f, 0, m))
        st, fbase, cap, in_arena = nst, [0] * F, ncap, False

    def local_pieces(d):
        """Rows this rank sends in dimension d: its local piece then its
        buffer piece, to a (step 1) and to b (step 2)."""
        a, b, keep_a, keep_b = nb[d]
        return (int(ls[2 * d]) if keep_a else 0), (int(ls[2 * d + 1]) if keep_b else 0)

    # local sends staged for the neighbours: every non-self dimension's sets
    # (and dimension 0's, whose place in the store is known now) in one pass;
    # the sets of a later self dimension are written straight into the store
    # when that dimension comes (their place depends on the earlier receives)
    stage_off, off = {}, 0
    for d in range(dim):
        if not selfd[d]:
            nla, nlb = local_pieces(d)
            stage_off[d] = off
            off += nla + nlb
    lbuf = [sel._buf(f"halo_local{f}", off * rbs[f]) for f in range(F)]

    def local_dsts(d, f, ia, ib):
        """Set -> destination of dimension d's local pieces, field f."""
        nla, nlb = local_pieces(d)
        rb = rbs[f]
        if selfd[d]:   # step 1 (to a = me) lands at ib, step 2 (to b = me) at ia
            return {2 * d: store(f, ib, nla) if nla else None,
                    2 * d + 1: store(f, ia, nlb) if nlb else None}
        o = stage_off[d]
        return {2 * d: lbuf[f][o * rb:(o + nla) * rb] if nla else None,
                2 * d + 1: lbuf[f][(o + nla) * rb:(o + nla + nlb) * rb] if nlb else None}

    def pack_local(dims, places):
        dsts = [[None] * S for _ in range(F)]
        for d in dims:
            for f in range(F):
                for k, t in local_dsts(d, f, *places.get(d, (0, 0))).items():
                    dsts[f][k] = t
        if any(t is not None for t in dsts[0]):
            sel.msel_pack_fields(lh, srcs, rbs, dsts, sum(sum(local_pieces(d)) for d in dims))

    first = [d for d in range(dim) if not selfd[d] or d == 0]
    if selfd[0]:
        nla, nlb = local_pieces(0)
        ensure(nla + nlb)
    pack_local(first, {0: (0, local_pieces(0)[1])} if selfd[0] else {})

    for d, (a, b, keep_a, keep_b) in enumerate(nb):
        sa, sb = 2 * d, 2 * d + 1
        # 3. the buffer's selections for this dimension (rows received so far)
        gc = np.zeros(2, dtype=np.int64)
        rg = np.zeros(2, dtype=np.int64)
        gh = None
        if d > 0:
            send_g = torch.zeros(2, dtype=torch.int64, device=dev)
            recv_g = torch.zeros(2, dtype=torch.int64, device=dev)
            if m:
                gh, gcount = sel.msel(store(FL, 0, m).view(torch.int16), m, [sa, sb], "_ghost")
                send_g.copy_(_encode_counts(gcount))
            if failed:   # keep announcing it: the neighbours' neighbours learn too
                send_g.fill_(_FAIL)
            if not keep_a:
                send_g[0].zero_()
            if not keep_b:
                send_g[1].zero_()
            _p2p(transport, [("send", a, send_g[0:1].view(torch.uint8)),
                           ("recv", b, recv_g[0:1].view(torch.uint8)),
                           ("send", b, send_g[1:2].view(torch.uint8)),
                           ("recv", a, recv_g[1:2].view(torch.uint8))])
            gc, rg = sel.to_host([send_g, recv_g])            # host sync per dimension
            gc, f1 = _decode(gc)
            rg, f2 = _decode(rg)
            # (sizes stay as announced -- the neighbours post receives of them)
            failed = failed or f1 or f2
        nla, nlb = local_pieces(d)
        nga, ngb = int(gc[0]), int(gc[1])
        # what it receives: from_b (step 1) and from_a (step 2), each a local
        # piece and a buffer piece of the sender
        rlb, rla = int(rl[sa]), int(rl[sb])
        rgb, rga = int(rg[0]), int(rg[1])
        new_m = m + rla + rga + rlb + rgb
        ensure(new_m)
        # concat(buffer, from_a, from_b) (redist.py:305): appended in place
        ia, ib = m, m + rla + rga
        if selfd[d] and d > 0:
            pack_local([d], {d: (ia, ib)})
        gsz = nga + ngb
        gbuf = None
        if gsz:
            if selfd[d]:
                gd = [[store(f, ib + nla, nga) if nga else None,
                       store(f, ia + nlb, ngb) if ngb else None] for f in range(F)]
            else:
                gbuf = [sel._buf(f"halo_ghost{f}", gsz * rbs[f]) for f in range(F)]
                gd = [[gbuf[f][: nga * rbs[f]] if nga else None,
                       gbuf[f][nga * rbs[f]:gsz * rbs[f]] if ngb else None] for f in range(F)]
            sel.msel_pack_fields(gh, [store(f, 0, m) for f in range(F)], rbs, gd, gsz)
        if selfd[d]:
            m = new_m
            continue
        ops = []
        o = stage_off[d]
        for step in (1, 2):
            to, frm = (a, b) if step == 1 else (b, a)
            nl, ng = (nla, nga) if step == 1 else (nlb, ngb)
            lo_, go_ = (o, 0) if step == 1 else (o + nla, nga)
            rl_, rg_, at = (rlb, rgb, ib) if step == 1 else (rla, rga, ia)
            for f in range(F):
                rb = rbs[f]
                if nl:
                    ops.append(("send", to, lbuf[f][lo_ * rb:(lo_ + nl) * rb]))
                if ng:
                    ops.append(("send", to, gbuf[f][go_ * rb:(go_ + ng) * rb]))
                if rl_:
                    ops.append(("recv", frm, store(f, at, rl_)))
                if rg_:
                    ops.append(("recv", frm, store(f, at + rl_, rg_)))
        _p2p(transport, ops)
        m = new_m
    # one agreement per call: every rank raises together if any scan failed
    if transport.any_failed(failed):
        check_counts([-1], [])
    if not m:
        empty = torch.empty(0, dtype=torch.uint8, device=dev)
        return empty, (empty if carry_pos else None), 0, in_arena
    return store(0, 0, m), (store(1, 0, m) if carry_pos else None), m, in_arena
