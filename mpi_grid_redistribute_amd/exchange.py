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


def check_counts(send_counts, recv_counts):
    """A failed device scan reports -1 counts (mgr_kernels.hip scan_onepass_kernel);
    a peer's failure arrives here as a -1 receive count, so every rank raises
    together instead of one rank leaving the others inside the exchange."""
    if (np.asarray(send_counts) < 0).any() or (np.asarray(recv_counts) < 0).any():
        raise MgrError("device scan failed (a look-back timed out on this rank or a peer): "
                       f"send counts {list(send_counts)}, receive counts {list(recv_counts)}")


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
             scratch=None, pack_all=None):
    """Run steps 1-4.  ``bin_counts``: int64 tensor [size] of rows per
    destination (on ``device``).  ``pack(field, send, redirect_bin, out,
    out_offset)`` packs field ``field`` (the redirect bin's rows into ``out``
    from byte ``out_offset``).  ``extra_rows(total_recv)``: spare
    rows to allocate after the received ones (the halo appends there).
    ``scratch(name, nbytes)``: a reusable device buffer (the send buffers),
    else fresh allocations.  ``pack_all(sends, outs, redirect_bin,
    out_offsets)``, when given, packs every field in one call instead (fields
    moved by one kernel, e.g. rows with their fine cells).  Returns (outs, layout); outs are new flat uint8
    tensors of (total_recv + extra) * row_bytes[f] bytes (>= 1 byte)."""
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
