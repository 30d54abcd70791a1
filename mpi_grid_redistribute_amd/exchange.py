"""Exchange orchestration shared by every transport (redist.py:199).

After the local stage has produced the per-destination row counts, one
redistribution does:
  1. count exchange    -> how many rows arrive from each source (host copy);
  2. layout            -> send offsets (bin-major packed buffer) and receive
                          offsets in source-rank order (S7), output size;
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


def exchange(transport, row_bytes, bin_counts, rank, device, pack, extra_rows=None):
    """Run steps 1-4.  ``bin_counts``: int64 tensor [size] of rows per
    destination (on ``device``).  ``pack(field, send, redirect_bin,
    redirect_out)`` packs field ``field``.  ``extra_rows(total_recv)``: spare
    rows to allocate after the received ones (the halo appends there).
    Returns (outs, layout); outs are flat uint8 tensors of (total_recv +
    extra) * row_bytes[f] bytes (>= 1 byte)."""
    sc, rc = transport.exchange_counts(bin_counts)
    lay = ExchangeLayout(send_counts=sc, recv_counts=rc, send_offsets=excl_cumsum(sc),
                         recv_offsets=excl_cumsum(rc), total_recv=int(rc.sum()),
                         total_send=int(sc.sum()), redirect_self=bool(transport.skips_self))
    size = len(sc)
    extra = int(extra_rows(lay.total_recv)) if extra_rows is not None else 0
    outs, sends = [], []
    for f, rb in enumerate(row_bytes):
        out = torch.empty(max((lay.total_recv + extra) * rb, 1), dtype=torch.uint8, device=device)
        n_send = lay.total_send
        if lay.redirect_self and size == 1:
            n_send = 0  # everything is the self segment
        snd = torch.empty(max(n_send * rb, 1), dtype=torch.uint8, device=device)
        if lay.redirect_self:
            pack(f, snd, rank, out[int(lay.recv_offsets[rank]) * rb:])
        else:
            pack(f, snd, -1, None)
        outs.append(out)
        sends.append(snd)
    transport.exchange_rows(sends, outs, list(row_bytes), sc, lay.send_offsets, rc,
                            lay.recv_offsets)
    return outs, lay
