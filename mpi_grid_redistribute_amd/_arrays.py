"""Adapters between caller arrays (torch GPU/CPU tensors, numpy arrays) and
the flat device byte buffers the kernels take.

The reference accepts numpy arrays indexed along axis 0 with any dtype,
structured records included (redist.py:126-129, S8), and mutates ``position``
in place (redist.py:68, S1).  Here:
  * torch tensors already on the GPU are used in place (zero copies);
  * numpy arrays / CPU tensors are staged to the GPU and the results (and
    the in-place position write-back) are copied back, so a numpy caller of
    the reference sees the same objects change.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

# position dtypes the binning kernels take: every float, integer and bool
# dtype (redist.py:68-69 bins any numeric numpy column).  float128 (x87
# extended precision) and complex are refused: the GPU has no extended float,
# and numpy's remainder is undefined for complex (the reference raises too).
_BOX_CODES = {"f2": _lib.MGR_F16, "f4": _lib.MGR_F32, "f8": _lib.MGR_F64, "i1": _lib.MGR_I8,
              "i2": _lib.MGR_I16, "i4": _lib.MGR_I32, "i8": _lib.MGR_I64, "u1": _lib.MGR_U8,
              "b1": _lib.MGR_B8, "u2": _lib.MGR_U16, "u4": _lib.MGR_U32, "u8": _lib.MGR_U64}
_NP_POS_CODES = {np.dtype(k): v for k, v in _BOX_CODES.items()}
_POS_CODES = {torch.float16: _lib.MGR_F16, torch.float32: _lib.MGR_F32,
              torch.float64: _lib.MGR_F64, torch.int8: _lib.MGR_I8, torch.int16: _lib.MGR_I16,
              torch.int32: _lib.MGR_I32, torch.int64: _lib.MGR_I64, torch.uint8: _lib.MGR_U8,
              torch.bool: _lib.MGR_B8}
for _name, _code in (("uint16", _lib.MGR_U16), ("uint32", _lib.MGR_U32), ("uint64", _lib.MGR_U64)):
    if hasattr(torch, _name):
        _POS_CODES[getattr(torch, _name)] = _code
_POS_NAMES = "float16/32/64, (u)int8-64, bool"
_ID_CODES = {torch.int32: _lib.MGR_I32, torch.int64: _lib.MGR_I64, torch.float32: _lib.MGR_F32,
             torch.float64: _lib.MGR_F64}


def device():
    return torch.device("cuda", torch.cuda.current_device())


def is_device_tensor(x):
    return isinstance(x, torch.Tensor) and x.is_cuda


class Rows:
    """A payload field: n rows of row_bytes opaque bytes on the device."""

    def __init__(self, obj, dev):
        self.obj = obj
        if isinstance(obj, torch.Tensor):
            if obj.dim() == 0:
                raise ValueError("data must have at least one dimension (rows on axis 0)")
            self.kind = "torch"
            self.dtype, self.trailing = obj.dtype, tuple(obj.shape[1:])
            t = obj if obj.is_cuda else obj.to(dev)
            t = t.contiguous()
            self.n = int(t.shape[0])
            self.row_bytes = int(t.element_size() * int(np.prod(self.trailing, dtype=np.int64)))
            self.flat = t.reshape(-1).view(torch.uint8) if t.numel() else torch.empty(
                0, dtype=torch.uint8, device=dev)
            self.out_device = obj.device
        else:
            a = np.asarray(obj)
            if a.ndim == 0:
                raise ValueError("data must have at least one dimension (rows on axis 0)")
            if a.dtype.hasobject:
                raise TypeError("object-dtype payloads are not supported (rows are moved as "
                                "bytes); the reference pickles them")
            self.kind = "numpy"
            self.dtype, self.trailing = a.dtype, tuple(a.shape[1:])
            self.host = a
            self.contig = np.ascontiguousarray(a)
            self.n = int(a.shape[0])
            self.row_bytes = int(a.dtype.itemsize * int(np.prod(self.trailing, dtype=np.int64)))
            flat = self.contig.reshape(-1).view(np.uint8) if a.size else np.zeros(0, np.uint8)
            self.flat = torch.from_numpy(flat).to(dev)
        if self.row_bytes == 0 and self.n:
            raise ValueError("zero-byte rows")

    def wrap(self, flat_out, m):
        """Output of m rows in the caller's type (new array, redist.py:199)."""
        if self.kind == "torch":
            if m == 0:
                return torch.empty((0,) + self.trailing, dtype=self.dtype, device=self.out_device)
            t = flat_out.view(self.dtype).reshape((m,) + self.trailing)
            return t if self.out_device.type == "cuda" else t.to(self.out_device)
        host = flat_out.cpu().numpy() if m else np.zeros(0, np.uint8)
        return host.view(self.dtype).reshape((m,) + self.trailing)

    def write_back_host(self):
        """numpy payload whose bytes were mutated on the device (position alias)."""
        if self.kind == "numpy" and self.n:
            dev_bytes = self.flat.cpu().numpy()
            np.copyto(self.host, dev_bytes.view(self.dtype).reshape(self.host.shape))


class Positions:
    """(N, >=dim) positions of any float, integer or bool dtype (redist.py
    bins any numeric column) as (device pointer, row stride, mgr_dtype code).

    ``finish()`` must run right after the binning kernel: it makes the
    caller's array hold the wrapped values (S1) before anything reads it."""

    def __init__(self, obj, dim, dev, data_rows: Rows | None = None):
        self.obj = obj
        self._copy_back = None
        self._alias_rows = None
        if isinstance(obj, torch.Tensor):
            if obj.dim() != 2 or obj.shape[1] < dim:
                raise ValueError(f"position must be (N, >= {dim}), got {tuple(obj.shape)}")
            if obj.dtype not in _POS_CODES:
                raise TypeError(f"position dtype {obj.dtype} not supported ({_POS_NAMES})")
            t = obj
            if not t.is_cuda or t.stride(1) != 1 or t.stride(0) < dim:
                t = obj.to(dev).contiguous()
                self._copy_back = ("torch", t)
            self.t = t
            self.n = int(t.shape[0])
            self.stride = int(t.stride(0)) if self.n else dim
            self.code = _POS_CODES[t.dtype]
            self.addr = t.data_ptr()
            return
        a = obj
        if not isinstance(a, np.ndarray):
            raise TypeError("position must be a numpy array or a torch tensor")
        if a.ndim != 2 or a.shape[1] < dim:
            raise ValueError(f"position must be (N, >= {dim}), got {a.shape}")
        if a.dtype not in _NP_POS_CODES:
            raise TypeError(f"position dtype {a.dtype} not supported ({_POS_NAMES})")
        self.n = int(a.shape[0])
        self.code = _NP_POS_CODES[a.dtype]
        isz = a.dtype.itemsize
        if (data_rows is not None and data_rows.kind == "numpy" and self.n
                and np.shares_memory(a, data_rows.host)):
            base = data_rows.host
            off = a.__array_interface__["data"][0] - base.__array_interface__["data"][0]
            ok = (base.flags.c_contiguous and off >= 0 and off % isz == 0
                  and a.strides[1] == isz and a.strides[0] % isz == 0 and a.strides[0] > 0)
            if not ok:
                raise NotImplementedError("position overlaps data in a layout other than a "
                                          "row-strided view of a C-contiguous data array")
            # the kernels read/write the positions inside the device copy of data
            self.addr = data_rows.flat.data_ptr() + off
            self.stride = a.strides[0] // isz
            self._alias_rows = data_rows
            self.t = None
            return
        c = np.ascontiguousarray(a)
        self.t = torch.from_numpy(c).to(dev)
        self.stride = int(a.shape[1])
        self.addr = self.t.data_ptr()
        self._copy_back = ("numpy", a)

    def finish(self):
        if self._copy_back is None:
            if self._alias_rows is not None:
                self._alias_rows.write_back_host()
            return
        kind, target = self._copy_back
        if kind == "torch":
            if target is not self.obj:
                self.obj.copy_(target)
        else:
            np.copyto(target, self.t.cpu().numpy())


def id_array(obj, dev):
    """rank_to_send as a device tensor of a kernel-supported dtype."""
    t = obj if isinstance(obj, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(obj))
    if t.dtype == torch.bool:
        t = t.to(torch.int64)
    elif t.dtype not in _ID_CODES:
        t = t.to(torch.float64 if t.is_floating_point() else torch.int64)
    t = t.to(dev).contiguous().reshape(-1)
    return t, _ID_CODES[t.dtype]


def pos_code(dtype):
    """mgr_dtype code of a position dtype (numpy or torch), or TypeError."""
    code = _POS_CODES.get(dtype) if isinstance(dtype, torch.dtype) else _NP_POS_CODES.get(
        np.dtype(dtype))
    if code is None:
        raise TypeError(f"position dtype {dtype} not supported ({_POS_NAMES})")
    return code


def box_dtype_code(box: np.ndarray):
    """numpy dtype of box_length (redist.py:46 keeps the caller's) -> mgr_dtype:
    with the positions' dtype it decides how numpy promotes the wrap and the
    quotient (S9, S11a; mgr_capi.hip promote).  bool promotes like uint8."""
    code = _BOX_CODES.get(box.dtype.kind + str(box.dtype.itemsize))
    if code is None:
        raise TypeError(f"box_length dtype {box.dtype} not supported (float16/32/64, "
                        "(u)int8-64, bool)")
    if box.dtype.kind in "iub" and box.size and np.abs(box.astype(np.float64)).max() >= 2.0 ** 53:
        raise NotImplementedError("integer box lengths of 2^53 or more")
    return code
