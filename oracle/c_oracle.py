"""ctypes binding of oracle/_build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/ and bench.py's cpu_baseline leg as the large-N checker; the
product library never loads it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

_P = ctypes.c_void_p
_I64 = ctypes.c_int64


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_bin.argtypes = [_P, ctypes.c_int, ctypes.c_int, _I64, _I64, ctypes.c_int, _P, _P,
                                 ctypes.c_int, _P, _P]
        L.oracle_bin.restype = None
        L.oracle_partition.argtypes = [_P, _I64, _I64, _P, _I64, _P, _P]
        L.oracle_partition.restype = _I64
        L.oracle_synth_uniform.argtypes = [ctypes.c_uint64, _I64, _I64, ctypes.c_int, _P, _P, _P]
        L.oracle_synth_uniform.restype = None
        L.oracle_fnv1a.argtypes = [_P, _I64]
        L.oracle_fnv1a.restype = ctypes.c_uint64
        L.oracle_pymod.argtypes = [ctypes.c_double, ctypes.c_double]
        L.oracle_pymod.restype = ctypes.c_double
        L.oracle_trunc_i64.argtypes = [ctypes.c_double]
        L.oracle_trunc_i64.restype = ctypes.c_int64
        L.oracle_local_partition_omp.argtypes = [_P, _I64, _I64, ctypes.c_int, _P, _P,
                                                 ctypes.c_int, _P, _I64, _P, _P, ctypes.c_int,
                                                 _P, _P]
        L.oracle_local_partition_omp.restype = _I64
        L.oracle_bin_ext.argtypes = [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _I64, _I64,
                                     ctypes.c_int, _P, _P, ctypes.c_int, _P, _P]
        L.oracle_bin_ext.restype = None
        L.oracle_d2h.argtypes = [ctypes.c_double]
        L.oracle_d2h.restype = ctypes.c_uint16
        L.oracle_f2h.argtypes = [ctypes.c_float]
        L.oracle_f2h.restype = ctypes.c_uint16
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


# oracle_bin_ext dtype codes (the O_* of mgr_oracle.c)
_CODES = {np.dtype(k): v for k, v in {"f4": 1, "f8": 2, "i4": 3, "i8": 4, "f2": 5, "i1": 6,
                                       "i2": 7, "u1": 8, "u2": 9, "u4": 10, "u8": 11,
                                       "b1": 12}.items()}
_EXT = {k: v for k, v in _CODES.items() if v > 2}


def bin_positions(position, grid_topology, box_length, periodic=True, compute_f32=None,
                  want_idx=False):
    """Bin ``position`` ((N, >=dim) float32/float64, C-contiguous rows) in place.

    Returns int64 cell ids (and per-dim indexes when ``want_idx``)."""
    if position.ndim == 2 and position.shape[0] == 0:   # an empty rank (numpy strides 0)
        cell = np.empty(0, dtype=np.int64)
        idx = np.empty((0, len(grid_topology)), dtype=np.int64)
        return (cell, idx) if want_idx else cell
    assert position.ndim == 2 and position.strides[1] == position.itemsize
    topo = np.ascontiguousarray(np.asarray(grid_topology).astype(np.int64))
    box_arr = np.asarray(box_length)
    dim = len(topo)
    if position.dtype in _EXT:
        # numpy itself names the types the wrap and the quotient compute in
        zp, zb = np.zeros(1, position.dtype), np.ones(1, box_arr.dtype)
        wmode = _CODES[(zp % zb[0]).dtype]
        dmode = _CODES[(zp / zb[0]).dtype]
        box = np.ascontiguousarray(box_arr.astype(np.float64))
        n = position.shape[0]
        cell = np.empty(n, dtype=np.int64)
        idx = np.empty((n, dim), dtype=np.int64) if want_idx else None
        lib().oracle_bin_ext(_ptr(position), _EXT[position.dtype], wmode, dmode, n,
                             position.strides[0] // position.itemsize, dim, _ptr(box), _ptr(topo),
                             int(bool(periodic)), _ptr(cell), _ptr(idx))
        return (cell, idx) if want_idx else cell
    is_f32 = position.dtype == np.float32
    assert is_f32 or position.dtype == np.float64
    if compute_f32 is None:
        compute_f32 = is_f32 and np.result_type(position.dtype, box_arr.dtype) == np.float32
    box = np.ascontiguousarray(box_arr.astype(np.float64))
    n = position.shape[0]
    row_stride = position.strides[0] // position.itemsize
    cell = np.empty(n, dtype=np.int64)
    idx = np.empty((n, dim), dtype=np.int64) if want_idx else None
    lib().oracle_bin(_ptr(position), int(is_f32), int(bool(compute_f32)), n, row_stride, dim,
                     _ptr(box), _ptr(topo), int(bool(periodic)), _ptr(cell), _ptr(idx))
    return (cell, idx) if want_idx else cell


def partition(data, dest, nbins):
    """Stable partition of rows of ``data`` by ``dest`` (int64); returns (out, offsets)."""
    data = np.ascontiguousarray(data)
    dest = np.ascontiguousarray(np.asarray(dest, dtype=np.int64))
    n = data.shape[0]
    row_bytes = data.itemsize * (int(np.prod(data.shape[1:])) if data.ndim > 1 else 1)
    out = np.empty_like(data)
    offsets = np.zeros(nbins + 1, dtype=np.int64)
    total = lib().oracle_partition(_ptr(data), n, row_bytes, _ptr(dest), nbins, _ptr(out),
                                   _ptr(offsets))
    return out[:total], offsets


def local_partition_workspace(n, nbins, threads):
    """Scratch of local_partition_omp (destinations, per-thread bin starts),
    allocated and touched once, outside any timed call."""
    ws = (np.zeros(max(int(n), 1), dtype=np.int32), np.zeros(int(threads) * int(nbins), np.int64))
    return ws


def local_partition_omp(position, data, grid_topology, box_length, periodic=True, threads=1,
                        out=None, workspace=None):
    """Threaded host restatement of the local stage (wrap + bin of f64
    positions in place, stable partition of ``data`` rows): the optimised
    CPU comparison point of bench.py.  ``workspace``: local_partition_workspace
    (else allocated inside the call).  Returns (out, offsets)."""
    assert position.dtype == np.float64 and position.strides[1] == 8
    topo = np.ascontiguousarray(np.asarray(grid_topology).astype(np.int64))
    box = np.ascontiguousarray(np.asarray(box_length, dtype=np.float64))
    data = np.ascontiguousarray(data)
    n = position.shape[0]
    row_bytes = data.itemsize * (int(np.prod(data.shape[1:])) if data.ndim > 1 else 1)
    if out is None:
        out = np.empty_like(data)
    offsets = np.zeros(int(np.prod(topo)) + 1, dtype=np.int64)
    lib().oracle_local_partition_omp(_ptr(position), n, position.strides[0] // 8, len(topo),
                                     _ptr(box), _ptr(topo), int(bool(periodic)), _ptr(data),
                                     row_bytes, _ptr(out), _ptr(offsets), int(threads),
                                     _ptr(workspace[0]) if workspace else None,
                                     _ptr(workspace[1]) if workspace else None)
    return out, offsets


def synth_uniform(seed, gid0, n, dim=3, box=1.0):
    box = np.ascontiguousarray(np.broadcast_to(np.asarray(box, dtype=np.float64), (dim,)))
    pos = np.empty((n, dim), dtype=np.float64)
    ids = np.empty(n, dtype=np.int64)
    lib().oracle_synth_uniform(seed, gid0, n, dim, _ptr(box), _ptr(pos), _ptr(ids))
    return pos, ids


def fnv1a(arr):
    arr = np.ascontiguousarray(arr)
    return int(lib().oracle_fnv1a(_ptr(arr), arr.nbytes))
