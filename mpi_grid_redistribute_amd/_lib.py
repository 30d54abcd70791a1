"""ctypes binding of libmgr.so (C ABI: include/mgr.h; measurement and test
hooks: include/mgr_instrument.h).

The HIP library is the only compute path: if it is missing or cannot be
loaded, every entry point raises -- there is no CPU or eager fallback.
``torch`` is imported first on purpose: torch ships its own libamdhip64 /
librccl, and loading it first makes libmgr.so bind to the same HIP runtime
and RCCL instance (same SONAMEs) instead of a second copy.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmgr.so")

MGR_OK = 0
MGR_F32, MGR_F64, MGR_I32, MGR_I64 = 1, 2, 3, 4
MGR_F16, MGR_I8, MGR_I16, MGR_U8, MGR_U16, MGR_U32, MGR_U64, MGR_B8 = 5, 6, 7, 8, 9, 10, 11, 12
# element bytes of the position dtypes (mgr_bin_count & co.)
POS_ITEMSIZE = {MGR_F16: 2, MGR_F32: 4, MGR_F64: 8, MGR_I8: 1, MGR_I16: 2, MGR_I32: 4,
                MGR_I64: 8, MGR_U8: 1, MGR_U16: 2, MGR_U32: 4, MGR_U64: 8, MGR_B8: 1}
UNIQUE_ID_BYTES = 128

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_PI64 = ctypes.POINTER(ctypes.c_int64)

# name: (restype, argtypes) -- mirrors include/mgr.h one for one.
SIGNATURES = {
    "mgr_last_error": (ctypes.c_char_p, []),
    "mgr_version": (ctypes.c_char_p, []),
    "mgr_plan_create": (_I, [_I, _P, _P, _I, _I, ctypes.POINTER(_P)]),
    "mgr_plan_create_fine": (_I, [_I, _P, _P, _P, _I, ctypes.POINTER(_P)]),
    "mgr_plan_destroy": (_I, [_P]),
    "mgr_plan_set_write_back": (_I, [_P, _I]),
    "mgr_tile_rows": (_I, [_I64, _I]),
    "mgr_ranked_tile_rows": (_I, [_I64, _I]),
    "mgr_workspace_bytes": (_I64, [_I64, _I, _I]),
    "mgr_dest_bytes": (_I, [_I]),
    "mgr_bin_count": (_I, [_P, _P, _I, _I64, _I64, _I, _P, _I, _P, _P]),
    "mgr_bin_count_fine": (_I, [_P, _P, _P, _I, _I64, _I64, _I, _P, _P, _I, _P, _P]),
    "mgr_count_ids": (_I, [_P, _I64, _I, _I, _P, _P, _P, _P]),
    "mgr_rank_ids": (_I, [_P, _I64, _I, _I, _P, _P, _P, _P, _P]),
    "mgr_pack_ranked": (_I, [_P, _I64, _I64, _P, _P, _P, _I, _I, _P, _P, _P]),
    "mgr_cell_ids": (_I, [_P, _P, _I, _I64, _I64, _I, _P, _P, _P]),
    "mgr_bin_ids": (_I, [_P, _P, _I, _I64, _P, _I, _P, _P]),
    "mgr_cell_number_from_indexes": (_I, [_P, _P, _I64, _I, _P, _P]),
    "mgr_scan": (_I, [_I64, _I, _I, _P, _P, _P]),
    "mgr_pack": (_I, [_P, _I64, _I64, _P, _I, _I, _I, _P, _P, _I, _P, _P]),
    "mgr_pack_ids": (_I, [_P, _I64, _I64, _P, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P, _P]),
    "mgr_pack_tiles": (_I, [_P, _I64, _I64, _P, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P, _I64, _I64,
                            _P]),
    "mgr_pack_fields": (_I, [_I, _P, _P, _I64, _P, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P, _I64,
                             _I64, _P]),
    "mgr_tile_offsets": (_I, [_P, _I64, _I, _I, _P, _I, _P, _P]),
    "mgr_partition_by_position": (_I, [_P, _P, _I, _I64, _I64, _I, _P, _I64, _P, _P, _P, _I,
                                       _P, _P]),
    "mgr_bin_starts": (_I, [_I64, _I, _I, _P, ctypes.POINTER(_P)]),
    "mgr_onepass_workspace_bytes": (_I64, [_I64, _I]),
    "mgr_partition_onepass": (_I, [_P, _P, _P, _I64, _I64, _I, _I64, _I, _P, _P, _I64, _P, _P, _P]),
    "mgr_halo_flags": (_I, [_P, _I, _I64, _I64, _I, _P, _P, _P, _P]),
    "mgr_bin_count_halo": (_I, [_P, _P, _I, _I64, _I64, _I, _P, _P, _P, _P, _I, _P, _P]),
    "mgr_msel_count": (_I, [_P, _I64, _I, _P, _I, _P, _P]),
    "mgr_msel_pack": (_I, [_P, _I64, _I64, _P, _I, _P, _I, _P, _P, _P]),
    "mgr_msel_pack_fields": (_I, [_I, _P, _P, _I64, _P, _I, _P, _I, _P, _P, _P]),
    "mgr_msel_pack_placed": (_I, [_I, _P, _P, _I64, _P, _I, _P, _I, _P, _P, _I64, _P]),
    "mgr_group_p2p": (_I, [_P, _I, _P, _P, _P, _P, _P]),
    "mgr_comm_unique_id": (_I, [_P]),
    "mgr_comm_create": (_I, [_P, _I, _I, ctypes.POINTER(_P)]),
    "mgr_comm_destroy": (_I, [_P]),
    "mgr_comm_rank": (_I, [_P]),
    "mgr_comm_size": (_I, [_P]),
    "mgr_comm_count": (_I, [_P]),
    "mgr_rccl_version": (_I, [ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "mgr_exchange_counts": (_I, [_P, _P, _P, _P]),
    "mgr_exchange_count_rows": (_I, [_P, _P, _P, _I, _P]),
    "mgr_exchange_rows": (_I, [_P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "mgr_exchange_schedule": (_I, [_I, _I, _I, _P, _P, _P, _P, _P, _I, _P, _I]),
    "mgr_comm_allreduce_max_f64": (_I, [_P, _P, _P, _I64, _P]),
    "mgr_synth_uniform": (_I, [ctypes.c_uint64, _I64, _I64, _I, _P, _P, _P, _P]),
}
# include/mgr_instrument.h: measurement and test hooks (not the boundary).
INSTRUMENT_SIGNATURES = {
    "mgr_test_hook": (_I, [ctypes.c_char_p, _I64]),
    "mgr_test_pos_modes": (_I, [_I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "mgr_profile_enable": (_I, [_I]),
    "mgr_profile_reset": (_I, []),
    "mgr_profile_select": (_I, [_I64]),
    "mgr_profile_read": (_I, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), _PI64]),
    "mgr_profile_kernel_id": (_I, [ctypes.c_char_p]),
}
MGR_WRITE_BACK_CHANGED, MGR_WRITE_BACK_ALL = 0, 1


class MgrError(RuntimeError):
    """A libmgr.so call returned a negative status."""


MGR_XOP_SEND, MGR_XOP_RECV, MGR_XOP_COPY = 0, 1, 2


class XOp(ctypes.Structure):
    """mgr_xop: one operation of a row exchange (include/mgr.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32), ("field", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("src_offset", ctypes.c_int64),
                ("dst_offset", ctypes.c_int64), ("bytes", ctypes.c_int64)]


def exchange_schedule(rank, size, row_bytes, send_counts, send_offsets, recv_counts,
                      recv_offsets, skip_self=True):
    """The RCCL operation list mgr_exchange_rows issues (host only, no GPU):
    [(kind, peer, field, src_offset, dst_offset, bytes), ...] in issue order."""
    nf = len(row_bytes)
    arr = lambda a, k: (ctypes.c_int64 * k)(*[int(x) for x in a])  # noqa: E731
    args = (int(rank), int(size), nf, arr(row_bytes, nf), arr(send_counts, size),
            arr(send_offsets, size), arr(recv_counts, size), arr(recv_offsets, size),
            int(bool(skip_self)))
    n = load().mgr_exchange_schedule(*args, None, 0)
    check(min(n, 0), "mgr_exchange_schedule")
    ops = (XOp * max(n, 1))()
    check(min(load().mgr_exchange_schedule(*args, ops, n), 0), "mgr_exchange_schedule")
    return [(o.kind, o.peer, o.field, o.src_offset, o.dst_offset, o.bytes) for o in ops[:n]]


_lib = None


def load():
    """Load libmgr.so (raises if it was not built -- run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libmgr.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in {**SIGNATURES, **INSTRUMENT_SIGNATURES}.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc, what=""):
    if rc != MGR_OK:
        msg = load().mgr_last_error().decode(errors="replace")
        raise MgrError(f"{what} failed ({rc}): {msg}")
    return rc


def call(name, *args):
    return check(getattr(load(), name)(*args), name)


def rccl_version():
    """(compiled, runtime) RCCL version codes (mgr_rccl_version)."""
    c, r = ctypes.c_int(0), ctypes.c_int(0)
    call("mgr_rccl_version", ctypes.byref(c), ctypes.byref(r))
    return c.value, r.value


def require_gpu():
    """The product path runs on the MI355X only; refuse loudly otherwise."""
    if not torch.cuda.is_available():
        raise RuntimeError("mpi_grid_redistribute_amd needs a ROCm GPU (MI355X, gfx950); "
                           "there is no CPU fallback")
    load()


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    """Device address of a torch tensor (None -> NULL)."""
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


def test_hook(key, value):
    """mgr_test_hook: make a fallback path run for the parity tests
    (include/mgr_instrument.h; results are unchanged, defaults are shipped)."""
    call("mgr_test_hook", key.encode(), int(value))


HOOK_DEFAULTS = {"tile_rounds": 0, "scan_chunk": 2048, "scan_max_chunks": 1024,
                 "scan_spins": 1 << 24, "pack_img_all": 0, "rank_rows": 0, "bin_unstaged": 0,
                 "bin_generic": 0, "pack_generic": 0, "scan_delay_bin": -1,
                 "scan_delay_sleeps": 0, "scan_end_spins": -1, "scan_poison_chunk": -1,
                 "fields_kernel": 0}


# --------------------------------------------------------------- profiler
# Profiler kernel names (mgr_internal.h KernelId).
PROFILE_KERNELS = ("bin_count", "scan", "pack", "cell_ids", "bin_ids", "cellnum_idx", "synth",
                   "exchange", "halo", "bin_fine", "count_ids", "pack_fine", "pack_narrow",
                   "halo_pack", "onepass")


_prof_on = False
_alg = {}


def profile_enable(on=True):
    global _prof_on
    call("mgr_profile_enable", int(bool(on)))
    _prof_on = bool(on)


def alg_add(kernel, nbytes):
    """Algorithmic bytes of a launch whose size only the host code knows
    (the halo's selections: rows scanned and rows copied), summed per
    profiler kernel name while profiling is enabled."""
    if _prof_on:
        _alg[kernel] = _alg.get(kernel, 0) + int(nbytes)


def alg_read(kernel):
    return _alg.get(kernel, 0)


def profile_select(kernels=None):
    """Time only these kernels (None: all).  Every timed launch adds two HIP
    event records to its stream, so a benchmark times just what it reports."""
    if kernels is None:
        call("mgr_profile_select", -1)
        return
    mask = 0
    for k in kernels:
        kid = load().mgr_profile_kernel_id(k.encode())
        if kid < 0:
            check(kid, "mgr_profile_kernel_id")
        mask |= 1 << kid
    call("mgr_profile_select", mask)


def profile_reset():
    call("mgr_profile_reset")
    _alg.clear()


def profile_read(kernel):
    ms = ctypes.c_double(0.0)
    cnt = ctypes.c_int64(0)
    call("mgr_profile_read", kernel.encode(), ctypes.byref(ms), ctypes.byref(cnt))
    return ms.value, cnt.value
