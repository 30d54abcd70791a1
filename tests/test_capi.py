"""CPU checks of the C ABI: libmgr.so loads and exports every symbol that
include/mgr.h declares; host-only entry points behave (no compute calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mgr.h")
INSTRUMENT = os.path.join(ROOT, "include", "mgr_instrument.h")


def header_functions(path=HEADER):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mgr_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from mpi_grid_redistribute_amd import _lib
    return _lib.load()


def test_header_declares_api():
    fns = header_functions()
    assert "mgr_bin_count" in fns and "mgr_pack" in fns and "mgr_exchange_rows" in fns
    assert len(fns) >= 25


def test_every_declared_symbol_exported(lib):
    from mpi_grid_redistribute_amd import _lib
    for name in header_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(header_functions())
    # the instrumentation header: exported, bound, and not in the boundary
    inst = header_functions(INSTRUMENT)
    for name in inst:
        assert hasattr(lib, name), name
    assert set(_lib.INSTRUMENT_SIGNATURES) == set(inst)
    assert not set(inst) & set(header_functions())


def test_test_hooks_validate(lib):
    from mpi_grid_redistribute_amd import _lib
    with pytest.raises(_lib.MgrError):
        _lib.test_hook("no_such_hook", 1)
    with pytest.raises(_lib.MgrError):
        _lib.test_hook("rank_rows", 1000)              # only 0 / 2048 / 4096
    for k, v in _lib.HOOK_DEFAULTS.items():            # every hook takes its default
        _lib.test_hook(k, v)
    assert not hasattr(lib, "mgr_tune")                # no process-wide product knobs


def test_plan_write_back_option(lib):
    import numpy as np
    topo = np.array([2, 2, 2], dtype=np.int64)
    box = np.array([1.0, 1.0, 1.0])
    h = ctypes.c_void_p()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert lib.mgr_plan_create(3, vp(topo), vp(box), 2, 8, ctypes.byref(h)) == 0
    assert lib.mgr_plan_set_write_back(h, 1) == 0 and lib.mgr_plan_set_write_back(h, 0) == 0
    assert lib.mgr_plan_set_write_back(h, 2) < 0
    assert lib.mgr_plan_set_write_back(None, 1) < 0
    assert lib.mgr_plan_destroy(h) == 0


def test_library_is_gfx950():
    so = os.path.join(ROOT, "mpi_grid_redistribute_amd", "libmgr.so")
    blob = open(so, "rb").read()
    assert b"gfx950" in blob


def test_host_only_entry_points(lib):
    assert lib.mgr_version().startswith(b"mgr ")
    assert lib.mgr_dest_bytes(8) == 1 and lib.mgr_dest_bytes(300) == 2
    tr = lib.mgr_tile_rows(32, 8)
    assert tr % 64 == 0 and 64 <= tr <= 4096
    assert lib.mgr_workspace_bytes(1 << 20, 8, tr) > 0
    assert lib.mgr_workspace_bytes(-1, 8, tr) < 0


def test_plan_validation(lib):
    import numpy as np
    topo = np.array([2, 2, 2], dtype=np.int64)
    box = np.array([1.0, 1.0, 1.0])
    h = ctypes.c_void_p()
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert lib.mgr_plan_create(3, vp(topo), vp(box), 2, 8, ctypes.byref(h)) == 0
    assert lib.mgr_plan_destroy(h) == 0
    # topology needs 8 ranks, only 7 (redist.py:43-44)
    rc = lib.mgr_plan_create(3, vp(topo), vp(box), 2, 7, ctypes.byref(h))
    assert rc < 0 and b"ranks" in lib.mgr_last_error()
    rc = lib.mgr_plan_create(0, vp(topo), vp(box), 2, 8, ctypes.byref(h))
    assert rc < 0


def test_profiler_names(lib):
    from mpi_grid_redistribute_amd import _lib
    _lib.profile_reset()
    for k in _lib.PROFILE_KERNELS:   # every id the library names, in enum order
        ms, cnt = _lib.profile_read(k)
        assert cnt == 0 and ms == 0.0
    _lib.profile_select(["bin_count", "pack"])
    _lib.profile_select(None)
    with pytest.raises(_lib.MgrError):
        _lib.profile_read("nope")


def test_product_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import mpi_grid_redistribute_amd as m
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.MPIGridRedistributor(None, [2], [1.0])
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.GridPartitioner([2], [1.0])


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No libmgr.so: the package raises at its first native call, naming the
    build step -- nothing falls back to a host path."""
    from mpi_grid_redistribute_amd import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libmgr.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load()


def test_msel_validation(lib):
    """mgr_msel_count / mgr_msel_pack argument checks run on the host before
    any launch."""
    buf = ctypes.create_string_buffer(64)
    p = ctypes.cast(buf, ctypes.c_void_p)
    bits = (ctypes.c_int * 2)(1, 2)                                    # flag masks
    bad = (ctypes.c_int * 2)(1, 1 << 16)
    assert lib.mgr_msel_count(p, 5, 0, bits, 4096, p, None) < 0        # no sets
    assert b"nsets" in lib.mgr_last_error()
    assert lib.mgr_msel_count(p, 5, 33, bits, 4096, p, None) < 0       # > 32 sets
    assert lib.mgr_msel_count(p, 5, 2, bad, 4096, p, None) < 0         # mask beyond 16 bits
    assert b"flag mask" in lib.mgr_last_error()
    zero = (ctypes.c_int * 2)(0, 1)
    assert lib.mgr_msel_count(p, 5, 2, zero, 4096, p, None) < 0        # empty mask
    assert lib.mgr_msel_count(p, 5, 2, bits, 100, p, None) < 0         # tile not a multiple of 64
    assert lib.mgr_msel_pack(p, 0, 5, p, 2, bits, 4096, p, p, None) < 0  # row_bytes < 1
    assert b"row_bytes" in lib.mgr_last_error()
    assert lib.mgr_msel_pack(None, 8, 5, p, 2, bits, 4096, p, p, None) < 0  # null source
    assert b"null" in lib.mgr_last_error()
    assert lib.mgr_msel_pack(None, 8, 0, None, 2, bits, 4096, None, None, None) == 0  # empty


def test_rank_ids_contract(lib):
    """mgr_rank_ids takes the ranked tiles only (mgr_ranked_tile_rows: 2048 or
    4096 rows, <= 2048 ids): other shapes are refused before any launch."""
    buf = ctypes.create_string_buffer(256)
    p = ctypes.cast(buf, ctypes.c_void_p)
    for tr in (256, 512, 1024, 3072):
        assert lib.mgr_rank_ids(p, 5, 512, tr, p, p, None, p, None) == -1, tr
        assert b"tile_rows" in lib.mgr_last_error()
    assert lib.mgr_rank_ids(p, 5, 2049, 4096, p, p, None, p, None) == -1
    assert b"nbins" in lib.mgr_last_error()
    assert lib.mgr_rank_ids(p, 0, 512, 4096, p, p, None, p, None) == 0   # empty: no launch


def test_position_and_box_dtypes(lib):
    """Every dtype code makes a plan and takes positions (every float,
    integer and bool dtype); unknown codes are refused; an integer box must
    hold integers below 2^53."""
    import numpy as np
    from mpi_grid_redistribute_amd import _lib
    topo = np.array([2], dtype=np.int64)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    h = ctypes.c_void_p()
    for code in range(1, 13):
        assert lib.mgr_plan_create(1, vp(topo), vp(np.array([4.0])), code, 2, ctypes.byref(h)) == 0
        buf = ctypes.create_string_buffer(64)
        p = ctypes.cast(buf, ctypes.c_void_p)
        for pc in (0, 13, -1):
            assert lib.mgr_bin_count(h, p, pc, 4, 1, 1, p, 64, p, None) == -1
            assert b"positions must be" in lib.mgr_last_error()
        for pc in range(1, 13):   # n = 0: validated, nothing launched
            assert lib.mgr_bin_count(h, p, pc, 0, 1, 1, p, 64, p, None) == 0
        assert lib.mgr_plan_destroy(h) == 0
    assert lib.mgr_plan_create(1, vp(topo), vp(np.array([4.0])), 13, 2, ctypes.byref(h)) < 0
    assert lib.mgr_plan_create(1, vp(topo), vp(np.array([2.5])), _lib.MGR_I64, 2,
                               ctypes.byref(h)) < 0
    assert b"integer box_length" in lib.mgr_last_error()


def test_box_dtype_codes():
    import numpy as np
    from mpi_grid_redistribute_amd import _lib
    from mpi_grid_redistribute_amd._arrays import box_dtype_code, pos_code
    exp = {np.float16: _lib.MGR_F16, np.float32: _lib.MGR_F32, np.float64: _lib.MGR_F64,
           np.int8: _lib.MGR_I8, np.int16: _lib.MGR_I16, np.int32: _lib.MGR_I32,
           np.int64: _lib.MGR_I64, np.uint8: _lib.MGR_U8, np.bool_: _lib.MGR_B8,
           np.uint16: _lib.MGR_U16, np.uint32: _lib.MGR_U32, np.uint64: _lib.MGR_U64}
    for dt, code in exp.items():
        assert box_dtype_code(np.ones(3, dt)) == code, dt
    assert box_dtype_code(np.array([1, 2])) == _lib.MGR_I64          # python ints (S11a)
    with pytest.raises(TypeError):
        box_dtype_code(np.ones(2, np.complex128))
    with pytest.raises(NotImplementedError):
        box_dtype_code(np.array([2 ** 60]))
    for dt in (np.float16, np.float32, np.float64, np.int8, np.int16, np.int32, np.int64,
               np.uint8, np.uint16, np.uint32, np.uint64, np.bool_):
        assert _lib.POS_ITEMSIZE[pos_code(dt)] == np.dtype(dt).itemsize
    for dt in (np.longdouble, np.complex64, np.complex128, object):
        with pytest.raises(TypeError):
            pos_code(dt)
    with pytest.raises(TypeError):
        box_dtype_code(np.ones(2, np.longdouble))


def test_promotion_table_matches_numpy(lib):
    """Every (position, box) dtype pair: the library's wrap type (numpy's
    position % box) and quotient type (position / box) equal numpy 2.2's own
    -- the promotion the reference's redist.py:68-69 arithmetic gets, with
    the box a strongly typed numpy scalar (S11).  Host only."""
    import ctypes
    import numpy as np
    from mpi_grid_redistribute_amd._arrays import pos_code
    dts = [np.float16, np.float32, np.float64, np.int8, np.int16, np.int32, np.int64,
           np.uint8, np.uint16, np.uint32, np.uint64, np.bool_]
    w, q = ctypes.c_int(), ctypes.c_int()
    for p in dts:
        for b in dts:
            zp, zb = np.zeros(1, p), np.ones(1, b)
            with np.errstate(all="ignore"):
                ew, eq = (zp % zb[0]).dtype, (zp / zb[0]).dtype
            assert lib.mgr_test_pos_modes(pos_code(p), pos_code(b), ctypes.byref(w),
                                          ctypes.byref(q)) == 0
            assert (w.value, q.value) == (pos_code(ew), pos_code(eq)), (p, b, ew, eq)
    assert lib.mgr_test_pos_modes(0, 2, ctypes.byref(w), ctypes.byref(q)) != 0
    assert lib.mgr_test_pos_modes(2, 13, ctypes.byref(w), ctypes.byref(q)) != 0
