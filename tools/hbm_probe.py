#!/usr/bin/env python3
"""Run tools/hbm_probe.hip variants on 2 GiB (+2 GiB) and print GB/s (read+write)."""
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_hbm_probe.so")
if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "hbm_probe.hip")):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-o", SO, os.path.join(HERE, "hbm_probe.hip")], check=True)
lib = ctypes.CDLL(SO)
lib.probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
nbytes = int(os.environ.get("PROBE_BYTES", 2 << 30))
x = torch.ones(nbytes, dtype=torch.uint8, device="cuda")
y = torch.empty_like(x)
names = ["copy_u1", "copy_u4", "copy_u8", "copy_u1_nt", "copy_u4_nt", "copy_u8_nt", "scatter8_u4",
         "read_u1", "read_u1_nt", "read_u4", "read_u4_nt", "read_u16_nt"]
res = {}
for w, name in enumerate(names):
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert lib.probe(w, x.data_ptr(), y.data_ptr(), nbytes // 16, s) == 0
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        lib.probe(w, x.data_ptr(), y.data_ptr(), nbytes // 16, s)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    moved = nbytes if name.startswith("read") else 2 * nbytes
    res[name] = round(moved / (ms / 1e3) / 1e9, 1)
print(json.dumps(res))

# cooperative-pack structure probes: 32-byte rows, one destination
lib.coop_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_int64, ctypes.c_void_p]
nrows = nbytes // 32
dest = torch.zeros(nrows, dtype=torch.uint8, device="cuda")
res2 = {}
for mode, name in enumerate(["coop_full", "coop_nobarrier", "coop_nodest"]):
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert lib.coop_probe(mode, x.data_ptr(), y.data_ptr(), dest.data_ptr(), nrows, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(x[:4096], y[:4096]) and torch.equal(x[-4096:], y[-4096:])
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        lib.coop_probe(mode, x.data_ptr(), y.data_ptr(), dest.data_ptr(), nrows, s)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    moved = 2 * nbytes + (nrows if mode < 2 else 0)
    res2[name] = round(moved / (ms / 1e3) / 1e9, 1)
    res2[name + "_ms_per_64M_rows"] = round(ms * (1 << 26) / nrows, 4)
print(json.dumps(res2))

# copy shapes (thread count, units per lane, unit order, cache policy)
lib.shape_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                            ctypes.c_char_p, ctypes.c_void_p]
res3 = {}
for which in range(lib.shape_count()):
    nm = ctypes.create_string_buffer(64)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        assert lib.shape_probe(which, x.data_ptr(), y.data_ptr(), nbytes // 16, nm, s) == 0
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
        lib.shape_probe(which, x.data_ptr(), y.data_ptr(), nbytes // 16, nm, s)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    res3[nm.value.decode()] = round(2 * nbytes / (ms / 1e3) / 1e9, 1)
print(json.dumps(res3))
