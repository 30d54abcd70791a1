#!/usr/bin/env python3
"""Run tools/align_probe.hip: a 2 GiB streaming copy with its 16-byte stores (or
loads) 0/4/8/12 bytes past a 16-byte boundary; prints GB/s (read + write).
Build first (on the CPU side): hipcc --offload-arch=gfx950 -O3 -shared -fPIC
-o tools/_align_probe.so tools/align_probe.hip"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "_align_probe.so"))
lib.mis_copy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                         ctypes.c_int, ctypes.c_void_p]
nbytes = int(os.environ.get("PROBE_BYTES", 2 << 30))
n16 = nbytes // 16
x = torch.randint(0, 255, (nbytes + 16,), dtype=torch.uint8, device="cuda")
y = torch.zeros_like(x)
s = torch.cuda.current_stream().cuda_stream
res = {}
for rep in range(2):
    for mis_load in (0, 1):
        for off in (0, 4, 8, 12):
            for _ in range(3):
                assert lib.mis_copy(mis_load, x.data_ptr(), y.data_ptr(), n16, off, s) == 0
            torch.cuda.synchronize()
            if rep == 0:   # the copy is right: the bytes moved by off
                if mis_load:
                    assert torch.equal(y[:4096], x[off:off + 4096])
                else:
                    assert torch.equal(y[off:off + 4096], x[:4096])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                lib.mis_copy(mis_load, x.data_ptr(), y.data_ptr(), n16, off, s)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / 10
            key = f"{'load' if mis_load else 'store'}_off{off}"
            res.setdefault(key, []).append(round(2 * nbytes / (ms / 1e3) / 1e9, 1))
print(json.dumps(res))
