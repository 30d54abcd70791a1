#!/usr/bin/env python3
"""Kernel A/B microbenchmark (GPU): per-kernel HIP-event times of the local
stage (bin_count, scan, pack) on BASELINE config 2 (KB_VARIANTS: JSON list
of {"topo", "input", "rec"} workloads and test hooks, include/mgr_instrument.h),
next to torch's device copy of the same payload as a practical HBM ceiling.
Library builds are compared by scripts/gpu_libs_ab.sh."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_grid_redistribute_amd as mgr  # noqa: E402
from mpi_grid_redistribute_amd import _lib  # noqa: E402

N = int(os.environ.get("KB_N", 1 << 26))
ITERS = int(os.environ.get("KB_ITERS", 10))


def run(variant):
    variant = dict(variant)
    topo = variant.pop("topo", None) or [2, 2, 2]
    clustered = variant.pop("input", "uniform") == "clustered"
    rb = variant.pop("rec", 32)
    for k, v in variant.items():
        _lib.test_hook(k, v)
    part = mgr.GridPartitioner(topo, [1.0] * len(topo))
    part.set_write_back("all")   # every step writes the wrapped positions back (bench.py)
    if rb == 36:   # config 5 record: f32 pos x3, vel x3, mass, i64 id; position = its view
        rec = torch.zeros((N, 36), dtype=torch.uint8, device="cuda")
        f = rec.view(torch.float32)
        f[:, :3] = torch.rand((N, 3), device="cuda")
        rec.view(torch.int32)[:, 7] = torch.arange(N, device="cuda", dtype=torch.int32)
        pos = f[:, :3]
    else:
        pos, rec = mgr.synth_clustered(N) if clustered else mgr.synth_uniform(N)
        if rb != 32:   # other payload widths: random bytes beside the (N,3) f64 positions
            rec = torch.randint(0, 256, (N, rb), dtype=torch.uint8, device="cuda")
    flat = rec.reshape(-1)
    for _ in range(3):
        part.partition_device(flat, rb, pos)
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(ITERS):
        part.partition_device(flat, rb, pos)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    # whole step (bin + scan + pack) without profiler events
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        part.partition_device(flat, rb, pos)
    b.record()
    torch.cuda.synchronize()
    out = {"step": round(a.elapsed_time(b) / ITERS, 4)}
    for k in ("bin_count", "scan", "pack"):
        ms, cnt = _lib.profile_read(k)
        out[k] = round(ms / max(cnt, 1), 4)
    out["bin_GBps"] = round(49 * N / (out["bin_count"] / 1e3) / 1e9, 1)
    out["pack_GBps"] = round((2 * rb + 1) * N / (out["pack"] / 1e3) / 1e9, 1)
    for k, v in _lib.HOOK_DEFAULTS.items():
        _lib.test_hook(k, v)
    del part, pos, rec, flat
    torch.cuda.empty_cache()
    return out


def copy_ceiling():
    x = torch.empty(N * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(ITERS):
        y.copy_(x)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / ITERS
    return {"copy_ms": round(ms, 4), "copy_GBps": round(2 * N * 32 / (ms / 1e3) / 1e9, 1)}


if __name__ == "__main__":
    vf = os.environ.get("KB_VARIANTS_FILE")
    variants = json.load(open(vf)) if vf else json.loads(os.environ.get("KB_VARIANTS", "[{}]"))
    repeat = int(os.environ.get("KB_REPEAT", 1))
    print(json.dumps({"n": N, **copy_ceiling()}), flush=True)
    results = {}
    for _ in range(repeat):          # interleaved A/B: box drift hits every variant alike
        for v in variants:
            r = run(v)
            results.setdefault(json.dumps(v, sort_keys=True), []).append(r)
            print(json.dumps({"variant": v, **r}), flush=True)
    if repeat > 1:
        for key, rs in results.items():
            med = {k: sorted(r[k] for r in rs)[len(rs) // 2] for k in rs[0]}
            print(json.dumps({"median_of": len(rs), "variant": json.loads(key), **med}), flush=True)
