#!/usr/bin/env python3
"""Benchmark: particles redistributed/sec (whole node), HBM / xGMI roofline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--soa]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...,
         or bare `python bench.py --gpus N`: with no WORLD_SIZE in the
         environment the script starts its N rank processes itself (children,
         127.0.0.1 rendezvous), relays rank 0's line and exits non-zero if a
         rank fails or the run exceeds --launch-timeout.

One step = one pass of the hot path over one batch of synthetic particles
already resident in HBM (SURVEY §8d generator, generated on the device):
  N = 1  BASELINE config 2: 64M (2^26) uniform particles, 2x2x2 virtual
         subdomains, local bin + scan + stable pack (no exchange);
         positions (N,3) f64 wrapped in place, payload 32-byte records
         [x, y, z f64, id i64].
  N > 1  BASELINE config 3 per GPU: 1B/8 = 125M particles per GPU (weak
         scaling), one GPU per grid cell (2x1x1, 2x2x1, 2x2x2), the full
         MPIGridRedistributor.redistribute_by_position: bin, scan, RCCL count
         all-to-all, pack, RCCL grouped send/recv over xGMI.

Rank 0 prints ONE JSON line.  ``roofline`` is the dominant kernel's
algorithmic bytes per launch over its average launch
time, measured with HIP events on its own stream during the timed steps;
``cpu_baseline`` times the NumPy restatement of the reference algorithm
(oracle/, the checker) on a bounded sample on this host's cores (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
# xGMI: 7 links per GPU at ~153.6 GB/s per link counting both directions
# (AMD's per-link figure; 7 x 153.6 = the quoted 1075 GB/s aggregate), i.e.
# 76.8 GB/s per link and direction.  A rank's exchange with k peers of a
# fully connected 8-GPU node uses k direct links, so its per-direction peak
# is k x 76.8 GB/s.  tools/p2p_probe.py measures the per-link rate.
XGMI_LINK_GBS_PER_DIR = 153.6 / 2
SEED = 20261015
N_CFG2 = 1 << 26                 # config 2: 64M on one GPU
N_CFG3_PER_GPU = 1_000_000_000 // 8  # config 3: 1B over 8 GPUs
N_CFG5_PER_GPU = 512_000_000 // 8    # config 5: 512M over 8 GPUs

# Algorithmic bytes per row of one launch (DESIGN.md §4 Measurement): what
# the kernel must read and write at least, per row it processes.
def row_bytes_per_kernel(cfg, halo, fine_tile_rows=2048, fine_bins=512, world=1, soa=False,
                         onepass=False):
    if cfg == 5 and onepass:
        ts = 2.0 * fine_bins / fine_tile_rows
        return {
            # one read of the 36-B records (their f32 positions in-box: no
            # write-back), the record into its bin's region, its fine id beside
            "onepass": 36 + 36 + 2,
            "count_ids": 2 + 2 + ts,
            "pack_fine": 2 + 2 + ts + 36 + 36,
        }
    if cfg == 5 and soa:
        # four arrays: pos f32 x3 (also the binned positions), vel f32 x3,
        # mass f32, id i64 -- 36 bytes a row in 12 + 12 + 4 + 8
        ts = 2.0 * fine_bins / fine_tile_rows
        return {
            "bin_fine": 12 + 1 + 2,          # read the (n,3) f32 positions, dest, fine id
            "pack": 1 + 36 + 2 + 36 + 2,     # dest, every field + fine id in, out
            "count_ids": 2 + 2 + ts,         # mgr_rank_ids
            # mgr_pack_ranked once per field: ids, ranks, starts + the field
            "pack_fine": 4 * (2 + 2 + ts) + 36 + 36,
        }
    if soa:   # configs 2 / 4 as two arrays: pos f64 x3 (binned, wrapped) + id i64
        return {
            "bin_count": 24 + 24 + 1,
            "pack": 1 + 24 + 8 + 24 + 8,
        }
    if cfg == 5:
        ts = 2.0 * fine_bins / fine_tile_rows        # u16 tile starts per row
        return {
            "bin_fine": 36 + 1 + 2,          # read the 36-B record (staged slab), dest, fine id
            "pack": 1 + 36 + 2 + 36 + 2,     # dest, record + fine id in, record + fine id out
            "count_ids": 2 + 2 + ts,         # mgr_rank_ids: ids in, ranks + tile starts out
            "pack_fine": 2 + 2 + ts + 36 + 36,   # mgr_pack_ranked: ids, ranks, starts, record
        }
    if halo:
        # one rank keeps its rows in order: the selections read the binning's
        # flags in place, no flag field travels with the pack
        fl = 2 + 2 if world > 1 else 0
        return {
            "bin_count": 24 + 24 + 1 + 2,    # positions in + wrapped out, dest, face flags
            "pack": 1 + 32 + 32 + fl,        # dest, record in + out (+ flags in + out)
        }
    return {
        "bin_count": 24 + 24 + 1,            # read pos, write wrapped pos, write dest
        "pack": 1 + 32 + 32,                 # read dest, read record, write record
    }


def xgmi_report(traffic, exch, dist, world, chunks):
    """Per-direction xGMI figures of one step: this rank's bytes sent to and
    received from other ranks (MPIGridRedistributor.last_traffic: the
    exchange's real layout, every field and side field, the halo's messages)
    over the time its RCCL groups took per step (HIP events around them, summed
    over the step's groups); each direction against k x 76.8 GB/s for the k
    peers it talks to.  The max over ranks of every figure is reported (the
    slowest rank bounds the step)."""
    per_step = exch["avg_ms"] * exch["launches"] / max(exch.get("steps", 1), 1)
    send, recv = traffic["send_bytes"], traffic["recv_bytes"]
    speers, rpeers = traffic["send_peers"], traffic["recv_peers"]
    vals = [float(send), float(recv), float(per_step), float(speers), float(rpeers)]
    if dist is not None and world > 1:
        t = torch.tensor(vals, dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = t.tolist()
    send, recv, ms, speers, rpeers = vals
    out = {"unit": "GB/s", "ms_per_step": ms, "link_peak_per_direction": XGMI_LINK_GBS_PER_DIR,
           "bytes_from": "exchange layout (MPIGridRedistributor.last_traffic), max over ranks",
           # which exchange the figures come from: the pipelined one (k chunk
           # messages per peer, exchange.exchange_pipelined) or one message
           "path": (f"pipelined, {chunks} chunks per peer (exchange_pipelined)" if chunks > 1
                    else "one message per peer (exchange)")}
    for name, b, k in (("send", send, speers), ("recv", recv, rpeers)):
        peak = k * XGMI_LINK_GBS_PER_DIR
        ach = b / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        out[name] = {"bytes": int(b), "peers": int(k), "achieved": ach, "peak": peak,
                     "frac": ach / peak if peak > 0 else None}
    fr = [out[d]["frac"] for d in ("send", "recv") if out[d]["frac"] is not None]
    out["frac"] = max(fr) if fr else None
    return out


RCCL_LOG_PREFIX = "/tmp/mgr_bench_rccl"


def rccl_log_env(environ):
    """N > 1: RCCL's connection lines ("Channel 00/0 : 0[0] -> 1[1] via
    P2P/IPC") to a per-process file, so the record can name the transport
    RCCL chose (init-time logging only).  A caller already logging at INFO or
    TRACE keeps its own destination (transports then unread); a lower level
    (VERSION, WARN -- some images preset one) is raised to INFO into the file."""
    if environ.get("NCCL_DEBUG", "").strip().upper() in ("INFO", "TRACE"):
        return None
    path = f"{RCCL_LOG_PREFIX}.{os.getpid()}.log"
    environ["NCCL_DEBUG"] = "INFO"
    environ["NCCL_DEBUG_SUBSYS"] = "INIT,P2P,SHM,NET"
    environ["NCCL_DEBUG_FILE"] = path
    return path


def rccl_transports(text):
    """Transports named by RCCL's connection lines: 'P2P/IPC', 'SHM/direct',
    'NET/Socket', ... (the first two fields after 'via')."""
    import re
    out = set()
    for m in re.finditer(r" via ([A-Za-z0-9_]+)(/[A-Za-z0-9_]+)?", text):
        out.add(m.group(1) + (m.group(2) or ""))
    return sorted(out)


def rccl_block(info, transports, world):
    """The scaling record's RCCL facts: versions (built against / loaded),
    the library path, ranks as RCCL counts them (must equal the world size)
    and the transports its connections use (P2P/IPC = xGMI on one node).
    A failed query is reported, not raised: the record still prints."""
    if "error" in info:
        return {"error": info["error"], "transports": transports}
    return {"version_compiled": info["version_compiled"],
            "version_runtime": info["version_runtime"], "library": info["library"],
            "nranks": info["nranks"], "nranks_ok": info["nranks"] == world,
            "transports": transports}


def exchange_ab_block(pipelined_ms, chunks, one_message_ms, steps):
    """The pipelined exchange (the product default at > 1 rank, chunks per
    peer) against one message per peer, same inputs, same ranks: the second
    timed in an untimed pass after the region."""
    return {"pipelined_ms_per_step": pipelined_ms, "chunks": chunks,
            "one_message_ms_per_step": one_message_ms, "one_message_steps": steps,
            "pipelined_speedup": (one_message_ms / pipelined_ms) if pipelined_ms > 0 else None,
            "in_timed_region": False}


def _m(n):
    """Workload size label: 2^26 -> 64M, 125_000_000 -> 125M."""
    return f"{n >> 20}M" if n % (1 << 20) == 0 else f"{n / 1e6:g}M"


def topology_for(n):
    dims = [1, 1, 1]
    k = 0
    while int(np.prod(dims)) < n:
        dims[k % 3] *= 2
        k += 1
    assert int(np.prod(dims)) == n, f"--gpus {n} must be a power of two"
    return dims


def cpu_baseline(n_per_rank=1 << 22):
    """The reference algorithm on this host's cores (oracle/, the checker): the
    NumPy restatement of redistribute_by_position (redist.py:157-199: in-place
    wrap + bin, one mask pass per destination, pickled all-to-all,
    concatenate) run as 8 spawned rank processes on a 2x2x2 grid -- the
    `mpirun -n 8` shape of BASELINE config 1 (mpi4py/mpirun are absent on the
    box; pipes carry the pickled all-to-all).  Bounded sample: 8 x 4M
    particles, the median of 5 iterations (slowest rank each) with the spread
    -- ~20 s of CPU work over the 8 cores."""
    from oracle import mp_baseline

    avail = len(os.sched_getaffinity(0))
    ranks = 8 if avail >= 8 else max(1, avail)
    topo = {8: (2, 2, 2), 4: (2, 2, 1), 2: (2, 1, 1)}.get(ranks, (1, 1, 1))
    n = int(n_per_rank)
    t0 = time.perf_counter()
    r = mp_baseline.run(size=int(np.prod(topo)), n_per_rank=n, iters=5, topo=topo)
    el = time.perf_counter() - t0
    return {"value": r["value"], "unit": "particles/s", "cores": r["ranks"], "kind": "port",
            "stat": "median", "spread": r["spread"],
            "sample": f"{r['ranks']} rank processes x {n} uniform particles, grid {list(topo)}, "
                      f"f64 (N,3) positions + 32-byte records, numpy {np.__version__} "
                      f"restatement of redist.py:157-199 with a pickled all-to-all over pipes "
                      f"(mpirun/mpi4py absent), median of 5 iterations "
                      f"{[round(x, 3) for x in r['seconds']]} s, {el:.1f} s wall"}


def cpu_baseline_cfg1():
    """BASELINE config 1's own shape on the oracle: 8 rank processes x 125k
    uniform particles (1M total) on a 2x2x2 grid, median of 7 iterations."""
    from oracle import mp_baseline

    avail = len(os.sched_getaffinity(0))
    if avail < 8:
        return None
    n = 125_000
    r = mp_baseline.run(size=8, n_per_rank=n, iters=7, topo=(2, 2, 2))
    return {"value": r["value"], "unit": "particles/s", "cores": r["ranks"], "kind": "port",
            "stat": "median", "spread": r["spread"],
            "sample": f"BASELINE config 1: 8 rank processes x {n} uniform particles (1M), grid "
                      f"[2, 2, 2], numpy restatement of redist.py:157-199, pickled all-to-all "
                      f"over pipes, median of 7 {[round(x, 4) for x in r['seconds']]} s"}


def cpu_baseline_c(iters=7):
    """Optimised host comparison point (oracle/, the checker): the threaded C
    restatement of the local stage (wrap + bin + stable partition, exactly the
    GPU step's work at N=1) on this host's cores, 16M particles of the same
    layout.  Output and scratch are allocated and touched by an untimed first
    call, then warm-up calls run until two agree; the timed calls allocate
    nothing.  The median of ``iters`` with the spread (min..max rate): single
    iterations on a shared host vary."""
    from oracle import c_oracle

    # 8 threads: the same core count as the 8-rank port baselines
    threads = min(8, len(os.sched_getaffinity(0)))
    n = 1 << 24
    pos, ids = c_oracle.synth_uniform(SEED, 0, n, 3, 1.0)
    rec = np.empty((n, 4), dtype=np.float64)
    rec[:, :3] = pos
    rec.view(np.int64)[:, 3] = ids
    out = np.empty_like(rec)
    ws = c_oracle.local_partition_workspace(n, 8, threads)
    # untimed: the first call touches out and scratch; the host's first few
    # passes over fresh arrays run up to 3x slower (pages still settling on
    # the threads' nodes), so warm up until two calls agree within 15 %
    prev = None
    for _ in range(8):
        t0 = time.perf_counter()
        c_oracle.local_partition_omp(pos, rec, [2, 2, 2], [1.0, 1.0, 1.0], threads=threads,
                                     out=out, workspace=ws)
        t = time.perf_counter() - t0
        if prev is not None and abs(t - prev) < 0.15 * min(t, prev):
            break
        prev = t
    secs = []
    for _ in range(iters):
        t0 = time.perf_counter()
        c_oracle.local_partition_omp(pos, rec, [2, 2, 2], [1.0, 1.0, 1.0], threads=threads,
                                     out=out, workspace=ws)
        secs.append(time.perf_counter() - t0)
    med = float(np.median(secs))
    return {"value": n / med, "unit": "particles/s", "cores": threads, "kind": "port",
            "stat": "median", "spread": [n / max(secs), n / min(secs)],
            "sample": f"{n} uniform particles, f64 (N,3) positions + 32-byte records, 2x2x2, "
                      f"threaded C restatement (oracle/mgr_oracle.c oracle_local_partition_omp) "
                      f"of the local stage, median of {iters} after untimed warm-up calls "
                      f"{[round(x, 3) for x in secs]} s"}


def load_traffic(kernel, workload):
    """HBM bytes/launch from a committed rocprofv3 PMC pass (profiles/traffic.json)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(p) as f:
            t = json.load(f)
        e = t.get(workload, {}).get(kernel)
        return None if e is None else float(e["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        return None


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(nranks, argv, timeout_s, script=None, python=None, grace_s=20.0, out=None):
    """The bare `python bench.py --gpus N` form: start N rank processes of
    ``script`` (this file) as children -- never exec -- with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, each in
    its own process group; relay rank 0's stdout (its JSON line) to ``out``;
    wait at most ``timeout_s`` for all of them.  A rank that fails gets its
    peers (likely stuck in a collective) killed after ``grace_s``; a timeout
    kills every group.  Returns 0 only if every rank exited 0 and rank 0
    printed a JSON line; else the first failing rank's code (124: timeout,
    3: no line)."""
    script = script or os.path.abspath(__file__)
    python = python or sys.executable
    out = out or sys.stdout
    port = _free_port()
    procs, lines = [], []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks),
                   LOCAL_WORLD_SIZE=str(nranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([python, script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else None,
                                      start_new_session=True, text=True))

    def relay():
        for line in procs[0].stdout:
            lines.append(line)
            out.write(line)
            out.flush()

    th = threading.Thread(target=relay, daemon=True)
    th.start()

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        for p in procs:
            p.wait()

    t_end = time.monotonic() + timeout_s
    first_fail, fail_at = None, None
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            break
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad and first_fail is None:
            first_fail, fail_at = bad[0], time.monotonic()
            print(f"bench launcher: rank {bad[0][0]} exited {bad[0][1]}", file=sys.stderr)
        now = time.monotonic()
        if now > t_end or (fail_at is not None and now - fail_at > grace_s):
            if now > t_end:
                print(f"bench launcher: timeout after {timeout_s:.0f} s, killing the ranks",
                      file=sys.stderr)
                first_fail = first_fail or (-1, 124)
            kill_all()
            break
        time.sleep(0.2)
    th.join(timeout=5)
    if first_fail is not None:
        return int(first_fail[1]) if first_fail[1] > 0 else 1
    codes = [p.returncode for p in procs]
    if any(c != 0 for c in codes):
        return next(c for c in codes if c != 0) or 1
    if not any(ln.lstrip().startswith("{") for ln in lines):
        print("bench launcher: rank 0 printed no JSON line", file=sys.stderr)
        return 3
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--particles", "--n", dest="n", type=int, default=0,
                    help="particles per GPU (default: config size)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prof", choices=("report", "all", "none"), default="report",
                    help="kernels timed with HIP events inside the timed region: report = "
                         "pack (+ exchange) only, all, none")
    ap.add_argument("--config", type=int, choices=(2, 3, 4, 5), default=0,
                    help="BASELINE config (default: 2 at one GPU, 3 for N > 1); 4 = clustered, "
                         "5 = 36-byte records + 8x8x8 fine-cell sort")
    ap.add_argument("--overload", type=float, default=0.0,
                    help="N > 1 / --exchange: overload (halo) length per dimension in box units; "
                         "the step then includes the halo exchange (redist.py:161-166)")
    ap.add_argument("--exchange", action="store_true",
                    help="run the N>1 path (config 3, RCCL exchange) even at one GPU")
    ap.add_argument("--chunks", type=int, default=0,
                    help="N > 1: pack the tiles in this many chunks, each chunk's rows sent "
                         "while the next is packed (exchange_pipelined); 0 = the product default "
                         "(redistributor.exchange_chunks_for)")
    ap.add_argument("--soa", action="store_true",
                    help="SoA payload: the fields as separate arrays moved by one multi-field "
                         "pack (config 5: pos f32 x3, vel f32 x3, mass f32, id i64; configs "
                         "2-4: pos f64 x3 + id i64); the position array is field 0")
    ap.add_argument("--classic", action="store_true",
                    help="config 5 at one GPU: the source partition by bin + scan + pack (the "
                         "records read twice) instead of the one-pass kernel")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="bare --gpus N > 1 (no WORLD_SIZE): seconds before the rank "
                         "processes are killed")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # bare multi-GPU launch: start the ranks as children before anything
        # touches the GPU (no exec from this process)
        return launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout)

    import mpi_grid_redistribute_amd as mgr
    from mpi_grid_redistribute_amd import _lib
    from mpi_grid_redistribute_amd.exchange import count_skew

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    # CPU baseline first: its rank processes are spawned before this process
    # touches the GPU
    cpu = cpu_baseline() if (world == 1 and not args.no_cpu_baseline) else None
    cpu_1 = cpu_baseline_cfg1() if (world == 1 and not args.no_cpu_baseline) else None
    cpu_c = cpu_baseline_c() if (world == 1 and not args.no_cpu_baseline) else None
    if os.environ.get("MGR_BENCH_SHARED_GPU") == "1":
        # rehearsal of the N>1 path on a 1-GPU box: every rank on GPU 0, each
        # its own RCCL "host" (socket transport) -- numbers are not xGMI ones
        os.environ["NCCL_HOSTID"] = f"mgr-bench-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        local = 0
    torch.cuda.set_device(local)
    dist = None
    multi = world > 1 or args.exchange
    rccl_log = rccl_log_env(os.environ) if world > 1 else None
    if multi:
        import torch.distributed as dist
        if world == 1:   # --exchange without a launcher: a one-rank group
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517"), ("RANK", "0"),
                         ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    cfg = args.config or (3 if multi else 2)
    onepass = cfg == 5 and not multi and not args.soa and not args.classic
    chunks = args.chunks or None      # None: the product's own choice
    if multi and cfg == 2:
        cfg = 3
    topo = topology_for(world) if multi else [2, 2, 2]
    rb, pos_desc = 32, "(N,3) float64, wrapped in place"
    if not multi:
        n = args.n or N_CFG2
        part = mgr.GridPartitioner([2, 2, 2], [1.0, 1.0, 1.0])
        if cfg == 5 and args.soa:
            # config 5 with the record's fields as four arrays (SoA): one fine
            # binning of the (n,3) f32 positions, ONE multi-field pack of the
            # four arrays + fine ids; at the destination the fine sort of every
            # field by the received ids
            workload = f"cfg5_{_m(n)}_soa_pos_vel_mass_id_2x2x2_local_partition_plus_fine_sort_888"
            rb, pos_desc = 36, "f32 (N,3) array, also payload field 0, wrapped in place"
            src = mgr.synth_wide_soa(n, seed=SEED, gid0=0)
            rcv = mgr.synth_wide_soa(n, seed=SEED + 1, gid0=0, hi=0.5)
            R1 = mgr.MPIGridRedistributor(None, [1, 1, 1], [0.5, 0.5, 0.5])
            flats = [t.reshape(-1).view(torch.uint8) for t in src]
            rbs = [12, 12, 4, 8]
            _, recv_fids, _ = mgr.GridPartitioner([1, 1, 1], [0.5] * 3).partition_fields_device(
                [t.reshape(-1).view(torch.uint8).clone() for t in rcv], rbs, rcv[0].clone(),
                fine_cells=[8, 8, 8])
            recv_fids = recv_fids.clone()

            def step():
                part.partition_fields_device(flats, rbs, src[0], fine_cells=[8, 8, 8])
                R1.fine_cell_sort(rcv, rcv[0], [8, 8, 8], fine_ids=recv_fids)
        elif cfg == 5:
            # one GPU's share of config 5: 64M 36-byte records; the local stage
            # (bin + scan + pack into 8 destinations) and the destination-side
            # fine-cell sort (8x8x8) of 64M rows inside one cell
            workload = f"cfg5_{_m(n)}_rec36_2x2x2_local_partition_plus_fine_sort_888"
            rb, pos_desc = 36, "f32 (N,3) view into the 36-byte records, wrapped in place"
            rec, pos = mgr.synth_wide(n, seed=SEED, gid0=0)
            recv, rpos = mgr.synth_wide(n, seed=SEED + 1, gid0=0, hi=0.5)
            # rank 0's cell of the 2x2x2 grid as a one-rank system (same fine bins)
            R1 = mgr.MPIGridRedistributor(None, [1, 1, 1], [0.5, 0.5, 0.5])
            flat = rec.reshape(-1)
            # the fine cells that arrive with the received rows: computed by
            # the sources' bin kernels (the source side of this step does the
            # same for its own 64M rows), here once before the timed region
            _, recv_fids, _ = mgr.GridPartitioner([1, 1, 1], [0.5] * 3).partition_device(
                recv.reshape(-1), 36, rpos, fine_cells=[8, 8, 8])
            recv_fids = recv_fids.clone()

            if not args.classic:
                # the one-pass source partition (mgr_partition_onepass): every
                # record read once, the output the send_buff list itself
                # (redist.py:195-198: per-destination regions)
                workload = workload.replace("_local_partition", "_onepass_partition")

                last = {}

                def step():
                    last["r"] = part.partition_onepass_device(flat, 36, pos, fine_cells=[8, 8, 8])
                    R1.fine_cell_sort(recv, rpos, [8, 8, 8], fine_ids=recv_fids)

                def onepass_check():
                    # every bin fit its region (a count above cap would need the
                    # classic redo, GridPartitioner.partition_lists)
                    _, _, cnt, cap = last["r"]
                    c = cnt.cpu().numpy()
                    return {"bin_counts_max": int(c.max()), "region_rows": int(cap),
                            "fits": bool((c >= 0).all() and (c <= cap).all())}
            else:
                def step():
                    part.partition_device(flat, 36, pos, fine_cells=[8, 8, 8])
                    R1.fine_cell_sort(recv, rpos, [8, 8, 8], fine_ids=recv_fids)
        else:
            if cfg == 4:
                workload = f"cfg4_{_m(n)}_clustered_2x2x2_local_partition"
                pos, rec = mgr.synth_clustered(n, seed=SEED, gid0=0)
            else:
                workload = f"cfg2_{_m(n)}_uniform_2x2x2_local_partition"
                pos, rec = mgr.synth_uniform(n, seed=SEED, gid0=0)
            flat = rec.reshape(-1)
            if args.soa:
                # two arrays: the positions (field 0, binned and wrapped) and the ids
                workload = workload.replace("_local_partition", "_soa_pos_id_local_partition")
                pos_desc = "(N,3) float64, also payload field 0, wrapped in place"
                ids = rec.view(torch.int64)[:, 3].contiguous()
                flats = [pos.reshape(-1).view(torch.uint8), ids.view(torch.uint8)]

                def step():
                    part.partition_fields_device(flats, [24, 8], pos)
            else:
                def step():
                    part.partition_device(flat, 32, pos)
    else:
        n = args.n or (N_CFG5_PER_GPU if cfg == 5 else N_CFG3_PER_GPU)
        comm = mgr.RcclComm.from_torch_distributed()
        R = mgr.MPIGridRedistributor(comm, topo, [1.0, 1.0, 1.0])
        R.exchange_chunks = chunks
        chunks = chunks or mgr.redistributor.exchange_chunks_for(world, 36 if cfg == 5 else 32)
        if cfg == 5 and args.soa:
            workload = f"cfg5_soa_per_gpu_{_m(n)}_full_exchange_plus_fine_sort_888"
            rb, pos_desc = 36, "f32 (N,3) array, also payload field 0, wrapped in place"
            soa = mgr.synth_wide_soa(n, seed=SEED, gid0=rank * n)

            def step_with(Rx):
                Rx.redistribute_by_position(soa, soa[0], fine_cells=[8, 8, 8])
        elif cfg == 5:
            workload = f"cfg5_rec36_per_gpu_{_m(n)}_full_exchange_plus_fine_sort_888"
            rb, pos_desc = 36, "f32 (N,3) view into the 36-byte records, wrapped in place"
            rec, pos = mgr.synth_wide(n, seed=SEED, gid0=rank * n)

            def step_with(Rx):
                Rx.redistribute_by_position(rec, pos, fine_cells=[8, 8, 8])
        else:
            if cfg == 4:
                workload = f"cfg4_clustered_per_gpu_{_m(n)}_full_exchange"
                pos, rec = mgr.synth_clustered(n, seed=SEED, gid0=rank * n)
            else:
                workload = f"cfg3_uniform_per_gpu_{_m(n)}_full_exchange"
                pos, rec = mgr.synth_uniform(n, seed=SEED, gid0=rank * n)

            ol = [args.overload] * 3 if args.overload > 0 else None
            if ol:
                workload += f"_halo{args.overload:g}"
            if args.soa:
                if ol:
                    raise SystemExit("--soa with --overload: the halo takes one payload array")
                workload = workload.replace("_full_exchange", "_soa_pos_id_full_exchange")
                pos_desc = "(N,3) float64, also payload field 0, wrapped in place"
                soa = (pos, rec.view(torch.int64)[:, 3].contiguous())
                del rec

                def step_with(Rx):
                    Rx.redistribute_by_position(soa, pos)
            else:
                def step_with(Rx):
                    Rx.redistribute_by_position(rec, pos, overload_lengths=ol)

        def step():
            step_with(R)

    # Fresh f64 input needs the in-place wrap written back (redist.py:68: x + L
    # rounds, so most in-box coordinates change on the first call).  The bin
    # kernel skips slabs whose bits did not change, which after the first
    # step is every slab of these re-used inputs; that would time a
    # repeat-call steady state, so every timed f64 step writes back as on
    # fresh input (a per-plan option of this bench's own partitioner or
    # redistributor, not process state).  f32 positions (config 5) wrap in f64
    # and round back to the same f32 bits (S9: x + L is exact), so fresh f32
    # input is clean and keeps the skip.
    if cfg != 5:
        (R if multi else part).set_write_back("all")

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    _lib.profile_reset()
    # HIP events go only around the dominant kernel (pack) and the RCCL
    # exchange inside the timed region: every timed launch adds two event
    # records to the stream (measured ~2-3 us of step time per kernel).  The
    # other kernels are timed in an untimed detail pass after the region.
    timed = {"report": ["pack", "exchange", "halo", "halo_pack", "pack_fine", "onepass"],
             "all": list(_lib.PROFILE_KERNELS),
             "none": []}[args.prof]
    _lib.profile_select(timed)
    _lib.profile_enable(bool(timed))
    barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)      # device time of the same steps (information)
    _lib.profile_enable(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kernels = {}
    for k in _lib.PROFILE_KERNELS:
        ms, cnt = _lib.profile_read(k)
        if cnt:
            kernels[k] = {"avg_ms": ms / cnt, "launches": cnt, "steps": args.steps,
                          "in_timed_region": True}
            if _lib.alg_read(k):   # host-counted bytes (the halo's selections)
                kernels[k]["alg_bytes_per_launch"] = _lib.alg_read(k) / cnt
    missing = [k for k in list(row_bytes_per_kernel(cfg, bool(args.overload > 0),
                                                    soa=args.soa, onepass=onepass)) + ["scan"]
               if k not in kernels]
    if missing:
        # detail pass (not timed): the kernels left out of the timed region
        _lib.profile_reset()
        _lib.profile_select(missing)
        _lib.profile_enable(True)
        for _ in range(min(args.steps, 5)):
            step()
        barrier()
        _lib.profile_enable(False)
        for k in missing:
            ms, cnt = _lib.profile_read(k)
            if cnt:
                kernels[k] = {"avg_ms": ms / cnt, "launches": cnt, "in_timed_region": False}
    _lib.profile_select(None)
    onepass_info = onepass_check() if onepass else None
    # the count matrix's max/mean (load imbalance of the
    # redistribution: rows each destination receives, max over mean) -- the
    # N=1 line's 1 x 8 row of virtual destinations, or the N>1 ranks' count rows
    # gathered after the timed region
    skew = None
    if not multi and cfg in (2, 4):
        skew = count_skew(part.last_counts.cpu().numpy().reshape(1, -1))
    elif multi:
        sc = torch.as_tensor(R.last_counts[0], dtype=torch.int64, device="cuda")
        rows = [torch.empty_like(sc) for _ in range(world)] if world > 1 else [sc]
        if world > 1:
            dist.all_gather(rows, sc)
        skew = count_skew(torch.stack(rows).cpu().numpy())
    xgmi = None
    if multi and "exchange" in kernels:
        xgmi = xgmi_report(R.last_traffic, kernels["exchange"], dist, world, chunks)
    rccl, exchange_ab, n1_same_ms = None, None, None
    if multi and world > 1:
        # untimed: one message per peer (exchange_chunks = 1) on the same
        # inputs, beside the pipelined steps of the timed region
        R.exchange_chunks = 1
        for _ in range(2):
            step()
        barrier()
        k1 = min(args.steps, 10)
        t1 = time.perf_counter()
        for _ in range(k1):
            step()
        barrier()
        t = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        R.exchange_chunks = args.chunks or None
        exchange_ab = exchange_ab_block(elapsed / args.steps * 1e3, chunks,
                                        float(t.item()) / k1 * 1e3, k1)
        # the same workload at N = 1: this rank's own rows through a one-rank
        # redistributor (bin + scan + pack, no exchange), untimed pass, max
        # over ranks -- the same-workload base of the scaling curve (the N = 1
        # bench line itself is config 2)
        R1 = mgr.MPIGridRedistributor(None, [1, 1, 1], [1.0, 1.0, 1.0])
        if cfg != 5:
            R1.set_write_back("all")
        for _ in range(2):
            step_with(R1)
        barrier()
        t1 = time.perf_counter()
        for _ in range(k1):
            step_with(R1)
        barrier()
        t = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        n1_same_ms = float(t.item()) / k1 * 1e3
        del R1
        mine = []
        if rccl_log:
            try:
                with open(rccl_log) as f:
                    mine = rccl_transports(f.read())
                if mine:      # an unparsed log stays in /tmp for a look
                    os.remove(rccl_log)
            except OSError:
                mine = []
        try:      # local queries only: a failure must not skip the collective below
            info = comm.rccl_info()
        except Exception as e:   # noqa: BLE001 -- reported in the record
            info = {"error": repr(e)}
        every = [None] * world
        dist.all_gather_object(every, mine)
        rccl = rccl_block(info, sorted({x for e in every for x in e}), world)
    # per-kernel algorithmic bytes per launch: per-row figure x the rows one
    # launch processes -- a step's launches of these kernels together cover
    # this rank's n rows (received rows at N > 1 are ~n for the uniform
    # inputs), so a pack pipelined in k chunks covers n / k per launch -- or
    # the host-counted bytes of the halo's selections
    fine_tr = (int(_lib.load().mgr_ranked_tile_rows(12 if args.soa else 36, 512)) if cfg == 5
               else 2048)
    for k, b in row_bytes_per_kernel(cfg, bool(args.overload > 0), fine_tr, world=world,
                                     soa=args.soa, onepass=onepass).items():
        if k in kernels and "alg_bytes_per_launch" not in kernels[k]:   # host-counted first
            e = kernels[k]
            per_step = e["launches"] / e["steps"] if e.get("steps") else 1
            e["launches_per_step"] = per_step
            e["alg_bytes_per_launch"] = b * n / max(per_step, 1)
    for k, e in kernels.items():
        if "alg_bytes_per_launch" in e:
            e["alg_GBps"] = e["alg_bytes_per_launch"] / (e["avg_ms"] / 1e3) / 1e9
    roofline = None
    timed_bytes = {k: e for k, e in kernels.items() if "alg_GBps" in e and e["in_timed_region"]}
    if timed_bytes:
        # the dominant kernel: the most device time per step
        dom = max(timed_bytes, key=lambda k: timed_bytes[k]["avg_ms"] * timed_bytes[k]["launches"])
        e = kernels[dom]
        roofline = {"bound": "hbm", "kernel": dom, "achieved": e["alg_GBps"],
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": e["alg_GBps"] / HBM_PEAK_GBS,
                    "traffic": load_traffic(dom, workload),
                    "alg_bytes_per_launch": e["alg_bytes_per_launch"]}

    total = n * world * args.steps
    value = total / elapsed
    if rank == 0:
        line = {
            "metric": "particles redistributed/sec (whole node)",
            "value": value, "unit": "particles/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "gpu_ms_per_step": gpu_ms / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if cfg == 5 else "f64",
            "data": {2: "synthetic (splitmix64 uniform, generated on device)",
                     3: "synthetic (splitmix64 uniform, generated on device)",
                     4: "synthetic (64 Gaussian halos + 20 % uniform, torch RNG on device)",
                     5: "synthetic (uniform 36-byte records, torch RNG on device)"}[cfg],
            "config": {"workload": workload, "particles_per_gpu": n,
                       "grid": topo, "payload_bytes": rb, "position": pos_desc,
                       "payload_layout": ("SoA: " + ("pos f32x3, vel f32x3, mass f32, id i64"
                                                     if cfg == 5 else "pos f64x3, id i64")
                                          + " as separate arrays") if args.soa
                       else "one record array",
                       "parallelism": f"{world} rank(s), one GPU per grid cell" if multi
                       else "1 GPU, 8 virtual subdomains",
                       "exchange_chunks": chunks if multi else None},
            "roofline": roofline,
            "kernels": kernels,
            "xgmi": xgmi,
            "rccl": rccl,
            "exchange_ab": exchange_ab,
            "n1_same_workload_ms": n1_same_ms,
            "onepass": onepass_info,
            "count_skew": skew,
            "cpu_baseline": cpu,
            "cpu_baseline_cfg1": cpu_1,
            "cpu_baseline_c": cpu_c,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
