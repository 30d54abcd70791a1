"""Multi-process CPU baseline: the reference algorithm run as P ranks.

TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's ``cpu_baseline`` leg).  The
reference runs under ``mpirun -n P`` with mpi4py; neither exists on the GPU
box, so each rank here is a spawned process running the NumPy restatement of
``redistribute_by_position`` (redist.py:157-199, oracle/redist_oracle.py):
in-place wrap + bin, one mask pass per destination, a pickled all-to-all
(mpi4py lowercase ``alltoall`` semantics: list by destination in, list by
source out) over pipes, and the concatenate.  Rank r holds the global ids
[r*n, (r+1)*n) of the SURVEY §8d generator, as the GPU bench does.
"""
from __future__ import annotations

import multiprocessing as mp
import threading
import time

import numpy as np


def _rank_main(rank, size, n, iters, conns, box, topo, seed, barrier, out_q):
    from oracle import redist_oracle as ro

    pos = ro.synth_uniform(seed, rank * n, n, 3, box[0])
    rec = np.zeros(n, dtype=[("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])
    rec["x"], rec["y"], rec["z"] = pos.T
    rec["id"] = np.arange(rank * n, (rank + 1) * n)
    geo = ro.Geometry(topo, box, size, rank)

    def alltoall(parts):
        got = [None] * size
        got[rank] = parts[rank]

        def sender():
            for k in range(1, size):
                conns[(rank + k) % size].send(parts[(rank + k) % size])

        t = threading.Thread(target=sender)
        t.start()
        for k in range(1, size):
            src = (rank - k) % size
            got[src] = conns[src].recv()
        t.join()
        return got

    times = []
    for _ in range(iters):
        barrier.wait()
        t0 = time.perf_counter()
        cell = ro.cell_number_from_position(geo, pos)               # redist.py:157
        parts = ro.stable_split(rec, cell, size)                    # :195-198
        out = np.concatenate(alltoall(parts))                       # :199
        barrier.wait()
        times.append(time.perf_counter() - t0)
        del out
    out_q.put((rank, times))


def run(size=8, n_per_rank=1 << 21, iters=3, topo=(2, 2, 2), box=(1.0, 1.0, 1.0),
        seed=20261015):
    """-> dict(value particles/s, cores, per-iteration seconds)."""
    ctx = mp.get_context("spawn")
    pipes = {}
    for a in range(size):
        for b in range(a + 1, size):
            pipes[(a, b)], pipes[(b, a)] = ctx.Pipe(duplex=True)
    barrier = ctx.Barrier(size)
    q = ctx.Queue()
    procs = []
    for r in range(size):
        conns = {p: pipes[(r, p)] for p in range(size) if p != r}
        procs.append(ctx.Process(target=_rank_main, args=(r, size, n_per_rank, iters, conns,
                                                           list(box), list(topo), seed, barrier,
                                                           q)))
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(size)]
    for p in procs:
        p.join(timeout=60)
    per_iter = np.max(np.array([t for _, t in sorted(res)]), axis=0)  # slowest rank
    med = float(np.median(per_iter))
    return {"value": size * n_per_rank / med, "seconds": per_iter.tolist(), "ranks": size,
            "n_per_rank": n_per_rank, "stat": "median",
            "spread": [size * n_per_rank / float(per_iter.max()),
                       size * n_per_rank / float(per_iter.min())]}
