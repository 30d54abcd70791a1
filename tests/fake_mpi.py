"""Threaded in-process stand-in for an mpi4py communicator (test infrastructure).

``alltoall`` follows mpi4py's lowercase semantics (redist.py:199): each rank
passes a list indexed by destination and gets back a list indexed by source.
Ranks are threads; a shared barrier separates deposit and collection.
"""
from __future__ import annotations

import threading

import numpy as np


class FakeWorld:
    def __init__(self, size):
        self.size = size
        self.barrier = threading.Barrier(size)
        self.slots = [None] * size


class FakeComm:
    def __init__(self, world, rank):
        self.world, self.rank = world, rank

    def Get_rank(self):
        return self.rank

    def Get_size(self):
        return self.world.size

    def alltoall(self, sendobj):
        w = self.world
        assert len(sendobj) == w.size
        w.slots[self.rank] = [np.array(x, copy=True) for x in sendobj]  # pickle == copy
        w.barrier.wait()
        out = [w.slots[s][self.rank] for s in range(w.size)]
        w.barrier.wait()
        return out


def run_ranks(size, fn):
    """Run fn(comm, rank) on ``size`` threads; re-raise the first failure."""
    world = FakeWorld(size)
    results = [None] * size
    errors = []

    def body(r):
        try:
            results[r] = fn(FakeComm(world, r), r)
        except BaseException as e:  # pragma: no cover
            errors.append((r, e))
            world.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(size)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0][1]
    return results
