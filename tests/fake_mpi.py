"""Threaded in-process stand-in for an mpi4py communicator (test infrastructure).

``alltoall`` follows mpi4py's lowercase semantics (redist.py:199): each rank
passes a list indexed by destination and gets back a list indexed by source.
Ranks are threads; a shared barrier separates deposit and collection.
``isend``/``irecv`` (the halo exchange, redist.py:289-303) are per
(source, destination, tag) FIFO queues: messages between one pair with one
tag are received in the order they were sent (MPI non-overtaking); a send
completes at once (eager, like mpi4py's pickled small messages).
"""
from __future__ import annotations

import queue
import threading

import numpy as np


class FakeWorld:
    def __init__(self, size):
        self.size = size
        self.barrier = threading.Barrier(size)
        self.slots = [None] * size
        self.lock = threading.Lock()
        self.queues = {}

    def q(self, src, dst, tag):
        with self.lock:
            return self.queues.setdefault((src, dst, tag), queue.Queue())


class _Req:
    def __init__(self, fn):
        self.fn = fn

    def wait(self):
        return self.fn()


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

    def isend(self, obj, dest, tag=0):
        self.world.q(self.rank, int(dest), tag).put(np.array(obj, copy=True))  # pickle == copy
        return _Req(lambda: None)

    def irecv(self, buf=None, source=0, tag=0):
        q = self.world.q(int(source), self.rank, tag)
        return _Req(lambda: q.get(timeout=120))


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
