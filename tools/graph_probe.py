"""Builder's probe: the config-2 step (GridPartitioner.partition_device:
bin + scan + pack) launched eagerly vs replayed from a captured HIP graph
(one step per graph, and ten steps per graph), same buffers, interleaved
repeats; checks the replayed output equals the eager one.  Prints JSON."""
import json
import time

import torch

import mpi_grid_redistribute_amd as mgr


def timeit(f, k):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3


def main():
    n = 1 << 26
    part = mgr.GridPartitioner([2, 2, 2], [1.0, 1.0, 1.0])
    part.set_write_back("all")
    pos, rec = mgr.synth_uniform(n, seed=20261015, gid0=0)
    flat = rec.reshape(-1)
    step = lambda: part.partition_device(flat, 32, pos)  # noqa: E731
    for _ in range(10):
        step()
    ref_out, ref_counts = [t.clone() for t in step()]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        out1, counts1 = step()
    g10 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g10):
        for _ in range(10):
            out10, counts10 = step()
    g1.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(out1, ref_out) and torch.equal(counts1, ref_counts))
    res = {"eager": [], "graph1": [], "graph10": []}
    for _ in range(3):
        res["eager"].append(timeit(step, 50))
        res["graph1"].append(timeit(g1.replay, 50))
        res["graph10"].append(timeit(g10.replay, 5) / 10)
    print(json.dumps({"ms_per_step": res, "replay_equals_eager": same}))


if __name__ == "__main__":
    main()
