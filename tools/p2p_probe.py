#!/usr/bin/env python3
"""xGMI point-to-point probe: the per-link, per-direction rate
that bench.py's xGMI roofline assumes (XGMI_LINK_GBS_PER_DIR).

Two ranks on two GPUs exchange buffers through the product transport
(RcclComm.p2p = one grouped ncclSend/ncclRecv, the call the halo exchange and
mgr_exchange_rows make), for message sizes 1 MiB .. 1 GiB:
  uni  rank 0 sends, rank 1 receives          (one direction of one link)
  bi   both ranks send and receive at once    (both directions)
Times are HIP events on the communicator's stream over ITERS repetitions.

  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
         tools/p2p_probe.py
Run directly on a box with fewer than two GPUs it prints a skip line and exits 0
(the 1-GPU test box has no xGMI link to measure).
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ITERS = int(os.environ.get("P2P_ITERS", 20))
SIZES = [1 << s for s in range(20, 31, 2)]   # 1 MiB .. 1 GiB


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world < 2 or torch.cuda.device_count() < 2:
        print(json.dumps({"probe": "p2p", "skipped": True,
                          "reason": f"needs 2 ranks on 2 GPUs (world {world}, "
                                    f"{torch.cuda.device_count()} GPU(s) visible)"}))
        return 0
    import torch.distributed as dist

    import mpi_grid_redistribute_amd as mgr

    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    comm = mgr.RcclComm.from_torch_distributed()
    peer = 1 - rank if rank < 2 else None
    res = []
    for size in SIZES:
        snd = torch.empty(size, dtype=torch.uint8, device="cuda").fill_(rank + 1)
        rcv = torch.empty(size, dtype=torch.uint8, device="cuda")
        for mode in ("uni", "bi"):
            if peer is None:
                ops = []
            elif mode == "uni":
                ops = [("send", peer, snd)] if rank == 0 else [("recv", peer, rcv)]
            else:
                ops = [("send", peer, snd), ("recv", peer, rcv)]
            for _ in range(3):
                comm.p2p(ops)
            torch.cuda.synchronize()
            dist.barrier()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(ITERS):
                comm.p2p(ops)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / ITERS
            t = torch.tensor([ms], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms = float(t.item())
            if mode == "bi" and peer is not None:
                assert int(rcv[0].item()) == peer + 1 and int(rcv[-1].item()) == peer + 1
            res.append({"bytes": size, "mode": mode, "ms": ms,
                        "GBps_per_direction": size / (ms / 1e3) / 1e9})
    if rank == 0:
        best = max(r["GBps_per_direction"] for r in res)
        print(json.dumps({"probe": "p2p", "ranks": world, "iters": ITERS, "results": res,
                          "best_GBps_per_direction": best}), flush=True)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
