"""One rank of the multi-process RCCL parity run (tests/test_gpu_multi.py).

Runs the product transport -- RcclComm, i.e. libmgr.so's mgr_exchange_counts,
mgr_exchange_rows (grouped ncclSend/ncclRecv, receives in place at
source-ordered offsets) and mgr_group_p2p (the halo's isend/irecv batches) --
between distinct ranks, and checks every rank's result bit-exact against the
reference's own outputs (tests/golden/*.npz) and the oracle.  Replaces
``comm.alltoall`` (redist.py:199) and the isend/irecv pairs (redist.py:289-303).

Environment: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT (torch.distributed
gloo rendezvous; it only carries the RCCL unique id), MGR_TEST_OUT (result
file), MGR_TEST_SHARED_GPU=1 when the ranks share GPU 0: each rank then
presents its own NCCL_HOSTID, so RCCL treats them as separate hosts and
connects them with its socket transport over loopback (correctness of the
exchange logic, not xGMI speed); otherwise rank r uses GPU r (xGMI).
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RANK = int(os.environ["RANK"])
WORLD = int(os.environ["WORLD_SIZE"])
SHARED = os.environ.get("MGR_TEST_SHARED_GPU") == "1"
if SHARED:   # before anything loads RCCL
    os.environ["NCCL_HOSTID"] = f"mgr-test-rank-{RANK}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_DEBUG", "WARN")
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import redist_oracle as ro  # noqa: E402  (checker)
from tests import golden_io as G  # noqa: E402

TOPO = {1: [1, 1, 1], 2: [2, 1, 1], 3: [3, 1, 1], 4: [2, 2, 1], 8: [2, 2, 2]}
BOX = [1.0, 1.0, 1.0]
CASE_TIMEOUT_S = float(os.environ.get("MGR_CASE_TIMEOUT", "60"))


def log(msg):
    print(f"[rank {RANK}/{WORLD} {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def as_bytes(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().contiguous().numpy().view(np.uint8).reshape(-1)
    return np.ascontiguousarray(x).view(np.uint8).reshape(-1)


def records(n, r, rng):
    rec = np.zeros(n, dtype=[("x", "f8"), ("y", "f8"), ("z", "f8"), ("id", "i8")])
    rec["id"] = np.arange(n) + 1_000_000 * r
    return rec


def case_redist_golden(mgr, comm, name, as_torch):
    f = G.load(name)
    data, pos = G.fixture_inputs(f, name, WORLD, as_torch)
    R = mgr.MPIGridRedistributor(comm, f["topology"], f["box"])
    out = R.redistribute_by_position(data[RANK], pos[RANK], periodic=bool(f["periodic"]))
    torch.cuda.synchronize()
    assert np.array_equal(as_bytes(pos[RANK]), as_bytes(f[f"r{RANK}_pos_out"])), "positions"
    exp = f[f"r{RANK}_out"]
    if as_torch:
        assert np.array_equal(as_bytes(out), as_bytes(exp)), "output bytes"
    else:
        assert G.same_bytes(out, exp), "output"


def case_halo_golden(mgr, comm, name, as_torch):
    f = G.load(name)
    data = f[f"r{RANK}_data"].copy()
    pos = f[f"r{RANK}_pos_in"].copy()
    if as_torch:
        data = torch.from_numpy(data.view(np.uint8).reshape(len(data), -1) if data.dtype.names
                                else data).cuda()
        pos = torch.from_numpy(pos).cuda()
    R = mgr.MPIGridRedistributor(comm, f["topology"], f["box"])
    out = R.redistribute_by_position(data, pos, overload_lengths=list(f["overload"]))
    torch.cuda.synchronize()
    assert np.array_equal(as_bytes(out), as_bytes(f[f"r{RANK}_out"])), "halo output"
    assert np.array_equal(as_bytes(pos), as_bytes(f[f"r{RANK}_pos_out"])), "positions"


def case_halo_direct_golden(mgr, comm, name):
    f = G.load(name)
    R = mgr.MPIGridRedistributor(comm, f["topology"], f["box"])
    out = R.exchange_overload_by_position(f[f"r{RANK}_data"], f[f"r{RANK}_pos"],
                                          list(f["overload"]), periodic=False)
    assert G.same_bytes(out, f[f"r{RANK}_out"]), "halo (direct, non-periodic)"


def rank_inputs(seed, sizes, lo=-0.5, hi=1.5, hot=None):
    """Every rank's input (each rank builds all of them: the oracle needs all)."""
    pos, data = [], []
    for r, n in enumerate(sizes):
        rng = np.random.default_rng(seed + r)
        p = rng.uniform(lo, hi, (n, 3))
        if hot is not None and n:   # skew: most rows into one rank's cell
            k = rng.random(n) < 0.8
            p[k] = rng.uniform(0.0, 0.5, (int(k.sum()), 3)) + np.asarray(hot)
        pos.append(p)
        data.append(records(n, r, rng))
    return pos, data


def case_random(mgr, comm, sizes, seed, as_torch, hot=None, return_positions=False, chunks=1):
    topo = TOPO[WORLD]
    pos, data = rank_inputs(seed, sizes, hot=hot)
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_all_ranks(topo, BOX, WORLD, data, pos_o)[RANK]
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    R.exchange_chunks = chunks
    d, p = data[RANK], pos[RANK]
    if as_torch:
        d = torch.from_numpy(d.view(np.uint8).reshape(len(d), 32)).cuda()
        p = torch.from_numpy(p).cuda()
    out = R.redistribute_by_position(d, p, return_positions=return_positions)
    torch.cuda.synchronize()
    if return_positions:
        out, opos = out
        want = np.stack([pos_o[s][i] for s, i in
                         zip(as_bytes(out).view(exp.dtype)["id"] // 1_000_000,
                             as_bytes(out).view(exp.dtype)["id"] % 1_000_000)]) \
            if len(exp) else np.zeros((0, 3))
        assert np.array_equal(as_bytes(opos), as_bytes(want)), "returned positions"
    assert np.array_equal(as_bytes(out), as_bytes(exp)), "output"
    assert np.array_equal(as_bytes(p), as_bytes(pos_o[RANK])), "wrapped positions"
    return len(exp)


def case_fine_fused(mgr, comm, fine, seed):
    """redistribute_by_position(fine_cells=...) over RCCL: the source's fine
    ids travel as a side field, the destination sorts by them -- against the
    oracle's redistribution + fine_cell_ids + stable sort."""
    topo = TOPO[WORLD]
    sizes = [int(np.random.default_rng(seed + r).integers(5_000, 40_000)) for r in range(WORLD)]
    pos, data = rank_inputs(seed, sizes)
    pos_o = [p.copy() for p in pos]
    loc = ro.redistribute_by_position_all_ranks(topo, BOX, WORLD, data, pos_o)[RANK]
    geos = [ro.Geometry(topo, BOX, WORLD, r) for r in range(WORLD)]
    lpos = ro.redistribute_by_cell_number_all_ranks(
        WORLD, pos_o, [ro.cell_number_from_position(g, p.copy()) for g, p in zip(geos, pos_o)])[RANK]
    fid = ro.fine_cell_ids(topo, fine, BOX, lpos)
    exp, exp_off = ro.fine_cell_sort(loc, fid, int(np.prod(fine)))
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    got, gpos, off = R.redistribute_by_position(data[RANK], pos[RANK], fine_cells=fine,
                                                return_positions=True)
    torch.cuda.synchronize()
    assert np.array_equal(as_bytes(got), as_bytes(exp)), "fine-sorted output"
    assert np.array_equal(np.asarray(off), exp_off), "fine offsets"
    assert np.array_equal(as_bytes(gpos), as_bytes(lpos[np.argsort(fid, kind="stable")])), \
        "fine-sorted positions"


REC36 = np.dtype([("pos", "f4", 3), ("vel", "f4", 3), ("mass", "f4"), ("id", "i8")])


def case_soa_golden(mgr, comm, name, as_torch):
    """SoA payload (several arrays) against the reference's multi-field
    pattern (make_golden.py make_soa: one binning, every field redistributed
    with the same destinations, redist.py:157-164)."""
    f = G.load(name)
    fields, pos = G.soa_inputs(f, WORLD, as_torch)
    R = mgr.MPIGridRedistributor(comm, f["topology"], f["box"])
    out = R.redistribute_by_position(tuple(fields[RANK]), pos[RANK], periodic=bool(f["periodic"]))
    torch.cuda.synchronize()
    assert np.array_equal(as_bytes(pos[RANK]), as_bytes(f[f"r{RANK}_pos_out"])), "positions"
    for i in range(int(f["nfields"])):
        assert np.array_equal(as_bytes(out[i]), as_bytes(f[f"r{RANK}_f{i}_out"])), f"field {i}"


def soa_inputs(seed, sizes):
    """Config 5's fields as four arrays per rank: pos f32 x3 (the position
    array itself), vel f32 x3, mass f32, id i64."""
    out = []
    for r, n in enumerate(sizes):
        rng = np.random.default_rng(seed + r)
        out.append([rng.uniform(-0.5, 1.5, (n, 3)).astype(np.float32),
                    rng.normal(size=(n, 3)).astype(np.float32),
                    rng.uniform(1, 2, n).astype(np.float32),
                    np.arange(n, dtype=np.int64) + 1_000_000 * r])
    return out


def case_soa_random(mgr, comm, seed, as_torch, chunks=1, fine=None):
    """SoA redistribution over RCCL (one count exchange, one RCCL group with a
    send per field and peer; pipelined when chunks > 1), skewed sizes with an
    empty rank, optionally with fine cells -- against the oracle's per-field
    restatement of redist.py:157-164 (+ fine_cell_ids and a stable sort)."""
    topo = TOPO[WORLD]
    sizes = [int(np.random.default_rng(seed + 7 * r).integers(2_000, 50_000)) for r in range(WORLD)]
    sizes[WORLD // 2] = 0
    fields = soa_inputs(seed, sizes)
    ofields = [[x.copy() for x in fl] for fl in fields]
    exp = ro.redistribute_fields_by_position_all_ranks(topo, BOX, WORLD, ofields,
                                                       [fl[0] for fl in ofields])[RANK]
    mine = fields[RANK]
    if as_torch:
        mine = [torch.from_numpy(x).cuda() for x in mine]
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    R.exchange_chunks = chunks
    if fine is None:
        out = R.redistribute_by_position(tuple(mine), mine[0])
        torch.cuda.synchronize()
        for i in range(4):
            assert np.array_equal(as_bytes(out[i]), as_bytes(exp[i])), f"field {i}"
    else:
        out, off = R.redistribute_by_position(mine, mine[0], fine_cells=fine)
        torch.cuda.synchronize()
        fid = ro.fine_cell_ids(topo, fine, BOX, exp[0])
        order = np.argsort(fid, kind="stable")
        for i in range(4):
            assert np.array_equal(as_bytes(out[i]), as_bytes(exp[i][order])), f"fine field {i}"
        assert np.array_equal(np.diff(np.asarray(off.cpu() if hasattr(off, "cpu") else off)),
                              np.bincount(fid, minlength=int(np.prod(fine)))), "fine offsets"
    assert np.array_equal(as_bytes(mine[0]), as_bytes(ofields[RANK][0])), "wrapped positions"


def case_fine_rec36(mgr, comm, fine, seed, as_torch, chunks=1):
    """BASELINE config 5's exact layout over RCCL: 36-byte records (f32 pos +
    vel + mass + i64 id), the position the f32 view into the record (the
    image pack moves the records, the fine cell travels as a u16 side field),
    fine_cells + return_positions, skewed sizes with an empty rank -- against
    the oracle's redistribution + fine_cell_ids + stable sort."""
    topo = TOPO[WORLD]
    sizes = [int(np.random.default_rng(seed + r).integers(5_000, 60_000)) for r in range(WORLD)]
    sizes[0] = 0
    data = []
    for r, n in enumerate(sizes):
        rng = np.random.default_rng(seed + 100 + r)
        rec = np.zeros(n, dtype=REC36)
        rec["pos"] = rng.uniform(-0.5, 1.5, (n, 3)).astype(np.float32)
        rec["vel"] = rng.standard_normal((n, 3)).astype(np.float32)
        rec["mass"] = rng.random(n).astype(np.float32)
        rec["id"] = np.arange(n) + 1_000_000 * r
        data.append(rec)
    pos_o = [np.ascontiguousarray(d["pos"]) for d in data]
    data_o = [d.copy() for d in data]
    loc = ro.redistribute_by_position_all_ranks(topo, BOX, WORLD, data_o, [p.copy() for p in pos_o])
    # the position is a view into the records: the in-place wrap (S1) shows
    # in the records that travel, so the expected rows carry wrapped positions
    geos = [ro.Geometry(topo, BOX, WORLD, r) for r in range(WORLD)]
    wrapped = [p.copy() for p in pos_o]
    dests = [ro.cell_number_from_position(g, w) for g, w in zip(geos, wrapped)]
    lpos = ro.redistribute_by_cell_number_all_ranks(WORLD, wrapped, dests)[RANK]
    src = [d.copy() for d in data]
    for r in range(WORLD):
        src[r]["pos"] = wrapped[r]
    exp_rows = ro.redistribute_by_cell_number_all_ranks(WORLD, src, dests)[RANK]
    fid = ro.fine_cell_ids(topo, fine, BOX, lpos)
    exp, exp_off = ro.fine_cell_sort(exp_rows, fid, int(np.prod(fine)))
    assert len(loc[RANK]) == len(exp_rows)
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    R.exchange_chunks = chunks
    d = data[RANK]
    if as_torch:
        # (an empty rank's (0, 36) array has a zero stride: build it fresh)
        raw = torch.zeros((len(d), 36), dtype=torch.uint8, device="cuda")
        if len(d):
            raw.copy_(torch.from_numpy(d.view(np.uint8).reshape(len(d), 36).copy()))
        got, gpos, off = R.redistribute_by_position(raw, raw.view(torch.float32)[:, :3],
                                                    fine_cells=fine, return_positions=True)
        off = off.cpu().numpy()
    else:
        got, gpos, off = R.redistribute_by_position(d, d["pos"], fine_cells=fine,
                                                    return_positions=True)
    torch.cuda.synchronize()
    assert np.array_equal(as_bytes(got), as_bytes(exp)), "fine-sorted 36-byte records"
    assert np.array_equal(np.asarray(off), exp_off), "fine offsets"
    want_pos = np.ascontiguousarray(lpos[np.argsort(fid, kind="stable")])
    assert np.array_equal(as_bytes(gpos), as_bytes(want_pos)), "fine-sorted positions"


def clustered_inputs(seed, sizes, halos=64):
    """Config-4-style input: per rank, Gaussian halos (centres anywhere in the
    box, sigma 0.01-0.05, tails leaving the box -> wrapped) plus 20 % uniform
    background."""
    pos, data = [], []
    crng = np.random.default_rng(seed)
    centres = crng.random((halos, 3))
    sig = crng.uniform(0.01, 0.05, halos)
    wts = crng.pareto(1.5, halos) + 0.1
    wts /= wts.sum()
    for r, n in enumerate(sizes):
        rng = np.random.default_rng(seed + 1 + r)
        h = rng.choice(halos, n, p=wts)
        p = centres[h] + rng.standard_normal((n, 3)) * sig[h][:, None]
        bg = rng.random(n) < 0.2
        p[bg] = rng.random((int(bg.sum()), 3))
        pos.append(p)
        data.append(records(n, r, rng))
    return pos, data


def case_clustered(mgr, comm, seed, as_torch):
    """Heavily skewed counts (Gaussian halos, config 4) with an empty rank,
    over RCCL, against the oracle."""
    topo = TOPO[WORLD]
    sizes = [int(np.random.default_rng(seed + 50 + r).integers(20_000, 80_000))
             for r in range(WORLD)]
    sizes[WORLD // 2] = 0
    pos, data = clustered_inputs(seed, sizes)
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_all_ranks(topo, BOX, WORLD, data, pos_o)[RANK]
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    d, p = data[RANK], pos[RANK]
    if as_torch:
        d = torch.from_numpy(d.view(np.uint8).reshape(len(d), 32)).cuda()
        p = torch.from_numpy(p).cuda()
    out = R.redistribute_by_position(d, p)
    torch.cuda.synchronize()
    assert np.array_equal(as_bytes(out), as_bytes(exp)), "clustered output"
    assert np.array_equal(as_bytes(p), as_bytes(pos_o[RANK])), "wrapped positions"
    t = R.last_traffic   # xGMI accounting: only rows that left this rank
    sc = np.bincount(ro.cell_number_from_position(ro.Geometry(topo, BOX, WORLD, RANK),
                                                  pos[RANK].copy() if not as_torch
                                                  else p.cpu().numpy().copy()),
                     minlength=WORLD)
    # the count message: one int64 per peer, or [total, k chunk counts] when
    # the exchange is pipelined in k chunks (the product default at > 1 rank)
    from mpi_grid_redistribute_amd.redistributor import exchange_chunks_for
    k = exchange_chunks_for(WORLD, 32)
    cbytes = 8 if k == 1 else 8 * (k + 1)
    sent = sum(int(sc[q]) * 32 + cbytes for q in range(WORLD) if q != RANK)
    assert t["send_bytes"] == sent, (t["send_bytes"], sent)


def case_halo_random(mgr, comm, ol, return_positions, seed, chunks=1):
    """The halo over RCCL at larger sizes (flags from the bin kernel, the
    multi-selection packs, grouped p2p): against the oracle; with
    return_positions the positions travel as a third field."""
    topo = TOPO[WORLD]
    sizes = [int(np.random.default_rng(seed + r).integers(10_000, 40_000)) for r in range(WORLD)]
    pos, data = rank_inputs(seed, sizes)
    pos_o = [p.copy() for p in pos]
    exp = ro.redistribute_by_position_overload_all_ranks(topo, BOX, WORLD, data, pos_o, ol)[RANK]
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    R.exchange_chunks = chunks
    out = R.redistribute_by_position(data[RANK], pos[RANK], overload_lengths=ol,
                                     return_positions=return_positions)
    torch.cuda.synchronize()
    if return_positions:
        out, opos = out
        ids = as_bytes(out).view(exp.dtype)["id"]
        want = np.stack([pos_o[s][i] for s, i in zip(ids // 1_000_000, ids % 1_000_000)])
        assert np.array_equal(as_bytes(opos), as_bytes(want)), "halo positions"
    assert np.array_equal(as_bytes(out), as_bytes(exp)), "halo output"


def case_cell_number(mgr, comm):
    rng = np.random.default_rng(99)
    data = [rng.integers(0, 255, (int(rng.integers(0, 5000)), 7)).astype(np.uint8)
            for _ in range(WORLD)]
    ids = [np.random.default_rng(500 + r).integers(-2, WORLD + 2, len(d)) for r, d in
           enumerate(data)]
    exp = ro.redistribute_by_cell_number_all_ranks(WORLD, data, ids)[RANK]
    R = mgr.MPIGridRedistributor(comm, [WORLD], [1.0])
    out = R.redistribute_by_cell_number(torch.from_numpy(data[RANK]).cuda(),
                                        torch.from_numpy(ids[RANK]).cuda())
    assert np.array_equal(out.cpu().numpy(), exp), "redistribute_by_cell_number"


def case_scan_failure(mgr, comm):
    """Every rank's scan gives up at once (test hook scan_spins = -1): all ranks
    raise together at the count exchange, nobody hangs in the row exchange."""
    from mpi_grid_redistribute_amd import _lib
    topo = TOPO[WORLD]
    pos, data = rank_inputs(7, [200_000] * WORLD)
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    _lib.test_hook("scan_spins", -1)
    try:
        R.redistribute_by_position(data[RANK], pos[RANK])
    except _lib.MgrError as e:
        assert "scan failed" in str(e), str(e)
    else:
        raise AssertionError("a failed scan did not raise")
    finally:
        _lib.test_hook("scan_spins", 1 << 24)
    # the communicator still works afterwards
    assert case_random(mgr, comm, [1000] * WORLD, 8, False) >= 0


def case_full_size(mgr, comm, kind, n):
    """BASELINE configs 3 / 4 at their full per-GPU size (125M rows per rank,
    32-byte records [x, y, z, id], uniform or clustered), the product path
    (redistribute_by_position over RCCL) checked by properties, every rank's
    input regenerated from its seed (the ids encode source rank and row):
      * sources in rank order (S7), each source's run in increasing id order
        (stable);
      * per-source row counts == the C oracle's bincount of that source's
        wrapped positions, and every received row's oracle cell is this rank;
      * every received row's 32 bytes == the source record with that id;
      * this rank's positions wrapped in place exactly as the C oracle wraps."""
    from oracle import c_oracle
    topo = TOPO[WORLD]
    seed = 20261015

    def gen(r):
        if kind == "uniform":
            return mgr.synth_uniform(n, seed=seed, gid0=r * n)
        return mgr.synth_clustered(n, seed=seed, gid0=r * n)

    pos, rec = gen(RANK)
    R = mgr.MPIGridRedistributor(comm, topo, BOX)
    out = R.redistribute_by_position(rec, pos)
    torch.cuda.synchronize()
    wrapped = pos.cpu().numpy()
    del pos, rec
    ids = out.view(torch.int64)[:, 3]
    src = torch.div(ids, n, rounding_mode="floor")
    assert bool((src[1:] >= src[:-1]).all()), "sources not in rank order (S7)"
    total = 0
    for s in range(WORLD):
        ps, rs = gen(s)
        ph = ps.cpu().numpy()
        del ps
        cells = c_oracle.bin_positions(ph, topo, BOX)        # wraps ph in place
        if s == RANK:
            assert np.array_equal(wrapped.view(np.uint64), ph.view(np.uint64)), "wrapped positions"
        sel = src == s
        run = ids[sel] - s * n
        cnt = int(np.count_nonzero(cells == RANK))
        assert run.numel() == cnt, f"source {s}: {run.numel()} rows, oracle {cnt}"
        assert bool((run[1:] > run[:-1]).all()), f"source {s}: order not stable"
        run_h = run.cpu().numpy()
        assert bool((cells[run_h] == RANK).all()), f"source {s}: rows of another cell"
        assert torch.equal(out[sel], rs[run]), f"source {s}: row bytes"
        total += cnt
        del rs, run, sel, cells, ph
    assert total == out.shape[0]
    return total


def main():
    out_path = os.environ["MGR_TEST_OUT"]
    results = {}
    dev = 0 if SHARED else RANK
    torch.cuda.set_device(dev)
    log("init gloo")
    dist.init_process_group("gloo", rank=RANK, world_size=WORLD)
    import mpi_grid_redistribute_amd as mgr
    log("creating RcclComm")
    comm = mgr.RcclComm.from_torch_distributed()
    log(f"RcclComm up (device {dev}, shared={SHARED})")
    cases = []
    if os.environ.get("MGR_TEST_SET") == "fullsize":
        n = int(os.environ.get("MGR_FULL_N", 125_000_000))
        cases = [("cfg3_uniform_full", lambda: case_full_size(mgr, comm, "uniform", n)),
                 ("cfg4_clustered_full", lambda: case_full_size(mgr, comm, "clustered", n))]
    else:
        cases = _parity_cases(mgr, comm)
    return _run_cases(cases, comm, out_path, results)


def _parity_cases(mgr, comm):
    cases = []
    for name in G.redist_cases():
        if int(G.load(name)["size"]) == WORLD:
            for as_torch in (False, True):
                cases.append((f"{name}[torch={as_torch}]",
                              lambda n=name, t=as_torch: case_redist_golden(mgr, comm, n, t)))
    for name in G.soa_cases():
        if int(G.load(name)["size"]) == WORLD:
            for as_torch in (False, True):
                cases.append((f"{name}[torch={as_torch}]",
                              lambda n=name, t=as_torch: case_soa_golden(mgr, comm, n, t)))
    for name in G.halo_cases():
        if int(G.load(name)["size"]) == WORLD:
            for as_torch in (False, True):
                cases.append((f"{name}[torch={as_torch}]",
                              lambda n=name, t=as_torch: case_halo_golden(mgr, comm, n, t)))
    for name in G.halo_direct_cases():
        if int(G.load(name)["size"]) == WORLD:
            cases.append((name, lambda n=name: case_halo_direct_golden(mgr, comm, n)))
    if WORLD in TOPO:
        sizes = [int(np.random.default_rng(r).integers(1000, 30_000)) for r in range(WORLD)]
        sizes[WORLD - 1] = 0   # an empty rank (the reference raises ValueError, S5)
        cases += [
            ("random_empty_rank", lambda: case_random(mgr, comm, sizes, 11, False)),
            ("random_torch", lambda: case_random(mgr, comm, sizes[::-1], 12, True)),
            ("skewed_hot_cell", lambda: case_random(mgr, comm, [40_000] * WORLD, 13, True,
                                                    hot=[0.5, 0.0, 0.0])),
            ("return_positions", lambda: case_random(mgr, comm, sizes, 14, False,
                                                     return_positions=True)),
            ("large_300k", lambda: case_random(mgr, comm, [300_000] * WORLD, 15, True)),
            ("scan_failure", lambda: case_scan_failure(mgr, comm)),
            ("fine_fused_888", lambda: case_fine_fused(mgr, comm, [8, 8, 8], 21)),
            ("fine_fused_234", lambda: case_fine_fused(mgr, comm, [2, 3, 4], 22)),
            ("fine_rec36_888", lambda: case_fine_rec36(mgr, comm, [8, 8, 8], 31, False)),
            ("fine_rec36_888_torch", lambda: case_fine_rec36(mgr, comm, [8, 8, 8], 32, True)),
            ("fine_rec36_245", lambda: case_fine_rec36(mgr, comm, [2, 4, 5], 33, True)),
            ("pipelined_empty_rank", lambda: case_random(mgr, comm, sizes, 51, True, chunks=3)),
            ("pipelined_large", lambda: case_random(mgr, comm, [300_000] * WORLD, 52, True,
                                                    chunks=4)),
            ("pipelined_skewed", lambda: case_random(mgr, comm, [40_000] * WORLD, 53, False,
                                                     hot=[0.5, 0.0, 0.0], chunks=2)),
            ("pipelined_fine_rec36", lambda: case_fine_rec36(mgr, comm, [8, 8, 8], 54, True,
                                                             chunks=3)),
            ("pipelined_halo", lambda: case_halo_random(mgr, comm, [0.06, 0.1, 0.04], True, 55,
                                                        chunks=3)),
            ("soa_random", lambda: case_soa_random(mgr, comm, 71, False)),
            ("soa_random_torch_pipelined", lambda: case_soa_random(mgr, comm, 72, True, chunks=3)),
            ("soa_fine_888", lambda: case_soa_random(mgr, comm, 73, True, fine=[8, 8, 8])),
            ("soa_fine_888_pipelined",
             lambda: case_soa_random(mgr, comm, 74, False, chunks=4, fine=[8, 8, 8])),
            ("clustered_empty_rank", lambda: case_clustered(mgr, comm, 41, False)),
            ("clustered_torch", lambda: case_clustered(mgr, comm, 42, True)),
            ("halo_random", lambda: case_halo_random(mgr, comm, [0.06, 0.1, 0.04], False, 23)),
            ("halo_random_positions",
             lambda: case_halo_random(mgr, comm, [0.06, 0.1, 0.04], True, 24)),
        ]
    cases.append(("cell_number_dropped_ids", lambda: case_cell_number(mgr, comm)))
    return cases


def _run_cases(cases, comm, out_path, results):
    for name, fn in cases:
        t0 = time.perf_counter()
        # a rank that fails before a collective leaves its peers waiting in
        # it: every case gets a watchdog that ends this rank (results so far
        # written) instead of hanging the whole run
        def _hung(n=name):
            log(f"{n}: HUNG (> {CASE_TIMEOUT_S} s), exiting")
            results[n] = f"FAIL: hung > {CASE_TIMEOUT_S} s"
            with open(out_path, "w") as fh:
                json.dump(results, fh)
            os._exit(4)
        dog = threading.Timer(CASE_TIMEOUT_S, _hung)
        dog.daemon = True
        dog.start()
        try:
            fn()
            results[name] = "ok"
        except Exception as e:   # record and go on: every rank runs every case
            results[name] = f"FAIL: {e!r}\n{traceback.format_exc()}"
        dog.cancel()
        log(f"{name}: {results[name].splitlines()[0]} ({time.perf_counter() - t0:.2f} s)")
        # keep the ranks in step between cases (a failed case must not skew
        # the next collective's pairing)
        dist.barrier()
    comm.close()
    dist.destroy_process_group()
    with open(out_path, "w") as fh:
        json.dump(results, fh)
    return 0 if all(v == "ok" for v in results.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
