"""mpi_grid_redistribute_amd -- MI355X-native particle -> Cartesian grid of
ranks redistribution (drop-in for dkorytov/mpi_grid_redistribute redist.py).

    from mpi_grid_redistribute_amd import MPIGridRedistributor, RcclComm
    comm = RcclComm.from_torch_distributed()          # one process per GPU
    R = MPIGridRedistributor(comm, [2, 2, 2], [1.0, 1.0, 1.0])
    local = R.redistribute_by_position(data, position)   # position wrapped in place

Compute: hand-written gfx950 HIP kernels in libmgr.so (C ABI include/mgr.h);
exchange: native RCCL grouped send/recv.  No CPU fallback.
"""
from . import _lib
from .comm import MpiHostComm, RcclComm, SelfComm, TorchDistComm, Transport
from .redistributor import GridPartitioner, MPIGridRedistributor, mpi_grid_redistribute

__all__ = ["MPIGridRedistributor", "GridPartitioner", "mpi_grid_redistribute", "RcclComm",
           "SelfComm", "MpiHostComm", "TorchDistComm", "Transport"]
__version__ = "0.1.0"


def synth_uniform(n, seed=20261015, gid0=0, dim=3, box=1.0, records=True, stream=None):
    """Device-side SURVEY §8d generator: (positions (n,dim) f64, 32-byte
    records [x,y,z,id] as an (n,32) uint8 tensor or None) on the GPU."""
    import ctypes

    import numpy as np
    import torch

    _lib.require_gpu()
    b = np.ascontiguousarray(np.broadcast_to(np.asarray(box, dtype=np.float64), (dim,)))
    pos = torch.empty((n, dim), dtype=torch.float64, device="cuda")
    rec = torch.empty((n, 32), dtype=torch.uint8, device="cuda") if records else None
    _lib.call("mgr_synth_uniform", ctypes.c_uint64(seed), int(gid0), int(n), int(dim),
              b.ctypes.data_as(ctypes.c_void_p), _lib.ptr(pos), _lib.ptr(rec),
              _lib.stream_handle(stream))
    torch.cuda.current_stream().synchronize()
    return pos, rec


def synth_clustered(n, seed=20261015, gid0=0, box=1.0, n_halos=64, sigma=0.02, frac_bg=0.2,
                    alpha=1.0, records=True):
    """BASELINE config 4 input: 80 % of the particles in
    ``n_halos`` Gaussian halos (sigma = 0.02 L, centres uniform in the box,
    halo weights ~ Pareto(alpha)), 20 % uniform background; offsets may leave
    the box (the wrap, S1/S3).  3-D; (positions (n,3) f64, 32-byte records
    [x,y,z,id]) on the GPU.  Test/bench input only (torch RNG)."""
    import torch

    _lib.require_gpu()
    g = torch.Generator(device="cuda").manual_seed(int(seed))
    L = torch.as_tensor(box, dtype=torch.float64, device="cuda").expand(3)
    centres = torch.rand((n_halos, 3), generator=g, dtype=torch.float64, device="cuda") * L
    w = (1.0 - torch.rand(n_halos, generator=g, dtype=torch.float64, device="cuda")) ** (-1.0 / alpha)
    # the halos are global (same seed on every rank); each rank's particles
    # come from its own stream (gid0)
    g.manual_seed(int(seed) ^ (int(gid0) * 0x9E3779B97F4A7C15 & 0x7FFFFFFFFFFFFFFF))
    halo = torch.multinomial(w / w.sum(), n, replacement=True, generator=g)
    pos = centres[halo] + torch.randn((n, 3), generator=g, dtype=torch.float64,
                                      device="cuda") * (sigma * L)
    bg = torch.rand(n, generator=g, device="cuda") < frac_bg
    pos[bg] = torch.rand((int(bg.sum()), 3), generator=g, dtype=torch.float64, device="cuda") * L
    rec = None
    if records:
        rec = torch.empty((n, 4), dtype=torch.float64, device="cuda")
        rec[:, :3] = pos
        rec.view(torch.int64)[:, 3] = torch.arange(gid0, gid0 + n, device="cuda")
        rec = rec.view(torch.uint8).reshape(n, 32)
    return pos.contiguous(), rec


def synth_wide_soa(n, seed=20261015, gid0=0, box=1.0, lo=0.0, hi=None):
    """BASELINE config 5 input as a SoA payload: the fields of synth_wide's
    records (same values) as four GPU arrays -- positions (n, 3) float32,
    velocities (n, 3) float32, masses (n,) float32, ids (n,) int64.  The
    positions array is both a payload field and the ``position`` argument.
    Test/bench input only."""
    import torch

    rec, pos = synth_wide(n, seed=seed, gid0=gid0, box=box, lo=lo, hi=hi)
    f = rec.view(torch.float32)
    out = (pos.contiguous(), f[:, 3:6].contiguous(), f[:, 6].contiguous(),
           rec[:, 28:36].contiguous().view(torch.int64).reshape(-1))
    del rec, f, pos
    return out


def synth_wide(n, seed=20261015, gid0=0, box=1.0, lo=0.0, hi=None):
    """BASELINE config 5 input: 36-byte records [pos f32 x3, vel f32 x3, mass
    f32, id i64] as an (n, 36) uint8 GPU tensor, positions uniform in
    [lo, hi)^3 (default the whole box), plus the (n, 3) float32 position view
    into the records (row stride 9 elements) that redistribute_by_position /
    fine_cell_sort take.  Test/bench input only (torch RNG)."""
    import torch

    _lib.require_gpu()
    hi = box if hi is None else hi
    g = torch.Generator(device="cuda").manual_seed(int(seed) ^ (int(gid0) * 0x9E3779B97F4A7C15
                                                               & 0x7FFFFFFFFFFFFFFF))
    rec = torch.empty((n, 36), dtype=torch.uint8, device="cuda")
    f = rec.view(torch.float32)                       # (n, 9)
    f[:, :3] = (lo + torch.rand((n, 3), generator=g, dtype=torch.float64, device="cuda")
                * (hi - lo)).to(torch.float32)
    f[:, 3:6] = torch.randn((n, 3), generator=g, device="cuda")
    f[:, 6] = 1.0
    ids = torch.arange(gid0, gid0 + n, dtype=torch.int64, device="cuda")
    rec.view(torch.int32)[:, 7] = (ids & 0xFFFFFFFF).to(torch.int32)
    rec.view(torch.int32)[:, 8] = (ids >> 32).to(torch.int32)
    return rec, f[:, :3]
