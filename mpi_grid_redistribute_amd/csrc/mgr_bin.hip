// Binning kernels of the hot path (gfx950): wrap + write back + destination
// + tile histogram (bin_count, redist.py:63-90, :157), cell ids / indexes
// (:63-90), rank ids -> bins (redistribute_by_cell_number, :169-198), and
// cell numbers from indexes (:73-85), with their launchers.
// Semantics notes: mgr_kernels.hip header; helpers: mgr_device.h.
#include "mgr_device.h"

namespace mgr {

// Kernel 1 of the hot path: wrap + write back positions, destination of
// every row, per-tile histogram (destination-major counts[b * T + tile]).
constexpr int kStageMaxRowBytes = 64;

// Kernel 1 body.  NU > 0: staged -- the 64-row slab of position rows
// (64 * rb bytes, rb <= 64, 16-byte aligned) is read with fully coalesced
// 16-byte loads into NU registers per lane DEPTH rounds ahead (two register
// sets when DEPTH == 2), parked in wave-private LDS for the per-row math, and
// written back the same way when a row of it changed.
// NU == 0: each lane reads and writes its own row.
// One workgroup per tile: its waves split the tile's 64-row rounds into
// contiguous runs (wave w: rows [w*rows_per_wave, ...)), bin them, and add
// their wave-aggregated counts into one LDS histogram for the tile.
// SIDE: also write a u16 per row to side_out -- its fine cell (kSideFine,
// FineGeom: the destination-side fine sort of config 5 then needs no second
// binning pass) or its halo face flags (kSideHalo, HaloGeom: the overload
// exchange then needs no flag pass over the received positions).
template <typename PosT, bool kPeriodic, typename DestT, int NU, int DIM, bool NT, int DEPTH,
          int SIDE, int GEO = kGeoAny>
__global__ __launch_bounds__(1024) void bin_count_kernel(PosT* __restrict__ pos, int64_t n,
                                                           int64_t stride, Geom g,
                                                           DestT* __restrict__ dest,
                                                           int32_t* __restrict__ counts,
                                                           int64_t T, int tile_rows,
                                                           int per_wave_lds, int skip_clean,
                                                           int xcd, uint64_t* __restrict__ scan_flags,
                                                           FineGeom fg, HaloGeom hg,
                                                           uint16_t* __restrict__ side_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    clear_scan_flags(scan_flags);
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int nwaves = blockDim.x >> 6;
    const int64_t tile = xcd ? xcd_tile(blockIdx.x, T) : (int64_t)blockIdx.x;
    int32_t* hist = (int32_t*)smem;
    uint8_t* stage = smem + align16(g.nbins * 4) + w * per_wave_lds;
    const int rows_per_wave = tile_rows / nwaves;
    const int64_t tile0 = tile * (int64_t)tile_rows;
    const int64_t row0 = tile0 + (int64_t)w * rows_per_wave;
    const int rows = (int)max((int64_t)0, min((int64_t)rows_per_wave, n - row0));
    const int rb = (int)(stride * (int64_t)sizeof(PosT));
    for (int b = threadIdx.x; b < g.nbins; b += blockDim.x) hist[b] = 0;
    __syncthreads();

    // destination byte + wave-aggregated histogram add of one round.  A full
    // round of 1-byte destinations is stored as 16 dwords (lane 4k gathers
    // lanes 4k..4k+3): byte stores cost ~5x their bytes in HBM writes.
    auto account = [&](unsigned b, bool valid, int r0) {
        if (sizeof(DestT) == 1 && rows - r0 >= 64) {
            const unsigned v1 = __shfl_down(b, 1, 64), v2 = __shfl_down(b, 2, 64),
                           v3 = __shfl_down(b, 3, 64);
            if ((lane & 3) == 0)
                *(uint32_t*)(dest + row0 + r0 + lane) =
                    (b & 0xffu) | ((v1 & 0xffu) << 8) | ((v2 & 0xffu) << 16) | (v3 << 24);
        } else if (valid) {
            dest[row0 + r0 + lane] = (DestT)b;
        }
        const unsigned long long peers = match_bin(b, valid, g.nbits);
        if (valid && rank_in(peers) == 0) atomicAdd(&hist[b], __popcll(peers));
    };
    // the side u16 of one round: a full round as 16 8-byte stores (lane 4k
    // gathers lanes 4k..4k+3), like the destination bytes
    const bool side8 = ((uintptr_t)side_out & 7) == 0;
    auto side_store = [&](unsigned v, bool valid, int r0) {
        if (SIDE == kSideNone) return;
        if (side8 && rows - r0 >= 64) {
            const unsigned v1 = __shfl_down(v, 1, 64), v2 = __shfl_down(v, 2, 64),
                           v3 = __shfl_down(v, 3, 64);
            if ((lane & 3) == 0)
                *(uint2*)(side_out + row0 + r0 + lane) =
                    make_uint2((v & 0xffffu) | (v1 << 16), (v2 & 0xffffu) | (v3 << 16));
        } else if (valid) {
            side_out[row0 + r0 + lane] = (uint16_t)v;
        }
    };

    if constexpr (NU > 0) {
        // Prefetch registers: named scalars (an array here was demoted to scratch).
        const uint4 z = make_uint4(0, 0, 0, 0);
        uint4 a0 = z, a1 = z, a2 = z, a3 = z, b0 = z, b1 = z, b2 = z, b3 = z;
        uint4 c0 = z, c1 = z, c2 = z, c3 = z, e0 = z, e1 = z, e2 = z, e3 = z;
        // Every lane issues every load, without branches (index clamped into
        // the slab; a slab past the wave's rows re-reads its last one), so the
        // compiler's wait for the oldest slab is a counted vmcnt that leaves
        // the younger one in flight.  A slab's last 16-byte unit may extend
        // past its last row: an aligned 16-byte read that starts inside the
        // buffer stays inside its page, and those bytes are never stored.
        const int last = (rows - 1) & ~63;   // start of the wave's last round
        auto load = [&](uint4& x0, uint4& x1, uint4& x2, uint4& x3, int r) {
            const int rr = r < rows ? r : last;   // past the end: the slab just read (L2)
            const int cu = (min(64, rows - rr) * rb + 15) / 16;
            const uint4* gs = (const uint4*)((const uint8_t*)pos + (row0 + rr) * rb);
            if (NU > 0) x0 = ld<NT>(gs + min(lane, cu - 1));
            if (NU > 1) x1 = ld<NT>(gs + min(lane + 64, cu - 1));
            if (NU > 2) x2 = ld<NT>(gs + min(lane + 128, cu - 1));
            if (NU > 3) x3 = ld<NT>(gs + min(lane + 192, cu - 1));
        };
        auto round = [&](uint4& x0, uint4& x1, uint4& x2, uint4& x3, int r0) {
            const int nr = min(64, rows - r0);
            const bool valid = lane < nr;
            const int units = nr * rb / 16;
            const int cu = (nr * rb + 15) / 16;
            uint8_t* gslab = (uint8_t*)pos + (row0 + r0) * rb;
            uint4* sg = (uint4*)stage;
            if (NU > 0 && lane < cu) sg[lane] = x0;
            if (NU > 1 && lane + 64 < cu) sg[lane + 64] = x1;
            if (NU > 2 && lane + 128 < cu) sg[lane + 128] = x2;
            if (NU > 3 && lane + 192 < cu) sg[lane + 192] = x3;
            // DEPTH slabs in flight while this one is binned.  DEPTH 1: only
            // a real next slab (one register set: nothing to count past);
            // DEPTH 2: unconditional (see load)
            if (DEPTH > 1 || r0 + 64 < rows) load(x0, x1, x2, x3, r0 + 64 * DEPTH);
            wave_sync();
            unsigned b = 0;
            bool dirty = false;
            long long sc = 0;
            if (valid)
                b = (unsigned)bin_row<PosT, kPeriodic, DIM, SIDE, GEO>((PosT*)(stage + lane * rb), g,
                                                                  nullptr, &dirty, &fg, &hg, &sc);
            side_store((unsigned)sc, valid, r0);
            // write the slab back only if a row of it changed (skip_clean)
            if (kPeriodic && (!skip_clean || __ballot(dirty) != 0ull)) {
                wave_sync();
                uint4* gd = (uint4*)gslab;
                if (NU > 0 && lane < units) st<NT>(gd + lane, sg[lane]);
                if (NU > 1 && lane + 64 < units) st<NT>(gd + lane + 64, sg[lane + 64]);
                if (NU > 2 && lane + 128 < units) st<NT>(gd + lane + 128, sg[lane + 128]);
                if (NU > 3 && lane + 192 < units) st<NT>(gd + lane + 192, sg[lane + 192]);
                if (nr * rb > units * 16 && lane < (nr * rb - units * 16) / 4)
                    ((uint32_t*)gslab)[units * 4 + lane] = ((const uint32_t*)stage)[units * 4 + lane];
            }
            account(b, valid, r0);
            wave_sync();
        };
        if (rows <= 0) goto done;   // a trailing wave of the last tile
        load(a0, a1, a2, a3, 0);
        if (DEPTH > 1) load(b0, b1, b2, b3, 64);
        if (DEPTH > 2) load(c0, c1, c2, c3, 128);
        if (DEPTH > 3) load(e0, e1, e2, e3, 192);
        wave_sync();
        {
            // DEPTH rounds on every trip, one register set each: the
            // loop-carried wait for the oldest set is then a counted vmcnt
            // that leaves the younger sets' slabs in flight
            int r0 = 0;
            for (; r0 + 64 * (DEPTH - 1) < rows; r0 += 64 * DEPTH) {
                round(a0, a1, a2, a3, r0);
                if (DEPTH > 1) round(b0, b1, b2, b3, r0 + 64);
                if (DEPTH > 2) round(c0, c1, c2, c3, r0 + 128);
                if (DEPTH > 3) round(e0, e1, e2, e3, r0 + 192);
            }
            if (r0 < rows) round(a0, a1, a2, a3, r0);
            if (DEPTH > 2 && r0 + 64 < rows) round(b0, b1, b2, b3, r0 + 64);
            if (DEPTH > 3 && r0 + 128 < rows) round(c0, c1, c2, c3, r0 + 128);
        }
    } else {
        for (int r0 = 0; r0 < rows; r0 += 64) {
            const bool valid = r0 + lane < rows;
            unsigned b = 0;
            bool dirty = false;
            long long sc = 0;
            if (valid)
                b = (unsigned)bin_row<PosT, kPeriodic, DIM, SIDE, GEO>(pos + (row0 + r0 + lane) * stride,
                                                                  g, nullptr, &dirty, &fg, &hg, &sc);
            side_store((unsigned)sc, valid, r0);
            account(b, valid, r0);
            wave_sync();
        }
    }
done:
    __syncthreads();
    for (int b = threadIdx.x; b < g.nbins; b += blockDim.x) counts[(int64_t)b * T + tile] = hist[b];
}

// get_cell_number_from_position / get_cell_indexes_from_position (API helpers).
template <typename PosT, bool kPeriodic>
__global__ __launch_bounds__(kBlock) void cell_ids_kernel(PosT* __restrict__ pos, int64_t n,
                                                          int64_t stride, Geom g,
                                                          int64_t* __restrict__ cell,
                                                          int64_t* __restrict__ idx) {
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t r = blockIdx.x * (int64_t)kBlock + threadIdx.x; r < n; r += step) {
        long long* ip = idx ? (long long*)(idx + r * g.dim) : nullptr;
        bool dirty = false;
        const long long c = bin_row<PosT, kPeriodic>(pos + r * stride, g, ip, &dirty);
        if (cell) cell[r] = c;
    }
}

// redistribute_by_cell_number ids -> bin (out of range / non-integral -> drop bin).
template <typename IdT, typename DestT>
__global__ __launch_bounds__(kBlock) void bin_ids_kernel(const IdT* __restrict__ ids, int64_t n,
                                                         int nbins, int nbits,
                                                         DestT* __restrict__ dest,
                                                         int32_t* __restrict__ counts, int64_t T,
                                                         int tile_rows, int per_wave_lds,
                                                         uint64_t* __restrict__ scan_flags) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    clear_scan_flags(scan_flags);
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
    if (tile >= T) return;
    int32_t* hist = (int32_t*)(smem + w * per_wave_lds);
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    const int nb = nbins + 1;
    for (int b = lane; b < nb; b += 64) hist[b] = 0;
    wave_sync();
    for (int r0 = 0; r0 < rows; r0 += 64) {
        const bool valid = r0 + lane < rows;
        unsigned b = 0;
        if (valid) {
            const IdT v = ids[row0 + r0 + lane];
            bool ok;
            if constexpr (std::is_floating_point<IdT>::value) {  // numpy float == int compare
                ok = (v >= (IdT)0) && (v < (IdT)nbins) && (v == (IdT)(long long)v);
            } else {
                ok = (v >= 0) && ((long long)v < (long long)nbins);
            }
            b = ok ? (unsigned)(long long)v : (unsigned)nbins;
            dest[row0 + r0 + lane] = (DestT)b;
        }
        const unsigned long long peers = match_bin(b, valid, nbits);
        if (valid && rank_in(peers) == 0) hist[b] += __popcll(peers);
        wave_sync();
    }
    for (int b = lane; b < nb; b += 64) counts[(int64_t)b * T + tile] = hist[b];
}

__global__ __launch_bounds__(kBlock) void cellnum_from_idx_kernel(const int64_t* __restrict__ idx,
                                                                  int64_t n, Geom g, int periodic,
                                                                  int64_t* __restrict__ cell) {
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t r = blockIdx.x * (int64_t)kBlock + threadIdx.x; r < n; r += step) {
        long long c = 0;
        for (int d = 0; d < g.dim; ++d) {
            long long k = idx[r * g.dim + d];
            if (periodic) {
                const long long nn = g.n[d];
                k = floormod_i64(floormod_i64(k, nn) + nn, nn);
            }
            c += g.off[d] * k;   // non-periodic: '&' range check never fires (redist.py:80)
        }
        cell[r] = c;
    }
}

// ============================================================ launchers
// The plan's geometry class for the bin kernel (bin_row_fast's GEO): every
// dimension with the fast wrap and a power-of-two box length, 32-bit index
// math, not a fine plan -- then kGeoF32 / kGeoF64 by the quotient's type
// (f32 positions with an f32 box compute in f32, everything else in f64).
int geo_kind(const Geom& g, bool pos_f32) {
    if (g.dim != 3 || g.fine || !g.fast32) return kGeoAny;
    const bool f32c = pos_f32 && g.compute_f32;
    for (int d = 0; d < 3; ++d) {
        if (f32c && !(g.fastf[d] && g.pow2f[d])) return kGeoAny;
        if (!f32c && !(g.fast[d] && g.pow2[d])) return kGeoAny;
    }
    return f32c ? kGeoF32 : kGeoF64;
}

template <typename PosT, bool kP, typename DestT, int NU, int DIM>
static hipError_t bin_count_t(const Geom& g, void* pos, int64_t n, int64_t stride, void* dest,
                              int tile_rows, const Workspace& ws, hipStream_t s,
                              const FineGeom* fg, const HaloGeom* hg, uint16_t* side_out) {
    // nontemporal slab loads/stores always (every A/B favoured them); one
    // slab in flight per wave (two measured slower with the write-back,
    // DESIGN.md §3.3)
    // the in-box fast path with the geometry at compile time when it is
    // simple (geo_kind): staged 3-D periodic slabs, the hot configurations
    auto k = fg ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideFine>
                : hg ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideHalo>
                     : bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideNone>;
    if constexpr (DIM == 3 && kP && NU > 0) {
        const int geo = hooks().bin_generic ? kGeoAny : geo_kind(g, sizeof(PosT) == 4);
        if (geo == kGeoF32)
            k = fg ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideFine, kGeoF32>
                   : hg ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideHalo, kGeoF32>
                        : bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideNone, kGeoF32>;
        else if (geo == kGeoF64)
            k = fg ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideFine, kGeoF64>
                   : hg ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideHalo, kGeoF64>
                        : bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1, kSideNone, kGeoF64>;
    }
    FineGeom f{};
    if (fg) f = *fg;
    HaloGeom h{};
    if (hg) h = *hg;
    const int rb = (int)(stride * (int64_t)sizeof(PosT));
    const int per_wave = NU > 0 ? align16(64 * rb) : 0;     // staging slab
    // waves per workgroup, whole rounds each: 1 for f32 positions (in-box rows
    // wrap to themselves: a read-mostly pass, which streams best with more
    // rounds per wave), 2 for f64 (the write-back) -- A/B: 1/2/4/8/16 waves,
    // DESIGN.md §3.1 and §3.3
    const int want = sizeof(PosT) == 4 ? 1 : 2;
    int nwaves = tile_rows / 64;
    while (nwaves > want || (tile_rows / 64) % nwaves) --nwaves;
    const int lds = align16(g.nbins * 4) + per_wave * nwaves;
    ensure_lds(k, lds);
    hipLaunchKernelGGL(k, dim3((unsigned)ws.T), dim3(64 * nwaves), (size_t)lds, s, (PosT*)pos, n,
                       stride, g, (DestT*)dest, ws.counts, ws.T, tile_rows, per_wave,
                       !g.write_back_all, g.nbins > 64, ws.flags, f, h,
                       side_out);
    return hipGetLastError();
}

template <typename PosT, bool kP, typename DestT, int NU>
static hipError_t bin_count_dim(const Geom& g, void* pos, int64_t n, int64_t stride, void* dest,
                                int tile_rows, const Workspace& ws, hipStream_t s,
                                const FineGeom* fg, const HaloGeom* hg, uint16_t* fo) {
    switch (g.dim) {
        case 1: return bin_count_t<PosT, kP, DestT, NU, 1>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
        case 2: return bin_count_t<PosT, kP, DestT, NU, 2>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
        case 3: return bin_count_t<PosT, kP, DestT, NU, 3>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
        default: return bin_count_t<PosT, kP, DestT, NU, 0>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
    }
}

template <typename PosT, bool kP, typename DestT>
static hipError_t bin_count_w(const Geom& g, void* pos, int64_t n, int64_t stride, void* dest,
                              int tile_rows, const Workspace& ws, hipStream_t s,
                              const FineGeom* fg, const HaloGeom* hg, uint16_t* fo) {
    const int64_t rb = stride * (int64_t)sizeof(PosT);
    if (!hooks().bin_unstaged && rb <= kStageMaxRowBytes && ((uintptr_t)pos & 15) == 0) {
        switch ((int)((rb + 15) / 16)) {   // 16-byte units per lane per 64-row slab
            case 1: return bin_count_dim<PosT, kP, DestT, 1>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
            case 2: return bin_count_dim<PosT, kP, DestT, 2>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
            case 3: return bin_count_dim<PosT, kP, DestT, 3>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
            default: return bin_count_dim<PosT, kP, DestT, 4>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
        }
    }
    return bin_count_dim<PosT, kP, DestT, 0>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
}

template <typename PosT, typename DestT>
static hipError_t bin_count_p(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                              void* dest, int tile_rows, const Workspace& ws, hipStream_t s,
                              const FineGeom* fg, const HaloGeom* hg, uint16_t* fo) {
    return periodic ? bin_count_w<PosT, true, DestT>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo)
                    : bin_count_w<PosT, false, DestT>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
}

template <typename PosT>
static hipError_t bin_count_d(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                              void* dest, int tile_rows, const Workspace& ws, hipStream_t s,
                              const FineGeom* fg, const HaloGeom* hg, uint16_t* fo) {
    if (dest_bytes(g.nbins) == 1)
        return bin_count_p<PosT, uint8_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fo);
    return bin_count_p<PosT, uint16_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fo);
}

// integer / float16 / bool positions (bin_coord_ext): each lane reads its
// own row (no slab staging: such rows need not be 4-byte multiples), run-time
// dimensionality -- the general path of every plan.
template <typename PosT, typename DestT>
static hipError_t bin_count_ext(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                                void* dest, int tile_rows, const Workspace& ws, hipStream_t s,
                                const FineGeom* fg, const HaloGeom* hg, uint16_t* fo) {
    return periodic ? bin_count_t<PosT, true, DestT, 0, 0>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo)
                    : bin_count_t<PosT, false, DestT, 0, 0>(g, pos, n, stride, dest, tile_rows, ws, s, fg, hg, fo);
}
template <typename PosT>
static hipError_t bin_count_ext_d(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                                  void* dest, int tile_rows, const Workspace& ws, hipStream_t s,
                                  const FineGeom* fg, const HaloGeom* hg, uint16_t* fo) {
    if (dest_bytes(g.nbins) == 1)
        return bin_count_ext<PosT, uint8_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fo);
    return bin_count_ext<PosT, uint16_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fo);
}

hipError_t launch_bin_count(const Geom& g, void* pos, int pos_dtype, int64_t n, int64_t stride,
                            int periodic, void* dest, int tile_rows, const Workspace& ws,
                            hipStream_t s, const FineGeom* fg, uint16_t* fine_out,
                            const HaloGeom* hg) {
    if (n <= 0) return hipSuccess;
    const int kid = fg ? K_BIN_FINE : K_BIN_COUNT;
    prof_begin(s, kid);
    hipError_t e;
    switch (pos_dtype) {
        case MGR_F32: e = bin_count_d<float>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_F64: e = bin_count_d<double>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_I32: e = bin_count_ext_d<int32_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_I64: e = bin_count_ext_d<int64_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_F16: e = bin_count_ext_d<f16_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_I8: e = bin_count_ext_d<int8_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_I16: e = bin_count_ext_d<int16_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_U8: e = bin_count_ext_d<uint8_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_U16: e = bin_count_ext_d<uint16_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_U32: e = bin_count_ext_d<uint32_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_U64: e = bin_count_ext_d<uint64_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        case MGR_B8: e = bin_count_ext_d<b8_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s, fg, hg, fine_out); break;
        default: e = hipErrorInvalidValue;
    }
    prof_end(s, kid);
    return e;
}

// Tile histogram of u16 bin ids (the fine cells that arrived with the rows,
// config 5): one workgroup per tile, LDS atomics (counts only, order free),
// destination-major counts[b * T + tile] for mgr_scan; the ids themselves
// are the pack's destination array (<= 256 bins: copied to the 1-byte
// destination array dest8 the pack then reads).
// Ids >= nbins (the caller's, e.g. of another fine grid) are clamped to
// nbins - 1 -- every table index stays in range -- and reported through
// *bad (nonzero), which the host turns into a raised error / -1 counts.
template <typename DestT>
__global__ __launch_bounds__(kBlock) void count_ids_kernel(const uint16_t* __restrict__ ids,
                                                           int64_t n, int nbins,
                                                           int32_t* __restrict__ counts, int64_t T,
                                                           int tile_rows,
                                                           uint64_t* __restrict__ scan_flags,
                                                           DestT* __restrict__ dest,
                                                           uint32_t* __restrict__ bad) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int32_t* hist = (int32_t*)smem;
    clear_scan_flags(scan_flags);
    // XCD-contiguous tiles: neighbouring tiles' counts share lines
    // (counts[b * T + tile]) and merge in one L2 instead of leaving it half-written
    const int64_t tile = xcd_tile(blockIdx.x, T);
    for (int b = threadIdx.x; b < nbins; b += kBlock) hist[b] = 0;
    __syncthreads();
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    bool oob = false;
    for (int i = threadIdx.x; i < rows; i += kBlock) {
        unsigned v = ids[row0 + i];
        if (v >= (unsigned)nbins) { v = nbins - 1; oob = true; }
        atomicAdd(&hist[v], 1);
        dest[row0 + i] = (DestT)v;
    }
    if (__any(oob) && lane_id() == 0 && bad) atomicOr(bad, 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += kBlock) counts[(int64_t)b * T + tile] = hist[b];
}

// Stable tile slots of u16 bin ids (the fine cells at the destination, config
// 5) for mgr_pack_ranked: one 256-thread workgroup per tile of TR rows (4
// waves x RPW rounds, in order).  Per row: its slot in the tile's bin-sorted
// order = the tile's start of its bin + the wave prefix of the bin + its rank
// among the wave's earlier rows of the bin; per tile: every bin's start inside
// the tile (tile_starts[t][b], tile-major, contiguous) and its count (counts[b
// * T + t], for mgr_scan).  The ranking work leaves the pack, which then only
// places rows.
// A round's peers by LDS atomics: every lane ORs its lane bit into its bin's
// 64-bit word of the wave, reads the word back (the peers), the leader clears
// it -- 3 LDS operations and a few VALU per round instead of nbits ballots
// with their 64-bit selects (the ballot match measured VALU-bound at ~180
// instructions per round: 0.223 vs 0.146-0.155 ms per 64M ids).  OR commutes,
// so the result does not depend on the order the LDS unit serves the lanes in.
// RPW: the rounds per wave (the ranked tiles are 2048 or 4096 rows).
template <int NW, int RPW>
__global__ __launch_bounds__(NW * 64) void rank_ids_kernel(
    const uint16_t* __restrict__ ids, int64_t n, int nbins,
    int32_t* __restrict__ counts, int64_t T, uint16_t* __restrict__ slots,
    uint16_t* __restrict__ tile_starts, uint64_t* __restrict__ scan_flags,
    uint32_t* __restrict__ bad) {
    constexpr int NT = NW * 64, TR = NW * 64 * RPW;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // [NW][nbins] peer words, then [NW][nbins] running counts
    unsigned long long* mk = (unsigned long long*)smem;
    uint16_t* wt = (uint16_t*)(smem + NW * nbins * 8);
    __shared__ int s_wsum[NW];
    clear_scan_flags(scan_flags);
    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const int64_t tile = xcd_tile(blockIdx.x, T);
    {   // zero the peer words and running counts in 16-byte stores (the LDS
        // regions are 16-byte aligned: nbins * 8 per wave, then the counts)
        typedef unsigned int z4_t __attribute__((ext_vector_type(4)));
        const int nz = (NW * nbins * 8 + align16(NW * nbins * 2)) / 16;
        z4_t* z = (z4_t*)smem;
        for (int i = tid; i < nz; i += NT) z[i] = z4_t{0u, 0u, 0u, 0u};
    }
    unsigned b[RPW];
    bool oob = false;   // ids >= nbins: clamped, reported through *bad
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int64_t row = tile * TR + (int64_t)(w * RPW + q) * 64 + lane;
        b[q] = row < n ? (unsigned)ids[row] : 0u;
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q)
        if (b[q] >= (unsigned)nbins) { b[q] = nbins - 1; oob = true; }
    if (__any(oob) && lane == 0 && bad) atomicOr(bad, 1u);
    __syncthreads();
    unsigned long long* mw = mk + w * nbins;
    uint16_t* ww = wt + w * nbins;
    int rk[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int64_t row = tile * TR + (int64_t)(w * RPW + q) * 64 + lane;
        const bool valid = row < n;
        if (valid) __hip_atomic_fetch_or(&mw[b[q]], 1ull << lane, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WAVEFRONT);
        wave_sync();
        const unsigned long long peers = valid ? mw[b[q]] : 0ull;
        const int r = rank_in(peers);
        const int before = valid ? (int)ww[b[q]] : 0;
        wave_sync();
        if (valid && r == 0) {
            ww[b[q]] = (uint16_t)(before + __popcll(peers));
            mw[b[q]] = 0ull;
        }
        wave_sync();
        rk[q] = before + r;
    }
    __syncthreads();
    // per bin (bin k*NT + tid): the tile count, the bins' starts in the tile
    // (block scan over the bins), then every wave's base of the bin = start +
    // the counts of the earlier waves (in place)
    int carry = 0;
    for (int k = 0; k * NT < nbins; ++k) {
        const int bb = k * NT + tid;
        int run = 0;
        int c[NW];
#pragma unroll
        for (int ww2 = 0; ww2 < NW; ++ww2) {
            c[ww2] = bb < nbins ? (int)wt[ww2 * nbins + bb] : 0;
            run += c[ww2];
        }
        if (bb < nbins) counts[(int64_t)bb * T + tile] = run;
        const int incl = wave_incl_dpp(run);
        if (lane == 63) s_wsum[w] = incl;
        __syncthreads();
        int wpre = 0, wall = 0;
#pragma unroll
        for (int ww2 = 0; ww2 < NW; ++ww2) {
            const int x = s_wsum[ww2];
            wpre += ww2 < w ? x : 0;
            wall += x;
        }
        if (bb < nbins) {
            int acc = carry + wpre + incl - run;
            tile_starts[tile * nbins + bb] = (uint16_t)acc;
#pragma unroll
            for (int ww2 = 0; ww2 < NW; ++ww2) {
                wt[ww2 * nbins + bb] = (uint16_t)acc;
                acc += c[ww2];
            }
        }
        carry += wall;
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int64_t row = tile * TR + (int64_t)(w * RPW + q) * 64 + lane;
        if (row < n) slots[row] = (uint16_t)(ww[b[q]] + rk[q]);
    }
}

hipError_t launch_rank_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows,
                           const Workspace& ws, uint16_t* slots, uint16_t* tile_starts,
                           uint32_t* bad, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    // the ranked tiles (ranked_tile_rows: <= 1024 bins, 2048 or 4096 rows);
    // 4 waves (16 waves measured 0.57 vs 0.31 ms at 64M rows, 512 bins)
    if (nbins < 1 || nbins > 2048 || (tile_rows != 2048 && tile_rows != 4096))
        return hipErrorNotSupported;
    const int lds = align16(kWaves * nbins * 2) + kWaves * nbins * 8;
    auto k = tile_rows == 4096 ? rank_ids_kernel<kWaves, 16> : rank_ids_kernel<kWaves, 8>;
    prof_begin(s, K_COUNT_IDS);
    ensure_lds(k, lds);
    hipLaunchKernelGGL(k, dim3((unsigned)ws.T), dim3(64 * kWaves), (size_t)lds, s, ids, n, nbins,
                       ws.counts, ws.T, slots, tile_starts, ws.flags, bad);
    prof_end(s, K_COUNT_IDS);
    return hipGetLastError();
}

hipError_t launch_count_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows,
                            const Workspace& ws, void* dest, uint32_t* bad, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    prof_begin(s, K_COUNT_IDS);
    const int lds = align16(nbins * 4);
    if (dest_bytes(nbins) == 1) {
        ensure_lds(count_ids_kernel<uint8_t>, lds);
        hipLaunchKernelGGL(count_ids_kernel<uint8_t>, dim3((unsigned)ws.T), dim3(kBlock), (size_t)lds,
                           s, ids, n, nbins, ws.counts, ws.T, tile_rows, ws.flags, (uint8_t*)dest, bad);
    } else {
        ensure_lds(count_ids_kernel<uint16_t>, lds);
        hipLaunchKernelGGL(count_ids_kernel<uint16_t>, dim3((unsigned)ws.T), dim3(kBlock), (size_t)lds,
                           s, ids, n, nbins, ws.counts, ws.T, tile_rows, ws.flags, (uint16_t*)dest, bad);
    }
    prof_end(s, K_COUNT_IDS);
    return hipGetLastError();
}

template <typename PosT>
static hipError_t cell_ids_t(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                             int64_t* cell, int64_t* idx, hipStream_t s) {
    const int grid = grid_for(n);
    if (periodic)
        hipLaunchKernelGGL((cell_ids_kernel<PosT, true>), dim3(grid), dim3(kBlock), 0, s,
                           (PosT*)pos, n, stride, g, cell, idx);
    else
        hipLaunchKernelGGL((cell_ids_kernel<PosT, false>), dim3(grid), dim3(kBlock), 0, s,
                           (PosT*)pos, n, stride, g, cell, idx);
    return hipGetLastError();
}

hipError_t launch_cell_ids(const Geom& g, void* pos, int pos_dtype, int64_t n, int64_t stride,
                           int periodic, int64_t* cell, int64_t* idx, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    prof_begin(s, K_CELL_IDS);
    hipError_t e;
    switch (pos_dtype) {
        case MGR_F32: e = cell_ids_t<float>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_F64: e = cell_ids_t<double>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_I32: e = cell_ids_t<int32_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_I64: e = cell_ids_t<int64_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_F16: e = cell_ids_t<f16_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_I8: e = cell_ids_t<int8_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_I16: e = cell_ids_t<int16_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_U8: e = cell_ids_t<uint8_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_U16: e = cell_ids_t<uint16_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_U32: e = cell_ids_t<uint32_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_U64: e = cell_ids_t<uint64_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        case MGR_B8: e = cell_ids_t<b8_t>(g, pos, n, stride, periodic, cell, idx, s); break;
        default: e = hipErrorInvalidValue;
    }
    prof_end(s, K_CELL_IDS);
    return e;
}

template <typename IdT, typename DestT>
static hipError_t bin_ids_t(const void* ids, int64_t n, int nbins, void* dest, int tile_rows,
                            const Workspace& ws, hipStream_t s) {
    auto k = bin_ids_kernel<IdT, DestT>;
    const int per_wave = align16((nbins + 1) * 4);
    const int wpb = waves_per_block(per_wave);
    const int lds = per_wave * wpb;
    ensure_lds(k, lds);
    const int64_t grid = (ws.T + wpb - 1) / wpb;
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * wpb), (size_t)lds, s, (const IdT*)ids,
                       n, nbins, nbits_for(nbins + 1), (DestT*)dest, ws.counts, ws.T, tile_rows,
                       per_wave, ws.flags);
    return hipGetLastError();
}

template <typename IdT>
static hipError_t bin_ids_d(const void* ids, int64_t n, int nbins, void* dest, int tile_rows,
                            const Workspace& ws, hipStream_t s) {
    if (dest_bytes(nbins + 1) == 1) return bin_ids_t<IdT, uint8_t>(ids, n, nbins, dest, tile_rows, ws, s);
    return bin_ids_t<IdT, uint16_t>(ids, n, nbins, dest, tile_rows, ws, s);
}

hipError_t launch_bin_ids(const void* ids, int ids_dtype, int64_t n, int nbins, void* dest,
                          int tile_rows, const Workspace& ws, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    prof_begin(s, K_BIN_IDS);
    hipError_t e;
    switch (ids_dtype) {
        case MGR_I32: e = bin_ids_d<int32_t>(ids, n, nbins, dest, tile_rows, ws, s); break;
        case MGR_I64: e = bin_ids_d<int64_t>(ids, n, nbins, dest, tile_rows, ws, s); break;
        case MGR_F32: e = bin_ids_d<float>(ids, n, nbins, dest, tile_rows, ws, s); break;
        default: e = bin_ids_d<double>(ids, n, nbins, dest, tile_rows, ws, s); break;
    }
    prof_end(s, K_BIN_IDS);
    return e;
}

hipError_t launch_cellnum_from_idx(const Geom& g, const int64_t* idx, int64_t n, int periodic,
                                   int64_t* cell, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    prof_begin(s, K_CELLNUM_IDX);
    hipLaunchKernelGGL(cellnum_from_idx_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, idx, n, g,
                       periodic, cell);
    prof_end(s, K_CELLNUM_IDX);
    return hipGetLastError();
}

}  // namespace mgr
