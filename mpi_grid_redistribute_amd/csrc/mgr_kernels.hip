// HIP kernels for gfx950 (MI355X): wrap+bin+histogram, device-wide scan,
// stable LDS-staged pack, id binning, synthetic input.
//
// Reference semantics (dkorytov/mpi_grid_redistribute, redist.py):
//   wrap   ((x % L) + L) % L, numpy floor remainder, written back  :68, :328-329
//   bin    trunc((t / L) * n) (x86 INT64_MIN on NaN/overflow)      :69-70
//   cell   sum_d offset[d] * ((k % n) + n) % n, row-major           :53-58, :83-84
//   split  data[rank_to_send == i], order kept                      :195-198
// Every float operation below is IEEE-exact and ordered as in numpy (built
// with -ffp-contract=off, no fast-math): the GPU results are bit-identical to
// the reference (tests/test_gpu_parity.py).
//
// Work decomposition: a "tile" is tile_rows consecutive rows (a multiple of
// 256), one 256-thread workgroup per tile.  Inside a tile, row i belongs to
// round i / 256 and lane (i % 256): rounds, then waves, then lanes follow the
// original row order, which is what makes the ballot ranks stable.

#include "mgr_internal.h"

#include <limits.h>

#include <type_traits>

namespace mgr {

Tune g_tune;

// ------------------------------------------------------------ scalar math
__device__ __forceinline__ long long trunc_i64(double v) {
    // numpy astype(int64) on x86 (cvttsd2si): NaN / out of range -> INT64_MIN (S10).
    // |v| < 2^31 (every in-box particle): one v_cvt_i32_f64.
    if (v > -2147483648.0 && v < 2147483648.0) return (long long)(int)v;
    return (v >= -9223372036854775808.0 && v < 9223372036854775808.0) ? (long long)v : LLONG_MIN;
}

// ---- x86/glibc NaN semantics (numpy runs on x86: SSE + glibc fmod) ----
// An invalid operation (fmod(inf, L), fmod(x, 0), inf - inf) yields the x86
// "default NaN" -- sign bit SET (0xFFF8... / 0xFFC00000); a NaN operand
// propagates quieted, first operand first.  The GPU's own default NaN is
// positive, so these cases are spelled out bit by bit.  They only occur on
// the slow path (non-finite input or box), never for in-box particles.
constexpr unsigned long long kDefaultNaN64 = 0xFFF8000000000000ull;
constexpr unsigned kDefaultNaN32 = 0xFFC00000u;

__device__ __forceinline__ double quiet64(double x) {
    return __longlong_as_double(__double_as_longlong(x) | 0x0008000000000000ll);
}
__device__ __forceinline__ float quiet32(float x) {
    return __uint_as_float(__float_as_uint(x) | 0x00400000u);
}
// cvtss2sd / cvtsd2ss on NaN: keep sign, quiet, shift the payload.
__device__ __forceinline__ double f32_to_f64_x86(float x) {
    if (!isnan(x)) return (double)x;
    const unsigned u = __float_as_uint(x) | 0x00400000u;
    const unsigned long long b = ((unsigned long long)(u >> 31) << 63) | 0x7FF0000000000000ull |
                                 ((unsigned long long)(u & 0x007FFFFFu) << 29);
    return __longlong_as_double((long long)b);
}
__device__ __forceinline__ float f64_to_f32_x86(double x) {
    if (!isnan(x)) return (float)x;
    const unsigned long long b = (unsigned long long)__double_as_longlong(x) | 0x0008000000000000ull;
    const unsigned u = ((unsigned)(b >> 63) << 31) | 0x7F800000u | (unsigned)((b >> 29) & 0x007FFFFFu);
    return __uint_as_float(u);
}

__device__ __forceinline__ double fmod_x86(double a, double b) {
    if (isnan(a)) return quiet64(a);
    if (isnan(b)) return quiet64(b);
    if (isinf(a) || b == 0.0) return __longlong_as_double((long long)kDefaultNaN64);
    if (isinf(b)) return a;
    return fmod(a, b);  // finite / finite nonzero: exact
}
__device__ __forceinline__ float fmodf_x86(float a, float b) {
    if (isnan(a)) return quiet32(a);
    if (isnan(b)) return quiet32(b);
    if (isinf(a) || b == 0.0f) return __uint_as_float(kDefaultNaN32);
    if (isinf(b)) return a;
    return fmodf(a, b);
}

// numpy npy_remainder: floor remainder, sign of the divisor.  A NaN result
// is final: every later x86 operation propagates it unchanged.
__device__ __forceinline__ double pymod(double a, double b) {
    double m = fmod_x86(a, b);
    if (b == 0.0 || isnan(m)) return m;
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

__device__ __forceinline__ float pymodf(float a, float b) {
    float m = fmodf_x86(a, b);
    if (b == 0.0f || isnan(m)) return m;
    if (m != 0.0f) {
        if ((b < 0.0f) != (m < 0.0f)) m += b;
    } else {
        m = copysignf(0.0f, b);
    }
    return m;
}

// ((x % L) + L) % L.  Fast path for 0 <= x < L (every in-box particle):
// x % L == x, y = x + L in [L, 2L], and fmod(y, L) == y - L exactly
// (Sterbenz), 0 when y == 2L.  Bit-identical to the general path.
// General path (outside the box, non-finite, odd boxes): out of line so its
// registers do not weigh on the streaming fast path.
__device__ __attribute__((noinline)) double wrap_f64_slow(double x, double L) {
    const double m = pymod(x, L);
    if (isnan(m)) return m;
    return pymod(m + L, L);
}

__device__ __attribute__((noinline)) float wrap_f32_slow(float x, float L) {
    const float m = pymodf(x, L);
    if (isnan(m)) return m;
    return pymodf(m + L, L);
}

__device__ __forceinline__ double wrap_f64(double x, double L, double twoL, int fast) {
    if (fast && x >= 0.0 && x < L) {
        const double y = x + L;
        return (y == twoL) ? 0.0 : y - L;
    }
    return wrap_f64_slow(x, L);
}

__device__ __forceinline__ float wrap_f32(float x, float L, float twoL, int fast) {
    if (fast && x >= 0.0f && x < L) {
        const float y = x + L;
        return (y == twoL) ? 0.0f : y - L;
    }
    return wrap_f32_slow(x, L);
}

__device__ __forceinline__ long long floormod_i64(long long a, long long n) {
    if (n == 0 || n == -1) return 0;
    long long r = a % n;
    if (r != 0 && ((r < 0) != (n < 0))) r += n;
    return r;
}

template <typename PosT>
__device__ __forceinline__ bool same_bits(PosT a, PosT b) {
    if constexpr (sizeof(PosT) == 8) return __double_as_longlong((double)a) == __double_as_longlong((double)b);
    else return __float_as_uint((float)a) == __float_as_uint((float)b);
}

// One coordinate: wrap (+ write back), bin, index wrap.  Returns the wrapped
// index; *raw gets trunc(t/L*n) before the index wrap (cell indexes API).
// The wrapped value is stored only when its bits differ from the input
// (the in-place mutation of redist.py:68 / :328-329 is then complete: an
// in-box coordinate wraps to itself) and *dirty records that a store happened.
template <typename PosT, bool kPeriodic>
__device__ __forceinline__ long long bin_coord(PosT* p, const Geom& g, int d, long long* raw,
                                               bool* dirty) {
    long long k;
    const PosT in = *p;
    if (sizeof(PosT) == 4 && g.compute_f32) {
        float x = (float)in;
        if (kPeriodic) {
            x = wrap_f32(x, g.Lf[d], g.twoLf[d], g.fastf[d]);
            if (!same_bits((PosT)x, in)) { *p = (PosT)x; *dirty = true; }
        }
        const float q = g.pow2f[d] ? x * g.invLf[d] : x / g.Lf[d];  // f32 / f32 -> f32
        k = trunc_i64((double)q * g.nd[d]);          // * int64 scalar -> f64
    } else {
        double x = sizeof(PosT) == 4 ? f32_to_f64_x86((float)in) : (double)in;
        if (kPeriodic) {
            const double t = wrap_f64(x, g.L[d], g.twoL[d], g.fast[d]);
            const PosT w = sizeof(PosT) == 4 ? (PosT)f64_to_f32_x86(t) : (PosT)t;  // round (S9)
            if (!same_bits(w, in)) { *p = w; *dirty = true; }
            x = sizeof(PosT) == 4 ? f32_to_f64_x86((float)w) : (double)w;  // bin reads it (S2)
        }
        k = trunc_i64((g.pow2[d] ? x * g.invL[d] : x / g.L[d]) * g.nd[d]);
    }
    if (raw) *raw = k;
    const long long n = g.n[d];
    if (!(k >= 0 && k < n)) k = floormod_i64(floormod_i64(k, n) + n, n);
    if (g.fine) k %= g.fmod[d];   // fine-cell plan: index inside the rank's cell
    return k;
}

// DIM > 0: compile-time dimensionality (the common 1-3); 0: runtime g.dim.
template <typename PosT, bool kPeriodic, int DIM = 0>
__device__ __forceinline__ long long bin_row(PosT* row, const Geom& g, long long* idx,
                                             bool* dirty) {
    long long cell = 0;
    if (DIM > 0) {
#pragma unroll
        for (int d = 0; d < DIM; ++d)
            cell += g.off[d] * bin_coord<PosT, kPeriodic>(row + d, g, d, idx ? idx + d : nullptr, dirty);
    } else {
        for (int d = 0; d < g.dim; ++d)
            cell += g.off[d] * bin_coord<PosT, kPeriodic>(row + d, g, d, idx ? idx + d : nullptr, dirty);
    }
    return cell;
}

// ------------------------------------------------------ wave primitives
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Lanes of this wave holding the same bin b (valid lanes only): nbits
// ballots, one per bit of the bin id (gfx950 wave64 ballot + popc match).
__device__ __forceinline__ unsigned long long match_bin(unsigned b, bool valid, int nbits) {
    unsigned long long peers = __ballot(valid);
    for (int i = 0; i < nbits; ++i) {
        const bool bit = (b >> i) & 1u;
        const unsigned long long m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return valid ? peers : 0ull;
}

__device__ __forceinline__ int rank_in(unsigned long long peers) {
    const unsigned lo = (unsigned)peers, hi = (unsigned)(peers >> 32);
    return __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
}

// Block-wide exclusive scan of one int64 per thread (256 threads).
__device__ __forceinline__ long long block_excl_scan(long long v, long long* total,
                                                     long long* s_w /* [kWaves] */) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    long long pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) {
        const long long t = s_w[i];
        pre += (i < w) ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

// ------------------------------------------------------ wave-private tiles
// A tile is tile_rows = 64 * R consecutive rows owned by ONE wavefront; a
// workgroup of wpb waves runs tiles blockIdx.x * wpb + wave.  Row
// (tile, round r, lane l) = tile * tile_rows + 64 r + l, so (round, lane)
// order IS the original row order: a ballot rank inside a round plus a
// running per-bin count across rounds is a stable rank.  Tiles never share
// data, so the kernels have no workgroup barriers at all.
__device__ __forceinline__ void wave_sync() {
    // LDS traffic of one wave is performed in order; this only stops the
    // compiler from moving LDS accesses across the point.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int W> struct Unit;
template <> struct Unit<16> { using T = uint4; };
template <> struct Unit<8> { using T = uint2; };
template <> struct Unit<4> { using T = uint32_t; };
template <> struct Unit<2> { using T = uint16_t; };
template <> struct Unit<1> { using T = uint8_t; };

// Copy nbytes (a multiple of 4) between 16-byte-aligned regions with one
// wave: W-byte units, 4-byte tail.
template <int W>
__device__ __forceinline__ void wave_copy(uint8_t* __restrict__ d, const uint8_t* __restrict__ s,
                                          int nbytes, int lane) {
    using U = typename Unit<W>::T;
    const int units = nbytes / W;
    for (int u = lane; u < units; u += 64) ((U*)d)[u] = ((const U*)s)[u];
    for (int q = units * (W / 4) + lane; q < nbytes / 4; q += 64)
        ((uint32_t*)d)[q] = ((const uint32_t*)s)[q];
}

__host__ __device__ inline int align16(int x) { return (x + 15) & ~15; }

// XCD-contiguous tile order.  Workgroups are dealt to the 8 XCDs round-robin
// (blockIdx % 8 labels the XCD, MI355X_MICROARCH.md "Workgroup dispatch"), so
// tile = blockIdx would put neighbouring tiles on different L2s.  This
// bijection gives each XCD label one contiguous run of T/8 tiles: the cache
// lines that two neighbouring tiles' output segments share are then written
// through ONE L2 and leave it as whole lines.  Speed only, never correctness.
__device__ __forceinline__ int64_t xcd_tile(int64_t bid, int64_t T) {
    const int64_t per = T >> 3;
    if (bid < per * 8) return (bid & 7) * per + (bid >> 3);
    return bid;
}

// Streaming accesses: NT selects the nontemporal (nt) cache policy for data
// that is read or written exactly once.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <bool NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (!NT) {
        return *p;
    } else if constexpr (sizeof(T) == 16) {
        const u32x4_t x = __builtin_nontemporal_load((const u32x4_t*)p);
        T r;
        __builtin_memcpy(&r, &x, 16);
        return r;
    } else if constexpr (sizeof(T) == 8) {
        const u32x2_t x = __builtin_nontemporal_load((const u32x2_t*)p);
        T r;
        __builtin_memcpy(&r, &x, 8);
        return r;
    } else {
        return __builtin_nontemporal_load(p);
    }
}
template <bool NT, typename T>
__device__ __forceinline__ void st(T* p, const T& v) {
    if constexpr (!NT) {
        *p = v;
    } else if constexpr (sizeof(T) == 16) {
        u32x4_t x;
        __builtin_memcpy(&x, &v, 16);
        __builtin_nontemporal_store(x, (u32x4_t*)p);
    } else if constexpr (sizeof(T) == 8) {
        u32x2_t x;
        __builtin_memcpy(&x, &v, 8);
        __builtin_nontemporal_store(x, (u32x2_t*)p);
    } else {
        __builtin_nontemporal_store(v, p);
    }
}

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
template <typename PosT, bool kPeriodic, typename DestT, int NU, int DIM, bool NT, int DEPTH>
__global__ __launch_bounds__(1024) void bin_count_kernel(PosT* __restrict__ pos, int64_t n,
                                                           int64_t stride, Geom g,
                                                           DestT* __restrict__ dest,
                                                           int32_t* __restrict__ counts,
                                                           int64_t T, int tile_rows,
                                                           int per_wave_lds, int skip_clean,
                                                           int xcd) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
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
            if (valid)
                b = (unsigned)bin_row<PosT, kPeriodic, DIM>((PosT*)(stage + lane * rb), g, nullptr, &dirty);
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
            if (valid)
                b = (unsigned)bin_row<PosT, kPeriodic, DIM>(pos + (row0 + r0 + lane) * stride, g,
                                                             nullptr, &dirty);
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
                                                         int tile_rows, int per_wave_lds) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
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

// ------------------------------------------------------------------ scan
__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const int32_t* __restrict__ counts,
                                                             int64_t M, int64_t chunk,
                                                             int64_t* __restrict__ partials) {
    __shared__ long long s_w[kWaves];
    const int64_t lo = blockIdx.x * chunk, hi = min(M, lo + chunk);
    long long acc = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) acc += counts[i];
    long long tot;
    block_excl_scan(acc, &tot, s_w);
    if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void scan_apply_kernel(const int32_t* __restrict__ counts,
                                                            int64_t M, int64_t chunk,
                                                            const int64_t* __restrict__ partials,
                                                            int64_t* __restrict__ offsets, int64_t T,
                                                            int64_t* __restrict__ bin_starts,
                                                            int nbins) {
    __shared__ long long s_w[kWaves];
    long long carry = 0;
    for (int j = threadIdx.x; j < (int)blockIdx.x; j += kBlock) carry += partials[j];
    long long tot;
    block_excl_scan(carry, &tot, s_w);
    carry = tot;
    const int64_t lo = blockIdx.x * chunk, hi = min(M, lo + chunk);
    for (int64_t base = lo; base < hi; base += kBlock) {
        const int64_t i = base + threadIdx.x;
        const long long v = (i < hi) ? counts[i] : 0;
        const long long ex = block_excl_scan(v, &tot, s_w) + carry;
        if (i < hi) {
            offsets[i] = ex;
            if (i % T == 0) bin_starts[i / T] = ex;
        }
        carry += tot;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) bin_starts[nbins] = carry;
}

__global__ void bin_totals_kernel(const int64_t* __restrict__ bin_starts, int nbins,
                                  int64_t* __restrict__ bin_counts) {
    for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < nbins; b += gridDim.x * blockDim.x)
        bin_counts[b] = bin_starts[b + 1] - bin_starts[b];
}

// ------------------------------------------------------------------ pack
// Kernel 3 of the hot path.  Per round: ballot match -> rank inside the
// wave; slot = tile segment start of the bin + running count + rank; the
// row is copied straight to its slot.  Same-bin lanes hold consecutive
// slots, so each store instruction writes a few contiguous runs, and the
// runs of consecutive rounds continue each other (merged in L2).
// kWide (rows > 256 B): the wave copies one row at a time, 64 lanes wide.
template <int W, typename DestT, bool kWide>
__global__ __launch_bounds__(kBlock) void pack_kernel(
    const uint8_t* __restrict__ src, int64_t upr /* W-units per row */, int64_t n,
    const DestT* __restrict__ dest, int nb, int nbits, int drop_bin,
    const int64_t* __restrict__ offsets, const int64_t* __restrict__ bin_starts, int64_t T,
    int tile_rows, int per_wave_lds, uint8_t* __restrict__ dst, int redirect_bin,
    uint8_t* __restrict__ redirect_dst) {
    using U = typename Unit<W>::T;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
    if (tile >= T) return;
    int64_t* goff = (int64_t*)(smem + w * per_wave_lds);
    int32_t* run = (int32_t*)(smem + w * per_wave_lds + align16(nb * 8));
    for (int b = lane; b < nb; b += 64) {
        int64_t o = offsets[(int64_t)b * T + tile];
        if (b == redirect_bin) o -= bin_starts[b];
        goff[b] = o;
        run[b] = 0;
    }
    wave_sync();
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    const U* __restrict__ s_u = (const U*)src;
    U* __restrict__ d_u = (U*)dst;
    U* __restrict__ r_u = (U*)redirect_dst;
    for (int r0 = 0; r0 < rows; r0 += 64) {
        const bool valid = r0 + lane < rows;
        const int64_t row = row0 + r0 + lane;
        const unsigned b = valid ? (unsigned)dest[row] : 0u;
        const unsigned long long peers = match_bin(b, valid, nbits);
        const int rk = rank_in(peers);
        int64_t slot = 0;
        if (valid) slot = goff[b] + run[b] + rk;
        wave_sync();
        if (valid && rk == 0) run[b] += __popcll(peers);
        const bool live = valid && (int)b != drop_bin;
        if (!kWide) {
            if (live) {
                const U* sp = s_u + row * upr;
                U* dp = ((int)b == redirect_bin ? r_u : d_u) + slot * upr;
                int64_t k = 0;
                for (; k + 4 <= upr; k += 4) {
                    const U a0 = sp[k], a1 = sp[k + 1], a2 = sp[k + 2], a3 = sp[k + 3];
                    dp[k] = a0; dp[k + 1] = a1; dp[k + 2] = a2; dp[k + 3] = a3;
                }
                for (; k < upr; ++k) dp[k] = sp[k];
            }
        } else {
            const unsigned long long todo = __ballot(live);
            for (int j = 0; j < 64; ++j) {
                if (!((todo >> j) & 1ull)) continue;
                const int bj = __shfl((int)b, j, 64);
                const int64_t sj = __shfl((long long)slot, j, 64);
                const U* sp = s_u + (row0 + r0 + j) * upr;
                U* dp = (bj == redirect_bin ? r_u : d_u) + sj * upr;
                for (int64_t k = lane; k < upr; k += 64) dp[k] = sp[k];
            }
        }
        wave_sync();
    }
}

// Register-resident pack for <= 64 bins and rows of <= 64 bytes (the
// common case, e.g. 8 grid cells x 32-byte records).  Lane l keeps the next
// free slot of bin l in a register; a row finds its slot with one
// cross-lane read (bpermute) of its bin's lane; per-bin round counts come
// from the same nbits ballots as the rank, so there is no LDS traffic.  The
// next round's destinations and rows are prefetched while the current
// round is ranked and stored.
template <int W, int UPR, bool NT, bool NTS>
__global__ __launch_bounds__(kBlock) void pack_small_kernel(
    const uint8_t* __restrict__ src, int64_t n, const uint8_t* __restrict__ dest,
    int nb, int nbits, int drop_bin, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ bin_starts, int64_t T, int tile_rows, uint8_t* __restrict__ dst,
    int redirect_bin, uint8_t* __restrict__ redirect_dst) {
    using U = typename Unit<W>::T;
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
    if (tile >= T) return;
    long long next_slot = 0;  // lane l: next free slot of bin l
    if (lane < nb) {
        next_slot = offsets[(int64_t)lane * T + tile];
        if (lane == redirect_bin) next_slot -= bin_starts[lane];
    }
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    // Round = 64 rows = 64*UPR units of W bytes, contiguous in src.  Lane l
    // moves units 64k + l (k < UPR): every load instruction reads 64*W
    // contiguous bytes.  The unit's row (compile-time division by UPR) gets
    // its slot from the lane that ranked it.
    const U* __restrict__ s_u = (const U*)src + row0 * UPR;
    U* __restrict__ d_u = (U*)dst;
    U* __restrict__ r_u = (U*)redirect_dst;
    unsigned nb_next = 0;
    U nv[UPR];
    if (lane < rows) nb_next = dest[row0 + lane];
#pragma unroll
    for (int k = 0; k < UPR; ++k)
        if (64 * k + lane < rows * UPR) nv[k] = ld<NT>(s_u + 64 * k + lane);
    for (int r0 = 0; r0 < rows; r0 += 64) {
        const int nr = min(64, rows - r0);
        const bool valid = lane < nr;
        const unsigned b = valid ? nb_next : 0u;
        U v[UPR];
#pragma unroll
        for (int k = 0; k < UPR; ++k) v[k] = nv[k];
        if (r0 + 64 < rows) {  // next round in flight
            const int nn = min(64, rows - r0 - 64);
            if (lane < nn) nb_next = dest[row0 + r0 + 64 + lane];
            const U* sp = s_u + (int64_t)(r0 + 64) * UPR;
#pragma unroll
            for (int k = 0; k < UPR; ++k)
                if (64 * k + lane < nn * UPR) nv[k] = ld<NT>(sp + 64 * k + lane);
        }
        // nbits ballots: rank inside the wave + per-bin counts for lane == bin
        unsigned long long peers = __ballot(valid);
        unsigned long long mine = peers;  // lanes whose bin == this lane's index
        for (int i = 0; i < nbits; ++i) {
            const unsigned long long m = __ballot((b >> i) & 1u);
            peers &= ((b >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        if (!valid) peers = 0;
        const long long base = __shfl(next_slot, (int)b, 64);
        next_slot += __popcll(mine);
        // per-row target: slot, or -1 (dropped / past the end); bit 62 = redirect
        long long tgt = -1;
        if (valid && (int)b != drop_bin)
            tgt = (base + rank_in(peers)) | ((int)b == redirect_bin ? (1ll << 62) : 0ll);
#pragma unroll
        for (int k = 0; k < UPR; ++k) {
            const int u = 64 * k + lane;
            const int r = u / UPR, part = u - r * UPR;
            const long long t = __shfl(tgt, r, 64);
            if (u < nr * UPR && t >= 0) {
                U* o = (t >> 62) ? r_u : d_u;
                st<NTS>(o + (t & ((1ll << 62) - 1)) * UPR + part, v[k]);
            }
        }
    }
}

// Block-cooperative pack for <= 64 bins and rows of <= 64 bytes: one
// workgroup per tile of R rounds, wave w ranks and moves round w (64 rows)
// in one shot -- the short-lived, fully parallel shape that streams best.
// The waves exchange their per-bin counts through a [R][64] LDS table (one
// barrier) to get each bin's base inside the tile.  Unit-transposed moves:
// lane l moves W-byte units 64k + l of the round, so each load instruction
// reads 64*W contiguous bytes; the unit's row gets its slot by shfl.
template <int W, int UPR, bool NT, int RPW, bool NTS>
__global__ __launch_bounds__(1024) void pack_coop_kernel(
    const uint8_t* __restrict__ src, int64_t n, const uint8_t* __restrict__ dest, int nb,
    int nbits, int drop_bin, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ bin_starts, int64_t T, int tile_rows, uint8_t* __restrict__ dst,
    int redirect_bin, uint8_t* __restrict__ redirect_dst, int xcd) {
    using U = typename Unit<W>::T;
    __shared__ int s_cnt[kMaxTileRows / 64][64];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = xcd ? xcd_tile(blockIdx.x, T) : (int64_t)blockIdx.x;
    // wave w moves rounds w*RPW .. w*RPW+RPW-1 of the tile
    const int64_t row0 = tile * (int64_t)tile_rows + 64 * RPW * w;
    // issue every load of the wave's rounds first
    int nr[RPW];
    unsigned b[RPW];
    U v[RPW][UPR];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        nr[q] = (int)max((int64_t)0, min((int64_t)64, n - row0 - 64 * q));
        b[q] = lane < nr[q] ? (unsigned)dest[row0 + 64 * q + lane] : 0u;
    }
    long long tbase = 0;
    if (lane < nb) {
        tbase = offsets[(int64_t)lane * T + tile];
        if (lane == redirect_bin) tbase -= bin_starts[lane];
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const U* __restrict__ sp = (const U*)src + (row0 + 64 * q) * UPR;
#pragma unroll
        for (int k = 0; k < UPR; ++k)
            if (64 * k + lane < nr[q] * UPR) v[q][k] = ld<NT>(sp + 64 * k + lane);
    }
    // rank inside each round; lane l counts bin l
    unsigned long long peers[RPW];
    int cnt[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const bool valid = lane < nr[q];
        unsigned long long pe = __ballot(valid);
        unsigned long long mine = pe;
        for (int i = 0; i < nbits; ++i) {
            const unsigned long long m = __ballot((b[q] >> i) & 1u);
            pe &= ((b[q] >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        peers[q] = valid ? pe : 0ull;
        cnt[q] = __popcll(mine);
        s_cnt[w * RPW + q][lane] = cnt[q];
    }
    __syncthreads();
    for (int j = 0; j < w * RPW; ++j) tbase += s_cnt[j][lane];
    U* __restrict__ d_u = (U*)dst;
    U* __restrict__ r_u = (U*)redirect_dst;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const long long base = __shfl(tbase, (int)b[q], 64);
        long long tgt = -1;
        if (lane < nr[q] && (int)b[q] != drop_bin)
            tgt = (base + rank_in(peers[q])) | ((int)b[q] == redirect_bin ? (1ll << 62) : 0ll);
        tbase += cnt[q];
#pragma unroll
        for (int k = 0; k < UPR; ++k) {
            const int u = 64 * k + lane;
            const int r = u / UPR, part = u - r * UPR;
            const long long t = __shfl(tgt, r, 64);
            if (u < nr[q] * UPR && t >= 0) {
                U* o = (t >> 62) ? r_u : d_u;
                st<NTS>(o + (t & ((1ll << 62) - 1)) * UPR + part, v[q][k]);
            }
        }
    }
}

// Many-destination pack (65..1024 bins, e.g. the 512 fine cells of config
// 5) in the cooperative shape: one workgroup of 16 waves per tile of R = 16*RPW
// rounds, wave w ranking and moving rounds w*RPW.. with unit-transposed
// coalesced loads and stores.  The per-(round, bin) counts go to an LDS table
// (uint16 [R][nbins], written by each peer group's leader lane), one pass
// turns every bin column into an exclusive prefix over the rounds, and a
// row's slot = the tile's segment start of its bin (staged once per tile in
// LDS) + its round's prefix + its ballot rank.
template <int W, int UPR, typename DestT, int RPW>
__global__ __launch_bounds__(1024) void pack_many_kernel(
    const uint8_t* __restrict__ src, int64_t n, const DestT* __restrict__ dest, int nb,
    int nbits, int drop_bin, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ bin_starts, int64_t T, int tile_rows, uint8_t* __restrict__ dst,
    int redirect_bin, uint8_t* __restrict__ redirect_dst, int xcd) {
    using U = typename Unit<W>::T;
    constexpr int R = 16 * RPW;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    long long* s_off = (long long*)smem;                       // [nb]
    uint16_t* tab = (uint16_t*)(smem + align16(nb * 8));       // [R][nb]
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = xcd ? xcd_tile(blockIdx.x, T) : (int64_t)blockIdx.x;
    const int64_t row0 = tile * (int64_t)tile_rows + 64 * RPW * w;
    for (int i = threadIdx.x; i < R * nb; i += blockDim.x) tab[i] = 0;
    for (int bb = threadIdx.x; bb < nb; bb += blockDim.x) {
        long long o = offsets[(int64_t)bb * T + tile];
        if (bb == redirect_bin) o -= bin_starts[bb];
        s_off[bb] = o;
    }
    int nr[RPW];
    unsigned b[RPW];
    U v[RPW][UPR];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        nr[q] = (int)max((int64_t)0, min((int64_t)64, n - row0 - 64 * q));
        b[q] = lane < nr[q] ? (unsigned)dest[row0 + 64 * q + lane] : 0u;
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const U* __restrict__ sp = (const U*)src + (row0 + 64 * q) * UPR;
#pragma unroll
        for (int k = 0; k < UPR; ++k)
            if (64 * k + lane < nr[q] * UPR) v[q][k] = sp[64 * k + lane];
    }
    __syncthreads();   // table zeroed, tile offsets staged
    unsigned long long peers[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const bool valid = lane < nr[q];
        peers[q] = match_bin(b[q], valid, nbits);
        if (valid && rank_in(peers[q]) == 0)
            tab[(w * RPW + q) * nb + b[q]] = (uint16_t)__popcll(peers[q]);
    }
    __syncthreads();
    for (int bb = threadIdx.x; bb < nb; bb += blockDim.x) {   // exclusive prefix per bin
        int run = 0;
        for (int r = 0; r < R; ++r) {
            const int c = tab[r * nb + bb];
            tab[r * nb + bb] = (uint16_t)run;
            run += c;
        }
    }
    __syncthreads();
    U* __restrict__ d_u = (U*)dst;
    U* __restrict__ r_u = (U*)redirect_dst;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        long long tgt = -1;
        if (lane < nr[q] && (int)b[q] != drop_bin)
            tgt = (s_off[b[q]] + tab[(w * RPW + q) * nb + b[q]] + rank_in(peers[q])) |
                  ((int)b[q] == redirect_bin ? (1ll << 62) : 0ll);
#pragma unroll
        for (int k = 0; k < UPR; ++k) {
            const int u = 64 * k + lane;
            const int r = u / UPR, part = u - r * UPR;
            const long long t = __shfl(tgt, r, 64);
            if (u < nr[q] * UPR && t >= 0) {
                U* o = (t >> 62) ? r_u : d_u;
                o[(t & ((1ll << 62) - 1)) * UPR + part] = v[q][k];
            }
        }
    }
}

// Destination-sorted pack for <= 64 bins and rows of <= 64 bytes.  As
// pack_coop_kernel, one workgroup per tile and wave w ranks round w; but the
// rows are first written into an LDS image of the tile SORTED by destination
// (bin, then original order), and the image is then streamed out in order:
// each store instruction writes 64*W contiguous bytes of one or two
// destination runs instead of ~nbins short runs.  LDS: the image
// (tile_rows * row bytes), the [rounds][64] count table and one bin byte per
// sorted row.
template <int W, int UPR, bool NT>
__global__ __launch_bounds__(1024) void pack_sorted_kernel(
    const uint8_t* __restrict__ src, int64_t n, const uint8_t* __restrict__ dest, int nb,
    int nbits, int drop_bin, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ bin_starts, int64_t T, int tile_rows, uint8_t* __restrict__ dst,
    int redirect_bin, uint8_t* __restrict__ redirect_dst, int xcd) {
    using U = typename Unit<W>::T;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int R = tile_rows >> 6;
    U* img = (U*)smem;
    int* s_cnt = (int*)(smem + (size_t)tile_rows * UPR * W);
    uint8_t* s_bin = (uint8_t*)(s_cnt + R * 64);
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = xcd ? xcd_tile(blockIdx.x, T) : (int64_t)blockIdx.x;
    const int64_t trow0 = tile * (int64_t)tile_rows;
    const int64_t row0 = trow0 + 64 * w;
    const int nr = (int)max((int64_t)0, min((int64_t)64, n - row0));
    const int trows = (int)min((int64_t)tile_rows, n - trow0);
    const bool valid = lane < nr;
    const unsigned b = valid ? (unsigned)dest[row0 + lane] : 0u;
    long long tbase = 0;
    if (lane < nb) {
        tbase = offsets[(int64_t)lane * T + tile];
        if (lane == redirect_bin) tbase -= bin_starts[lane];
    }
    const U* __restrict__ sp = (const U*)src + row0 * UPR;
    U v[UPR];
#pragma unroll
    for (int k = 0; k < UPR; ++k)
        if (64 * k + lane < nr * UPR) v[k] = ld<NT>(sp + 64 * k + lane);
    unsigned long long peers = __ballot(valid);
    unsigned long long mine = peers;
    for (int i = 0; i < nbits; ++i) {
        const unsigned long long m = __ballot((b >> i) & 1u);
        peers &= ((b >> i) & 1u) ? m : ~m;
        mine &= ((lane >> i) & 1) ? m : ~m;
    }
    if (!valid) peers = 0;
    s_cnt[w * 64 + lane] = __popcll(mine);
    __syncthreads();
    // lane = bin: rows of this bin in earlier rounds, and in the whole tile
    int before = 0, tot = 0;
    for (int j = 0; j < R; ++j) {
        const int c = s_cnt[j * 64 + lane];
        before += (j < w) ? c : 0;
        tot += c;
    }
    // exclusive scan of the per-bin tile totals over the lanes: local bin start
    int lstart = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(lstart, o, 64);
        if (lane >= o) lstart += y;
    }
    lstart -= tot;
    const int lpos = __shfl(lstart + before, (int)b, 64) + rank_in(peers);
#pragma unroll
    for (int k = 0; k < UPR; ++k) {
        const int u = 64 * k + lane;
        const int r = u / UPR, part = u - r * UPR;
        const int t = __shfl(lpos, r, 64);
        if (u < nr * UPR) img[t * UPR + part] = v[k];
    }
    if (valid) s_bin[lpos] = (uint8_t)b;
    __syncthreads();
    // stream the sorted image out: wave w writes sorted units [w*64*UPR, ...)
    const long long delta = tbase - lstart;   // lane = bin: global slot - local position
    U* __restrict__ d_u = (U*)dst;
    U* __restrict__ r_u = (U*)redirect_dst;
#pragma unroll
    for (int k = 0; k < UPR; ++k) {
        const int u = w * 64 * UPR + 64 * k + lane;
        const int p = u / UPR, part = u - p * UPR;
        const int bb = p < trows ? (int)s_bin[p] : 0;
        const long long dl = __shfl(delta, bb, 64);
        if (p < trows && bb != drop_bin) {
            U* o = bb == redirect_bin ? r_u : d_u;
            o[(p + dl) * UPR + part] = img[u];
        }
    }
}

// ---------------------------------------------------------- halo (f1)
// exchange_overload_by_position (redist.py:202-309) selects, per dimension
// d, the rows with position[:, d] > limits[d,1] - ol[d] (sent to the right
// neighbour, :271/:274) and position[:, d] < limits[d,0] + ol[d] (to the
// left, :272/:275).  numpy compares the float32/float64 column against the
// float64 threshold in float64 (exact), NaN selects nothing.
struct HaloThr { double hi[MGR_MAX_DIM]; double lo[MGR_MAX_DIM]; };

// flags[r] bit 2d: coordinate d > hi[d]; bit 2d+1: coordinate d < lo[d].
template <typename PosT>
__global__ __launch_bounds__(kBlock) void halo_flags_kernel(const PosT* __restrict__ pos,
                                                            int64_t n, int64_t stride, int dim,
                                                            HaloThr t,
                                                            uint16_t* __restrict__ flags) {
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t r = blockIdx.x * (int64_t)kBlock + threadIdx.x; r < n; r += step) {
        unsigned f = 0;
        for (int d = 0; d < dim; ++d) {
            const double x = sizeof(PosT) == 4 ? f32_to_f64_x86((float)pos[r * stride + d])
                                               : (double)pos[r * stride + d];
            f |= (x > t.hi[d] ? 1u : 0u) << (2 * d);
            f |= (x < t.lo[d] ? 1u : 0u) << (2 * d + 1);
        }
        flags[r] = (uint16_t)f;
    }
}

// Selection as a 2-bin partition for mgr_scan / mgr_pack: bin 0 = selected
// ((flags & mask) != 0), bin 1 = not (the drop bin).  Wave-private tiles of
// tile_rows rows; counts[b * T + tile].
__global__ __launch_bounds__(kBlock) void select_count_kernel(const uint16_t* __restrict__ flags,
                                                              int64_t n, unsigned mask,
                                                              uint8_t* __restrict__ dest,
                                                              int32_t* __restrict__ counts,
                                                              int64_t T, int tile_rows) {
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = (int64_t)blockIdx.x * kWaves + w;
    if (tile >= T) return;
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    int sel = 0, all = 0;
    for (int r0 = 0; r0 < rows; r0 += 64) {
        const bool valid = r0 + lane < rows;
        bool on = false;
        if (valid) {
            on = (flags[row0 + r0 + lane] & mask) != 0;
            dest[row0 + r0 + lane] = on ? 0 : 1;
        }
        sel += __popcll(__ballot(on));
        all += __popcll(__ballot(valid));
    }
    if (lane == 0) {
        counts[tile] = sel;
        counts[T + tile] = all - sel;
    }
}

// --------------------------------------------------------- synthetic data
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Box8 { double v[MGR_MAX_DIM]; };

__global__ __launch_bounds__(kBlock) void synth_uniform_kernel(uint64_t seed, int64_t gid0,
                                                               int64_t n, int dim, Box8 box,
                                                               double* __restrict__ pos,
                                                               double* __restrict__ rec) {
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += step) {
        const uint64_t gid = (uint64_t)(gid0 + i);
        double c[MGR_MAX_DIM];
#pragma unroll
        for (int d = 0; d < MGR_MAX_DIM; ++d) {
            if (d < dim) {
                const uint64_t h = splitmix64(seed ^ (3ull * gid + (uint64_t)d));
                c[d] = (double)(h >> 11) * 0x1.0p-53 * box.v[d];
                if (pos) pos[i * dim + d] = c[d];
            }
        }
        if (rec) {
            double2* r2 = (double2*)(rec + i * 4);
            r2[0] = make_double2(c[0], c[1]);
            double2 t;
            t.x = c[2];
            long long id = (long long)gid;
            t.y = __longlong_as_double(id);
            r2[1] = t;
        }
    }
}

// ============================================================ launchers
static int grid_for(int64_t n, int per_block_rows = kBlock) {
    int64_t g = (n + per_block_rows - 1) / per_block_rows;
    if (g > 256 * 16) g = 256 * 16;   // grid-stride beyond 16 blocks per CU
    return (int)(g < 1 ? 1 : g);
}

int64_t num_tiles(int64_t n, int tile_rows) { return (n + tile_rows - 1) / tile_rows; }

int dest_bytes(int nbins) { return nbins <= 256 ? 1 : (nbins <= 65536 ? 2 : 4); }

int nbits_for(int nbins) {
    int b = 0;
    while ((1 << b) < nbins) ++b;
    return b;
}

static int64_t a256(int64_t x) { return (x + 255) & ~(int64_t)255; }

int64_t workspace_bytes(int64_t n, int nbins, int tile_rows) {
    const int64_t T = num_tiles(n, tile_rows);
    const int64_t M = (int64_t)nbins * (T > 0 ? T : 1);
    return a256(M * 4) + a256(M * 8) + a256((nbins + 1) * 8) + a256(kScanMaxBlocks * 8);
}

Workspace carve(void* base, int64_t n, int nbins, int tile_rows) {
    Workspace ws;
    ws.T = num_tiles(n, tile_rows);
    const int64_t M = (int64_t)nbins * (ws.T > 0 ? ws.T : 1);
    char* p = (char*)base;
    ws.counts = (int32_t*)p;     p += a256(M * 4);
    ws.offsets = (int64_t*)p;    p += a256(M * 8);
    ws.bin_starts = (int64_t*)p; p += a256((nbins + 1) * 8);
    ws.partials = (int64_t*)p;
    return ws;
}

template <typename K>
static void ensure_lds(K kernel, int bytes) {
    if (bytes > 64 * 1024)
        (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Waves per workgroup for a per-wave LDS footprint: 4 when a 4-wave
// workgroup stays within 64 KiB, fewer otherwise (never above 160 KiB).
static int waves_per_block(int per_wave_lds) {
    if (per_wave_lds * kWaves <= 64 * 1024) return kWaves;
    int w = (160 * 1024) / (per_wave_lds > 0 ? per_wave_lds : 1);
    return w < 1 ? 1 : (w > kWaves ? kWaves : w);
}

template <typename PosT, bool kP, typename DestT, int NU, int DIM>
static hipError_t bin_count_t(const Geom& g, void* pos, int64_t n, int64_t stride, void* dest,
                              int tile_rows, const Workspace& ws, hipStream_t s) {
    // nontemporal slab loads/stores always (every A/B favoured them); one or
    // two slabs in flight per wave (deeper measured no faster)
    auto k = g_tune.bin_depth >= 2 ? bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 2>
                                   : bin_count_kernel<PosT, kP, DestT, NU, DIM, true, 1>;
    const int rb = (int)(stride * (int64_t)sizeof(PosT));
    const int per_wave = NU > 0 ? align16(64 * rb) : 0;     // staging slab
    int nwaves = tile_rows / 64;                 // <= bin_waves waves, whole rounds each
    while (nwaves > g_tune.bin_waves || (tile_rows / 64) % nwaves) --nwaves;
    const int lds = align16(g.nbins * 4) + per_wave * nwaves;
    ensure_lds(k, lds);
    hipLaunchKernelGGL(k, dim3((unsigned)ws.T), dim3(64 * nwaves), (size_t)lds, s, (PosT*)pos, n,
                       stride, g, (DestT*)dest, ws.counts, ws.T, tile_rows, per_wave,
                       g_tune.bin_skip_clean, g_tune.xcd_bin);
    return hipGetLastError();
}

template <typename PosT, bool kP, typename DestT, int NU>
static hipError_t bin_count_dim(const Geom& g, void* pos, int64_t n, int64_t stride, void* dest,
                                int tile_rows, const Workspace& ws, hipStream_t s) {
    switch (g.dim) {
        case 1: return bin_count_t<PosT, kP, DestT, NU, 1>(g, pos, n, stride, dest, tile_rows, ws, s);
        case 2: return bin_count_t<PosT, kP, DestT, NU, 2>(g, pos, n, stride, dest, tile_rows, ws, s);
        case 3: return bin_count_t<PosT, kP, DestT, NU, 3>(g, pos, n, stride, dest, tile_rows, ws, s);
        default: return bin_count_t<PosT, kP, DestT, NU, 0>(g, pos, n, stride, dest, tile_rows, ws, s);
    }
}

template <typename PosT, bool kP, typename DestT>
static hipError_t bin_count_w(const Geom& g, void* pos, int64_t n, int64_t stride, void* dest,
                              int tile_rows, const Workspace& ws, hipStream_t s) {
    const int64_t rb = stride * (int64_t)sizeof(PosT);
    if (g_tune.bin_staged && rb <= kStageMaxRowBytes && ((uintptr_t)pos & 15) == 0) {
        switch ((int)((rb + 15) / 16)) {   // 16-byte units per lane per 64-row slab
            case 1: return bin_count_dim<PosT, kP, DestT, 1>(g, pos, n, stride, dest, tile_rows, ws, s);
            case 2: return bin_count_dim<PosT, kP, DestT, 2>(g, pos, n, stride, dest, tile_rows, ws, s);
            case 3: return bin_count_dim<PosT, kP, DestT, 3>(g, pos, n, stride, dest, tile_rows, ws, s);
            default: return bin_count_dim<PosT, kP, DestT, 4>(g, pos, n, stride, dest, tile_rows, ws, s);
        }
    }
    return bin_count_dim<PosT, kP, DestT, 0>(g, pos, n, stride, dest, tile_rows, ws, s);
}

template <typename PosT, typename DestT>
static hipError_t bin_count_p(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                              void* dest, int tile_rows, const Workspace& ws, hipStream_t s) {
    return periodic ? bin_count_w<PosT, true, DestT>(g, pos, n, stride, dest, tile_rows, ws, s)
                    : bin_count_w<PosT, false, DestT>(g, pos, n, stride, dest, tile_rows, ws, s);
}

template <typename PosT>
static hipError_t bin_count_d(const Geom& g, void* pos, int64_t n, int64_t stride, int periodic,
                              void* dest, int tile_rows, const Workspace& ws, hipStream_t s) {
    if (dest_bytes(g.nbins) == 1)
        return bin_count_p<PosT, uint8_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s);
    return bin_count_p<PosT, uint16_t>(g, pos, n, stride, periodic, dest, tile_rows, ws, s);
}

hipError_t launch_bin_count(const Geom& g, void* pos, int pos_f32, int64_t n, int64_t stride,
                            int periodic, void* dest, int tile_rows, const Workspace& ws,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    prof_begin(s, K_BIN_COUNT);
    hipError_t e = pos_f32 ? bin_count_d<float>(g, pos, n, stride, periodic, dest, tile_rows, ws, s)
                           : bin_count_d<double>(g, pos, n, stride, periodic, dest, tile_rows, ws, s);
    prof_end(s, K_BIN_COUNT);
    return e;
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

hipError_t launch_cell_ids(const Geom& g, void* pos, int pos_f32, int64_t n, int64_t stride,
                           int periodic, int64_t* cell, int64_t* idx, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    prof_begin(s, K_CELL_IDS);
    hipError_t e = pos_f32 ? cell_ids_t<float>(g, pos, n, stride, periodic, cell, idx, s)
                           : cell_ids_t<double>(g, pos, n, stride, periodic, cell, idx, s);
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
                       per_wave);
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

hipError_t launch_scan(int64_t n, int nbins, int tile_rows, const Workspace& ws,
                       int64_t* bin_counts, hipStream_t s) {
    if (n <= 0 || ws.T == 0) {
        hipError_t e = hipMemsetAsync(ws.bin_starts, 0, (size_t)(nbins + 1) * 8, s);
        if (e == hipSuccess && bin_counts) e = hipMemsetAsync(bin_counts, 0, (size_t)nbins * 8, s);
        return e;
    }
    const int64_t M = (int64_t)nbins * ws.T;
    int64_t G = (M + 2047) / 2048;
    if (G > kScanMaxBlocks) G = kScanMaxBlocks;
    if (G < 1) G = 1;
    int64_t chunk = (M + G - 1) / G;
    G = (M + chunk - 1) / chunk;
    prof_begin(s, K_SCAN_REDUCE);
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)G), dim3(kBlock), 0, s, ws.counts, M,
                       chunk, ws.partials);
    prof_end(s, K_SCAN_REDUCE);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    prof_begin(s, K_SCAN_APPLY);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)G), dim3(kBlock), 0, s, ws.counts, M,
                       chunk, ws.partials, ws.offsets, ws.T, ws.bin_starts, nbins);
    prof_end(s, K_SCAN_APPLY);
    e = hipGetLastError();
    if (e != hipSuccess || !bin_counts) return e;
    prof_begin(s, K_BIN_TOTALS);
    hipLaunchKernelGGL(bin_totals_kernel, dim3((nbins + 255) / 256), dim3(256), 0, s,
                       ws.bin_starts, nbins, bin_counts);
    prof_end(s, K_BIN_TOTALS);
    return hipGetLastError();
}

// pack_many_kernel tiles: 64 rounds (4096 rows) up to 512 bins, 32 rounds up
// to 1024 bins -- the uint16 [rounds][nbins] LDS table stays <= 64 KiB.
static int many_tile_rows(int nbins) { return nbins <= 512 ? 4096 : 2048; }

int pack_tile_rows(int64_t row_bytes, int nbins) {
    if (g_tune.tile_rounds > 0) return 64 * g_tune.tile_rounds;
    // <= 16 bins: 512-row tiles (bin: 4 waves x 2 rounds; pack: 8 waves x
    // 1 round; A/B against 1024 at 8 bins: bin -3 %, pack within noise);
    // <= 64 bins: 1024 rows (64 bins: pack 0.92 vs 1.07 ms at 512: longer
    // same-bin runs); more bins: longer tiles keep the [nbins][tiles]
    // histogram small next to the payload.
    if (nbins <= 16) return 512 * g_tune.pack_rpw;
    if (nbins <= 64) return 1024 * g_tune.pack_rpw;
    if (g_tune.pack_many && nbins <= 1024 && row_bytes <= 64) return many_tile_rows(nbins);
    int r = 16;
    while (r < kMaxTileRows / 64 && (int64_t)nbins * 4 > (int64_t)r * 8) r *= 2;
    return 64 * r;
}

template <int W, typename DestT, bool kWide>
static hipError_t pack_t(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nb,
                         int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                         int redirect_bin, void* redirect_dst, hipStream_t s) {
    auto k = pack_kernel<W, DestT, kWide>;
    const int per_wave = align16(nb * 8) + align16(nb * 4);
    const int wpb = waves_per_block(per_wave);
    const int lds = per_wave * wpb;
    ensure_lds(k, lds);
    const int64_t grid = (ws.T + wpb - 1) / wpb;
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * wpb), (size_t)lds, s,
                       (const uint8_t*)src, row_bytes / W, n, (const DestT*)dest, nb,
                       nbits_for(nb), drop_bin, ws.offsets, ws.bin_starts, ws.T, tile_rows,
                       per_wave, (uint8_t*)dst, redirect_bin, (uint8_t*)redirect_dst);
    return hipGetLastError();
}

template <int W, int UPR>
static hipError_t pack_small_u(const void* src, int64_t n, const void* dest, int nb, int drop_bin,
                               int tile_rows, const Workspace& ws, void* dst, int redirect_bin,
                               void* redirect_dst, hipStream_t s) {
    if (g_tune.pack_sorted && tile_rows <= 1024) {
        const int threads = tile_rows;   // one wave per 64-row round of the tile
        const int lds = tile_rows * UPR * W + (tile_rows / 64) * 64 * 4 + tile_rows;
#define MGR_PSS(NT_)                                                                          \
        {                                                                                     \
        ensure_lds(pack_sorted_kernel<W, UPR, NT_>, lds);                                      \
        hipLaunchKernelGGL((pack_sorted_kernel<W, UPR, NT_>), dim3((unsigned)ws.T), dim3(threads), \
                           (size_t)lds, s, (const uint8_t*)src, n, (const uint8_t*)dest, nb,   \
                           nbits_for(nb), drop_bin, ws.offsets, ws.bin_starts, ws.T, tile_rows, \
                           (uint8_t*)dst, redirect_bin, (uint8_t*)redirect_dst, g_tune.xcd_pack); }
        if (g_tune.pack_nt) MGR_PSS(true)
        else MGR_PSS(false)
#undef MGR_PSS
        return hipGetLastError();
    }
    if (g_tune.pack_coop) {
        // one wave per RPW 64-row rounds of the tile (<= 16 waves)
        const int rpw = tile_rows > 1024 ? 2 : 1;
        const int threads = tile_rows / rpw;
#define MGR_PCK(NT_, RPW_, NTS_)                                                              \
        hipLaunchKernelGGL((pack_coop_kernel<W, UPR, NT_, RPW_, NTS_>), dim3((unsigned)ws.T), \
                           dim3(threads), 0, s, (const uint8_t*)src, n, (const uint8_t*)dest, nb, \
                           nbits_for(nb), drop_bin, ws.offsets, ws.bin_starts, ws.T, tile_rows, \
                           (uint8_t*)dst, redirect_bin, (uint8_t*)redirect_dst, g_tune.xcd_pack)
        if (g_tune.pack_nt >= 2) {
            if (rpw == 2) MGR_PCK(true, 2, true); else MGR_PCK(true, 1, true);
        } else if (g_tune.pack_nt == 1) {
            if (rpw == 2) MGR_PCK(true, 2, false); else MGR_PCK(true, 1, false);
        } else {
            if (rpw == 2) MGR_PCK(false, 2, false); else MGR_PCK(false, 1, false);
        }
#undef MGR_PCK
        return hipGetLastError();
    }
    const int64_t grid = (ws.T + kWaves - 1) / kWaves;
#define MGR_PSK(NT_, NTS_)                                                                  \
    hipLaunchKernelGGL((pack_small_kernel<W, UPR, NT_, NTS_>), dim3((unsigned)grid), dim3(kBlock), \
                       0, s, (const uint8_t*)src, n, (const uint8_t*)dest, nb, nbits_for(nb),    \
                       drop_bin, ws.offsets, ws.bin_starts, ws.T, tile_rows, (uint8_t*)dst,     \
                       redirect_bin, (uint8_t*)redirect_dst)
    if (g_tune.pack_nt >= 2) MGR_PSK(true, true);
    else if (g_tune.pack_nt == 1) MGR_PSK(true, false);
    else MGR_PSK(false, false);
#undef MGR_PSK
    return hipGetLastError();
}

// Compile-time units per row for rows of <= 64 bytes in 16/8/4-byte units
// (registers, no scratch); returns hipErrorNotSupported for other shapes.
template <int W>
static hipError_t pack_small_t(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                               int nb, int drop_bin, int tile_rows, const Workspace& ws,
                               void* dst, int redirect_bin, void* redirect_dst, hipStream_t s) {
#define MGR_PS(U_) case U_: return pack_small_u<W, U_>(src, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    if (W >= 4) {
        switch ((int)(row_bytes / W)) {
            MGR_PS(1) MGR_PS(2) MGR_PS(3) MGR_PS(4)
            default: break;
        }
        if (W <= 8) {
            switch ((int)(row_bytes / W)) {
                MGR_PS(5) MGR_PS(6) MGR_PS(7) MGR_PS(8)
                default: break;
            }
        }
        if (W == 4) {
            switch ((int)(row_bytes / W)) {
                MGR_PS(9) MGR_PS(10) MGR_PS(11) MGR_PS(12) MGR_PS(13) MGR_PS(14) MGR_PS(15) MGR_PS(16)
                default: break;
            }
        }
    }
#undef MGR_PS
    return hipErrorNotSupported;
}

template <int W, int UPR, typename DestT>
static hipError_t pack_many_u(const void* src, int64_t n, const void* dest, int nb, int drop_bin,
                              int tile_rows, const Workspace& ws, void* dst, int redirect_bin,
                              void* redirect_dst, hipStream_t s) {
    const int lds = align16(nb * 8) + (tile_rows / 64) * nb * 2;
#define MGR_PMK(RPW_)                                                                          \
    {                                                                                          \
        auto k = pack_many_kernel<W, UPR, DestT, RPW_>;                                        \
        ensure_lds(k, lds);                                                                    \
        hipLaunchKernelGGL(k, dim3((unsigned)ws.T), dim3(1024), (size_t)lds, s,                \
                           (const uint8_t*)src, n, (const DestT*)dest, nb, nbits_for(nb),      \
                           drop_bin, ws.offsets, ws.bin_starts, ws.T, tile_rows, (uint8_t*)dst, \
                           redirect_bin, (uint8_t*)redirect_dst, g_tune.xcd_pack);             \
    }
    if (tile_rows == 4096) MGR_PMK(4)
    else MGR_PMK(2)
#undef MGR_PMK
    return hipGetLastError();
}

template <int W, typename DestT>
static hipError_t pack_many_t(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                              int nb, int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                              int redirect_bin, void* redirect_dst, hipStream_t s) {
#define MGR_PM(U_) case U_: return pack_many_u<W, U_, DestT>(src, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    switch ((int)(row_bytes / W)) {
        MGR_PM(1) MGR_PM(2) MGR_PM(3) MGR_PM(4)
        default: break;
    }
    if (W <= 8) {
        switch ((int)(row_bytes / W)) {
            MGR_PM(5) MGR_PM(6) MGR_PM(7) MGR_PM(8)
            default: break;
        }
    }
    if (W == 4) {
        switch ((int)(row_bytes / W)) {
            MGR_PM(9) MGR_PM(10) MGR_PM(11) MGR_PM(12) MGR_PM(13) MGR_PM(14) MGR_PM(15) MGR_PM(16)
            default: break;
        }
    }
#undef MGR_PM
    return hipErrorNotSupported;
}

template <int W>
static hipError_t pack_w(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nb,
                         int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                         int redirect_bin, void* redirect_dst, hipStream_t s) {
    if constexpr (W >= 4) {
        if (g_tune.pack_many && nb > 64 && nb <= 1024 && row_bytes <= 64 &&
            tile_rows == many_tile_rows(nb)) {
            const hipError_t e = dest_bytes(nb) == 1
                ? pack_many_t<W, uint8_t>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s)
                : pack_many_t<W, uint16_t>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
            if (e != hipErrorNotSupported) return e;
        }
    }
    if (g_tune.pack_small && nb <= 64 && row_bytes <= 64 && W >= 4) {
        const hipError_t e = pack_small_t<W>(src, row_bytes, n, dest, nb, drop_bin, tile_rows,
                                             ws, dst, redirect_bin, redirect_dst, s);
        if (e != hipErrorNotSupported) return e;
    }
    const bool wide = row_bytes > 256;
    if (dest_bytes(nb) == 1)
        return wide ? pack_t<W, uint8_t, true>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s)
                    : pack_t<W, uint8_t, false>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    return wide ? pack_t<W, uint16_t, true>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s)
                : pack_t<W, uint16_t, false>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
}

hipError_t launch_pack(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                       int nbins, int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                       int redirect_bin, void* redirect_dst, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    // Widest unit dividing the row and every base address.
    uintptr_t a = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)row_bytes;
    if (redirect_dst) a |= (uintptr_t)redirect_dst;
    prof_begin(s, K_PACK);
    hipError_t e;
    if ((a & 15) == 0) e = pack_w<16>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    else if ((a & 7) == 0) e = pack_w<8>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    else if ((a & 3) == 0) e = pack_w<4>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    else if ((a & 1) == 0) e = pack_w<2>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    else e = pack_w<1>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    prof_end(s, K_PACK);
    return e;
}

hipError_t launch_halo_flags(const void* pos, int pos_f32, int64_t n, int64_t stride, int dim,
                             const double* hi, const double* lo, uint16_t* flags, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    HaloThr t;
    for (int d = 0; d < MGR_MAX_DIM; ++d) {
        t.hi[d] = d < dim ? hi[d] : 0.0;
        t.lo[d] = d < dim ? lo[d] : 0.0;
    }
    prof_begin(s, K_HALO);
    if (pos_f32)
        hipLaunchKernelGGL(halo_flags_kernel<float>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                           (const float*)pos, n, stride, dim, t, flags);
    else
        hipLaunchKernelGGL(halo_flags_kernel<double>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                           (const double*)pos, n, stride, dim, t, flags);
    prof_end(s, K_HALO);
    return hipGetLastError();
}

hipError_t launch_select_count(const uint16_t* flags, int64_t n, unsigned mask, uint8_t* dest,
                               int tile_rows, const Workspace& ws, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t grid = (ws.T + kWaves - 1) / kWaves;
    prof_begin(s, K_HALO);
    hipLaunchKernelGGL(select_count_kernel, dim3((unsigned)grid), dim3(kBlock), 0, s, flags, n,
                       mask, dest, ws.counts, ws.T, tile_rows);
    prof_end(s, K_HALO);
    return hipGetLastError();
}

hipError_t launch_synth_uniform(uint64_t seed, int64_t gid0, int64_t n, int dim,
                                const double* box, double* pos, void* rec32, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    Box8 b;
    for (int d = 0; d < MGR_MAX_DIM; ++d) b.v[d] = d < dim ? box[d] : 0.0;
    prof_begin(s, K_SYNTH);
    hipLaunchKernelGGL(synth_uniform_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, seed, gid0, n,
                       dim, b, pos, (double*)rec32);
    prof_end(s, K_SYNTH);
    return hipGetLastError();
}

}  // namespace mgr
