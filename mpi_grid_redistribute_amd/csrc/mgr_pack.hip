// Pack kernels of the hot path (gfx950): the stable partition of every
// payload field into the bin-major send buffer / output (redist.py:195-198,
// send_buff[i] = data[rank_to_send == i], order kept), with their launchers
// and tile-size policy.  Helpers: mgr_device.h.
#include <vector>

#include "mgr_device.h"

namespace mgr {


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
    int64_t t0, int64_t tn, int tile_rows, int per_wave_lds, uint8_t* __restrict__ dst,
    int redirect_bin, uint8_t* __restrict__ redirect_dst, const uint32_t* __restrict__ scan_err) {
    using U = typename Unit<W>::T;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tl = (int64_t)blockIdx.x * (blockDim.x >> 6) + w;
    if (tl >= tn || scan_failed(scan_err)) return;
    const int64_t tile = t0 + tl;
    int64_t* goff = (int64_t*)(smem + w * per_wave_lds);
    int32_t* run = (int32_t*)(smem + w * per_wave_lds + align16(nb * 8));
    for (int b = lane; b < nb; b += 64) {
        goff[b] = seg_start(offsets, bin_starts, T, tile, b, redirect_bin);
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

// Block-cooperative pack for <= 64 bins and rows of <= 64 bytes: one
// workgroup per tile of R rounds, wave w ranks and moves round w (64 rows)
// in one shot -- the short-lived, fully parallel shape that streams best.
// The waves exchange their per-bin counts through a [R][64] LDS table (one
// barrier) to get each bin's base inside the tile.  Unit-transposed moves:
// lane l moves W-byte units 64k + l of the round, so each load instruction
// reads 64*W contiguous bytes; the unit's row gets its slot by shfl.
// (A/B, same box: issuing every load branch-free before the first wait, as
// the image pack does, made this kernel slower -- 0.86 vs 0.77 ms at config 2
// -- so the destination bytes are waited for before the payload loads go out.)
template <int W, int UPR, int RPW>
__global__ __launch_bounds__(1024) void pack_coop_kernel(
    const uint8_t* __restrict__ src, int64_t n, const uint8_t* __restrict__ dest, int nb,
    int nbits, int drop_bin, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ bin_starts, int64_t T, int64_t t0, int64_t tn, int tile_rows,
    uint8_t* __restrict__ dst, int redirect_bin, uint8_t* __restrict__ redirect_dst, int xcd,
    int sel, const uint32_t* __restrict__ scan_err, const uint16_t* __restrict__ id_src,
    uint16_t* __restrict__ id_dst, uint16_t* __restrict__ id_red) {
    using U = typename Unit<W>::T;
    __shared__ int s_cnt[kCoopMaxRounds][64];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = t0 + (xcd ? xcd_tile_c(blockIdx.x, tn, xcd) : (int64_t)blockIdx.x);
    // wave w moves rounds w*RPW .. w*RPW+RPW-1 of the tile
    const int64_t row0 = tile * (int64_t)tile_rows + 64 * RPW * w;
    // issue every load of the wave's rounds first
    int nr[RPW];
    unsigned b[RPW];
    U v[RPW][UPR];
    unsigned idv[RPW];   // side field: every row's 2-byte id (fine cell), moved alike
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        nr[q] = (int)max((int64_t)0, min((int64_t)64, n - row0 - 64 * q));
        b[q] = lane < nr[q] ? (unsigned)dest[row0 + 64 * q + lane] : 0u;
        idv[q] = id_src && lane < nr[q] ? (unsigned)id_src[row0 + 64 * q + lane] : 0u;
    }
    long long tbase = 0;
    if (lane < nb) tbase = seg_start(offsets, bin_starts, T, tile, lane, redirect_bin);
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const U* __restrict__ sp = (const U*)src + (row0 + 64 * q) * UPR;
        if (sel) {
            // selection (most rows dropped): load only the units of kept rows
#pragma unroll
            for (int k = 0; k < UPR; ++k) {
                const int u = 64 * k + lane;
                const int rb = __shfl((int)b[q], u / UPR, 64);
                if (u < nr[q] * UPR && rb != drop_bin) v[q][k] = sp[u];
            }
        } else {
#pragma unroll
            for (int k = 0; k < UPR; ++k)
                if (64 * k + lane < nr[q] * UPR) v[q][k] = sp[64 * k + lane];
        }
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
    if (scan_failed(scan_err)) return;
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
        if (id_src && tgt >= 0)
            ((tgt >> 62) ? id_red : id_dst)[tgt & ((1ll << 62) - 1)] = (uint16_t)idv[q];
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

// Multi-field (SoA) pack in the cooperative shape of pack_coop_kernel, for
// the common field signatures (compile time): one wave per 64-row round,
// the round ranked ONCE for every field (ballot match, per-bin bases through
// LDS behind one barrier), then every field's rows moved straight from
// registers -- unit-transposed: lane l loads the W-byte units 64 k + l of
// the field's round (each load instruction reads 64 W contiguous bytes), the
// unit's row gets its slot by shfl, same-bin rows of a round land in
// consecutive slots (contiguous runs that L2 merges with the neighbouring
// rounds').  No LDS image: a few instructions per field and round, where the
// image kernel (pack_fields_kernel) spends a permutation and a 16-byte unit
// walk per field.  CF<U>: one field, U = W * 32 + UPR (UPR = row_bytes / W
// units of W bytes), 0 = no field.
template <int U>
struct CoopField {
    static constexpr int W = U >> 5, UPR = U & 31;
    using T = typename Unit<(W ? W : 4)>::T;
    T v[UPR ? UPR : 1];
    __device__ __forceinline__ void load(const uint8_t* __restrict__ src, int64_t row0, int nr,
                                         int lane) {
        if constexpr (U != 0) {
            const T* __restrict__ sp = (const T*)src + row0 * UPR;
#pragma unroll
            for (int k = 0; k < UPR; ++k)
                if (64 * k + lane < nr * UPR) v[k] = sp[64 * k + lane];
        }
    }
    // tgt: this lane's row's slot (bit 62: the redirect output), < 0: not written
    __device__ __forceinline__ void store(uint8_t* __restrict__ dst, uint8_t* __restrict__ red,
                                          long long tgt, int nr, int lane) const {
        if constexpr (U != 0) {
            T* __restrict__ d_u = (T*)dst;
            T* __restrict__ r_u = (T*)red;
#pragma unroll
            for (int k = 0; k < UPR; ++k) {
                const int u = 64 * k + lane;
                const int r = u / UPR, part = u - r * UPR;
                const long long t = __shfl(tgt, r, 64);
                if (u < nr * UPR && t >= 0) {
                    T* o = (t >> 62) ? r_u : d_u;
                    o[(t & ((1ll << 62) - 1)) * UPR + part] = v[k];
                }
            }
        }
    }
};

struct CoopFieldPtrs {
    const uint8_t* src[4];
    uint8_t* dst[4];
    uint8_t* red[4];
};

template <int U0, int U1, int U2, int U3>
__global__ __launch_bounds__(1024) void pack_coop_fields_kernel(
    CoopFieldPtrs fp, int64_t n, const uint8_t* __restrict__ dest, int nb, int nbits,
    int drop_bin, const int64_t* __restrict__ offsets, const int64_t* __restrict__ bin_starts,
    int64_t T, int64_t t0, int64_t tn, int tile_rows, int redirect_bin, int xcd,
    const uint32_t* __restrict__ scan_err, const uint16_t* __restrict__ id_src,
    uint16_t* __restrict__ id_dst, uint16_t* __restrict__ id_red) {
    __shared__ int s_cnt[kCoopMaxRounds][64];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = t0 + (xcd ? xcd_tile_c(blockIdx.x, tn, xcd) : (int64_t)blockIdx.x);
    const int64_t row0 = tile * (int64_t)tile_rows + 64 * w;
    const int nr = (int)max((int64_t)0, min((int64_t)64, n - row0));
    // the destination bytes first, waited for, then every field's loads
    // (pack_coop_kernel: 0.77 vs 0.86 ms against issuing everything at once)
    const unsigned b = lane < nr ? (unsigned)dest[row0 + lane] : 0u;
    const unsigned idv = id_src && lane < nr ? (unsigned)id_src[row0 + lane] : 0u;
    long long tbase = 0;
    if (lane < nb) tbase = seg_start(offsets, bin_starts, T, tile, lane, redirect_bin);
    CoopField<U0> f0;
    CoopField<U1> f1;
    CoopField<U2> f2;
    CoopField<U3> f3;
    f0.load(fp.src[0], row0, nr, lane);
    f1.load(fp.src[1], row0, nr, lane);
    f2.load(fp.src[2], row0, nr, lane);
    f3.load(fp.src[3], row0, nr, lane);
    // rank inside the round; lane l counts bin l
    const bool valid = lane < nr;
    unsigned long long pe = __ballot(valid), mine = pe;
    for (int i = 0; i < nbits; ++i) {
        const unsigned long long m = __ballot((b >> i) & 1u);
        pe &= ((b >> i) & 1u) ? m : ~m;
        mine &= ((lane >> i) & 1) ? m : ~m;
    }
    if (!valid) pe = 0ull;
    s_cnt[w][lane] = __popcll(mine);
    __syncthreads();
    if (scan_failed(scan_err)) return;
    for (int j = 0; j < w; ++j) tbase += s_cnt[j][lane];
    const long long base = __shfl(tbase, (int)b, 64);
    long long tgt = -1;
    if (valid && (int)b != drop_bin)
        tgt = (base + rank_in(pe)) | ((int)b == redirect_bin ? (1ll << 62) : 0ll);
    if (id_src && tgt >= 0) ((tgt >> 62) ? id_red : id_dst)[tgt & ((1ll << 62) - 1)] = (uint16_t)idv;
    f0.store(fp.dst[0], fp.red[0], tgt, nr, lane);
    f1.store(fp.dst[1], fp.red[1], tgt, nr, lane);
    f2.store(fp.dst[2], fp.red[2], tgt, nr, lane);
    f3.store(fp.dst[3], fp.red[3], tgt, nr, lane);
}

// Multi-selection pack (the halo's sends, msel counts + mgr_scan with nbins
// = nsets), up to kSelFields fields of the same rows in one launch.  Set k's
// rows of field f go, in row order, to dsts[f][k] (null: set k is not
// written), so one launch places a set straight where it is consumed (a
// staging buffer for a neighbour, or the halo store itself when the
// neighbour is this rank).  One wave per tile, kSelChunk rows at a time: the
// chunk's flags are read once (chunk_flags); per set, the lanes' membership
// masks and a wave prefix list the set's rows in row order in LDS (u16 entry:
// chunk row | set << 10), the sets one after the other; then one copy loop
// per field moves every listed row -- 64 / upr rows per instruction, W-byte
// units (the widest the field's alignment allows), groups of kSelDepth
// instructions, two groups in flight -- to its set's next output row.  Rows
// wider than 64 units are copied one after the other, lanes across the row.
// The gathers read whole lines for sparse rows (PMC: 3.3 GB read for 1.3 GB
// of rows at the halo's density), so the kernel runs near the HBM rate of
// the lines it must touch (profiles/round4/ab_notes.md).
constexpr int kSelCap = 2048;   // LDS entries per wave (>= kSelChunk)
static_assert(kSelCap >= kSelChunk, "a set of one chunk must fit an empty list");
constexpr int kSelDepth = 4;    // copy instructions per group (round 3: 8 in flight, 1.17 vs 1.10 ms)
constexpr int kSelFields = 3;
struct SelFields {
    const uint8_t* src[kSelFields];
    int64_t row_bytes[kSelFields];
    int wlog[kSelFields];                 // log2 of the copy unit
    uint8_t* dst[kSelFields][kMaxSets];
};

// Lanes without a row (past the list's end, or past cap) store to a per-wave
// slot of this buffer, so every copy group issues exactly kSelDepth loads and
// kSelDepth stores: the counts s_waitcnt works with stay static.
__device__ uint4 g_sel_trash[256][64];

template <int W>
__device__ __forceinline__ void sel_copy(const uint8_t* __restrict__ src, int64_t row_bytes,
                                         uint8_t* const* dst, const long long* at,
                                         const int* start, const uint16_t* list, int fill,
                                         int lane, long long cap, uint8_t* trash) {
    // global address space throughout: pointers read from LDS or by readlane
    // are generic to the compiler, and a flat access counts on lgkmcnt too, so
    // every LDS read of the list waited for all copies in flight
    using U = __attribute__((address_space(1))) typename Unit<W>::T;
    const int64_t upr = row_bytes / W;
    const U* sp = (const U*)src;
    if (upr <= 64) {
        const int per = 64 / (int)upr;   // rows per copy instruction
        const int lr = lane / (int)upr;
        const int u = lane - lr * (int)upr;
        const int step = kSelDepth * per;
        const int ng = (fill + step - 1) / step;
        // group g: kSelDepth loads into v, targets into o (entry 0 of the
        // list, a row of this chunk, stands in for a lane without a row)
        auto load = [&](int g, typename Unit<W>::T (&v)[kSelDepth], U* (&o)[kSelDepth]) {
#pragma unroll
            for (int q = 0; q < kSelDepth; ++q) {
                const int i = g * step + q * per + lr;
                const bool ok = lr < per && i < fill;
                const unsigned e = list[ok ? i : 0];
                const int k = (int)(e >> 10);
                const long long row = at[k] + (i - start[k]);
                o[q] = ok && row < cap ? (U*)dst[k] + row * upr + u : (U*)trash;
                v[q] = sp[(int64_t)(e & 1023u) * upr + u];
            }
        };
        auto store = [&](const typename Unit<W>::T (&v)[kSelDepth], U* const (&o)[kSelDepth]) {
#pragma unroll
            for (int q = 0; q < kSelDepth; ++q) *o[q] = v[q];
        };
        // two groups in flight: group g+1's loads are issued before group g's
        // stores, so waiting for a group's loads never waits for the stores
        // before it (one vmcnt counts loads and stores, retired in order)
        typename Unit<W>::T va[kSelDepth], vb[kSelDepth];
        U* oa[kSelDepth];
        U* ob[kSelDepth];
        load(0, va, oa);
        for (int g = 0;; g += 2) {
            load(g + 1, vb, ob);
            store(va, oa);
            if (g + 1 >= ng) break;
            load(g + 2, va, oa);
            store(vb, ob);
            if (g + 2 >= ng) break;
        }
    } else {
        for (int i = 0; i < fill; ++i) {
            const unsigned e = list[i];
            const int k = (int)(e >> 10);
            const long long row = at[k] + (i - start[k]);
            if (row >= cap) continue;
            const U* rs = sp + (int64_t)(e & 1023u) * upr;
            U* rd = (U*)dst[k] + row * upr;
            for (int64_t q = lane; q < upr; q += 64) rd[q] = rs[q];
        }
    }
}

template <int NB>
__global__ __launch_bounds__(256) void msel_pack_kernel(
    SelFields fs, int nf, int64_t n, const uint16_t* __restrict__ flags, int nsets, SetMasks masks,
    const int64_t* __restrict__ offsets, const int64_t* __restrict__ set_starts, int64_t T,
    int tile_rows, long long cap, const uint32_t* __restrict__ scan_err) {
    __shared__ uint16_t list_s[4][kSelCap];
    __shared__ uint8_t* dst_s[4][kSelFields][kMaxSets];
    __shared__ long long at_s[4][kMaxSets];    // next output row of every set
    __shared__ int start_s[4][kMaxSets], cnt_s[4][kMaxSets];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = (int64_t)blockIdx.x * 4 + w;
    if (tile >= T || scan_failed(scan_err)) return;
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    uint8_t* trash = (uint8_t*)&g_sel_trash[tile & 255][lane];
    uint16_t* list = list_s[w];
    long long* at = at_s[w];
    int* start = start_s[w];
    int* cnt = cnt_s[w];
    uint32_t live = 0;   // sets with a destination (in field 0: all fields alike)
#pragma unroll
    for (int k = 0; k < kMaxSets; ++k) {
        if (k >= nsets) break;
        if (fs.dst[0][k]) live |= 1u << k;
        if (lane == k) {
#pragma unroll
            for (int f = 0; f < kSelFields; ++f) dst_s[w][f][k] = fs.dst[f][k];
            // set_starts == nullptr: the sets back to back from dst (placed on the device)
            at[k] = offsets[(int64_t)k * T + tile] - (set_starts ? set_starts[k] : 0);
            cnt[k] = 0;
        }
    }
    wave_sync();
    const int nbits = mask_bits(masks, nsets);
    // Per-lane copies of what the loops index at run time (lane k: set k's
    // mask; lane f: field f's source, row bytes, unit width), read by
    // readlane: a kernel-argument array indexed at run time is a memory load
    // whose s_waitcnt vmcnt(0) drained every copy and prefetch in flight --
    // once per set and per field of every chunk.
    const unsigned lmask = lane < nsets ? (unsigned)masks.m[lane] : 0u;
    const unsigned long long lsrc = lane < nf ? (unsigned long long)fs.src[lane] : 0ull;
    const long long lrb = lane < nf ? fs.row_bytes[lane] : 0;
    const int lwl = lane < nf ? fs.wlog[lane] : 0;
    uint32_t fn[kSelWords];   // the next chunk's flags, loaded a chunk ahead
    chunk_flags(flags, row0, min(kSelChunk, rows), lane, fn);
    for (int c0 = 0; c0 < rows; c0 += kSelChunk) {
        uint32_t fw[kSelWords];
#pragma unroll
        for (int i = 0; i < kSelWords; ++i) fw[i] = fn[i];
        if (c0 + kSelChunk < rows)
            chunk_flags(flags, row0 + c0 + kSelChunk, min(kSelChunk, rows - c0 - kSelChunk), lane, fn);
        FlagPlanes fp;
        flag_planes_t<NB>(fw, nbits, fp);
        auto flush = [&](int fill) {
            wave_sync();
            for (int f = 0; f < nf; ++f) {
                const long long rb = readlane64(lrb, f);
                const uint8_t* sp = (const uint8_t*)readlane64(lsrc, f) + (row0 + c0) * rb;
                uint8_t* const* d = dst_s[w][f];
                switch (__builtin_amdgcn_readlane(lwl, f)) {
                    case 4: sel_copy<16>(sp, rb, d, at, start, list, fill, lane, cap, trash); break;
                    case 3: sel_copy<8>(sp, rb, d, at, start, list, fill, lane, cap, trash); break;
                    case 2: sel_copy<4>(sp, rb, d, at, start, list, fill, lane, cap, trash); break;
                    case 1: sel_copy<2>(sp, rb, d, at, start, list, fill, lane, cap, trash); break;
                    default: sel_copy<1>(sp, rb, d, at, start, list, fill, lane, cap, trash); break;
                }
            }
            wave_sync();
            if (lane < nsets) {
                at[lane] += cnt[lane];
                cnt[lane] = 0;
            }
            wave_sync();
        };
        // the sets' lists, flushed when the next set does not fit: ONE call
        // site of flush (its copy loops are most of the kernel's code; inlined
        // at two or three sites the kernel ran 2x slower)
        int k = 0;
        for (;;) {
            int fill = 0;
            bool full = false;
            for (; k < nsets; ++k) {
                if (!((live >> k) & 1u)) continue;
                uint32_t m = set_mask_t<NB>(fp, (unsigned)__builtin_amdgcn_readlane((int)lmask, k), nbits);
                if (!__ballot(m != 0u)) continue;   // an empty set costs no prefix
                int total;
                // bit-sliced ballot prefix (A/B: 1.122 vs 1.162 ms with the
                // __shfl_up scan)
                int pos = wave_excl_small<5>(__popc(m), &total);   // popc(m) <= 16
                if (!total) continue;
                if (fill + total > kSelCap) {   // (fill > 0: a set is <= kSelChunk rows)
                    full = true;
                    break;                       // set k again after the flush
                }
                if (lane == 0) {
                    start[k] = fill;
                    cnt[k] = total;
                }
                pos += fill;
                while (m) {
                    const int j = __builtin_ctz(m);
                    m &= m - 1u;
                    list[pos++] = (uint16_t)((16 * lane + j) | (k << 10));
                }
                fill += total;
            }
            if (fill) flush(fill);
            if (!full) break;
        }
    }
}

hipError_t launch_msel_pack(int nfields, const void* const* srcs, const int64_t* row_bytes,
                            int64_t n, const uint16_t* flags, int nsets, const int* masks,
                            int tile_rows, const Workspace& ws, void* const* dsts, hipStream_t s,
                            int64_t cap_rows) {
    if (n <= 0) return hipSuccess;
    if (nfields < 1 || nfields > kSelFields || nsets < 1 || nsets > kMaxSets)
        return hipErrorInvalidValue;
    SetMasks sb{};
    for (int k = 0; k < nsets; ++k) sb.m[k] = (uint16_t)masks[k];
    SelFields fs{};
    for (int f = 0; f < nfields; ++f) {
        fs.src[f] = (const uint8_t*)srcs[f];
        fs.row_bytes[f] = row_bytes[f];
        uintptr_t a = (uintptr_t)srcs[f] | (uintptr_t)row_bytes[f];
        for (int k = 0; k < nsets; ++k) {
            // a set is written in every field or in none (field 0 decides);
            // placed mode (cap_rows >= 0): every set of field f from dsts[f]
            fs.dst[f][k] = cap_rows >= 0 ? (uint8_t*)dsts[f]
                           : dsts[0 * nsets + k] ? (uint8_t*)dsts[f * nsets + k] : nullptr;
            a |= (uintptr_t)fs.dst[f][k];
        }
        fs.wlog[f] = (a & 15) == 0 ? 4 : (a & 7) == 0 ? 3 : (a & 3) == 0 ? 2 : (a & 1) == 0 ? 1 : 0;
    }
    unsigned u = 0;
    for (int k = 0; k < nsets; ++k) u |= (unsigned)sb.m[k];
    const int nb = flag_bits_class(u ? 32 - __builtin_clz(u) : 0);
    auto kern = nb == 2 ? msel_pack_kernel<2> : nb == 4 ? msel_pack_kernel<4>
              : nb == 6 ? msel_pack_kernel<6> : nb == 8 ? msel_pack_kernel<8>
                        : msel_pack_kernel<0>;
    const dim3 grid((unsigned)((ws.T + 3) / 4));
    prof_begin(s, K_HALO_PACK);
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, fs, nfields, n, flags, nsets, sb,
                       ws.offsets, cap_rows >= 0 ? nullptr : ws.bin_starts, ws.T, tile_rows,
                       cap_rows >= 0 ? (long long)cap_rows : (long long)INT64_MAX, ws.scan_err);
    prof_end(s, K_HALO_PACK);
    return hipGetLastError();
}

// Image pack for rows of RB bytes, RB a multiple of 4 but not of 16 (e.g.
// the 36-byte records of config 5), <= 64 bins: the cooperative shape of
// pack_coop_kernel (one wave per 64-row round, per-bin bases exchanged
// through LDS behind one barrier) but every global access is 16 bytes wide.
// The round (64 * RB bytes, 16-byte aligned) is loaded in 16-byte units,
// parked in wave-private LDS, each row moved to its slot of a round image
// ordered by destination (bin-major, stable), and the image stored back in
// 16-byte units: a unit inside one bin's run is one 16-byte store to the
// run's (4-byte aligned) place in the output, a unit straddling two runs is
// stored dword by dword.  Plain 4-byte units would need RB/4 load and RB/4
// store instructions per round instead of ~RB/16.
template <int RB, int RPW, bool SEL>
__global__ __launch_bounds__(1024) void pack_img_kernel(
    const uint8_t* __restrict__ src, int64_t n, const uint8_t* __restrict__ dest, int nb,
    int nbits, int drop_bin, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ bin_starts, int64_t T, int64_t t0, int64_t tn, int tile_rows,
    uint8_t* __restrict__ dst, int redirect_bin, uint8_t* __restrict__ redirect_dst, int xcd,
    const uint32_t* __restrict__ scan_err, const uint16_t* __restrict__ id_src,
    uint16_t* __restrict__ id_dst, uint16_t* __restrict__ id_red) {
    static_assert(RB % 4 == 0 && RB % 16 != 0 && RB <= 64, "image pack row size");
    constexpr int WR = 64 * RPW;                    // rows per wave (RPW consecutive rounds)
    constexpr int RBYTES = WR * RB;                 // the wave's rows, a multiple of 16
    constexpr int NU = (RBYTES / 16 + 63) / 64;     // 16-byte units per lane
    constexpr int DW = RB / 4;
    constexpr int WAVE_LDS = RBYTES + 64 * 8 + WR;  // image, per-bin output address, row bins
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int nw = blockDim.x >> 6;
    int* s_cnt = (int*)smem;                                    // [nw][64]
    uint8_t* img = smem + nw * 64 * 4 + w * WAVE_LDS;
    unsigned long long* gaddr = (unsigned long long*)(img + RBYTES);
    uint8_t* ibin = img + RBYTES + 64 * 8;
    uint32_t* imgw = (uint32_t*)img;
    const int64_t tile = t0 + (xcd ? xcd_tile_c(blockIdx.x, tn, xcd) : (int64_t)blockIdx.x);
    const int64_t row0 = tile * (int64_t)tile_rows + (int64_t)WR * w;
    const int nrows = (int)max((int64_t)0, min((int64_t)WR, n - row0));
    const int nbytes = nrows * RB;
    // every load issued first, branch-free (clamped indices; rows past n are
    // masked by valid / nbytes afterwards): the first wait -- for the
    // destination bytes -- leaves the payload and side loads in flight
    unsigned braw[RPW], b[RPW], idv[RPW];
    bool valid[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        valid[q] = 64 * q + lane < nrows;
        const int64_t r = min(row0 + 64 * q + lane, n - 1);
        braw[q] = (unsigned)dest[r];
        idv[q] = id_src ? (unsigned)id_src[r] : 0u;  // side field
    }
    const SegLoad seg = seg_load(offsets, bin_starts, T, tile, lane, nb, redirect_bin);
    const uint8_t* __restrict__ sp = src + row0 * RB;
    u32x4_t v[NU];
    if constexpr (!SEL) {
        // a 16-byte unit that starts inside the array stays inside its page;
        // units past the wave's rows re-read the array's last one (never stored)
        const int64_t xmax = ((n * RB - 1) & ~(int64_t)15) - row0 * RB;
#pragma unroll
        for (int k = 0; k < NU; ++k)
            v[k] = *(const u32x4_t*)(sp + min((int64_t)(16 * (64 * k + lane)), xmax));
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) b[q] = valid[q] ? braw[q] : 0u;
    long long tbase = lane < nb ? seg_value(seg, lane, redirect_bin) : 0;
#pragma unroll
    for (int k = 0; k < NU && SEL; ++k) {
        const int x = 16 * (64 * k + lane);
        bool need = true;
        {   // selection: skip units whose rows (at most two, RB > 16) are all dropped
            const int r0 = min(x / RB, WR - 1), r1 = min((x + 15) / RB, WR - 1);
            int b0 = 0, b1 = 0;
#pragma unroll
            for (int q = 0; q < RPW; ++q) {
                const int t0 = __shfl((int)b[q], r0 & 63, 64), t1 = __shfl((int)b[q], r1 & 63, 64);
                if ((r0 >> 6) == q) b0 = t0;
                if ((r1 >> 6) == q) b1 = t1;
            }
            need = b0 != drop_bin || b1 != drop_bin;
        }
        if (!need) {
        } else if (x + 16 <= nbytes) {
            v[k] = *(const u32x4_t*)(sp + x);
        } else if (x < nbytes) {            // last partial unit of the array
            const uint32_t* q = (const uint32_t*)(sp + x);
            v[k] = u32x4_t{q[0], x + 4 < nbytes ? q[1] : 0u, x + 8 < nbytes ? q[2] : 0u,
                           x + 12 < nbytes ? q[3] : 0u};
        }
    }
    // rank inside each round; lane l counts bin l per round, cnt over the wave
    unsigned long long pe[RPW];
    int cq[RPW], cnt = 0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        unsigned long long p = __ballot(valid[q]), mine = p;
        for (int i = 0; i < nbits; ++i) {
            const unsigned long long m = __ballot((b[q] >> i) & 1u);
            p &= ((b[q] >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        pe[q] = p;
        cq[q] = __popcll(mine);
        cnt += cq[q];
    }
    s_cnt[w * 64 + lane] = cnt;
#pragma unroll
    for (int k = 0; k < NU; ++k) {
        const int x = 16 * (64 * k + lane);
        if (x < nbytes) *(u32x4_t*)(img + x) = v[k];
    }
    __syncthreads();
    if (scan_failed(scan_err)) return;
    for (int j = 0; j < w; ++j) tbase += s_cnt[j * 64 + lane];
    // wave image order: exclusive prefix of the wave's bin counts
    const int excl = wave_incl_dpp(cnt) - cnt;
    int slot[RPW];
    int run = excl;   // lane b: bin b's next image slot, round by round
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        slot[q] = __shfl(run, (int)b[q], 64) + (valid[q] ? rank_in(pe[q]) : 0);
        run += cq[q];
    }
    if (lane < nb) {
        uint8_t* base = lane == redirect_bin ? redirect_dst : dst;
        gaddr[lane] = lane == drop_bin ? 0ull
                                       : (unsigned long long)(base + (tbase - excl) * (long long)RB);
    }
    if (id_src) {   // the row's output row: its bin's (tile base - wave image start) + image slot
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const long long gr = __shfl(tbase - excl, (int)b[q], 64) + slot[q];
            if (valid[q] && (int)b[q] != drop_bin)
                ((int)b[q] == redirect_bin ? id_red : id_dst)[gr] = (uint16_t)idv[q];
        }
    }
    uint32_t row[RPW][DW];
#pragma unroll
    for (int q = 0; q < RPW; ++q)
        if (valid[q]) {
#pragma unroll
            for (int p = 0; p < DW; ++p) row[q][p] = imgw[(64 * q + lane) * DW + p];
        }
    wave_sync();
#pragma unroll
    for (int q = 0; q < RPW; ++q)
        if (valid[q]) {
#pragma unroll
            for (int p = 0; p < DW; ++p) imgw[slot[q] * DW + p] = row[q][p];
            ibin[slot[q]] = (uint8_t)b[q];
        }
    wave_sync();
#pragma unroll
    for (int k = 0; k < NU; ++k) {
        const int x = 16 * (64 * k + lane);
        if (x < nbytes) store_img_unit<RB, true>(img, ibin, gaddr, x, nbytes);
    }
}

// Multi-field (SoA) pack, <= 64 bins: the fields of the same rows -- e.g.
// positions, velocities, masses and ids held as separate arrays -- moved by
// ONE launch that reads every row's destination byte once and ranks it once
// (redist.py:195-198 applied to every field with the same rank_to_send, the
// :160-164 pattern).  The cooperative shape of pack_img_kernel: one wave per
// 128 rows (two 64-row rounds), per-bin bases exchanged through LDS behind
// one barrier.  Every field's 128 rows (128 * rb bytes, 16-byte aligned) are
// copied into wave-private LDS by LDS-DMA (global_load_lds_dwordx4: no
// registers, every field's loads in flight at once), and each field in turn
// is permuted in place into its destination-ordered image (a row's slot is
// shared by all fields) and streamed out in 16-byte units (store_img_unit: a
// unit inside one bin's run is one 16-byte store to the run's 4-byte-aligned
// place, a unit straddling two runs goes dword by dword).  Field row sizes
// of 4..64 bytes (4-byte multiples) run a pass with the size at compile time
// (LDS accesses at immediate offsets, division by a constant); wider ones a
// generic pass that gathers the image's dwords through the inverse
// permutation.  The optional 2-byte side field (fine cells) is stored per
// row as in pack_img_kernel.
constexpr int kFieldsMax = 8;          // fields per launch
constexpr int kFieldsWR = 128;         // rows per wave
struct PackFieldsArgs {
    const uint8_t* src[kFieldsMax];
    uint8_t* dst[kFieldsMax];
    uint8_t* red[kFieldsMax];
    int rb[kFieldsMax];          // row bytes, 4-byte multiples
    int loff[kFieldsMax];        // byte offset of field f's rows in a wave's LDS area
    int nf;
    int wave_lds;                // LDS bytes per wave
};
// a wave's LDS after the fields' rows: per-bin output address (one field at
// a time), per-bin image row offset, slot -> wave row, slot -> bin
constexpr int kFieldsTail = 64 * 8 + 64 * 8 + 2 * kFieldsWR;

// Any 4-byte-multiple row size (the generic pass): every 16-byte unit of the
// image gathered dword by dword from the rows in row order through the
// inverse permutation (slot -> row); rowoff[bin] = the output row of the
// bin's image slot 0.
__device__ __forceinline__ void fields_pass_any(const uint8_t* rows, int rb, const uint8_t* inv,
                                                const uint8_t* ibin, const long long* rowoff,
                                                unsigned long long dbase, unsigned long long rbase,
                                                int redirect_bin, int drop_bin, int nrows,
                                                int lane) {
    const uint32_t rinv = (uint32_t)(0x100000000ull / (unsigned)rb + 1);   // x / rb, x < 2^18
    const int nbytes = nrows * rb;
    auto addr = [&](int bb) -> unsigned long long {
        return (bb == redirect_bin ? rbase : dbase) + (unsigned long long)(rowoff[bb] * rb);
    };
    for (int x = 16 * lane; x < nbytes; x += 1024) {
        int s[4];
        u32x4_t q;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int xd = min(x + 4 * d, nbytes - 4);
            s[d] = (int)__umulhi((unsigned)xd, rinv);
            q[d] = *(const uint32_t*)(rows + (int)inv[s[d]] * rb + (xd - s[d] * rb));
        }
        const int bf = ibin[s[0]], bl = ibin[s[3]];
        if (x + 16 <= nbytes && bf == bl) {
            if (bf != drop_bin) gstore<u32x4_a4>(addr(bf) + x, q);
        } else {
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int xd = x + 4 * d;
                const int bd = ibin[s[d]];
                if (xd < nbytes && bd != drop_bin) gstore<uint32_t>(addr(bd) + xd, q[d]);
            }
        }
    }
}

__global__ __launch_bounds__(1024) void pack_fields_kernel(
    PackFieldsArgs fa, int64_t n, const uint8_t* __restrict__ dest, int nb, int nbits,
    int drop_bin, const int64_t* __restrict__ offsets, const int64_t* __restrict__ bin_starts,
    int64_t T, int64_t t0, int64_t tn, int tile_rows, int redirect_bin, int xcd,
    const uint32_t* __restrict__ scan_err, const uint16_t* __restrict__ id_src,
    uint16_t* __restrict__ id_dst, uint16_t* __restrict__ id_red) {
    constexpr int WR = kFieldsWR, RPW = WR / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    const int nw = blockDim.x >> 6;
    int* s_cnt = (int*)smem;                                    // [nw][64]
    uint8_t* wl = smem + nw * 64 * 4 + w * fa.wave_lds;         // the fields' rows
    uint8_t* tail = wl + fa.wave_lds - kFieldsTail;
    unsigned long long* gaddr = (unsigned long long*)tail;      // [64]
    long long* rowoff = (long long*)(tail + 64 * 8);            // [64]
    uint8_t* inv = tail + 64 * 16;                              // slot -> wave row
    uint8_t* ibin = inv + WR;                                   // slot -> bin
    const int64_t tile = t0 + (xcd ? xcd_tile_c(blockIdx.x, tn, xcd) : (int64_t)blockIdx.x);
    const int64_t row0 = tile * (int64_t)tile_rows + (int64_t)WR * w;
    const int nrows = __builtin_amdgcn_readfirstlane((int)max((int64_t)0, min((int64_t)WR, n - row0)));
    unsigned braw[RPW], b[RPW], idv[RPW];
    bool valid[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        valid[q] = 64 * q + lane < nrows;
        const int64_t r = min(row0 + 64 * q + lane, n - 1);
        braw[q] = (unsigned)dest[r];
        idv[q] = id_src ? (unsigned)id_src[r] : 0u;
    }
    const SegLoad seg = seg_load(offsets, bin_starts, T, tile, lane, nb, redirect_bin);
    // every field's rows into LDS: unit x = 16 * (64 i + lane) of the field's
    // 128 rows lands at loff + x (LDS-DMA: wave-uniform base + lane * 16;
    // lanes past the rows are masked off, so nothing lands beyond them); the
    // last unit of the array reads up to 12 bytes past its end, inside the
    // 16-byte-aligned unit's page
#pragma unroll
    for (int f = 0; f < kFieldsMax; ++f) {
        if (f >= fa.nf) break;
        const int rb = fa.rb[f];
        const int nbytes = nrows * rb;
        const uint8_t* sp = fa.src[f] + row0 * rb;
        for (int i = 0; 1024 * i < nbytes; ++i) {
            const int x = 16 * (64 * i + lane);
            if (x < nbytes)
                __builtin_amdgcn_global_load_lds(
                    (const void*)(sp + x),
                    (__attribute__((address_space(3))) void*)(wl + fa.loff[f] + 1024 * i), 16, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) b[q] = valid[q] ? braw[q] : 0u;
    long long tbase = lane < nb ? seg_value(seg, lane, redirect_bin) : 0;
    // rank inside each round; lane l counts bin l per round, cnt over the wave
    unsigned long long pe[RPW];
    int cq[RPW], cnt = 0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        unsigned long long p = __ballot(valid[q]), mine = p;
        for (int i = 0; i < nbits; ++i) {
            const unsigned long long m = __ballot((b[q] >> i) & 1u);
            p &= ((b[q] >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        pe[q] = p;
        cq[q] = __popcll(mine);
        cnt += cq[q];
    }
    s_cnt[w * 64 + lane] = cnt;
    __syncthreads();   // (also retires the LDS-DMA loads: vmcnt(0) before the barrier)
    if (scan_failed(scan_err)) return;
    for (int j = 0; j < w; ++j) tbase += s_cnt[j * 64 + lane];
    // wave image order: exclusive prefix of the wave's bin counts
    const int excl = wave_incl_dpp(cnt) - cnt;
    int run = excl;   // lane b: bin b's next image slot, round by round
    int slot[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        // (shuffles in uniform control flow: a bpermute from a lane outside
        // the exec mask does not read that lane's value)
        slot[q] = __shfl(run, (int)b[q], 64) + (valid[q] ? rank_in(pe[q]) : 0);
        const long long gr = id_src ? __shfl(tbase - excl, (int)b[q], 64) + slot[q] : 0;
        run += cq[q];
        if (valid[q]) {
            inv[slot[q]] = (uint8_t)(64 * q + lane);
            ibin[slot[q]] = (uint8_t)b[q];
            if (id_src && (int)b[q] != drop_bin)
                ((int)b[q] == redirect_bin ? id_red : id_dst)[gr] = (uint16_t)idv[q];
        }
    }
    const long long ro = tbase - excl;   // lane b: output row of bin b's image slot 0
    if (lane < nb) rowoff[lane] = ro;
    // per-lane copies of the fields' run-time values (lane f: field f), read
    // with readlane: a kernel-argument array indexed at run time would be a
    // memory load (msel_pack_kernel)
    const int lrb = lane < fa.nf ? fa.rb[lane] : 0;
    const int lloff = lane < fa.nf ? fa.loff[lane] : 0;
    const unsigned long long ldst = lane < fa.nf ? (unsigned long long)fa.dst[lane] : 0ull;
    const unsigned long long lred = lane < fa.nf ? (unsigned long long)fa.red[lane] : 0ull;
#pragma unroll 1
    for (int f = 0; f < fa.nf; ++f) {
        const int rb = __builtin_amdgcn_readlane(lrb, f);
        uint8_t* rows = wl + __builtin_amdgcn_readlane(lloff, f);
        const unsigned long long dbase = readlane64(ldst, f), rbase = readlane64(lred, f);
        wave_sync();   // the previous field's stores have read gaddr
        if (lane < nb)
            gaddr[lane] = lane == drop_bin ? 0ull
                          : (lane == redirect_bin ? rbase : dbase) + (unsigned long long)(ro * rb);
        wave_sync();
        switch (rb) {
#define MGR_FP(RB_) case RB_: image_pass<RB_, kFieldsWR / 64>(rows, ibin, gaddr, slot, valid, nrows, lane); break;
            MGR_FP(4) MGR_FP(8) MGR_FP(12) MGR_FP(16) MGR_FP(20) MGR_FP(24) MGR_FP(28) MGR_FP(32)
            MGR_FP(36) MGR_FP(40) MGR_FP(44) MGR_FP(48) MGR_FP(52) MGR_FP(56) MGR_FP(60) MGR_FP(64)
#undef MGR_FP
            default:
                fields_pass_any(rows, rb, inv, ibin, rowoff, dbase, rbase, redirect_bin, drop_bin,
                                nrows, lane);
        }
    }
}

// Multi-field pack with one destination-ordered image per WORKGROUP and
// field (the tile's rows of a field, bin-major): every bin's rows of the tile
// leave as ONE contiguous run per field (tile_rows / nbins rows: 256 B of the
// 4-byte masses at 512-row tiles and 8 bins) instead of one run per wave --
// SoA fields are narrow, and per-wave runs of a few rows leave most store
// instructions writing partial lines.  Loads as pack_fields_kernel (every
// field's rows of a wave by LDS-DMA into wave-private staging, ranked once);
// then per field: the wave's rows into a tile image at their tile slots
// (row -> slot, a compile-time row size), a barrier, the tile image streamed
// out in 16-byte units by the whole workgroup (store_img_unit), a barrier.
// (A/B on the config-5 SoA rows, 512-row tiles: this 1.16-1.23 ms; two
// alternating images, one barrier per field, 1.33; every field's image at
// once with ONE barrier per tile 1.60 -- a tile's stores all at its end.)
template <int RB>
__device__ __forceinline__ void tile_field_permute(const uint8_t* rows, uint8_t* img,
                                                   const int* tslot, const bool* valid, int lane) {
    constexpr int DW = RB / 4;
    constexpr int RPW = kFieldsWR / 64;
    const uint32_t* r32 = (const uint32_t*)rows;
    uint32_t* i32 = (uint32_t*)img;
#pragma unroll
    for (int q = 0; q < RPW; ++q)
        if (valid[q]) {
            uint32_t v[DW];
#pragma unroll
            for (int p = 0; p < DW; ++p) v[p] = r32[(64 * q + lane) * DW + p];
#pragma unroll
            for (int p = 0; p < DW; ++p) i32[tslot[q] * DW + p] = v[p];
        }
}

template <int RB>
__device__ __forceinline__ void tile_field_store(const uint8_t* img, const uint8_t* ibin,
                                                 const unsigned long long* gaddr, int tile_bytes) {
    for (int x = 16 * (int)threadIdx.x; x < tile_bytes; x += 16 * (int)blockDim.x)
        store_img_unit<RB, true>(img, ibin, gaddr, x, tile_bytes);
}

__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(6))) void pack_fields_tile_kernel(
    PackFieldsArgs fa, int64_t n, const uint8_t* __restrict__ dest, int nb, int nbits,
    int drop_bin, const int64_t* __restrict__ offsets, const int64_t* __restrict__ bin_starts,
    int64_t T, int64_t t0, int64_t tn, int tile_rows, int redirect_bin, int xcd,
    const uint32_t* __restrict__ scan_err, const uint16_t* __restrict__ id_src,
    uint16_t* __restrict__ id_dst, uint16_t* __restrict__ id_red, int img_bytes) {
    constexpr int WR = kFieldsWR, RPW = WR / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ unsigned long long s_gaddr[64];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    const int nw = blockDim.x >> 6;
    uint8_t* img = smem;                                        // [img_bytes]
    uint8_t* ibin = smem + img_bytes;                           // [tile_rows]
    uint8_t* wl = ibin + align16(tile_rows) + w * fa.wave_lds;  // the wave's staged rows
    // the waves' bin counts [nw][64], after the staging (sized by the waves,
    // so six 512-row workgroups of config 5's SoA fields fit a CU's LDS)
    int (*s_cnt)[64] = (int (*)[64])(ibin + align16(tile_rows) + nw * fa.wave_lds);
    const int64_t tile = t0 + (xcd ? xcd_tile_c(blockIdx.x, tn, xcd) : (int64_t)blockIdx.x);
    const int64_t tile0 = tile * (int64_t)tile_rows;
    const int64_t row0 = tile0 + (int64_t)WR * w;
    const int nrows = __builtin_amdgcn_readfirstlane((int)max((int64_t)0, min((int64_t)WR, n - row0)));
    const int trows = (int)min((int64_t)tile_rows, n - tile0);
    unsigned braw[RPW], b[RPW], idv[RPW];
    bool valid[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        valid[q] = 64 * q + lane < nrows;
        const int64_t r = min(row0 + 64 * q + lane, n - 1);
        braw[q] = (unsigned)dest[r];
        idv[q] = id_src ? (unsigned)id_src[r] : 0u;
    }
    const SegLoad seg = seg_load(offsets, bin_starts, T, tile, lane, nb, redirect_bin);
#pragma unroll
    for (int f = 0; f < kFieldsMax; ++f) {
        if (f >= fa.nf) break;
        const int rb = fa.rb[f];
        const int nbytes = nrows * rb;
        const uint8_t* sp = fa.src[f] + row0 * rb;
        for (int i = 0; 1024 * i < nbytes; ++i) {
            const int x = 16 * (64 * i + lane);
            if (x < nbytes)
                __builtin_amdgcn_global_load_lds(
                    (const void*)(sp + x),
                    (__attribute__((address_space(3))) void*)(wl + fa.loff[f] + 1024 * i), 16, 0, 0);
        }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) b[q] = valid[q] ? braw[q] : 0u;
    // rank inside each round; lane l counts bin l over the wave's rounds
    unsigned long long pe[RPW];
    int cq[RPW], cnt = 0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        unsigned long long p = __ballot(valid[q]), mine = p;
        for (int i = 0; i < nbits; ++i) {
            const unsigned long long m = __ballot((b[q] >> i) & 1u);
            p &= ((b[q] >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        pe[q] = p;
        cq[q] = __popcll(mine);
        cnt += cq[q];
    }
    s_cnt[w][lane] = cnt;
    __syncthreads();   // (also retires the LDS-DMA loads)
    if (scan_failed(scan_err)) return;
    // lane b: the tile's count of bin b, the earlier waves' count, the bin's
    // start in the tile image (exclusive over the bins)
    int tot = 0, wpre = 0;
    for (int j = 0; j < nw; ++j) {
        const int c = s_cnt[j][lane];
        tot += c;
        wpre += j < w ? c : 0;
    }
    if (lane >= nb) tot = 0;
    const int tstart = wave_incl_dpp(tot) - tot;
    const int wexcl = wave_incl_dpp(cnt) - cnt;   // the wave's own bin-major order
    const int toff = tstart + wpre - wexcl;        // lane b: wave slot -> tile slot
    int run = wexcl;
    int tslot[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        // (shuffles in uniform control flow)
        const int ws = __shfl(run, (int)b[q], 64) + (valid[q] ? rank_in(pe[q]) : 0);
        tslot[q] = ws + __shfl(toff, (int)b[q], 64);
        run += cq[q];
        if (valid[q]) ibin[tslot[q]] = (uint8_t)b[q];
    }
    // lane b (wave 0): the bin's output row of tile image slot 0
    const long long obase = (lane < nb ? seg_value(seg, lane, redirect_bin) : 0) - tstart;
    if (id_src) {
        const long long ob = obase;
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const long long gr = __shfl(ob, (int)b[q], 64) + tslot[q];
            if (valid[q] && (int)b[q] != drop_bin)
                ((int)b[q] == redirect_bin ? id_red : id_dst)[gr] = (uint16_t)idv[q];
        }
    }
    const int lrb = lane < fa.nf ? fa.rb[lane] : 0;
    const int lloff = lane < fa.nf ? fa.loff[lane] : 0;
    const unsigned long long ldst = lane < fa.nf ? (unsigned long long)fa.dst[lane] : 0ull;
    const unsigned long long lred = lane < fa.nf ? (unsigned long long)fa.red[lane] : 0ull;
    // per field: the wave's rows into the tile image at their slots, a
    // barrier, the image streamed out, a barrier before the next field's
#pragma unroll 1
    for (int f = 0; f < fa.nf; ++f) {
        const int rb = __builtin_amdgcn_readlane(lrb, f);
        const uint8_t* rows = wl + __builtin_amdgcn_readlane(lloff, f);
        uint8_t* fimg = img;
        unsigned long long* ga = s_gaddr;
        if (w == 0 && lane < nb) {
            const unsigned long long dbase = readlane64(ldst, f), rbase = readlane64(lred, f);
            ga[lane] = lane == drop_bin ? 0ull
                       : (lane == redirect_bin ? rbase : dbase) + (unsigned long long)(obase * rb);
        }
        switch (rb) {
#define MGR_TFP(RB_) case RB_: tile_field_permute<RB_>(rows, fimg, tslot, valid, lane); break;
            MGR_TFP(4) MGR_TFP(8) MGR_TFP(12) MGR_TFP(16) MGR_TFP(20) MGR_TFP(24) MGR_TFP(28)
            MGR_TFP(32) MGR_TFP(36) MGR_TFP(40) MGR_TFP(44) MGR_TFP(48) MGR_TFP(52) MGR_TFP(56)
            MGR_TFP(60) MGR_TFP(64)
#undef MGR_TFP
            default: break;   // (the launcher sends only 4..64-byte rows)
        }
        __syncthreads();   // the image, ibin and the field's addresses complete
        switch (rb) {
#define MGR_TFS(RB_) case RB_: tile_field_store<RB_>(fimg, ibin, ga, trows * RB_); break;
            MGR_TFS(4) MGR_TFS(8) MGR_TFS(12) MGR_TFS(16) MGR_TFS(20) MGR_TFS(24) MGR_TFS(28)
            MGR_TFS(32) MGR_TFS(36) MGR_TFS(40) MGR_TFS(44) MGR_TFS(48) MGR_TFS(52) MGR_TFS(56)
            MGR_TFS(60) MGR_TFS(64)
#undef MGR_TFS
            default: break;
        }
        __syncthreads();   // the image is reused by the next field
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
    const int64_t* __restrict__ bin_starts, int64_t T, int64_t t0, int64_t tn, int tile_rows,
    uint8_t* __restrict__ dst, int redirect_bin, uint8_t* __restrict__ redirect_dst, int xcd,
    const uint32_t* __restrict__ scan_err) {
    using U = typename Unit<W>::T;
    constexpr int R = 16 * RPW;                                // rounds per super-round
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    long long* s_off = (long long*)smem;                       // [nb] running bin bases
    uint16_t* tab = (uint16_t*)(smem + align16(nb * 8));       // [R][nb]
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = t0 + (xcd ? xcd_tile_c(blockIdx.x, tn, xcd) : (int64_t)blockIdx.x);
    if (scan_failed(scan_err)) return;
    for (int bb = threadIdx.x; bb < nb; bb += blockDim.x)
        s_off[bb] = seg_start(offsets, bin_starts, T, tile, bb, redirect_bin);
    U* __restrict__ d_u = (U*)dst;
    U* __restrict__ r_u = (U*)redirect_dst;
    // the tile's super-rounds of 64 * R rows, in order: a bin's rows of
    // consecutive super-rounds continue each other's output run, so the
    // tile writes one run of ~tile_rows / nb rows per bin
    for (int64_t sr0 = tile * (int64_t)tile_rows; sr0 < min(n, (tile + 1) * (int64_t)tile_rows);
         sr0 += 64 * R) {
        const int64_t row0 = sr0 + 64 * RPW * w;
        for (int i = threadIdx.x; i < R * nb; i += blockDim.x) tab[i] = 0;
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
        __syncthreads();   // table zeroed (and, first time, tile offsets staged)
        unsigned long long peers[RPW];
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const bool valid = lane < nr[q];
            peers[q] = match_bin(b[q], valid, nbits);
            if (valid && rank_in(peers[q]) == 0)
                tab[(w * RPW + q) * nb + b[q]] = (uint16_t)__popcll(peers[q]);
        }
        __syncthreads();
        // per bin (one per thread, nb <= 1024): exclusive prefix over the
        // super-round's rounds; the total moves the bin's running base later
        int total = 0;
        if (threadIdx.x < nb) {
            const int bb = threadIdx.x;
            for (int r = 0; r < R; ++r) {
                const int c = tab[r * nb + bb];
                tab[r * nb + bb] = (uint16_t)total;
                total += c;
            }
        }
        __syncthreads();
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
        __syncthreads();   // every base and prefix read before they move on
        if (threadIdx.x < nb) s_off[threadIdx.x] += total;
    }
}

typedef unsigned int u32x3_a4 __attribute__((ext_vector_type(3), aligned(4)));
typedef unsigned int u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));

// One row of NDW dwords (4-byte aligned) into registers: 16-byte loads and a tail.
template <int NDW>
__device__ __forceinline__ void load_row_dw(const uint8_t* __restrict__ p, uint32_t (&v)[NDW]) {
    int i = 0;
#pragma unroll
    for (; i + 4 <= NDW; i += 4) {
        const u32x4_a4 x = *(const u32x4_a4*)(p + 4 * i);
        v[i] = x[0]; v[i + 1] = x[1]; v[i + 2] = x[2]; v[i + 3] = x[3];
    }
    if constexpr (NDW % 4 == 3) {
        const u32x3_a4 x = *(const u32x3_a4*)(p + 4 * i);
        v[i] = x[0]; v[i + 1] = x[1]; v[i + 2] = x[2];
    } else if constexpr (NDW % 4 == 2) {
        const u32x2_a4 x = *(const u32x2_a4*)(p + 4 * i);
        v[i] = x[0]; v[i + 1] = x[1];
    } else if constexpr (NDW % 4 == 1) {
        v[i] = *(const uint32_t*)(p + 4 * i);
    }
}

constexpr int kFineTR = 2048;      // ranked tiles when a 4096-row image does not fit
constexpr int kFineWaves = 16;     // ranked pack: 1024 threads

// ============================================================ launchers
// The 2-byte side field of a pack (mgr_pack_ids: the fine cells or halo
// flags travelling with the rows), handed down the launchers explicitly
// (NULL: none).  The coop and image launchers take it into their kernel and
// mark it used; other paths leave it to a second (2-byte-row) pack.
struct SideField {
    const uint16_t* src = nullptr;
    uint16_t* dst = nullptr;
    uint16_t* red = nullptr;
    bool used = false;
};

// pack_many_kernel: one super-round of 64 * R rows per tile (the uint16
// [R][nbins] LDS table stays <= 128 KiB at 4096 rows and 1024 bins; A/B: 2-16
// super-rounds per tile, i.e. longer per-bin runs, measured slower).
// Up to 512 bins 2048-row super-rounds (8x8x8 cells, 64M 36-byte rows: pack
// 1.43-1.49 vs 1.55-1.70 ms at 4096 rows and 1.70 at 1024; the bin kernel and
// the scan pay ~+0.05 ms each for the twice larger histogram; whole sort 2.17-2.24
// vs 2.19-2.34 ms; 120 cells 1.85 vs 2.03 ms); above 512 bins 4096 rows (1024
// cells: 2.53 vs 2.84 ms -- there the [bins][tiles] histogram dominates).
// profiles/round1/fine_many_ab.log, fine_shapes_ab.log.
static int many_round_rows(int nbins) { return nbins <= 512 ? 2048 : 4096; }

int pack_tile_rows(int64_t row_bytes, int nbins) {
    const int tr = hooks().tile_rounds;   // one snapshot
    if (tr > 0) return 64 * tr;
    // <= 16 bins: 512-row tiles (bin: 4 waves x 2 rounds; pack: 8 waves x
    // 1 round; A/B against 1024 at 8 bins: bin -3 %, pack within noise);
    // <= 64 bins: 1024 rows (64 bins: pack 0.92 vs 1.07 ms at 512: longer
    // same-bin runs); more bins: longer tiles keep the [nbins][tiles]
    // histogram small next to the payload.
    // rows the image pack takes (4-byte, not 16-byte multiples, 24..60 B, e.g.
    // config 5's 36-B records): 1024-row tiles (2 rounds x 8 waves per image
    // workgroup; A/B at 36 B: bin 0.382 vs 0.418, scan 0.014 vs 0.023, pack
    // 0.850 vs 0.856 ms per 64M)
    const bool img = row_bytes % 4 == 0 && row_bytes % 16 != 0 && row_bytes >= 24 && row_bytes <= 60;
    if (nbins <= 16) return img ? 1024 : 512;
    if (nbins <= 64) return 1024;
    if (nbins <= 1024 && row_bytes <= 64) return many_round_rows(nbins);
    int r = 16;
    while (r < 4096 / 64 && (int64_t)nbins * 4 > (int64_t)r * 8) r *= 2;
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
    const int64_t grid = (ws.tn + wpb - 1) / wpb;
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * wpb), (size_t)lds, s,
                       (const uint8_t*)src, row_bytes / W, n, (const DestT*)dest, nb,
                       nbits_for(nb), drop_bin, ws.offsets, ws.bin_starts, ws.T, ws.t0, ws.tn,
                       tile_rows,
                       per_wave, (uint8_t*)dst, redirect_bin, (uint8_t*)redirect_dst, ws.scan_err);
    return hipGetLastError();
}

template <int W, int UPR>
static hipError_t pack_coop_u(const void* src, int64_t n, const void* dest, int nb, int drop_bin,
                              int tile_rows, const Workspace& ws, void* dst, int redirect_bin,
                              void* redirect_dst, hipStream_t s, SideField* side, const Hooks& h) {
    if (h.pack_generic || tile_rows > 2048) return hipErrorNotSupported;
    // one wave per RPW 64-row rounds of the tile (<= 16 waves)
    const int rpw = tile_rows > 1024 ? 2 : 1;
    const int threads = tile_rows / rpw;
#define MGR_PCK(RPW_)                                                                         \
    hipLaunchKernelGGL((pack_coop_kernel<W, UPR, RPW_>), dim3((unsigned)ws.tn), dim3(threads), 0, \
                       s, (const uint8_t*)src, n, (const uint8_t*)dest, nb, nbits_for(nb),     \
                       drop_bin, ws.offsets, ws.bin_starts, ws.T, ws.t0, ws.tn, tile_rows,     \
                       (uint8_t*)dst,                                                          \
                       redirect_bin, (uint8_t*)redirect_dst, kXcdPackChunk, sel, ws.scan_err, \
                       side ? side->src : nullptr, side ? side->dst : nullptr,         \
                       side ? side->red : nullptr)
    // selection packs (2 bins, one dropped: the halo's rows to send) skip
    // the loads of dropped rows; elsewhere loads go out before the bins are known
    const int sel = nb <= 2 && drop_bin >= 0;
    if (side) side->used = side->src != nullptr;
    if (rpw == 2) MGR_PCK(2); else MGR_PCK(1);
#undef MGR_PCK
    return hipGetLastError();
}

// Compile-time units per row for rows of <= 64 bytes in 16/8/4-byte units
// (registers, no scratch); returns hipErrorNotSupported for other shapes.
template <int W>
static hipError_t pack_coop_t(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                               int nb, int drop_bin, int tile_rows, const Workspace& ws,
                               void* dst, int redirect_bin, void* redirect_dst, hipStream_t s,
                               SideField* side, const Hooks& h) {
#define MGR_PS(U_) case U_: return pack_coop_u<W, U_>(src, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side, h);
    if constexpr (W >= 4) {
        switch ((int)(row_bytes / W)) {
            MGR_PS(1) MGR_PS(2) MGR_PS(3) MGR_PS(4)
            default: break;
        }
        if constexpr (W <= 8) {
            switch ((int)(row_bytes / W)) {
                MGR_PS(5) MGR_PS(6) MGR_PS(7) MGR_PS(8)
                default: break;
            }
        }
        if constexpr (W == 4) {
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
    const int round_rows = many_round_rows(nb);
    if (tile_rows % round_rows) return hipErrorNotSupported;
    const int lds = align16(nb * 8) + (round_rows / 64) * nb * 2;
#define MGR_PMK(RPW_)                                                                          \
    {                                                                                          \
        auto k = pack_many_kernel<W, UPR, DestT, RPW_>;                                        \
        ensure_lds(k, lds);                                                                    \
        hipLaunchKernelGGL(k, dim3((unsigned)ws.tn), dim3(1024), (size_t)lds, s,               \
                           (const uint8_t*)src, n, (const DestT*)dest, nb, nbits_for(nb),      \
                           drop_bin, ws.offsets, ws.bin_starts, ws.T, ws.t0, ws.tn, tile_rows, \
                           (uint8_t*)dst,                                                      \
                           redirect_bin, (uint8_t*)redirect_dst, kXcdPackChunk, ws.scan_err); \
    }
    if (round_rows == 4096) MGR_PMK(4)
    else if (round_rows == 2048) MGR_PMK(2)
    else return hipErrorNotSupported;
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
    if constexpr (W <= 8) {
        switch ((int)(row_bytes / W)) {
            MGR_PM(5) MGR_PM(6) MGR_PM(7) MGR_PM(8)
            default: break;
        }
    }
    if constexpr (W == 4) {
        switch ((int)(row_bytes / W)) {
            MGR_PM(9) MGR_PM(10) MGR_PM(11) MGR_PM(12) MGR_PM(13) MGR_PM(14) MGR_PM(15) MGR_PM(16)
            default: break;
        }
    }
#undef MGR_PM
    return hipErrorNotSupported;
}

template <int RB>
static hipError_t pack_img_t(const void* src, int64_t n, const void* dest, int nb, int drop_bin,
                             int tile_rows, const Workspace& ws, void* dst, int redirect_bin,
                             void* redirect_dst, hipStream_t s, SideField* side) {
    // two 64-row rounds per wave (A/B, 36-B records: 0.90-0.92 vs 1.02-1.05
    // ms per 64M with one, 4: 1.17 -- a wave's fixed per-round chain of load,
    // count exchange, LDS permutation and store then moves twice the rows);
    // tiles that are not a multiple of two rounds go to the coop pack
    constexpr int rpw = kImgRoundsPerWave;
    if (tile_rows % (64 * rpw)) return hipErrorNotSupported;
    const int nw = tile_rows / (64 * rpw);
    const int lds = nw * 64 * 4 + nw * (64 * rpw * RB + 64 * 8 + 64 * rpw);
    const bool sel = nb <= 2 && drop_bin >= 0;
    auto k = sel ? pack_img_kernel<RB, rpw, true> : pack_img_kernel<RB, rpw, false>;
    ensure_lds(k, lds);
    hipLaunchKernelGGL(k, dim3((unsigned)ws.tn), dim3(64 * nw), (size_t)lds, s,
                       (const uint8_t*)src, n, (const uint8_t*)dest, nb, nbits_for(nb), drop_bin,
                       ws.offsets, ws.bin_starts, ws.T, ws.t0, ws.tn, tile_rows, (uint8_t*)dst,
                       redirect_bin,
                       (uint8_t*)redirect_dst, kXcdPackChunk, ws.scan_err,
                       side ? side->src : nullptr, side ? side->dst : nullptr,
                       side ? side->red : nullptr);
    if (side) side->used = side->src != nullptr;
    return hipGetLastError();
}

static int g_cus = 0;   // compute units of the current device (persistent grids)
static int device_cus() {
    if (g_cus <= 0) {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
            g_cus = c;
        if (g_cus <= 0) g_cus = 256;
    }
    return g_cus;
}

// Ranked sorted-image pack (mgr_pack_ranked), the stable sort of 65..1024
// bins (config 5's fine cells): every row's rank inside (tile, bin) and every
// tile's bin starts come from mgr_rank_ids, so a tile is: load (a tile
// ahead), rows into the LDS image at tile_start[bin] + rank, stream the image
// out in 16-byte units (a unit inside one bin's run is one 16-byte store to
// the run's place, a unit straddling two runs goes dword by dword).
// Persistent: one 1024-thread workgroup per CU (the image fills most of the
// LDS) walks its XCD's tiles, the workgroups of an XCD on adjacent tiles at a
// time (the lines their runs share meet in one L2).  No ballots, no per-tile
// count table, three barriers per tile.
template <int RB, int TR>
__global__ __launch_bounds__(1024) void pack_ranked_kernel(
    const uint8_t* __restrict__ src, int64_t n, const uint16_t* __restrict__ ids,
    const uint16_t* __restrict__ ranks, const uint16_t* __restrict__ tile_starts, int nb,
    const int64_t* __restrict__ offsets, int64_t T, uint8_t* __restrict__ dst,
    const uint32_t* __restrict__ scan_err) {
    static_assert(RB % 4 == 0 && RB <= 64, "ranked pack row size");
    constexpr int NW = kFineWaves, RPW = TR / 64 / NW;
    constexpr int NDW = RB / 4;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* img = (uint32_t*)smem;
    uint8_t* p = smem + align16(TR * RB);
    uint16_t* ibin = (uint16_t*)p;                 p += align16(TR * 2);
    unsigned long long* gaddr = (unsigned long long*)p;
    if (scan_failed(scan_err)) return;
    const int tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    // tile walk: XCD x owns tiles [x*per, (x+1)*per), its gx workgroups on
    // gx adjacent tiles at a time, so the lines that adjacent tiles' runs
    // share meet in one L2 (A/B: all 8 XCDs on one region of the input at a
    // time measured no better)
    const int64_t per = (T + 7) >> 3;
    const int gx = (int)(gridDim.x >> 3), kx = (int)(blockIdx.x >> 3), xx = (int)(blockIdx.x & 7);
    const int64_t first = (int64_t)xx * per + kx;
    const int64_t stride = gx;
    const int64_t last = min(T, (int64_t)xx * per + per);
    const int mb = min(tid, nb - 1);
    struct Set {
        uint32_t v[RPW][NDW];
        unsigned b[RPW];
        unsigned rk[RPW];
        long long seg;
        unsigned ls;
    };
    auto load = [&](Set& S, int64_t t) __attribute__((always_inline)) {
        t = min(t, last - 1);
        S.seg = offsets[(int64_t)mb * T + t];
        S.ls = tile_starts[t * nb + mb];
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int64_t row = min(t * TR + (int64_t)(w * RPW + q) * 64 + lane, n - 1);
            S.b[q] = min((unsigned)ids[row], (unsigned)(nb - 1));   // ids >= nb: clamped (mgr_rank_ids reports them)
            S.rk[q] = ranks[row];
            load_row_dw<NDW>(src + row * RB, S.v[q]);
        }
    };
    // (A/Bs, round 4, profiles/round4/ab_notes.md: a branch-free scatter,
    // which let the compiler keep the next tile's loads in flight through the
    // store phase, measured SLOWER (1.14 vs 1.10 ms, with or without a fully
    // unrolled store loop); so did the rows stored straight from registers
    // to their slots by small workgroups, no LDS image (1.50-1.96 ms).  With
    // every store sent sequentially to the tile's own region this kernel
    // takes 0.95 ms: the one 1024-thread workgroup per CU that the image
    // needs is the ceiling, the run scatter adds 0.15 ms.)
    auto process = [&](Set& S, int64_t t) __attribute__((always_inline)) {
        const int tr = (int)min((int64_t)TR, n - t * TR);
        if (tid < nb) gaddr[tid] = (unsigned long long)(dst + (S.seg - (long long)S.ls) * (long long)RB);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            if ((w * RPW + q) * 64 + lane < tr) {
                const int lpos = S.rk[q];   // the row's slot in the tile (mgr_rank_ids)
#pragma unroll
                for (int i = 0; i < NDW; ++i) img[lpos * NDW + i] = S.v[q][i];
                ibin[lpos] = (uint16_t)S.b[q];
            }
        }
        __syncthreads();
        const int nbytes = tr * RB;
        // (the image pack's two-address unit store, store_img_unit, measured
        // 12 % slower here)
        for (int x = 16 * tid; x < nbytes; x += 16 * 1024) {
            const u32x4_t q = *(const u32x4_t*)((const uint8_t*)img + x);
            const int bf = ibin[x / RB];
            if (x + 16 <= nbytes && ibin[(x + 15) / RB] == bf) {
                gstore<u32x4_a4>(gaddr[bf] + x, q);
            } else {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const int xd = x + 4 * d;
                    if (xd < nbytes) gstore<uint32_t>(gaddr[ibin[xd / RB]] + xd, q[d]);
                }
            }
        }
        __syncthreads();   // the image, ibin and gaddr are reused by the next tile
    };
    Set A, B;
    int64_t t = first;
    if (t >= last) return;
    load(A, t);
    for (;;) {
        load(B, t + stride);
        process(A, t);
        t += stride;
        if (t >= last) break;
        load(A, t + stride);
        process(B, t);
        t += stride;
        if (t >= last) break;
    }
}

// LDS of the ranked pack: the tile image, its row bins and per-bin output
// addresses.
static int ranked_lds_bytes(int tile_rows, int64_t row_bytes, int nbins) {
    return align16(tile_rows * (int)row_bytes) + align16(tile_rows * 2) + nbins * 8;
}
// Ranked tiles: 4096 rows when their image fits the LDS (36-byte rows: 157 KiB),
// else 2048.  Longer tiles halve the [bins][tiles] histogram the scan walks and
// the per-tile fixed work (A/B: profiles/round2/ab_notes.md).
int ranked_tile_rows(int64_t row_bytes, int nbins) {
    if (row_bytes < 1 || row_bytes % 4 || row_bytes > 64 || nbins < 1 || nbins > 1024) return 0;
    const int want = hooks().rank_rows;
    if (want != 2048 && ranked_lds_bytes(4096, row_bytes, nbins) <= 160 * 1024) return 4096;
    return ranked_lds_bytes(kFineTR, row_bytes, nbins) <= 160 * 1024 ? kFineTR : 0;
}

hipError_t launch_pack_ranked(const void* src, int64_t row_bytes, int64_t n, const uint16_t* ids,
                              const uint16_t* ranks, const uint16_t* tile_starts, int nbins,
                              int tile_rows, const Workspace& ws, void* dst, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if ((tile_rows != kFineTR && tile_rows != 4096) || row_bytes % 4 || row_bytes > 64 ||
        ((uintptr_t)src & 3) || ((uintptr_t)dst & 3))
        return hipErrorNotSupported;
    const int lds = ranked_lds_bytes(tile_rows, row_bytes, nbins);
    if (lds > 160 * 1024) return hipErrorNotSupported;
    prof_begin(s, K_PACK_FINE);
    hipError_t e = hipErrorNotSupported;
    // one persistent workgroup per CU (A/B, round 6: as many per CU as the LDS
    // holds -- two to four for the 4..12-byte fields of a SoA payload --
    // measured slower, 0.41 vs 0.36 ms per field launch at 64M rows)
    int64_t grid = ((int64_t)device_cus() + 7) / 8 * 8;
    const int64_t need = (ws.T + 7) / 8 * 8;
    if (grid > need) grid = need;
#define MGR_PRT(RB_, TR_)                                                                     \
    {                                                                                         \
        auto k = pack_ranked_kernel<RB_, TR_>;                                                \
        ensure_lds(k, lds);                                                                   \
        hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(1024), (size_t)lds, s,               \
                           (const uint8_t*)src, n, ids, ranks, tile_starts, nbins,            \
                           ws.offsets, ws.T, (uint8_t*)dst, ws.scan_err);                     \
        e = hipGetLastError();                                                                \
    }
#define MGR_PR(RB_)                                                                           \
    case RB_:                                                                                 \
        if (tile_rows == 4096) MGR_PRT(RB_, 4096) else MGR_PRT(RB_, kFineTR)                  \
        break;
    switch ((int)row_bytes) {
        MGR_PR(4) MGR_PR(8) MGR_PR(12) MGR_PR(16) MGR_PR(20) MGR_PR(24) MGR_PR(28) MGR_PR(32)
        MGR_PR(36)
        default: break;
    }
    if (e == hipErrorNotSupported && tile_rows == kFineTR) {
        switch ((int)row_bytes) {
#undef MGR_PR
#define MGR_PR(RB_) case RB_: MGR_PRT(RB_, kFineTR) break;
            MGR_PR(40) MGR_PR(44) MGR_PR(48) MGR_PR(52) MGR_PR(56) MGR_PR(60) MGR_PR(64)
            default: break;
        }
    }
#undef MGR_PR
#undef MGR_PRT
    prof_end(s, K_PACK_FINE);
    return e;
}

// Rows of 24..60 (pack_img 2: 12..60) bytes, 4-byte multiples but not 16-byte ones: the
// image pack (16-byte global accesses) when the source is 16-byte aligned,
// the outputs 4-byte aligned, <= 64 bins and <= 16 waves per tile.
static hipError_t pack_img(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                           int nb, int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                           int redirect_bin, void* redirect_dst, hipStream_t s, SideField* side,
                           const Hooks& h) {
    uintptr_t a = (uintptr_t)dst | (uintptr_t)row_bytes;
    if (redirect_dst) a |= (uintptr_t)redirect_dst;
    // pack_img 1: rows of >= 24 bytes (A/B: 36 B 0.90 vs 1.05 ms, 40 B 0.97 vs
    // 1.00, 24 B 0.70 vs 0.71; 12 B 0.56 vs 0.48 -- the LDS passes cost more
    // than narrow units for small rows); 2: every size it takes (tests)
    const int64_t min_rb = h.pack_img_all ? 12 : 24;
    if (((uintptr_t)src & 15) || (a & 3) || row_bytes % 16 == 0 ||
        row_bytes < min_rb || row_bytes > 60 || nb > 64 || tile_rows > 1024 ||
        dest_bytes(nb) != 1)
        return hipErrorNotSupported;
#define MGR_PI(RB_) case RB_: return pack_img_t<RB_>(src, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side);
    switch ((int)row_bytes) {
        MGR_PI(12) MGR_PI(20) MGR_PI(24) MGR_PI(28) MGR_PI(36) MGR_PI(40) MGR_PI(44)
        MGR_PI(52) MGR_PI(56) MGR_PI(60)
        default: break;
    }
#undef MGR_PI
    return hipErrorNotSupported;
}

template <int W>
static hipError_t pack_w(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nb,
                         int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                         int redirect_bin, void* redirect_dst, hipStream_t s, SideField* side,
                         const Hooks& h) {
    if constexpr (W >= 4) {
        if (nb > 64 && nb <= 1024 && row_bytes <= 64 && tile_rows == many_round_rows(nb)) {
            const hipError_t e = dest_bytes(nb) == 1
                ? pack_many_t<W, uint8_t>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s)
                : pack_many_t<W, uint16_t>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
            if (e != hipErrorNotSupported) return e;
        }
    }
    if constexpr (W == 2) {   // 2-byte rows (the fine cells travelling with config-5 rows)
        if (nb <= 64 && row_bytes == 2) {
            const hipError_t e = pack_coop_u<2, 1>(src, n, dest, nb, drop_bin, tile_rows, ws, dst,
                                                   redirect_bin, redirect_dst, s, nullptr, h);
            if (e != hipErrorNotSupported) return e;
        }
    }
    if (nb <= 64 && row_bytes <= 64 && W >= 4) {
        const hipError_t e = pack_coop_t<W>(src, row_bytes, n, dest, nb, drop_bin, tile_rows,
                                             ws, dst, redirect_bin, redirect_dst, s, side, h);
        if (e != hipErrorNotSupported) return e;
    }
    const bool wide = row_bytes > 256;
    if (dest_bytes(nb) == 1)
        return wide ? pack_t<W, uint8_t, true>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s)
                    : pack_t<W, uint8_t, false>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
    return wide ? pack_t<W, uint16_t, true>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s)
                : pack_t<W, uint16_t, false>(src, row_bytes, n, dest, nb, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s);
}

static hipError_t launch_pack_rows(const void* src, int64_t row_bytes, int64_t n,
                                   const void* dest, int nbins, int drop_bin, int tile_rows,
                                   const Workspace& ws, void* dst, int redirect_bin,
                                   void* redirect_dst, hipStream_t s, SideField* side);

hipError_t launch_pack(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                       int nbins, int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                       int redirect_bin, void* redirect_dst, hipStream_t s, const uint16_t* ids_src,
                       uint16_t* ids_dst, uint16_t* ids_red) {
    if (n <= 0) return hipSuccess;
    SideField side{ids_src, ids_dst, ids_red, false};
    hipError_t e = launch_pack_rows(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst,
                                    redirect_bin, redirect_dst, s, ids_src ? &side : nullptr);
    const bool rest = ids_src && !side.used;
    if (e != hipSuccess || !rest) return e;
    // the kernel that moved the rows cannot carry the ids: a 2-byte-row pack
    return launch_pack_rows(ids_src, 2, n, dest, nbins, drop_bin, tile_rows, ws, ids_dst,
                            redirect_bin, ids_red, s, nullptr);
}

// The cooperative multi-field kernel for a field signature it is built for
// (hipErrorNotSupported otherwise): each field's unit width -- the widest of
// 16/8/4 bytes dividing its row and every pointer -- and units per row.
static int coop_unit(const void* src, int64_t rb, const void* dst, const void* red) {
    uintptr_t a = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)rb;
    if (red) a |= (uintptr_t)red;
    const int W = (a & 15) == 0 ? 16 : (a & 7) == 0 ? 8 : (a & 3) == 0 ? 4 : 0;
    if (!W || rb / W > 16) return -1;
    return W * 32 + (int)(rb / W);
}

static hipError_t pack_coop_fields(int nf, const void* const* srcs, const int64_t* row_bytes,
                                   int64_t n, const void* dest, int nbins, int drop_bin,
                                   int tile_rows, const Workspace& ws, void* const* dsts,
                                   int redirect_bin, void* const* reds, hipStream_t s,
                                   const uint16_t* ids_src, uint16_t* ids_dst, uint16_t* ids_red) {
    int u[4] = {0, 0, 0, 0};
    CoopFieldPtrs fp{};
    for (int f = 0; f < nf; ++f) {
        u[f] = coop_unit(srcs[f], row_bytes[f], dsts[f], reds ? reds[f] : nullptr);
        if (u[f] < 0) return hipErrorNotSupported;
        fp.src[f] = (const uint8_t*)srcs[f];
        fp.dst[f] = (uint8_t*)dsts[f];
        fp.red[f] = reds ? (uint8_t*)reds[f] : nullptr;
    }
    auto sig = [&](int a, int b, int c, int d) { return u[0] == a && u[1] == b && u[2] == c && u[3] == d; };
    constexpr int F4x1 = 4 * 32 + 1, F4x3 = 4 * 32 + 3, F8x1 = 8 * 32 + 1, F8x3 = 8 * 32 + 3,
                  F16x2 = 16 * 32 + 2, F4x9 = 4 * 32 + 9, F16x1 = 16 * 32 + 1, F8x2 = 8 * 32 + 2;
    const int threads = tile_rows;   // one wave per 64-row round
#define MGR_PCF(A, B, C, D)                                                                          {                                                                                                    prof_begin(s, K_PACK);                                                                           hipLaunchKernelGGL((pack_coop_fields_kernel<A, B, C, D>), dim3((unsigned)ws.tn),                                     dim3(threads), 0, s, fp, n, (const uint8_t*)dest, nbins,                                          nbits_for(nbins), drop_bin, ws.offsets, ws.bin_starts, ws.T, ws.t0,                               ws.tn, tile_rows, redirect_bin, kXcdPackChunk, ws.scan_err, ids_src,                              ids_dst, ids_red);                                                             prof_end(s, K_PACK);                                                                             return hipGetLastError();                                                                    }
    // config 5's fields as arrays: pos f32 x3, vel f32 x3, mass f32, id i64
    if (sig(F4x3, F4x3, F4x1, F8x1)) MGR_PCF(F4x3, F4x3, F4x1, F8x1)
    // f64 positions + i64 ids; 32-byte records + their f64 positions (return_positions)
    if (sig(F8x3, F8x1, 0, 0)) MGR_PCF(F8x3, F8x1, 0, 0)
    if (sig(F16x2, F8x3, 0, 0)) MGR_PCF(F16x2, F8x3, 0, 0)
    // 36-byte records + their f32 positions (config 5 with return_positions)
    if (sig(F4x9, F4x3, 0, 0)) MGR_PCF(F4x9, F4x3, 0, 0)
    // positions f32 x3 + ids i64 / f64 x2 + i64
    if (sig(F4x3, F8x1, 0, 0)) MGR_PCF(F4x3, F8x1, 0, 0)
    if (sig(F16x1, F8x1, 0, 0)) MGR_PCF(F16x1, F8x1, 0, 0)
    if (sig(F8x3, F8x3, F8x1, 0)) MGR_PCF(F8x3, F8x3, F8x1, 0)
    if (sig(F4x3, F4x3, F8x1, 0)) MGR_PCF(F4x3, F4x3, F8x1, 0)
    if (sig(F8x2, F8x1, 0, 0)) MGR_PCF(F8x2, F8x1, 0, 0)
#undef MGR_PCF
    return hipErrorNotSupported;
}

// mgr_pack_fields: several fields of the same rows, one ranking.  With one
// field this is launch_pack (the coop / image kernels A/B'd for it).  With
// more, the fields pack_fields_kernel takes (4-byte-multiple rows, 16-byte
// aligned sources, 4-byte aligned outputs, <= 64 bins on 1-byte
// destinations, tiles of 128-row waves) move in as few launches as their LDS
// rows allow -- one for every realistic SoA set -- carrying the side field;
// any other field is packed by launch_pack on the same destinations.
hipError_t launch_pack_fields(int nf, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                              const void* dest, int nbins, int drop_bin, int tile_rows,
                              const Workspace& ws, void* const* dsts, int redirect_bin,
                              void* const* reds, hipStream_t s, const uint16_t* ids_src,
                              uint16_t* ids_dst, uint16_t* ids_red) {
    if (n <= 0) return hipSuccess;
    if (nf == 1)
        return launch_pack(srcs[0], row_bytes[0], n, dest, nbins, drop_bin, tile_rows, ws, dsts[0],
                           redirect_bin, reds ? reds[0] : nullptr, s, ids_src, ids_dst, ids_red);
    const Hooks& h = hooks();
    const int nw = tile_rows / kFieldsWR;
    const bool shape = !h.pack_generic && nbins <= 64 && dest_bytes(nbins) == 1 &&
                       tile_rows % kFieldsWR == 0 && nw >= 1 && nw <= 16;
    // rows of one wave's fields, within the LDS a workgroup may take
    const int budget = (160 * 1024 - nw * 256) / max(nw, 1) - kFieldsTail;
    std::vector<int> fast, slow;
    for (int f = 0; f < nf; ++f) {
        uintptr_t a = (uintptr_t)dsts[f] | (uintptr_t)row_bytes[f];
        if (redirect_bin >= 0 && reds) a |= (uintptr_t)reds[f];
        const bool ok = shape && row_bytes[f] >= 4 && row_bytes[f] % 4 == 0 &&
                        (int64_t)kFieldsWR * row_bytes[f] <= budget &&
                        ((uintptr_t)srcs[f] & 15) == 0 && (a & 3) == 0;
        (ok ? fast : slow).push_back(f);
    }
    if (fast.size() < 2) {   // nothing to share: each field by its own kernel
        slow.insert(slow.end(), fast.begin(), fast.end());
        fast.clear();
    }
    bool side_done = ids_src == nullptr;
    int max_rb = 0;
    for (const int f : fast) max_rb = max(max_rb, (int)row_bytes[f]);
    const int want = h.fields_kernel;   // test hook: 0 = the product's choice
    if ((want == 0 || want == 2) && fast.size() == (size_t)nf && nf <= kFieldsMax &&
        max_rb <= 64 && nw <= 16) {
        // every field in the tile-image kernel when they fit one launch
        int rows = 0;
        PackFieldsArgs fa{};
        for (const int f : fast) {
            fa.src[fa.nf] = (const uint8_t*)srcs[f];
            fa.dst[fa.nf] = (uint8_t*)dsts[f];
            fa.red[fa.nf] = reds ? (uint8_t*)reds[f] : nullptr;
            fa.rb[fa.nf] = (int)row_bytes[f];
            fa.loff[fa.nf] = rows;
            rows += kFieldsWR * (int)row_bytes[f];
            ++fa.nf;
        }
        fa.wave_lds = rows;
        const int img = align16(tile_rows * max_rb);
        const int lds = img + align16(tile_rows) + nw * fa.wave_lds + nw * 64 * 4;
        if (lds <= 150 * 1024) {
            ensure_lds(pack_fields_tile_kernel, lds);
            prof_begin(s, K_PACK);
            hipLaunchKernelGGL(pack_fields_tile_kernel, dim3((unsigned)ws.tn), dim3(64 * nw),
                               (size_t)lds, s, fa, n, (const uint8_t*)dest, nbins,
                               nbits_for(nbins), drop_bin, ws.offsets, ws.bin_starts, ws.T, ws.t0,
                               ws.tn, tile_rows, redirect_bin, kXcdPackChunk, ws.scan_err, ids_src,
                               ids_dst, ids_red, img);
            prof_end(s, K_PACK);
            return hipGetLastError();
        }
    }
    if ((want == 0 || want == 3) && fast.size() == (size_t)nf && nf <= 4 &&
        tile_rows <= 64 * kCoopMaxRounds && tile_rows / 64 <= 16) {
        // every field in the cooperative multi-field kernel when the fields'
        // signature is one it is built for
        const hipError_t e = pack_coop_fields(nf, srcs, row_bytes, n, dest, nbins, drop_bin,
                                              tile_rows, ws, dsts, redirect_bin, reds, s, ids_src,
                                              ids_dst, ids_red);
        if (e != hipErrorNotSupported) return e;
    }
    size_t i = 0;
    while (i < fast.size()) {
        PackFieldsArgs fa{};
        int rows = 0;
        for (; i < fast.size() && fa.nf < kFieldsMax; ++i) {
            const int f = fast[i];
            const int rb = (int)row_bytes[f];
            if (rows + kFieldsWR * rb > budget) break;
            fa.src[fa.nf] = (const uint8_t*)srcs[f];
            fa.dst[fa.nf] = (uint8_t*)dsts[f];
            fa.red[fa.nf] = reds ? (uint8_t*)reds[f] : nullptr;
            fa.rb[fa.nf] = rb;
            fa.loff[fa.nf] = rows;
            rows += kFieldsWR * rb;   // a multiple of 512 bytes
            ++fa.nf;
        }
        fa.wave_lds = rows + kFieldsTail;
        const int lds = nw * 64 * 4 + nw * fa.wave_lds;
        ensure_lds(pack_fields_kernel, lds);
        prof_begin(s, K_PACK);
        hipLaunchKernelGGL(pack_fields_kernel, dim3((unsigned)ws.tn), dim3(64 * nw), (size_t)lds, s,
                           fa, n, (const uint8_t*)dest, nbins, nbits_for(nbins), drop_bin,
                           ws.offsets, ws.bin_starts, ws.T, ws.t0, ws.tn, tile_rows, redirect_bin,
                           kXcdPackChunk, ws.scan_err, side_done ? nullptr : ids_src, ids_dst,
                           ids_red);
        prof_end(s, K_PACK);
        side_done = true;
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    for (const int f : slow) {
        const hipError_t e = launch_pack(srcs[f], row_bytes[f], n, dest, nbins, drop_bin, tile_rows,
                                         ws, dsts[f], redirect_bin, reds ? reds[f] : nullptr, s,
                                         side_done ? nullptr : ids_src, ids_dst, ids_red);
        side_done = true;
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

static hipError_t launch_pack_rows(const void* src, int64_t row_bytes, int64_t n,
                                   const void* dest, int nbins, int drop_bin, int tile_rows,
                                   const Workspace& ws, void* dst, int redirect_bin,
                                   void* redirect_dst, hipStream_t s, SideField* side) {
    // Widest unit dividing the row and every base address.
    uintptr_t a = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)row_bytes;
    if (redirect_dst) a |= (uintptr_t)redirect_dst;
    // profiler: narrow (< 4-byte) rows apart
    const int kid = row_bytes < 4 ? K_PACK_NARROW : K_PACK;
    const Hooks& h = hooks();   // one snapshot for the whole launch
    prof_begin(s, kid);
    hipError_t e = pack_img(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst,
                            redirect_bin, redirect_dst, s, side, h);
    if (e != hipErrorNotSupported) {
        prof_end(s, kid);
        return e;
    }
    if ((a & 15) == 0) e = pack_w<16>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side, h);
    else if ((a & 7) == 0) e = pack_w<8>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side, h);
    else if ((a & 3) == 0) e = pack_w<4>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side, h);
    else if ((a & 1) == 0) e = pack_w<2>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side, h);
    else e = pack_w<1>(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst, redirect_bin, redirect_dst, s, side, h);
    prof_end(s, kid);
    return e;
}

}  // namespace mgr
