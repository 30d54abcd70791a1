// One-pass source partition (gfx950): bin + rank + scatter of records whose
// positions sit inside the rows (config 5's 36-byte records with their f32
// position view, S9), reading every record ONCE.  The classic path reads the
// record lines twice -- the bin pass fetches the whole lines its positions
// sit in, the pack reads them again (116 B/row for 36-byte rows with fine
// ids) -- this kernel moves 36 + 36 + 2 = 74 B/row.
//
// Output: the reference's send_buff list itself (redist.py:195-198,
// send_buff[i] = data[rank_to_send == i], original order kept): bin b's rows
// go to their own region out + b * cap * row_bytes (and their fine ids to
// fine_out + b * cap), in order.  No global bin starts are needed before a
// row is placed: a tile's place inside every bin's region is the sum of the
// earlier tiles' counts of that bin, found by a decoupled look-back per bin
// over the tiles (the one-pass scan's word format, mgr_device.h: status +
// poison + value in one 64-bit word, bounded polls).  Tiles take tickets in
// dispatch order, so a tile only ever waits on tiles that already run.
// bin_counts[b] = bin b's rows (the last tile's inclusive prefix); rows at
// or past cap are not written -- the caller compares the counts with cap
// (overflow: redo with the classic path, whose bin pass re-reads the stored,
// already wrapped positions with periodic = 0 and bins them identically, S2).
// A look-back that gives up (bounded polls) poisons its prefix: every later
// tile writes nothing and the counts read -1.
#include "mgr_device.h"

namespace mgr {

constexpr int kOneWR = 128;   // rows per wave (two 64-row rounds)
constexpr int kOneNW = 8;     // waves per workgroup: 1024-row tiles
constexpr int kOneTile = kOneWR * kOneNW;

struct OnePassCtl {
    uint32_t ticket;   // tiles in dispatch order
    uint32_t err;      // a look-back gave up
};

int64_t onepass_tiles(int64_t n) { return (n + kOneTile - 1) / kOneTile; }

// [T][nbins] look-back words, then the control words; zeroed before a launch.
int64_t onepass_workspace_bytes(int64_t n, int nbins) {
    return (onepass_tiles(n) * (int64_t)nbins) * 8 + (int64_t)sizeof(OnePassCtl) + 8;
}

static int onepass_lds_bytes(int nw, int rb, int nb) {
    const int nbe = (nb + 1) & ~1;
    return nw * (kOneWR * rb + 8 * nbe + 2 * kOneWR) + 16 * nbe + 4 * nw * nb;
}

template <typename PosT, bool kP, int SIDE, int GEO, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(8))) void onepass_partition_kernel(
    uint8_t* __restrict__ data, int rb, int pos_off, int64_t n, Geom g, FineGeom fg,
    uint8_t* __restrict__ out, uint16_t* __restrict__ fine_out, int64_t cap,
    int64_t* __restrict__ bin_counts, uint64_t* __restrict__ words, int64_t T, int spins,
    int write_all) {
    constexpr int WR = kOneWR, RPW = WR / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ int s_tile, s_poison;
    OnePassCtl* ctl = (OnePassCtl*)(words + T * g.nbins);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    const int nb = g.nbins;
    if (threadIdx.x == 0) {
        s_tile = (int)__hip_atomic_fetch_add(&ctl->ticket, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        s_poison = 0;
    }
    __syncthreads();
    const int64_t tile = s_tile;
    // LDS (onepass_lds_bytes): per wave its rows, the bins' output addresses,
    // the inverse permutation and the slots' bins; then the waves' bin counts
    // and the tile's bases and counts -- sized by the bins, so 8-bin 36-byte
    // rows take < 40 KiB and, with <= 64 VGPRs (amdgpu_waves_per_eu(8)), four
    // workgroups fit a CU: a tile waiting on its look-back leaves three to keep
    // memory busy (A/B, 64M config-5 rows: 1.19-1.20 ms against 1.39 with the
    // 64-entry tables and three per CU; 512-row tiles, eight per CU: 1.60; a
    // persistent grid taking tiles by ticket: 1.40, and 2.64 with the next
    // ticket taken during the look-back -- the held tile delays its successors)
    const int nbe = (nb + 1) & ~1;
    const int wave_lds = WR * rb + 8 * nbe + 2 * WR;
    uint8_t* wl = smem + w * wave_lds;
    unsigned long long* gaddr = (unsigned long long*)(wl + WR * rb);   // WR * rb: a multiple of 512
    uint8_t* inv = (uint8_t*)(gaddr + nbe);
    uint8_t* ibin = inv + WR;
    long long* s_base = (long long*)(smem + NW * wave_lds);
    long long* s_agg = s_base + nbe;
    int* s_cnt = (int*)(s_agg + nbe);   // [NW][nb]
    const int64_t row0 = tile * (int64_t)(WR * NW) + (int64_t)WR * w;
    const int nrows = __builtin_amdgcn_readfirstlane(
        (int)max((int64_t)0, min((int64_t)WR, n - row0)));
    const int nbytes = nrows * rb;
    uint8_t* gp = data + row0 * rb;
    // the wave's records into LDS (LDS-DMA: wave-uniform base + lane * 16;
    // lanes past the rows masked off; the array's last unit reads up to 12
    // bytes past its end, inside the 16-byte-aligned unit's page)
    for (int i = 0; 1024 * i < nbytes; ++i) {
        const int x = 16 * (64 * i + lane);
        if (x < nbytes)
            __builtin_amdgcn_global_load_lds(
                (const void*)(gp + x), (__attribute__((address_space(3))) void*)(wl + 1024 * i), 16,
                0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wave_sync();
    // bin every row from its LDS copy (the wrap is written into the copy, S1)
    unsigned b[RPW], side[RPW];
    bool valid[RPW];
    bool dirty = false;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int r = 64 * q + lane;
        valid[q] = r < nrows;
        b[q] = 0;
        side[q] = 0;
        if (valid[q]) {
            long long sc = 0;
            b[q] = (unsigned)bin_row<PosT, kP, 3, SIDE, GEO>((PosT*)(wl + r * rb + pos_off), g,
                                                             nullptr, &dirty, &fg, nullptr, &sc);
            side[q] = (unsigned)sc;
        }
    }
    wave_sync();
    // the caller's array holds the wrapped positions (redist.py:68 in place):
    // the wave's rows go back when one of them changed (or always, write_all)
    if (kP && (write_all || __ballot(dirty) != 0ull)) {
        const int full = nbytes & ~15;
        for (int x = 16 * lane; x < full; x += 1024)
            *(u32x4_t*)(gp + x) = *(const u32x4_t*)(wl + x);
        for (int x = full + 4 * lane; x < nbytes; x += 256)
            *(uint32_t*)(gp + x) = *(const uint32_t*)(wl + x);
    }
    // rank inside each round; lane l counts bin l over the wave's rounds
    unsigned long long pe[RPW];
    int cq[RPW], cnt = 0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        unsigned long long p = __ballot(valid[q]), mine = p;
        for (int i = 0; i < g.nbits; ++i) {
            const unsigned long long m = __ballot((b[q] >> i) & 1u);
            p &= ((b[q] >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        pe[q] = p;
        cq[q] = __popcll(mine);
        cnt += cq[q];
    }
    if (lane < nb) s_cnt[w * nb + lane] = cnt;
    __syncthreads();
    // the tile's count of every bin, published at once (wave 0, lane b) so
    // later tiles can look past this one before its prefix is known
    if (w == 0 && lane < nb) {
        long long agg = 0;
#pragma unroll
        for (int j = 0; j < NW; ++j) agg += s_cnt[j * nb + lane];
        s_agg[lane] = agg;
        flag_store(words + tile * nb + lane, (tile == 0 ? kScanInc : kScanAgg) | (uint64_t)agg);
    }
    __syncthreads();
    // the earlier tiles' counts of every bin, by wave 0: lane k * nbp + b
    // reads bin b's word of tile base - k (nbp = bins rounded up to a power of
    // two, a window of 64 / nbp tiles per bin and round trip: 8 for 8 bins),
    // summing up to the nearest inclusive prefix.  (A/B, round 6: one wave per
    // bin reading 64 tiles per round trip measured slower -- every look-back
    // word is an agent-scope load past the XCD's L2 -- and one lane per bin
    // polling one tile at a time too.)
    if (w == 0) {
        const int nbp = nb <= 1 ? 1 : 1 << (32 - __clz(nb - 1));
        const int win = 64 / nbp;
        const int bb = lane & (nbp - 1), k = lane / nbp;
        unsigned long long grp = 0;   // the lanes of one bin: bits bb, bb + nbp, ...
        for (int j = 0; j < win; ++j) grp |= 1ull << (j * nbp);
        grp <<= bb;
        bool done = bb >= nb || tile == 0;
        long long excl = 0;
        uint64_t poison = 0;
        for (int64_t base = tile - 1;; base -= win) {
            const int64_t idx = base - k;
            uint64_t v = kScanInc;
            if (!done && idx >= 0) v = flag_poll(words + idx * nb + bb, 1, poison ? 0 : spins);
            const unsigned long long im = __ballot(!done && (v >> 62) >= 2) & grp;
            const int first = im ? __ffsll((long long)im) - 1 : 64;   // nearest inclusive of my bin
            const bool used = !done && lane <= first;
            long long x = used ? (long long)(v & kScanVal) : 0;
            if (__ballot(used && (v & kScanPoison)) & grp) poison = kScanPoison;
            for (int o = nbp; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
            excl += x;
            if (im) done = true;
            if (__ballot(!done) == 0ull) break;
        }
        if (k == 0 && bb < nb) {
            if (tile > 0)
                flag_store(words + tile * nb + bb, kScanInc | poison | (uint64_t)(excl + s_agg[bb]));
            s_base[bb] = excl;
            if (tile == T - 1) bin_counts[bb] = poison ? -1 : excl + s_agg[bb];
            if (poison) {
                s_poison = 1;
                __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    if (s_poison || nrows == 0) return;
    // this wave's rows of bin b start at the tile's base + the earlier waves' counts
    long long tbase = 0;
    if (lane < nb) {
        tbase = s_base[lane];
        for (int j = 0; j < w; ++j) tbase += s_cnt[j * nb + lane];
    }
    const int excl = wave_incl_dpp(cnt) - cnt;   // the bins' image starts (bin-major)
    int run = excl;
    int slot[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        // (shuffles in uniform control flow)
        slot[q] = __shfl(run, (int)b[q], 64) + (valid[q] ? rank_in(pe[q]) : 0);
        const long long orow = __shfl(tbase - excl, (int)b[q], 64) + slot[q];   // row in the region
        run += cq[q];
        if (valid[q]) {
            inv[slot[q]] = (uint8_t)(64 * q + lane);
            ibin[slot[q]] = (uint8_t)b[q];
            if (SIDE == kSideFine && orow < cap)
                fine_out[(int64_t)b[q] * cap + orow] = (uint16_t)side[q];
        }
    }
    // lane b: region row of bin b's image slot 0; a bin whose rows of this
    // wave would reach cap writes none of them (the caller sees count > cap
    // and redoes the partition)
    const long long ro = tbase - excl;
    if (lane < nb) {
        gaddr[lane] = tbase + cnt > cap ? 0ull
                      : (unsigned long long)(out + ((int64_t)lane * cap + ro) * rb);
    }
    wave_sync();
    // the destination-ordered image streamed out in 16-byte units
    switch (rb) {
        case 32: image_pass<32, RPW>(wl, ibin, gaddr, slot, valid, nrows, lane); break;
        case 36: image_pass<36, RPW>(wl, ibin, gaddr, slot, valid, nrows, lane); break;
        default: {   // any 4-byte multiple: gathered through the inverse permutation
            const uint32_t rinv = (uint32_t)(0x100000000ull / (unsigned)rb + 1);
            for (int x = 16 * lane; x < nbytes; x += 1024) {
                int s[4];
                u32x4_t v;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const int xd = min(x + 4 * d, nbytes - 4);
                    s[d] = (int)__umulhi((unsigned)xd, rinv);
                    v[d] = *(const uint32_t*)(wl + (int)inv[s[d]] * rb + (xd - s[d] * rb));
                }
                const int bf = ibin[s[0]], bl = ibin[s[3]];
                const unsigned long long af = gaddr[bf];
                if (x + 16 <= nbytes && bf == bl) {
                    if (af) gstore<u32x4_a4>(af + x, v);
                } else {
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const int xd = x + 4 * d;
                        const unsigned long long ad = gaddr[ibin[s[d]]];
                        if (xd < nbytes && ad) gstore<uint32_t>(ad + xd, v[d]);
                    }
                }
            }
        }
    }
}

template <typename PosT, bool kP, int SIDE>
static hipError_t onepass_t(const Geom& g, const FineGeom& fg, void* data, int rb, int pos_off,
                            int64_t n, void* out, uint16_t* fine_out, int64_t cap,
                            int64_t* bin_counts, uint64_t* words, hipStream_t s) {
    const Hooks& h = hooks();   // one snapshot for the launch
    constexpr int NW = kOneNW;
    auto k = onepass_partition_kernel<PosT, kP, SIDE, kGeoAny, NW>;
    if constexpr (kP) {
        const int geo = h.bin_generic ? kGeoAny : geo_kind(g, sizeof(PosT) == 4);
        if (geo == kGeoF32) k = onepass_partition_kernel<PosT, kP, SIDE, kGeoF32, NW>;
        else if (geo == kGeoF64) k = onepass_partition_kernel<PosT, kP, SIDE, kGeoF64, NW>;
    }
    const int64_t T = onepass_tiles(n);
    const int lds = onepass_lds_bytes(NW, rb, g.nbins);
    ensure_lds(k, lds);
    hipLaunchKernelGGL(k, dim3((unsigned)T), dim3(64 * NW), (size_t)lds, s, (uint8_t*)data, rb,
                       pos_off, n, g, fg, (uint8_t*)out, fine_out, cap, bin_counts, words, T,
                       h.scan_spins, g.write_back_all);
    return hipGetLastError();
}

template <typename PosT>
static hipError_t onepass_d(const Geom& g, const FineGeom* fg, void* data, int rb, int pos_off,
                            int64_t n, int periodic, void* out, uint16_t* fine_out, int64_t cap,
                            int64_t* bin_counts, uint64_t* words, hipStream_t s) {
    FineGeom f{};
    if (fg) f = *fg;
    if (periodic)
        return fg ? onepass_t<PosT, true, kSideFine>(g, f, data, rb, pos_off, n, out, fine_out, cap, bin_counts, words, s)
                  : onepass_t<PosT, true, kSideNone>(g, f, data, rb, pos_off, n, out, fine_out, cap, bin_counts, words, s);
    return fg ? onepass_t<PosT, false, kSideFine>(g, f, data, rb, pos_off, n, out, fine_out, cap, bin_counts, words, s)
              : onepass_t<PosT, false, kSideNone>(g, f, data, rb, pos_off, n, out, fine_out, cap, bin_counts, words, s);
}

hipError_t launch_onepass(const Geom& g, const FineGeom* fg, void* data, int64_t row_bytes,
                          int64_t pos_off, int pos_dtype, int64_t n, int periodic, void* out,
                          uint16_t* fine_out, int64_t cap, int64_t* bin_counts, void* workspace,
                          hipStream_t s) {
    const int psz = pos_dtype == MGR_F32 ? 4 : pos_dtype == MGR_F64 ? 8 : 0;
    // shapes this kernel takes; the caller runs the classic path otherwise
    if (!psz || g.dim != 3 || g.nbins > 64 || row_bytes % 4 || row_bytes < 4 ||
        row_bytes > 128 || pos_off < 0 || pos_off % psz || pos_off + 3 * psz > row_bytes ||
        ((uintptr_t)data & 15) || ((uintptr_t)out & 3) || ((uintptr_t)fine_out & 1) || cap < 0)
        return hipErrorNotSupported;
    if (n <= 0) return hipMemsetAsync(bin_counts, 0, (size_t)g.nbins * 8, s);
    uint64_t* words = (uint64_t*)workspace;
    hipError_t e = hipMemsetAsync(words, 0, (size_t)onepass_workspace_bytes(n, g.nbins), s);
    if (e != hipSuccess) return e;
    prof_begin(s, K_ONEPASS);
    e = psz == 4 ? onepass_d<float>(g, fg, data, (int)row_bytes, (int)pos_off, n, periodic, out,
                                    fine_out, cap, bin_counts, words, s)
                 : onepass_d<double>(g, fg, data, (int)row_bytes, (int)pos_off, n, periodic, out,
                                     fine_out, cap, bin_counts, words, s);
    prof_end(s, K_ONEPASS);
    return e;
}

}  // namespace mgr
