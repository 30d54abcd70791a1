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

//
// Translation units: mgr_bin.hip (binning), mgr_pack.hip (pack), this file
// (test hooks, workspace, scan, halo selection, synthetic input); shared
// device helpers in mgr_device.h.

#include "mgr_device.h"

#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace mgr {

// The test-hook snapshots: every published set is kept until exit (a launch
// may still hold a reference to an older one; there are a handful per test
// run), the current one behind an atomic pointer.
static const Hooks kShipped{};
static std::atomic<const Hooks*> g_hooks{&kShipped};
static std::mutex g_hooks_mu;

const Hooks& hooks() { return *g_hooks.load(std::memory_order_acquire); }

int set_hook(const char* key, int64_t v) {
    std::lock_guard<std::mutex> lk(g_hooks_mu);
    static std::vector<std::unique_ptr<Hooks>> kept;
    auto h = std::make_unique<Hooks>(hooks());
    auto in = [&](int64_t lo, int64_t hi) { return v >= lo && v <= hi; };
    if (!strcmp(key, "tile_rounds") && in(0, 64)) h->tile_rounds = (int)v;
    else if (!strcmp(key, "scan_chunk") && in(256, 1 << 20)) h->scan_chunk = (int)v;
    else if (!strcmp(key, "scan_max_chunks") && in(1, kScanFlags)) h->scan_max_chunks = (int)v;
    else if (!strcmp(key, "scan_spins") && in(-1, 1 << 30)) h->scan_spins = (int)v;
    else if (!strcmp(key, "pack_img_all") && in(0, 1)) h->pack_img_all = (int)v;
    else if (!strcmp(key, "rank_rows") && (v == 0 || v == 2048 || v == 4096)) h->rank_rows = (int)v;
    else if (!strcmp(key, "bin_unstaged") && in(0, 1)) h->bin_unstaged = (int)v;
    else if (!strcmp(key, "bin_generic") && in(0, 1)) h->bin_generic = (int)v;
    else if (!strcmp(key, "pack_generic") && in(0, 1)) h->pack_generic = (int)v;
    else if (!strcmp(key, "scan_delay_bin") && in(-1, MGR_MAX_BINS)) h->scan_delay_bin = (int)v;
    else if (!strcmp(key, "scan_delay_sleeps") && in(0, 1 << 16)) h->scan_delay_sleeps = (int)v;
    else if (!strcmp(key, "scan_end_spins") && in(-1, 1 << 30)) h->scan_end_spins = (int)v;
    else if (!strcmp(key, "scan_poison_chunk") && in(-1, 1 << 30)) h->scan_poison_chunk = (int)v;
    else if (!strcmp(key, "fields_kernel") && in(0, 3)) h->fields_kernel = (int)v;
    else return -1;
    g_hooks.store(h.get(), std::memory_order_release);
    kept.push_back(std::move(h));
    return 0;
}

// ------------------------------------------------------------------ scan
// One-pass scan (decoupled look-back).  Chunks never straddle a bin: chunk
// j covers counts [b*T + c*chunk, b*T + min(T, (c+1)*chunk)) of bin b = j /
// cpb, c = j % cpb, one workgroup each.  A chunk publishes its aggregate,
// then wave 0 looks back 64 predecessors at a time until it meets one that
// already published its inclusive prefix, publishes its own inclusive
// prefix, and the workgroup writes the chunk's exclusive offsets.  Status
// and value share one 64-bit word (mgr_device.h), stored and polled with
// agent-scope atomics (sc1, coherent across the XCDs' L2s).
// Forward progress: a workgroup takes its chunk id j from an atomic ticket,
// so chunks 0..j-1 were all taken by workgroups that are already running
// (no assumption about dispatch order), and a chunk only waits on those.
// Every poll is bounded; a look-back that gives up marks its words
// poisoned, sets ScanCtl::err (every pack kernel then writes nothing), and
// the chunk with the last ticket -- which waits until every other chunk is
// done -- writes -1 into every bin count: the failure reaches the host at
// the count read it already does, never as silently wrong offsets.
// The count producers zero the words and ScanCtl (clear_scan_flags).
// ITEMS consecutive counts per thread (a TILE of ITEMS * 256 per pass): a
// chunk that fits one tile is read once, kept in registers, and scanned with
// one block scan; longer chunks loop over tiles.
template <int ITEMS>
__global__ __launch_bounds__(kBlock) void scan_onepass_kernel(const int32_t* __restrict__ counts,
                                                              int64_t T, int64_t chunk, int cpb,
                                                              int nbins,
                                                              uint64_t* __restrict__ flags,
                                                              int64_t* __restrict__ offsets,
                                                              int64_t* __restrict__ bin_starts,
                                                              int64_t* __restrict__ bin_counts,
                                                              int spins, ScanTest tst) {
    constexpr int TILE = ITEMS * kBlock;
    __shared__ long long s_w[kWaves];
    __shared__ long long s_excl;
    __shared__ int s_j, s_poison;
    __shared__ uint64_t s_incl;   // the inclusive word (test hook: stored late)
    ScanCtl* ctl = scan_ctl(flags);
    if (threadIdx.x == 0) {
        s_j = (int)__hip_atomic_fetch_add(&ctl->ticket, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        s_poison = 0;
    }
    __syncthreads();
    const int j = s_j;
    const int b = j / cpb, c = j - b * cpb;
    const int64_t lo = (int64_t)b * T + (int64_t)c * chunk;
    const int64_t hi = (int64_t)b * T + min(T, (int64_t)(c + 1) * chunk);
    const bool one_tile = hi - lo <= TILE;
    const int64_t mine = lo + (int64_t)threadIdx.x * ITEMS;
    int v[ITEMS];
    long long acc = 0;
    if (one_tile) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            v[k] = mine + k < hi ? counts[mine + k] : 0;
            acc += v[k];
        }
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) acc += counts[i];
    }
    long long agg;
    const long long tex = block_excl_scan(acc, &agg, s_w);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        long long excl = 0;
        // test hook: this chunk's prefix is published poisoned -- every
        // prefix built on it carries the bit, the scan reports a failure
        uint64_t poison = j == tst.poison_chunk ? kScanPoison : 0;
        // test hook: the chunk ending bin tst.delay_bin stores its inclusive
        // word only after counting itself done
        const bool late = tst.delay_bin >= 0 && j == (tst.delay_bin + 1) * cpb - 1 &&
                          j != (int)gridDim.x - 1;
        if (j == 0) {
            if (lane == 0 && !late) flag_store(&flags[0], kScanInc | poison | (uint64_t)agg);
            if (lane == 0) s_incl = kScanInc | poison | (uint64_t)agg;
        } else {
            if (lane == 0) flag_store(&flags[j], kScanAgg | (uint64_t)agg);
            for (int base = j - 1;; base -= 64) {
                const int idx = base - lane;
                // after a give-up, no more waiting: one look per word
                const uint64_t w = idx >= 0 ? flag_poll(&flags[idx], 1, poison ? 0 : spins)
                                            : kScanInc;
                const unsigned long long inc = __ballot((w >> 62) >= 2);
                long long x = (long long)(w & kScanVal);
                // lanes up to the nearest predecessor with an inclusive prefix
                const bool used = !(inc && lane > __ffsll((long long)inc) - 1);
                if (!used) x = 0;
                if (__ballot(used && (w & kScanPoison))) poison = kScanPoison;
#pragma unroll
                for (int o = 32; o; o >>= 1) x += __shfl_xor(x, o, 64);
                excl += x;
                if (inc) break;
            }
            if (lane == 0 && !late) flag_store(&flags[j], kScanInc | poison | (uint64_t)(excl + agg));
            if (lane == 0) s_incl = kScanInc | poison | (uint64_t)(excl + agg);
        }
        if (lane == 0) {
            s_excl = excl;
            if (poison) {
                s_poison = 1;
                __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    long long carry = s_excl;
    if (c == 0 && threadIdx.x == 0) bin_starts[b] = carry;
    if (one_tile) {
        long long ex = carry + tex;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            if (mine + k < hi) offsets[mine + k] = ex;
            ex += v[k];
        }
    } else {
        for (int64_t base = lo; base < hi; base += TILE) {
            const int64_t m = base + (int64_t)threadIdx.x * ITEMS;
            long long t = 0;
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                v[k] = m + k < hi ? counts[m + k] : 0;
                t += v[k];
            }
            long long tot;
            long long ex = block_excl_scan(t, &tot, s_w) + carry;
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                if (m + k < hi) offsets[m + k] = ex;
                ex += v[k];
            }
            carry += tot;
        }
    }
    __syncthreads();
    // one word counts the finished chunks (bits 0-31) and the failed ones
    // (bits 32-63): relaxed atomics on ONE location are seen in order, so no
    // fences (a release here costs an L2 write-back per workgroup)
    constexpr uint64_t kDoneMask = 0xFFFFFFFFull;
    if (j != (int)gridDim.x - 1) {
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(&ctl->done, 1ull + (s_poison ? (1ull << 32) : 0ull),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tst.delay_bin >= 0 && j == (tst.delay_bin + 1) * cpb - 1) {
                // test hook (scan_delay_bin): this chunk is seen done long
                // before its inclusive word -- the visibility order relaxed
                // atomics on two words allow -- so the last ticket must poll
                // the bin-end words (tests/test_gpu_api.py scan race test)
                for (int i = 0; i < tst.delay_sleeps; ++i) __builtin_amdgcn_s_sleep(127);
                flag_store(&flags[j], s_incl);
            }
        }
        return;
    }
    // The last ticket: wait until every other chunk is done (all of them hold
    // earlier tickets, so they are running and their polls are bounded), then
    // every bin's total from the inclusive prefixes at the bin ends -- or -1
    // everywhere when any look-back gave up.
    if (threadIdx.x == 0) {
        const uint64_t others = gridDim.x - 1;
        int spin = 0;
        uint64_t v;
        while (((v = __hip_atomic_load(&ctl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) &
                kDoneMask) < others) {
            if (spins < 0 || ++spin > (1 << 26)) {   // a lost chunk: fail loudly
                v |= 1ull << 32;
                __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (v >> 32) s_poison = 1;
    }
    __syncthreads();
    const bool failed = s_poison != 0;
    const long long total = s_excl + agg;
    if (bin_counts) {
        // Every bin's total from the inclusive words at the bin ends.  Each
        // chunk counted itself done AFTER storing its word, but relaxed
        // atomics on two locations are not ordered for another reader: the
        // done count can be seen before the word.  So the words are polled
        // (bounded, like every look-back) rather than read once -- one look
        // could read a bin end's aggregate as its prefix (a wrong count).
        const int end_spins = tst.end_spins >= 0 ? tst.end_spins : spins;   // hook: 0 = one look
        for (int bb = threadIdx.x; bb < nbins; bb += kBlock) {
            bool bad = failed;
            long long st = 0, en = total;
            if (bb > 0) {
                const uint64_t w = flag_poll(&flags[bb * cpb - 1], 2, end_spins);
                st = (long long)(w & kScanVal);
                bad |= (w & kScanPoison) != 0;
            }
            if (bb < nbins - 1) {
                const uint64_t w = flag_poll(&flags[(bb + 1) * cpb - 1], 2, end_spins);
                en = (long long)(w & kScanVal);
                bad |= (w & kScanPoison) != 0;
            }
            if (bad && !failed)
                __hip_atomic_store(&ctl->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bin_counts[bb] = bad ? -1 : en - st;
        }
    }
    if (threadIdx.x == 0) bin_starts[nbins] = failed ? -1 : total;
}

// ---------------------------------------------------------- halo (f1)
// exchange_overload_by_position (redist.py:202-309) selects, per dimension
// d, the rows with position[:, d] > limits[d,1] - ol[d] (sent to the right
// neighbour, :271/:274) and position[:, d] < limits[d,0] + ol[d] (to the
// left, :272/:275).  numpy compares the column (any float, integer or bool
// dtype) against the float64 threshold in float64 (pos_as_f64), NaN selects
// nothing.
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
            const double x = pos_as_f64(pos[r * stride + d]);
            f |= (x > t.hi[d] ? 1u : 0u) << (2 * d);
            f |= (x < t.lo[d] ? 1u : 0u) << (2 * d + 1);
        }
        flags[r] = (uint16_t)f;
    }
}

// Multi-selection counts (the halo's sends, redist.py:271-275, all at once):
// set s selects the rows whose flags hold every bit of masks.m[s] -- a row
// may be in several sets (near an edge or a corner).  Wave-private tiles of
// tile_rows rows read in kSelChunk-row chunks (chunk_flags); counts[s * T +
// tile] for mgr_scan with nbins = nsets, whose offsets then lay the sets out
// one after the other, each in row order.
template <int NB>
__global__ __launch_bounds__(kBlock) void msel_count_kernel(const uint16_t* __restrict__ flags,
                                                            int64_t n, int nsets, SetMasks masks,
                                                            int32_t* __restrict__ counts,
                                                            int64_t T, int tile_rows,
                                                            uint64_t* __restrict__ scan_flags) {
    clear_scan_flags(scan_flags);
    const int w = threadIdx.x >> 6, lane = lane_id();
    const int64_t tile = (int64_t)blockIdx.x * kWaves + w;
    if (tile >= T) return;
    const int64_t row0 = tile * (int64_t)tile_rows;
    const int rows = (int)min((int64_t)tile_rows, n - row0);
    if constexpr (NB > 0) {
        // NB flag bits at compile time: a histogram of the rows' flag codes
        // (the low NB bits; code 0 is in no set), then superset sums over the
        // NB bits -- a set's count is the sum of every code holding its mask
        // (one LDS add per flagged row instead of a membership test per set)
        constexpr int NC = 1 << NB;
        __shared__ int hist_s[kWaves][NC];
        int* hist = hist_s[w];
        for (int i = lane; i < NC; i += 64) hist[i] = 0;
        // the next chunk's flags are in flight while this one is counted
        uint32_t fn[kSelWords];
        chunk_flags(flags, row0, min(kSelChunk, rows), lane, fn);
        wave_sync();
        for (int c0 = 0; c0 < rows; c0 += kSelChunk) {
            uint32_t fw[kSelWords];
#pragma unroll
            for (int i = 0; i < kSelWords; ++i) fw[i] = fn[i];
            if (c0 + kSelChunk < rows)
                chunk_flags(flags, row0 + c0 + kSelChunk, min(kSelChunk, rows - c0 - kSelChunk),
                            lane, fn);
#pragma unroll
            for (int i = 0; i < kSelWords; ++i) {
                const unsigned f0 = fw[i] & (NC - 1), f1 = (fw[i] >> 16) & (NC - 1);
                if (f0) atomicAdd(&hist[f0], 1);
                if (f1) atomicAdd(&hist[f1], 1);
            }
        }
        wave_sync();
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            for (int c = lane; c < NC; c += 64)
                if (!((c >> b) & 1)) hist[c] += hist[c | (1 << b)];
            wave_sync();
        }
        // one set per lane: the tile's counts go out as parallel stores
        for (int k = lane; k < nsets; k += 64) {
            const unsigned m = masks.m[k];
            counts[(int64_t)k * T + tile] = m ? hist[m] : rows;
        }
    } else {
        int c[kMaxSets];
#pragma unroll
        for (int k = 0; k < kMaxSets; ++k) c[k] = 0;
        const int nbits = mask_bits(masks, nsets);
        for (int c0 = 0; c0 < rows; c0 += kSelChunk) {
            uint32_t fw[kSelWords];
            chunk_flags(flags, row0 + c0, min(kSelChunk, rows - c0), lane, fw);
            FlagPlanes fp;
            flag_planes(fw, nbits, fp);
#pragma unroll
            for (int k = 0; k < kMaxSets; ++k)
                if (k < nsets) c[k] += __popc(set_mask_m(fp, masks.m[k], nbits));
        }
#pragma unroll
        for (int k = 0; k < kMaxSets; ++k) {
            if (k < nsets) {
                const int t = wave_sum(c[k]);
                if (lane == 0) counts[(int64_t)k * T + tile] = t;
            }
        }
    }
}

hipError_t launch_msel_count(const uint16_t* flags, int64_t n, int nsets, const int* masks,
                             int tile_rows, const Workspace& ws, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    SetMasks sm{};
    unsigned u = 0;
    for (int k = 0; k < nsets; ++k) {
        sm.m[k] = (uint16_t)masks[k];
        u |= (unsigned)sm.m[k];
    }
    const int nb = flag_bits_class(u ? 32 - __builtin_clz(u) : 0);
    const int64_t grid = (ws.T + kWaves - 1) / kWaves;
    auto k = nb == 2 ? msel_count_kernel<2> : nb == 4 ? msel_count_kernel<4>
           : nb == 6 ? msel_count_kernel<6> : nb == 8 ? msel_count_kernel<8>
                     : msel_count_kernel<0>;
    prof_begin(s, K_HALO);
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(kBlock), 0, s, flags, n, nsets, sm,
                       ws.counts, ws.T, tile_rows, ws.flags);
    prof_end(s, K_HALO);
    return hipGetLastError();
}

// Offsets of chosen tile boundaries (mgr_tile_offsets): out[i][b] = the first
// row of bin b at tile tiles[i] in the packed layout (offsets[b][t]; at t = T
// the bin's end, bin_starts[b + 1]).  The tiles ride in the kernarg segment.
struct TileList {
    int64_t t[64];
};
__global__ void tile_offsets_kernel(const int64_t* __restrict__ offsets,
                                    const int64_t* __restrict__ bin_starts, int64_t T, int nbins,
                                    TileList tl, int ntiles, int64_t* __restrict__ out) {
    const int i = blockIdx.x, b = threadIdx.x + blockIdx.y * blockDim.x;
    if (i >= ntiles || b >= nbins) return;
    const int64_t t = tl.t[i];
    out[(int64_t)i * nbins + b] = t >= T ? bin_starts[b + 1] : offsets[(int64_t)b * T + t];
}

hipError_t launch_tile_offsets(const Workspace& ws, int nbins, const int64_t* tiles, int ntiles,
                               int64_t* out, hipStream_t s) {
    for (int i0 = 0; i0 < ntiles; i0 += 64) {
        TileList tl{};
        const int k = ntiles - i0 < 64 ? ntiles - i0 : 64;
        for (int i = 0; i < k; ++i) tl.t[i] = tiles[i0 + i];
        hipLaunchKernelGGL(tile_offsets_kernel, dim3(k, (nbins + 255) / 256), dim3(256), 0, s,
                           ws.offsets, ws.bin_starts, ws.T, nbins, tl, k, out + (int64_t)i0 * nbins);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
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
// ============================================================ launchers
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
    return a256(M * 4) + a256(M * 8) + a256((nbins + 1) * 8) +
           a256((kScanFlags + kScanCtlWords) * 8);
}

Workspace carve(void* base, int64_t n, int nbins, int tile_rows) {
    Workspace ws;
    ws.T = num_tiles(n, tile_rows);
    ws.t0 = 0;
    ws.tn = ws.T;
    const int64_t M = (int64_t)nbins * (ws.T > 0 ? ws.T : 1);
    char* p = (char*)base;
    ws.counts = (int32_t*)p;     p += a256(M * 4);
    ws.offsets = (int64_t*)p;    p += a256(M * 8);
    ws.bin_starts = (int64_t*)p; p += a256((nbins + 1) * 8);
    ws.flags = (uint64_t*)p;
    ws.scan_err = &((const ScanCtl*)(ws.flags + kScanFlags))->err;
    return ws;
}

hipError_t launch_scan(int64_t n, int nbins, int tile_rows, const Workspace& ws,
                       int64_t* bin_counts, hipStream_t s) {
    if (n <= 0 || ws.T == 0) {
        // no producer ran: clear the control words too (packs read err)
        hipError_t e = hipMemsetAsync(ws.bin_starts, 0, (size_t)(nbins + 1) * 8, s);
        if (e == hipSuccess) e = hipMemsetAsync(ws.flags + kScanFlags, 0, sizeof(ScanCtl), s);
        if (e == hipSuccess && bin_counts) e = hipMemsetAsync(bin_counts, 0, (size_t)nbins * 8, s);
        return e;
    }
    const Hooks& h = hooks();                         // one snapshot per launch
    const int64_t target = h.scan_chunk;               // counts per chunk (workgroup)
    int64_t cpb = (ws.T + target - 1) / target;
    int64_t cap = min((int64_t)h.scan_max_chunks, (int64_t)kScanFlags) / nbins;
    if (cap < 1) cap = 1;                             // nbins <= MGR_MAX_BINS = kScanFlags
    if (cpb > cap) cpb = cap;
    const int64_t chunk = (ws.T + cpb - 1) / cpb;
    cpb = (ws.T + chunk - 1) / chunk;                 // no empty chunk
    prof_begin(s, K_SCAN);
    auto k = chunk <= 8 * kBlock ? scan_onepass_kernel<8> : scan_onepass_kernel<16>;
    hipLaunchKernelGGL(k, dim3((unsigned)(nbins * cpb)), dim3(kBlock), 0, s, ws.counts, ws.T,
                       chunk, (int)cpb, nbins, ws.flags, ws.offsets, ws.bin_starts, bin_counts,
                       h.scan_spins, ScanTest{h.scan_delay_bin, h.scan_delay_sleeps,
                                              h.scan_end_spins, h.scan_poison_chunk});
    prof_end(s, K_SCAN);
    return hipGetLastError();
}

template <typename PosT>
static void halo_flags_t(const void* pos, int64_t n, int64_t stride, int dim, const HaloThr& t,
                         uint16_t* flags, hipStream_t s) {
    hipLaunchKernelGGL(halo_flags_kernel<PosT>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const PosT*)pos, n, stride, dim, t, flags);
}

hipError_t launch_halo_flags(const void* pos, int pos_dtype, int64_t n, int64_t stride, int dim,
                             const double* hi, const double* lo, uint16_t* flags, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    HaloThr t;
    for (int d = 0; d < MGR_MAX_DIM; ++d) {
        t.hi[d] = d < dim ? hi[d] : 0.0;
        t.lo[d] = d < dim ? lo[d] : 0.0;
    }
    prof_begin(s, K_HALO);
    switch (pos_dtype) {
        case MGR_F32: halo_flags_t<float>(pos, n, stride, dim, t, flags, s); break;
        case MGR_F64: halo_flags_t<double>(pos, n, stride, dim, t, flags, s); break;
        case MGR_I32: halo_flags_t<int32_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_I64: halo_flags_t<int64_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_I8: halo_flags_t<int8_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_I16: halo_flags_t<int16_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_U8: halo_flags_t<uint8_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_U16: halo_flags_t<uint16_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_U32: halo_flags_t<uint32_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_U64: halo_flags_t<uint64_t>(pos, n, stride, dim, t, flags, s); break;
        case MGR_B8: halo_flags_t<b8_t>(pos, n, stride, dim, t, flags, s); break;
        default: halo_flags_t<f16_t>(pos, n, stride, dim, t, flags, s); break;
    }
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
