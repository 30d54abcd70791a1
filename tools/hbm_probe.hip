// HBM ceiling probe (tools only, not part of libmgr): streaming copy variants
// to find what the MI355X sustains for the access shapes the kernels use.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const v4u* __restrict__ s, v4u* __restrict__ d,
                                              int64_t n) {
    const int64_t base = ((int64_t)blockIdx.x * U) * 256 + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + k * 256;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + k * 256;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[k], d + i);
            else d[i] = v[k];
        }
    }
}

// 8-way scatter: each 64-lane wave copies its 64 16-byte units to 8
// destination regions (lane & 7 picks the region), runs of 8 units.
template <int U>
__global__ __launch_bounds__(256) void scatter8_k(const v4u* __restrict__ s, v4u* __restrict__ d,
                                                  int64_t n) {
    const int64_t region = n / 8;
    const int64_t base = ((int64_t)blockIdx.x * U) * 256 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + k * 256;
        if (i < n) {
            const int lane = threadIdx.x & 63;
            const int64_t wave_id = i >> 6;
            const int r = lane >> 3;
            const int64_t j = (int64_t)r * region + wave_id * 8 + (lane & 7);
            if (j < n) d[j] = s[i];
        }
    }
}

// Read-only stream: each thread reads U units and folds them; the store
// never fires (magic never matches) but keeps the loads alive.
template <int U, bool NT>
__global__ __launch_bounds__(256) void read_k(const v4u* __restrict__ s, v4u* __restrict__ d,
                                              int64_t n, unsigned magic) {
    const int64_t base = ((int64_t)blockIdx.x * U) * 256 + threadIdx.x;
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + k * 256;
        if (i < n) {
            const v4u v = NT ? __builtin_nontemporal_load(s + i) : s[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == magic) d[base] = v4u{acc, 0, 0, 0};
}

// Pack-structure probes on 32-byte rows, one destination (dest bytes all 0,
// so every slot is the row itself): what the cooperative pack's parts cost.
// MODE 0: full (dest load, 3 ballots, LDS count exchange + barrier, slot shfl)
// MODE 1: no LDS exchange / barrier;  MODE 2: no dest load either (pure
// unit-transposed copy in the same 512-thread shape).
template <int MODE>
__global__ __launch_bounds__(512) void coop_probe_k(const v4u* __restrict__ s, v4u* __restrict__ d,
                                                    const unsigned char* __restrict__ dest,
                                                    int64_t nrows) {
    __shared__ int s_cnt[8][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row0 = (int64_t)blockIdx.x * 512 + 64 * w;
    const int nr = (int)max((int64_t)0, min((int64_t)64, nrows - row0));
    unsigned b = 0;
    if (MODE < 2) b = lane < nr ? dest[row0 + lane] : 0u;
    v4u v0, v1;
    if (lane < 2 * nr) v0 = s[row0 * 2 + lane];
    if (64 + lane < 2 * nr) v1 = s[row0 * 2 + 64 + lane];
    long long base = row0;
    unsigned long long pe = __ballot(lane < nr);
    if (MODE < 2) {
        unsigned long long mine = pe;
        for (int i = 0; i < 3; ++i) {
            const unsigned long long m = __ballot((b >> i) & 1u);
            pe &= ((b >> i) & 1u) ? m : ~m;
            mine &= ((lane >> i) & 1) ? m : ~m;
        }
        if (MODE == 0) {
            base = (int64_t)blockIdx.x * 512;
            s_cnt[w][lane] = __popcll(mine);
            __syncthreads();
            for (int j = 0; j < w; ++j) base += s_cnt[j][lane];
        }
        base = __shfl(base, (int)b, 64);
    }
    const unsigned lo = (unsigned)pe, hi = (unsigned)(pe >> 32);
    const long long tgt = base + __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
    {
        const int u = lane, r = u >> 1, part = u & 1;
        const long long t = __shfl(tgt, r, 64);
        if (u < 2 * nr) d[t * 2 + part] = v0;
    }
    {
        const int u = 64 + lane, r = u >> 1, part = u & 1;
        const long long t = __shfl(tgt, r, 64);
        if (u < 2 * nr) d[t * 2 + part] = v1;
    }
}

extern "C" int coop_probe(int mode, const void* s, void* d, const void* dest, int64_t nrows,
                          void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const dim3 g((unsigned)((nrows + 511) / 512));
    const v4u* S = (const v4u*)s;
    v4u* D = (v4u*)d;
    const unsigned char* B = (const unsigned char*)dest;
    switch (mode) {
        case 0: hipLaunchKernelGGL(coop_probe_k<0>, g, dim3(512), 0, st, S, D, B, nrows); break;
        case 1: hipLaunchKernelGGL(coop_probe_k<1>, g, dim3(512), 0, st, S, D, B, nrows); break;
        case 2: hipLaunchKernelGGL(coop_probe_k<2>, g, dim3(512), 0, st, S, D, B, nrows); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Copy shapes: a block of THREADS threads moves THREADS*UPL 16-byte units;
// WAVEMAJOR: wave w owns units [w*64*UPL, (w+1)*64*UPL) (the pack's round
// layout); else unit k*THREADS + tid.  NTL/NTS: nontemporal loads/stores.
template <int THREADS, int UPL, bool WAVEMAJOR, bool NTL, bool NTS>
__global__ __launch_bounds__(THREADS) void shape_k(const v4u* __restrict__ s, v4u* __restrict__ d,
                                                   int64_t n) {
    const int64_t b0 = (int64_t)blockIdx.x * THREADS * UPL;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    v4u v[UPL];
#pragma unroll
    for (int k = 0; k < UPL; ++k) {
        const int64_t i = WAVEMAJOR ? b0 + (int64_t)w * 64 * UPL + 64 * k + lane
                                    : b0 + (int64_t)k * THREADS + threadIdx.x;
        if (i < n) v[k] = NTL ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < UPL; ++k) {
        const int64_t i = WAVEMAJOR ? b0 + (int64_t)w * 64 * UPL + 64 * k + lane
                                    : b0 + (int64_t)k * THREADS + threadIdx.x;
        if (i < n) {
            if (NTS) __builtin_nontemporal_store(v[k], d + i);
            else d[i] = v[k];
        }
    }
}

#define SHAPES(X) \
    X(256, 1, false, false, false) X(512, 1, false, false, false) X(1024, 1, false, false, false) \
    X(256, 2, true, false, false) X(512, 2, true, false, false) X(512, 2, false, false, false) \
    X(512, 2, true, true, false) X(512, 2, true, false, true) X(512, 2, true, true, true) \
    X(1024, 2, true, false, false) X(256, 4, true, false, false) X(128, 2, true, false, false)

extern "C" int shape_count(void) {
    int c = 0;
#define CNT(T, U, W, L, S) ++c;
    SHAPES(CNT)
#undef CNT
    return c;
}

extern "C" int shape_probe(int which, const void* s, void* d, int64_t n16, char* name, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    int c = 0;
#define RUN(T, U, W, L, S)                                                                      \
    if (c++ == which) {                                                                         \
        snprintf(name, 64, "t%d_u%d_%s%s%s", T, U, W ? "wave" : "strided", L ? "_ntl" : "",     \
                 S ? "_nts" : "");                                                              \
        hipLaunchKernelGGL((shape_k<T, U, W, L, S>), dim3((unsigned)((n16 + T * U - 1) / (T * U))), \
                           dim3(T), 0, st, (const v4u*)s, (v4u*)d, n16);                         \
        return hipGetLastError() == hipSuccess ? 0 : -2;                                        \
    }
    SHAPES(RUN)
#undef RUN
    return -1;
}

extern "C" int probe(int which, const void* s, void* d, int64_t n16, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const v4u* S = (const v4u*)s;
    v4u* D = (v4u*)d;
    auto grid = [&](int u) { return dim3((unsigned)((n16 + 256LL * u - 1) / (256LL * u))); };
    switch (which) {
        case 0: hipLaunchKernelGGL((copy_k<1, false>), grid(1), dim3(256), 0, st, S, D, n16); break;
        case 1: hipLaunchKernelGGL((copy_k<4, false>), grid(4), dim3(256), 0, st, S, D, n16); break;
        case 2: hipLaunchKernelGGL((copy_k<8, false>), grid(8), dim3(256), 0, st, S, D, n16); break;
        case 3: hipLaunchKernelGGL((copy_k<1, true>), grid(1), dim3(256), 0, st, S, D, n16); break;
        case 4: hipLaunchKernelGGL((copy_k<4, true>), grid(4), dim3(256), 0, st, S, D, n16); break;
        case 5: hipLaunchKernelGGL((copy_k<8, true>), grid(8), dim3(256), 0, st, S, D, n16); break;
        case 6: hipLaunchKernelGGL((scatter8_k<4>), grid(4), dim3(256), 0, st, S, D, n16); break;
        case 7: hipLaunchKernelGGL((read_k<1, false>), grid(1), dim3(256), 0, st, S, D, n16, 0xDEADBEEFu); break;
        case 8: hipLaunchKernelGGL((read_k<1, true>), grid(1), dim3(256), 0, st, S, D, n16, 0xDEADBEEFu); break;
        case 9: hipLaunchKernelGGL((read_k<4, false>), grid(4), dim3(256), 0, st, S, D, n16, 0xDEADBEEFu); break;
        case 10: hipLaunchKernelGGL((read_k<4, true>), grid(4), dim3(256), 0, st, S, D, n16, 0xDEADBEEFu); break;
        case 11: hipLaunchKernelGGL((read_k<16, true>), grid(16), dim3(256), 0, st, S, D, n16, 0xDEADBEEFu); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
