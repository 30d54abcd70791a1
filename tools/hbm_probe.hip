// HBM ceiling probe (tools only, not part of libmgr): streaming copy variants
// to find what the MI355X sustains for the access shapes the kernels use.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
