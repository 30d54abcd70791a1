// Store-alignment probe (tools only, not part of libmgr): a streaming copy
// whose 16-byte stores (global_store_dwordx4) land OFF bytes past a 16-byte
// boundary (0, 4, 8, 12), and the same with the loads misaligned instead.
// Question: do the packs' image stores -- 16-byte units at gaddr[bin] + x,
// 4-byte aligned whenever the bin's output row * row bytes is not a multiple
// of 16 (36-, 12-, 4-byte rows) -- pay for their misalignment?
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u4a4 __attribute__((ext_vector_type(4), aligned(4)));

template <bool MIS_LOAD>
__global__ __launch_bounds__(256) void mis_copy_k(const uint8_t* __restrict__ s,
                                                  uint8_t* __restrict__ d, int64_t n16, int off) {
    const int64_t base = ((int64_t)blockIdx.x * 4) * 256 + threadIdx.x;
    u4a4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * 256;
        if (i < n16) v[k] = *(const u4a4*)(s + 16 * i + (MIS_LOAD ? off : 0));
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + k * 256;
        if (i < n16) *(u4a4*)(d + 16 * i + (MIS_LOAD ? 0 : off)) = v[k];
    }
}

// n16 units are copied; both buffers must hold 16 * n16 + 16 bytes.
extern "C" int mis_copy(int mis_load, const void* s, void* d, int64_t n16, int off, void* stream) {
    if (off < 0 || off > 15) return -1;
    const dim3 g((unsigned)((n16 + 1023) / 1024));
    if (mis_load)
        hipLaunchKernelGGL(mis_copy_k<true>, g, dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)s, (uint8_t*)d, n16, off);
    else
        hipLaunchKernelGGL(mis_copy_k<false>, g, dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)s, (uint8_t*)d, n16, off);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
