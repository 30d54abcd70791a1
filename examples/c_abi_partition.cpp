// The C ABI without Python or torch: a host program that calls libmgr.so
// (include/mgr.h) on hipMalloc'd buffers -- bin + scan + stable pack of n
// particles into a 2x2x2 grid (redist.py:157-198, BASELINE config 2's local
// stage) -- and checks the device results byte for byte against a plain C++
// restatement of the reference's arithmetic (numpy's floor
// remainder, in-place wrap, trunc(t / L * n), row-major cell, stable
// partition).  Exit 0 and one "ok" line when everything matches.
//
//   hipcc -O2 -Iinclude examples/c_abi_partition.cpp -Lmpi_grid_redistribute_amd -lmgr \
//         -Wl,-rpath,'$ORIGIN/../../mpi_grid_redistribute_amd' -o examples/bin/c_abi_partition
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mgr.h"

#define CHECK_MGR(x)                                                                  \
    do {                                                                              \
        int rc_ = (x);                                                                \
        if (rc_ != MGR_OK) {                                                          \
            std::fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, mgr_last_error()); \
            return 2;                                                                 \
        }                                                                             \
    } while (0)
#define CHECK_HIP(x)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                 \
            return 2;                                                                           \
        }                                                                                       \
    } while (0)

// numpy's float64 remainder (floor semantics, sign of the divisor)
static double pymod(double a, double b) {
    double m = std::fmod(a, b);
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = std::copysign(0.0, b);
    }
    return m;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : (int64_t)1 << 22;
    const int dim = 3, nbins = 8;
    const int64_t topo[3] = {2, 2, 2};
    const double box[3] = {1.0, 1.0, 1.0};
    const int64_t rb = 32;   // record [x, y, z, id]

    // host input: uniform in [-0.5, 1.5) (a quarter of the coordinates outside the box)
    std::vector<double> pos(3 * n);
    std::vector<uint8_t> rec(rb * n);
    uint64_t s = 20261018;
    for (int64_t r = 0; r < n; ++r) {
        for (int d = 0; d < 3; ++d) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            pos[3 * r + d] = (double)(s >> 11) * 0x1.0p-53 * 2.0 - 0.5;
        }
        std::memcpy(&rec[rb * r], &pos[3 * r], 24);
        std::memcpy(&rec[rb * r + 24], &r, 8);
    }

    mgr_plan* plan = nullptr;
    CHECK_MGR(mgr_plan_create(dim, topo, box, MGR_F64, nbins, &plan));
    const int tile_rows = mgr_tile_rows(rb, nbins);
    const int64_t wsb = mgr_workspace_bytes(n, nbins, tile_rows);
    void *d_pos, *d_rec, *d_dest, *d_ws, *d_out;
    int64_t* d_counts;
    CHECK_HIP(hipMalloc(&d_pos, 24 * n));
    CHECK_HIP(hipMalloc(&d_rec, rb * n));
    CHECK_HIP(hipMalloc(&d_dest, n * mgr_dest_bytes(nbins)));
    CHECK_HIP(hipMalloc(&d_ws, wsb));
    CHECK_HIP(hipMalloc(&d_out, rb * n));
    CHECK_HIP(hipMalloc((void**)&d_counts, 8 * nbins));
    CHECK_HIP(hipMemcpy(d_pos, pos.data(), 24 * n, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_rec, rec.data(), rb * n, hipMemcpyHostToDevice));
    hipStream_t st;
    CHECK_HIP(hipStreamCreate(&st));

    CHECK_MGR(mgr_bin_count(plan, d_pos, MGR_F64, n, 3, 1, d_dest, tile_rows, d_ws, st));
    CHECK_MGR(mgr_scan(n, nbins, tile_rows, d_ws, d_counts, st));
    CHECK_MGR(mgr_pack(d_rec, rb, n, d_dest, nbins, -1, tile_rows, d_ws, d_out, -1, nullptr, st));
    CHECK_HIP(hipStreamSynchronize(st));

    std::vector<double> wrapped(3 * n);
    std::vector<uint8_t> out(rb * n);
    int64_t counts[8];
    CHECK_HIP(hipMemcpy(wrapped.data(), d_pos, 24 * n, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(out.data(), d_out, rb * n, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(counts, d_counts, sizeof counts, hipMemcpyDeviceToHost));

    // the reference's arithmetic on the host
    std::vector<int> cell(n);
    int64_t exp_counts[8] = {0};
    int64_t bad_wrap = 0;
    for (int64_t r = 0; r < n; ++r) {
        int64_t c = 0;
        for (int d = 0; d < 3; ++d) {
            const double L = box[d];
            const double t = pymod(pymod(pos[3 * r + d], L) + L, L);   // redist.py:328-329
            if (std::memcmp(&t, &wrapped[3 * r + d], 8) != 0) ++bad_wrap;
            int64_t k = (int64_t)(t / L * (double)topo[d]);           // :69-70
            k = ((k % topo[d]) + topo[d]) % topo[d];                    // :83-84
            c = c * topo[d] + k;                                        // row-major (S4)
        }
        cell[r] = (int)c;
        ++exp_counts[c];
    }
    std::vector<uint8_t> exp(rb * n);
    int64_t at[8];
    int64_t acc = 0;
    for (int b = 0; b < nbins; ++b) {
        at[b] = acc;
        acc += exp_counts[b];
    }
    for (int64_t r = 0; r < n; ++r) std::memcpy(&exp[rb * at[cell[r]]++], &rec[rb * r], rb);

    const bool counts_ok = std::memcmp(counts, exp_counts, sizeof counts) == 0;
    const bool rows_ok = std::memcmp(out.data(), exp.data(), rb * n) == 0;
    std::printf("c_abi_partition %s: n=%lld wrap_mismatches=%lld counts_ok=%d rows_ok=%d "
                "counts=[%lld %lld %lld %lld %lld %lld %lld %lld] (%s, %s)\n",
                counts_ok && rows_ok && !bad_wrap ? "ok" : "FAILED", (long long)n,
                (long long)bad_wrap, (int)counts_ok, (int)rows_ok, (long long)counts[0],
                (long long)counts[1], (long long)counts[2], (long long)counts[3],
                (long long)counts[4], (long long)counts[5], (long long)counts[6],
                (long long)counts[7], mgr_version(), mgr_last_error());
    mgr_plan_destroy(plan);
    for (void* p : {d_pos, d_rec, d_dest, d_ws, d_out, (void*)d_counts}) CHECK_HIP(hipFree(p));
    CHECK_HIP(hipStreamDestroy(st));
    return counts_ok && rows_ok && !bad_wrap ? 0 : 1;
}
