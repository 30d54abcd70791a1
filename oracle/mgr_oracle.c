/*
 * CPU oracle (C restatement) of the reference redistribution path.
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / large-N verifier.  The product
 * library (libmgr.so) never links or calls anything here.
 *
 * Restates redist.py (dkorytov/mpi_grid_redistribute) from SURVEY.md §0 S11:
 *   pymod(a,b){m=fmod(a,b); if(m!=0){if((b<0)!=(m<0)) m+=b;} else m=copysign(0,b);}
 *   t = pymod(pymod(x,L)+L, L)                 redist.py:68, :328-329 (S1)
 *   k = trunc_i64(t/L*(double)n)               redist.py:69-70        (S2, S10)
 *   k = ((k%n)+n)%n  (floor-mod)               redist.py:83-84, :90   (S3)
 *   cell = sum_d offset[d]*k[d], row-major     redist.py:53-58, :84   (S4)
 * float32 positions: wrap in f64, round to f32 on write-back, bin from the
 * f32 value in f64 (S9); f32 positions with an f32 box compute the wrap and
 * the quotient in f32 (numpy result_type), the *n in f64.
 * Stable split + source-ordered concat: redist.py:195-199 (S6, S7).
 *
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared (oracle/Makefile).  No
 * -ffast-math: every operation must be IEEE-exact.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* x86 cvttsd2si semantics of numpy astype(int64): NaN/out-of-range -> INT64_MIN (S10). */
static int64_t trunc_i64(double v) {
    if (v >= -9223372036854775808.0 && v < 9223372036854775808.0) return (int64_t)v;
    return INT64_MIN;
}

/* numpy npy_remainder for doubles (floor-remainder, result takes the divisor's sign). */
static double pymod(double a, double b) {
    double m = fmod(a, b);
    if (b == 0.0) return m;
    if (m != 0.0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}

static float pymodf(float a, float b) {
    float m = fmodf(a, b);
    if (b == 0.0f) return m;
    if (m != 0.0f) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = copysignf(0.0f, b);
    }
    return m;
}

/* numpy int64 remainder (Python floor-mod); n == 0 -> 0 like numpy. */
static int64_t floormod_i64(int64_t a, int64_t n) {
    if (n == 0) return 0;
    if (n == -1) return 0;
    int64_t r = a % n;
    if (r != 0 && ((r < 0) != (n < 0))) r += n;
    return r;
}

double oracle_pymod(double a, double b) { return pymod(a, b); }
float oracle_pymodf(float a, float b) { return pymodf(a, b); }
int64_t oracle_trunc_i64(double v) { return trunc_i64(v); }

/*
 * Bin n rows of positions (row r, coordinate d at pos[r*row_stride + d]).
 *   pos_is_f32  : element type float (else double)
 *   compute_f32 : only with pos_is_f32 -- box is float32 (numpy f32 % f32)
 *   periodic    : wrap + in-place write-back (redist.py:67-68)
 * Outputs: cell[r] (int64, row-major cell id), idx[r*dim+d] (optional).
 */
static int64_t bin_one(void* pos, int pos_is_f32, int compute_f32, int64_t r, int64_t row_stride,
                       int dim, const double* box, const int64_t* topo, const int64_t* offset,
                       int periodic, int64_t* idx, int fast) {
    int64_t c = 0;
    for (int d = 0; d < dim; ++d) {
        int64_t k;
        if (pos_is_f32) {
            float* p = (float*)pos + r * row_stride + d;
            if (compute_f32) {
                float L = (float)box[d];
                if (periodic) *p = pymodf(pymodf(*p, L) + L, L);
                float q = *p / L;
                k = trunc_i64((double)q * (double)topo[d]);
            } else {
                double L = box[d];
                if (periodic) *p = (float)pymod(pymod((double)*p, L) + L, L);
                k = trunc_i64((double)*p / L * (double)topo[d]);
            }
        } else {
            double* p = (double*)pos + r * row_stride + d;
            double L = box[d];
            if (periodic) {
                const double x = *p;
                if (fast && x >= 0.0 && x < L) {
                    /* in-box: x % L == x and (x + L) % L == (x + L) - L exactly
                     * (Sterbenz), 0 when x + L rounds to 2L -- the same value as the
                     * general path (checked by tests/test_oracle.py) */
                    const double y = x + L;
                    *p = (y == L + L) ? 0.0 : y - L;
                } else {
                    *p = pymod(pymod(x, L) + L, L);
                }
            }
            k = trunc_i64(*p / L * (double)topo[d]);
        }
        if (idx) idx[r * dim + d] = k;
        if (fast && k >= 0 && k < topo[d])
            c += offset[d] * k;   /* ((k % n) + n) % n == k: skip the integer divisions */
        else
            c += offset[d] * floormod_i64(floormod_i64(k, topo[d]) + topo[d], topo[d]);
    }
    return c;
}

void oracle_bin(void* pos, int pos_is_f32, int compute_f32, int64_t n, int64_t row_stride,
                int dim, const double* box, const int64_t* topo, int periodic,
                int64_t* cell, int64_t* idx) {
    int64_t offset[64];
    int64_t off = 1;
    for (int d = dim - 1; d >= 0; --d) { offset[d] = off; off *= topo[d]; }
    for (int64_t r = 0; r < n; ++r)
        cell[r] = bin_one(pos, pos_is_f32, compute_f32, r, row_stride, dim, box, topo, offset,
                          periodic, idx, 0);
}

/* ---- integer / float16 / bool positions (redist.py:68-69 on any numpy column).
 * numpy 2.2.6 float16 conversions, restated from their documented behaviour:
 * round to nearest even with overflow to inf; NaN keeps sign and payload
 * (shifted), never quieted, forced nonzero; half arithmetic = the float32
 * operation rounded back.  Written independently of the device version
 * (mgr_device.h): plain value arithmetic for the rounding. */
static float h2f(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    float v;
    uint32_t b;
    if (e == 0x1fu) {
        b = s | 0x7f800000u | (m << 13);
        memcpy(&v, &b, 4);
        return v;
    }
    v = e ? ldexpf((float)(m | 0x400u), (int)e - 25) : ldexpf((float)m, -24);
    return (h & 0x8000u) ? -v : v;
}
static double h2d(uint16_t h) {
    if (((h >> 10) & 0x1fu) == 0x1fu) {
        const uint64_t b = ((uint64_t)(h & 0x8000u) << 48) | 0x7ff0000000000000ull |
                           ((uint64_t)(h & 0x3ffu) << 42);
        double v;
        memcpy(&v, &b, 8);
        return v;
    }
    return (double)h2f(h);
}
/* |x| (finite, < 65520) to float16 bits by value: scale to the half's ulp and
 * round half to even with nearbyint (default rounding mode). */
static uint16_t mag_to_half(double a) {
    if (a < 0x1p-14) return (uint16_t)nearbyint(a * 0x1p24);     /* subnormal (or 0x400) */
    int e;
    frexp(a, &e);                      /* a = f * 2^e, f in [0.5, 1) */
    const double ulp = ldexp(1.0, e - 11);
    double q = nearbyint(a / ulp);     /* 1024..2048 significand units */
    int he = e - 1 + 15;               /* biased half exponent of a */
    if (q >= 2048.0) { q /= 2.0; he += 1; }
    if (he >= 31) return 0x7c00u;
    return (uint16_t)((he << 10) | ((int)q - 1024));
}
static uint16_t d2h(double x) {
    uint64_t b;
    memcpy(&b, &x, 8);
    const uint16_t s = (uint16_t)((b >> 48) & 0x8000u);
    if (isnan(x)) {
        uint16_t r = (uint16_t)(0x7c00u + ((b & 0xfffffffffffffull) >> 42));
        if (r == 0x7c00u) r++;
        return (uint16_t)(s | r);
    }
    const double a = fabs(x);
    if (a >= 65520.0) return (uint16_t)(s | 0x7c00u);   /* also inf */
    return (uint16_t)(s | mag_to_half(a));
}
static uint16_t f2h(float x) {
    if (isnan(x)) {
        uint32_t b;
        memcpy(&b, &x, 4);
        uint16_t r = (uint16_t)(0x7c00u + ((b & 0x7fffffu) >> 13));
        if (r == 0x7c00u) r++;
        return (uint16_t)(((b >> 16) & 0x8000u) | r);
    }
    return d2h((double)x);   /* float -> double is exact: one rounding */
}
/* numpy's float -> int32 cast on x86 (cvttsd2si, 32-bit): NaN / out of range -> INT32_MIN */
static int32_t trunc_i32(double v) {
    if (v > -2147483649.0 && v < 2147483648.0) return (int32_t)v;
    return INT32_MIN;
}

uint16_t oracle_d2h(double x) { return d2h(x); }
uint16_t oracle_f2h(float x) { return f2h(x); }
double oracle_h2d(uint16_t h) { return h2d(h); }

enum { O_F32 = 1, O_F64 = 2, O_I32 = 3, O_I64 = 4, O_F16 = 5, O_I8 = 6, O_I16 = 7, O_U8 = 8,
       O_U16 = 9, O_U32 = 10, O_U64 = 11, O_B8 = 12 };

static int o_bits(int t) {
    switch (t) {
        case O_I8: case O_U8: case O_B8: return 8;
        case O_I16: case O_U16: case O_F16: return 16;
        case O_I32: case O_U32: case O_F32: return 32;
        default: return 64;
    }
}
static int o_signed(int t) { return t == O_I8 || t == O_I16 || t == O_I32 || t == O_I64; }

/* an integer / bool column element, widened (unsigned 64-bit: its bits) */
static int64_t o_load(const void* pos, int t, int64_t e) {
    switch (t) {
        case O_I8: return ((const int8_t*)pos)[e];
        case O_I16: return ((const int16_t*)pos)[e];
        case O_I32: return ((const int32_t*)pos)[e];
        case O_I64: return ((const int64_t*)pos)[e];
        case O_U8: return ((const uint8_t*)pos)[e];
        case O_U16: return ((const uint16_t*)pos)[e];
        case O_U32: return ((const uint32_t*)pos)[e];
        case O_B8: return ((const uint8_t*)pos)[e] != 0;
        default: return (int64_t)((const uint64_t*)pos)[e];
    }
}
static void o_store(void* pos, int t, int64_t e, int64_t v) {   /* C truncation; bool != 0 */
    switch (t) {
        case O_I8: case O_U8: ((uint8_t*)pos)[e] = (uint8_t)v; break;
        case O_B8: ((uint8_t*)pos)[e] = v != 0; break;
        case O_I16: case O_U16: ((uint16_t*)pos)[e] = (uint16_t)v; break;
        case O_I32: case O_U32: ((uint32_t*)pos)[e] = (uint32_t)v; break;
        default: ((uint64_t*)pos)[e] = (uint64_t)v; break;
    }
}
static double o_as_f64(int t, int64_t v) {
    return t == O_U64 ? (double)(uint64_t)v : (double)v;
}
/* numpy's float -> integer cast on x86, written out (not left to the C
 * compiler: out-of-range conversions are undefined in C): 32-bit cvttsd2si
 * for <= 32-bit signed and <= 16-bit unsigned types, 64-bit for int64,
 * uint32 / uint64 offset by 2^(w-1) at and above it; bool != 0. */
static int64_t o_from_f64(int t, double x) {
    if (t == O_B8) return x != 0.0;
    if (t == O_I64) return trunc_i64(x);
    if (t == O_U64)
        return x >= 9223372036854775808.0
                   ? (int64_t)((uint64_t)trunc_i64(x - 9223372036854775808.0) ^ 0x8000000000000000ull)
                   : trunc_i64(x);
    if (t == O_U32)
        return x >= 2147483648.0 ? (int64_t)((uint32_t)trunc_i32(x - 2147483648.0) ^ 0x80000000u)
                                 : (int64_t)(uint32_t)trunc_i32(x);
    return trunc_i32(x);
}
/* numpy's integer remainder at type w (floor-mod signed, plain unsigned,
 * x % 0 == 0), ((x % L) + L) % L with the + L wrapping at w's width */
static int64_t o_wrap_int(int64_t x, int64_t L, int w) {
    const int bits = o_bits(w), sgn = o_signed(w);
    const uint64_t mask = bits == 64 ? ~0ull : (1ull << bits) - 1ull;
    if (sgn) {
        uint64_t s = (uint64_t)floormod_i64(x, L) + (uint64_t)L;
        s &= mask;
        if (bits < 64 && ((s >> (bits - 1)) & 1ull)) s |= ~mask;
        return floormod_i64((int64_t)s, L);
    }
    const uint64_t ux = (uint64_t)x, uL = (uint64_t)L;
    if (uL == 0) return 0;
    return (int64_t)(((ux % uL + uL) & mask) % uL);
}

/* Bin n rows of integer / float16 / bool positions (pos_dtype O_*).  wmode:
 * numpy's type of position % box, dmode: of position / box -- the caller
 * takes both from numpy itself (c_oracle.bin_positions).  The wrap is stored
 * back cast to the column's type; binning reads the stored value (S2). */
void oracle_bin_ext(void* pos, int pos_dtype, int wmode, int dmode, int64_t n, int64_t row_stride,
                    int dim, const double* box, const int64_t* topo, int periodic, int64_t* cell,
                    int64_t* idx) {
    int64_t offset[64];
    int64_t off = 1;
    for (int d = dim - 1; d >= 0; --d) { offset[d] = off; off *= topo[d]; }
    for (int64_t r = 0; r < n; ++r) {
        int64_t c = 0;
        for (int d = 0; d < dim; ++d) {
            const int64_t e = r * row_stride + d;
            const double L = box[d];
            const float Lf = (float)L;
            double xs;   /* the stored value as float64 */
            if (pos_dtype == O_F16) {
                uint16_t* p = (uint16_t*)pos + e;
                if (periodic) {
                    if (wmode == O_F64) {
                        *p = d2h(pymod(pymod(h2d(*p), L) + L, L));
                    } else if (wmode == O_F32) {
                        *p = f2h(pymodf(pymodf(h2f(*p), Lf) + Lf, Lf));
                    } else {   /* half arithmetic: each step rounded to float16 */
                        const uint16_t m = f2h(pymodf(h2f(*p), Lf));
                        const uint16_t y = f2h(h2f(m) + Lf);
                        *p = f2h(pymodf(h2f(y), Lf));
                    }
                }
                xs = h2d(*p);
            } else {
                if (periodic) {
                    const int64_t x = o_load(pos, pos_dtype, e);
                    int64_t t;
                    if (wmode == O_F64) {
                        t = o_from_f64(pos_dtype, pymod(pymod(o_as_f64(pos_dtype, x), L) + L, L));
                    } else if (wmode == O_F32) {   /* <= 16-bit: exact in float32 */
                        t = o_from_f64(pos_dtype, (double)pymodf(pymodf((float)x, Lf) + Lf, Lf));
                    } else if (wmode == O_F16) {   /* 8-bit: exact in float16 */
                        const uint16_t m = f2h(pymodf((float)x, Lf));
                        const uint16_t y = f2h(h2f(m) + Lf);
                        t = o_from_f64(pos_dtype, (double)h2f(f2h(pymodf(h2f(y), Lf))));
                    } else {
                        t = o_wrap_int(x, (int64_t)L, wmode);
                    }
                    o_store(pos, pos_dtype, e, t);
                }
                xs = o_as_f64(pos_dtype, o_load(pos, pos_dtype, e));
            }
            double q;
            if (dmode == O_F64) q = xs / L;
            else if (dmode == O_F32) q = (double)((float)xs / Lf);
            else q = (double)h2f(f2h((float)xs / Lf));
            const int64_t k = trunc_i64(q * (double)topo[d]);
            if (idx) idx[r * dim + d] = k;
            c += offset[d] * floormod_i64(floormod_i64(k, topo[d]) + topo[d], topo[d]);
        }
        cell[r] = c;
    }
}

/*
 * The local stage on the host's cores (bench.py cpu_baseline_c): wrap + bin
 * of f64 positions and a stable partition of the rows, threaded: every
 * thread bins a contiguous chunk and counts its bins, the per-(thread, bin)
 * starts follow in (bin, thread) order, and every thread scatters its own
 * chunk -- the same result as oracle_bin + oracle_partition.  Returns rows
 * written; offsets[nbins+1].  dest_ws (int32 [n]) and start_ws (int64
 * [nthreads * nbins]): caller-owned scratch, so a timed call allocates and
 * first-touches nothing (NULL: allocated here).
 */
int64_t oracle_local_partition_omp(double* pos, int64_t n, int64_t row_stride, int dim,
                                   const double* box, const int64_t* topo, int periodic,
                                   const void* data, int64_t row_bytes, void* out,
                                   int64_t* offsets, int nthreads, int32_t* dest_ws,
                                   int64_t* start_ws) {
    int64_t offset[64];
    int64_t off = 1;
    for (int d = dim - 1; d >= 0; --d) { offset[d] = off; off *= topo[d]; }
    const int64_t nbins = off;
    if (nthreads < 1) nthreads = 1;
    int32_t* dest = dest_ws ? dest_ws : (int32_t*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int32_t));
    int64_t* start = start_ws ? start_ws
                              : (int64_t*)malloc((size_t)nthreads * (size_t)nbins * sizeof(int64_t));
    memset(start, 0, (size_t)nthreads * (size_t)nbins * sizeof(int64_t));
    const char* src = (const char*)data;
    char* dst = (char*)out;
    int fast = 1;   /* the in-box fast wrap needs L > 0 with 2L finite */
    for (int d = 0; d < dim; ++d)
        if (!(box[d] > 0.0) || !isfinite(box[d] + box[d])) fast = 0;
#pragma omp parallel num_threads(nthreads)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num(), T = omp_get_num_threads();
#else
        const int t = 0, T = 1;
#endif
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        int64_t* h = start + (int64_t)t * nbins;
        for (int64_t r = lo; r < hi; ++r) {
            const int64_t c = bin_one(pos, 0, 0, r, row_stride, dim, box, topo, offset, periodic,
                                      NULL, fast);
            dest[r] = (int32_t)c;
            h[c]++;
        }
#pragma omp barrier
#pragma omp single
        {
            int64_t run = 0;
            for (int64_t b = 0; b < nbins; ++b) {
                offsets[b] = run;
                for (int u = 0; u < T; ++u) {
                    const int64_t c = start[(int64_t)u * nbins + b];
                    start[(int64_t)u * nbins + b] = run;
                    run += c;
                }
            }
            offsets[nbins] = run;
        }
        if (row_bytes == 32) {   /* the bench layout: fixed-size copies the compiler inlines */
            for (int64_t r = lo; r < hi; ++r)
                memcpy(dst + (h[dest[r]]++) * 32, src + r * 32, 32);
        } else {
            for (int64_t r = lo; r < hi; ++r)
                memcpy(dst + (h[dest[r]]++) * row_bytes, src + r * row_bytes, (size_t)row_bytes);
        }
    }
    const int64_t total = offsets[nbins];
    if (!start_ws) free(start);
    if (!dest_ws) free(dest);
    return total;
}

/*
 * Stable counting-sort partition of n rows of row_bytes by dest[r] in
 * [0, nbins); rows with dest outside are dropped (redist.py:195-198, S6).
 * offsets[nbins+1] receives the segment starts.  Returns rows written.
 */
int64_t oracle_partition(const void* data, int64_t n, int64_t row_bytes, const int64_t* dest,
                         int64_t nbins, void* out, int64_t* offsets) {
    int64_t* cur = (int64_t*)calloc((size_t)nbins + 1, sizeof(int64_t));
    for (int64_t r = 0; r < n; ++r)
        if (dest[r] >= 0 && dest[r] < nbins) cur[dest[r] + 1]++;
    for (int64_t b = 0; b < nbins; ++b) cur[b + 1] += cur[b];
    for (int64_t b = 0; b <= nbins; ++b) offsets[b] = cur[b];
    const char* src = (const char*)data;
    char* dst = (char*)out;
    for (int64_t r = 0; r < n; ++r) {
        int64_t b = dest[r];
        if (b < 0 || b >= nbins) continue;
        memcpy(dst + (cur[b]++) * row_bytes, src + r * row_bytes, (size_t)row_bytes);
    }
    int64_t total = offsets[nbins];
    free(cur);
    return total;
}

/* splitmix64 finaliser and the §8d uniform generator (same stream as the device one). */
static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

uint64_t oracle_splitmix64(uint64_t x) { return splitmix64(x); }

void oracle_synth_uniform(uint64_t seed, int64_t gid0, int64_t n, int dim, const double* box,
                          double* pos, int64_t* ids) {
    for (int64_t i = 0; i < n; ++i) {
        uint64_t gid = (uint64_t)(gid0 + i);
        for (int d = 0; d < dim; ++d) {
            uint64_t h = splitmix64(seed ^ (3ULL * gid + (uint64_t)d));
            pos[i * dim + d] = (double)(h >> 11) * 0x1.0p-53 * box[d];
        }
        if (ids) ids[i] = (int64_t)gid;
    }
}

/* FNV-1a over a byte range: order-sensitive digest for large-N parity. */
uint64_t oracle_fnv1a(const void* p, int64_t nbytes) {
    const unsigned char* b = (const unsigned char*)p;
    uint64_t h = 0xcbf29ce484222325ULL;
    for (int64_t i = 0; i < nbytes; ++i) { h ^= b[i]; h *= 0x100000001b3ULL; }
    return h;
}
