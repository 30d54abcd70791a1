// Device-side building blocks shared by the kernel translation units
// (mgr_bin.hip, mgr_pack.hip, mgr_kernels.hip): IEEE/x86-exact scalar math
// of the reference's wrap and binning, wave primitives, one-pass scan words,
// streaming load/store policies, XCD-aware tile order; plus launch helpers.
#pragma once

#include "mgr_internal.h"

#include <limits.h>

#include <type_traits>

namespace mgr {

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
static __device__ __attribute__((noinline)) double wrap_f64_slow(double x, double L) {
    const double m = pymod(x, L);
    if (isnan(m)) return m;
    return pymod(m + L, L);
}

static __device__ __attribute__((noinline)) float wrap_f32_slow(float x, float L) {
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

// ---- float16 positions: numpy 2.2.6's software half conversions (its
// half.hpp, restated): round to nearest even, overflow to inf, subnormals
// kept; a NaN keeps its sign and shifted payload and is NEVER quieted (a
// payload that would shift out becomes 1, so it stays a NaN).  numpy's half
// arithmetic is the float32 operation rounded back (checked against numpy on
// 2M random bit patterns, NaNs included).  Bit manipulation only: nothing
// depends on the GPU's own half conversion or denormal modes.
struct f16_t {
    uint16_t u;
};

__device__ __forceinline__ float h2f(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    if (e == 0x1fu) return __uint_as_float(s | 0x7f800000u | (m << 13));
    if (e == 0) return __uint_as_float(s | __float_as_uint((float)m * 0x1p-24f));   // exact
    return __uint_as_float(s | ((e + 112u) << 23) | (m << 13));
}
__device__ __forceinline__ double h2d(uint16_t h) {
    if (((h >> 10) & 0x1fu) == 0x1fu)
        return __longlong_as_double((long long)(((unsigned long long)(h & 0x8000u) << 48) |
                                                0x7ff0000000000000ull |
                                                ((unsigned long long)(h & 0x3ffu) << 42)));
    return (double)h2f(h);   // exact
}
// Round the magnitude `mag` (an integer in units of 2^-shift half-ulps) to
// nearest even: the kept bits r = mag >> shift, ties by the low bit of r.
template <typename U>
__device__ __forceinline__ uint32_t rne_shift(U mag, int shift) {
    const U r = mag >> shift, rem = mag & (((U)1 << shift) - 1), half = (U)1 << (shift - 1);
    return (uint32_t)(r + ((rem > half || (rem == half && (r & 1))) ? 1 : 0));
}
__device__ __forceinline__ uint16_t f2h(float x) {
    const uint32_t f = __float_as_uint(x), s = (f >> 16) & 0x8000u, a = f & 0x7fffffffu;
    if (a >= 0x7f800000u) {   // inf / NaN
        if (a == 0x7f800000u) return (uint16_t)(s | 0x7c00u);
        uint32_t r = 0x7c00u + ((a & 0x7fffffu) >> 13);
        if (r == 0x7c00u) ++r;
        return (uint16_t)(s | r);
    }
    if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00u);          // >= 65520: inf
    if (a >= 0x38800000u) return (uint16_t)(s | rne_shift<uint32_t>(a - 0x38000000u, 13));  // normal
    if (a < 0x33000000u) return (uint16_t)s;                        // <= 2^-25 (tie to 0) and below
    const int e = (int)(a >> 23);                                   // subnormal half: units of 2^-24
    return (uint16_t)(s | rne_shift<uint32_t>((a & 0x7fffffu) | 0x800000u, 126 - e));
}
__device__ __forceinline__ uint16_t d2h(double x) {   // direct, no double rounding via float
    const unsigned long long d = (unsigned long long)__double_as_longlong(x);
    const uint32_t s = (uint32_t)(d >> 48) & 0x8000u;
    const unsigned long long a = d & 0x7fffffffffffffffull;
    if (a >= 0x7ff0000000000000ull) {
        if (a == 0x7ff0000000000000ull) return (uint16_t)(s | 0x7c00u);
        uint32_t r = 0x7c00u + (uint32_t)((a & 0xfffffffffffffull) >> 42);
        if (r == 0x7c00u) ++r;
        return (uint16_t)(s | r);
    }
    if (a >= 0x40effe0000000000ull) return (uint16_t)(s | 0x7c00u);                 // >= 65520
    if (a >= 0x3f10000000000000ull)                                                  // >= 2^-14
        return (uint16_t)(s | rne_shift<unsigned long long>(a - 0x3f00000000000000ull, 42));
    if (a < 0x3e60000000000000ull) return (uint16_t)s;                              // <= 2^-25
    const int e = (int)(a >> 52);
    return (uint16_t)(s | rne_shift<unsigned long long>((a & 0xfffffffffffffull) | (1ull << 52),
                                                        1051 - e));
}

// x86 cvttsd2si (numpy's float -> int casts on the in-place write-back of
// integer positions): NaN / out of range -> the "integer indefinite" MIN.
__device__ __forceinline__ int trunc_i32(double v) {
    return (v > -2147483649.0 && v < 2147483648.0) ? (int)v : INT_MIN;
}

// numpy bool positions (one byte, 0 / 1).
struct b8_t {
    uint8_t u;
};

// The positions' dtypes beyond float32 / float64: every integer width,
// float16 and bool (bin_coord_ext).
template <typename P>
constexpr bool kExtPos = std::is_integral<P>::value || std::is_same<P, f16_t>::value ||
                         std::is_same<P, b8_t>::value;

// A stored position as numpy promotes it against a float64 scalar (the
// quotient of integer positions, the halo's float64 comparisons).
template <typename PosT>
__device__ __forceinline__ double pos_as_f64(PosT v) {
    if constexpr (std::is_same<PosT, f16_t>::value) return h2d(v.u);
    else if constexpr (std::is_same<PosT, b8_t>::value) return v.u ? 1.0 : 0.0;
    else if constexpr (std::is_same<PosT, float>::value) return f32_to_f64_x86(v);
    else return (double)v;   // 64-bit integers: round to nearest, as numpy's cast
}

// numpy's float -> integer casts on x86 (the in-place write-back of integer
// positions wrapped in a float type; probed on numpy 2.2.6, pinned by
// tests/golden/bin_dtypes.npz, and -- the NaN / out-of-range branches, from
// zero, negative and infinite boxes -- by tests/golden/bin_dtype_edges.npz,
// both made by the reference): <= 32-bit signed and <= 16-bit unsigned
// types through a 32-bit cvttsd2si (NaN / out of range -> INT_MIN, then the
// low bits), int64 through the 64-bit one; uint32 / uint64: values at or
// above 2^(w-1) converted after subtracting it, the top bit flipped back;
// bool: != 0.  A float32 / float16 wrap converts exactly to float64 first.
template <typename P>
__device__ __forceinline__ P pos_from_f64(double t) {
    if constexpr (std::is_same<P, b8_t>::value) {
        return b8_t{(uint8_t)(t != 0.0 ? 1 : 0)};
    } else if constexpr (std::is_same<P, int64_t>::value) {
        return (P)trunc_i64(t);
    } else if constexpr (std::is_same<P, uint64_t>::value) {
        return t >= 9223372036854775808.0
                   ? (uint64_t)trunc_i64(t - 9223372036854775808.0) ^ 0x8000000000000000ull
                   : (uint64_t)trunc_i64(t);
    } else if constexpr (std::is_same<P, uint32_t>::value) {
        return t >= 2147483648.0 ? (uint32_t)trunc_i32(t - 2147483648.0) ^ 0x80000000u
                                 : (uint32_t)trunc_i32(t);
    } else {
        return (P)(unsigned)trunc_i32(t);
    }
}
template <typename P>
__device__ __forceinline__ P pos_from_int(long long t) {   // C truncation, as numpy's casts
    if constexpr (std::is_same<P, b8_t>::value) return b8_t{(uint8_t)(t != 0 ? 1 : 0)};
    else return (P)t;
}
template <typename P>
__device__ __forceinline__ long long pos_int(P v) {   // unsigned 64-bit: the bits
    if constexpr (std::is_same<P, b8_t>::value) return v.u ? 1 : 0;
    else return (long long)v;
}

template <typename PosT>
__device__ __forceinline__ bool same_bits(PosT a, PosT b) {
    if constexpr (std::is_same<PosT, f16_t>::value || std::is_same<PosT, b8_t>::value) return a.u == b.u;
    else if constexpr (std::is_integral<PosT>::value) return a == b;
    else if constexpr (sizeof(PosT) == 8) return __double_as_longlong((double)a) == __double_as_longlong((double)b);
    else return __float_as_uint((float)a) == __float_as_uint((float)b);
}

// One coordinate: wrap (+ write back), bin, index wrap.  Returns the wrapped
// index; *raw gets trunc(t/L*n) before the index wrap (cell indexes API).
// The wrapped value is stored only when its bits differ from the input
// (the in-place mutation of redist.py:68 / :328-329 is then complete: an
// in-box coordinate wraps to itself) and *dirty records that a store happened.
// SIDE, a per-row side output computed from the same values:
//   kSideFine: the coordinate's fine index (FineGeom) from the same quotient
//     t/L -- exactly what the fine plan computes from the stored position;
//   kSideHalo: the coordinate's two face flags against its cell's limits
//     (HaloGeom): bit 0 = x > (k+1)*cl - ol, bit 1 = x < k*cl + ol, the
//     float64 comparisons of redist.py:271-276 for the rank the row lands on.
constexpr int kSideNone = 0, kSideFine = 1, kSideHalo = 2;

// The index stage of one coordinate, every position dtype alike: k =
// trunc(q * n) (and kf = trunc(q * n_fine)) from the quotient, the integer
// wrap of :90, the fine / halo side value from xs (the stored coordinate as
// float64).
template <int SIDE>
__device__ __forceinline__ long long coord_index(long long k, long long kf, double xs,
                                                 const Geom& g, int d, long long* raw,
                                                 const FineGeom* fg, const HaloGeom* hg,
                                                 long long* side) {
    if (raw) *raw = k;
    const long long n = g.n[d];
    if (!(k >= 0 && k < n)) k = floormod_i64(floormod_i64(k, n) + n, n);
    if (g.fine) k %= g.fmod[d];   // fine-cell plan: index inside the rank's cell
    if (SIDE == kSideFine) {
        const long long nf = fg->n[d];
        if (!(kf >= 0 && kf < nf)) kf = floormod_i64(floormod_i64(kf, nf) + nf, nf);
        // kf % f without a 64-bit division: kf - f*k when the coarse index k
        // is kf's cell (always, up to rounding at a cell face), else the
        // remainder itself
        const long long f = fg->fmod[d];
        long long m = kf - f * k;
        if (!(m >= 0 && m < f)) m = kf % f;
        *side = m;
    }
    if (SIDE == kSideHalo) {
        // limits (redist.py:110-111): k * cl and (k + 1) * cl, int64 * float64
        const double hi = (double)(k + 1) * hg->cl[d] - hg->ol[d];
        const double lo = (double)k * hg->cl[d] + hg->ol[d];
        *side = (xs > hi ? 1 : 0) | (xs < lo ? 2 : 0);
    }
    return k;
}

// One coordinate of an integer / float16 / bool position (kExtPos): numpy
// 2.2.6's promotion of `position[:, d] % box[d]` (Geom::wmode) and of
// `position[:, d] / box[d]` (Geom::dmode), mgr_capi.hip pos_modes:
//   * integer positions, integer box: integer remainder at the promoted type
//     (floor-mod for signed, plain for unsigned; the `+ L` wraps at its
//     width), stored back truncated to the column's width; the quotient is
//     float64 (true division);
//   * integer / bool positions, float box: the wrap in the promoted float
//     type (float64; float32 for <= 16-bit integers against a float32 box;
//     float16 for 8-bit ones against a float16 box), stored back by numpy's
//     x86 float -> int cast (pos_from_f64), the quotient from the stored
//     value in the same float type;
//   * float16 positions: the wrap in float64 / float32 rounded to float16 on
//     the write-back (as S9 for float32), or -- box float16 / 8-bit integer --
//     every operation in float32 rounded to float16 (numpy's half arithmetic);
//     the quotient in float64, float32 or float16 alike, then * n in float64.
// The general path only (no fast in-box variant): these dtypes are for
// parity with the reference's inputs, not the bench's hot configurations.
static __device__ __forceinline__ long long wrap_int(long long x, long long L, int wmode) {
    const int bits = (wmode == MGR_I8 || wmode == MGR_U8) ? 8
                   : (wmode == MGR_I16 || wmode == MGR_U16) ? 16
                   : (wmode == MGR_I32 || wmode == MGR_U32) ? 32 : 64;
    const bool sgn = wmode == MGR_I8 || wmode == MGR_I16 || wmode == MGR_I32 || wmode == MGR_I64;
    auto norm = [&](unsigned long long v) -> unsigned long long {   // to the type's value
        if (bits == 64) return v;
        const unsigned long long m = (1ull << bits) - 1ull;
        v &= m;
        if (sgn && ((v >> (bits - 1)) & 1ull)) v |= ~m;
        return v;
    };
    if (sgn) {
        const long long m = floormod_i64(x, L);   // numpy: x % 0 == 0
        const long long s = (long long)norm((unsigned long long)m + (unsigned long long)L);
        return floormod_i64(s, L);
    }
    const unsigned long long ux = (unsigned long long)x, uL = (unsigned long long)L;
    if (uL == 0ull) return 0;
    const unsigned long long s = norm(ux % uL + uL);
    return (long long)(s % uL);
}
static __device__ __forceinline__ uint16_t wrap_f16(uint16_t x, float L) {
    const float m = pymodf(h2f(x), L);
    const uint16_t mh = f2h(m);
    if (isnan(m)) return mh;   // a NaN propagates unchanged (x86)
    const uint16_t yh = f2h(h2f(mh) + L);
    return f2h(pymodf(h2f(yh), L));
}

template <typename PosT, bool kPeriodic, int SIDE>
__device__ __forceinline__ long long bin_coord_ext(PosT* p, const Geom& g, int d, long long* raw,
                                                   bool* dirty, const FineGeom* fg,
                                                   const HaloGeom* hg, long long* side) {
    const PosT in = *p;
    PosT s = in;   // the stored value binning reads back (S2)
    if (kPeriodic) {
        if constexpr (std::is_same<PosT, f16_t>::value) {
            if (g.wmode == MGR_F64)
                s.u = d2h(wrap_f64(h2d(in.u), g.L[d], g.twoL[d], g.fast[d]));
            else if (g.wmode == MGR_F32)
                s.u = f2h(wrap_f32(h2f(in.u), g.Lf[d], g.twoLf[d], g.fastf[d]));
            else
                s.u = wrap_f16(in.u, g.Lf[d]);
        } else {
            if (g.wmode == MGR_F64)
                s = pos_from_f64<PosT>(wrap_f64(pos_as_f64(in), g.L[d], g.twoL[d], g.fast[d]));
            else if (g.wmode == MGR_F32)   // <= 16-bit integers / bool: exact in float32
                s = pos_from_f64<PosT>((double)wrap_f32((float)pos_as_f64(in), g.Lf[d],
                                                        g.twoLf[d], g.fastf[d]));
            else if (g.wmode == MGR_F16)   // 8-bit integers / bool: exact in float16
                s = pos_from_f64<PosT>((double)h2f(wrap_f16(f2h((float)pos_as_f64(in)), g.Lf[d])));
            else
                s = pos_from_int<PosT>(wrap_int(pos_int(in), g.Li[d], g.wmode));
        }
        if (!same_bits(s, in)) { *p = s; *dirty = true; }
    }
    long long k, kf = 0;
    const double xs = pos_as_f64(s);
    double q;   // the quotient as the float64 the `* n` promotes it to
    if (g.dmode == MGR_F64) {
        q = xs / g.L[d];
    } else {   // the quotient in float32, or float16 (the stored value is exact in either)
        float qf = (float)xs / g.Lf[d];
        if (g.dmode == MGR_F16) qf = h2f(f2h(qf));
        q = (double)qf;
    }
    k = trunc_i64(q * g.nd[d]);
    if (SIDE == kSideFine) kf = trunc_i64(q * fg->nd[d]);
    return coord_index<SIDE>(k, kf, xs, g, d, raw, fg, hg, side);
}

template <typename PosT, bool kPeriodic, int SIDE = kSideNone>
__device__ __forceinline__ long long bin_coord(PosT* p, const Geom& g, int d, long long* raw,
                                               bool* dirty, const FineGeom* fg = nullptr,
                                               const HaloGeom* hg = nullptr,
                                               long long* side = nullptr) {
    if constexpr (kExtPos<PosT>) {
        return bin_coord_ext<PosT, kPeriodic, SIDE>(p, g, d, raw, dirty, fg, hg, side);
    } else {
    long long k, kf = 0;
    double xs = 0.0;   // the stored (wrapped) coordinate, as numpy compares it
    const PosT in = *p;
    if (sizeof(PosT) == 4 && g.compute_f32) {
        float x = (float)in;
        if (kPeriodic) {
            x = wrap_f32(x, g.Lf[d], g.twoLf[d], g.fastf[d]);
            if (!same_bits((PosT)x, in)) { *p = (PosT)x; *dirty = true; }
        }
        const float q = g.pow2f[d] ? x * g.invLf[d] : x / g.Lf[d];  // f32 / f32 -> f32
        k = trunc_i64((double)q * g.nd[d]);          // * int64 scalar -> f64
        if (SIDE == kSideFine) kf = trunc_i64((double)q * fg->nd[d]);
        if (SIDE == kSideHalo) xs = f32_to_f64_x86(x);
    } else {
        double x = sizeof(PosT) == 4 ? f32_to_f64_x86((float)in) : (double)in;
        if (kPeriodic) {
            const double t = wrap_f64(x, g.L[d], g.twoL[d], g.fast[d]);
            const PosT w = sizeof(PosT) == 4 ? (PosT)f64_to_f32_x86(t) : (PosT)t;  // round (S9)
            if (!same_bits(w, in)) { *p = w; *dirty = true; }
            x = sizeof(PosT) == 4 ? f32_to_f64_x86((float)w) : (double)w;  // bin reads it (S2)
        }
        const double q = g.pow2[d] ? x * g.invL[d] : x / g.L[d];
        k = trunc_i64(q * g.nd[d]);
        if (SIDE == kSideFine) kf = trunc_i64(q * fg->nd[d]);
        if (SIDE == kSideHalo) xs = x;
    }
    return coord_index<SIDE>(k, kf, xs, g, d, raw, fg, hg, side);
    }
}

// In-box fast path of bin_row: every coordinate in [0, L_d) with the fast
// wrap (every in-box particle).  The same values as bin_coord, in 32-bit
// integer arithmetic: an in-box quotient x/L lies in [0, 1], so trunc(q*n)
// lies in [0, n] (n < 2^30, Geom::fast32) and the floor-mod reduces to
// n -> 0; the cell number is below nbins.  NaN fails the range test, so the
// x86 NaN rules never arise here.  Returns false (nothing written) when a
// coordinate is outside; bin_row then takes the general path.
// GEO: the plan's geometry at compile time where it is simple (geo_kind):
// kGeoAny -- read every flag from g; kGeoF32 / kGeoF64 -- every dimension
// has the fast wrap and a power-of-two box length (x / L == x * (1/L)), the
// quotient is computed in f32 / f64, and the plan is not a fine plan.  The
// values are the same; only the per-row flag tests and branches go away.
constexpr int kGeoAny = 0, kGeoF32 = 1, kGeoF64 = 2;

template <typename PosT, bool kPeriodic, int DIM, int SIDE, int GEO = kGeoAny>
__device__ __forceinline__ bool bin_row_fast(PosT* row, const Geom& g, bool* dirty,
                                             const FineGeom* fg, const HaloGeom* hg,
                                             long long* cell_out, long long* side) {
    const bool f32c = GEO == kGeoF32 ? true
                    : GEO == kGeoF64 ? false
                                     : (sizeof(PosT) == 4 && g.compute_f32);
    PosT in[DIM];
    bool inb = true;
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
        in[d] = row[d];
        if (f32c) inb = inb && (GEO != kGeoAny || g.fastf[d]) && (float)in[d] >= 0.0f && (float)in[d] < g.Lf[d];
        else inb = inb && (GEO != kGeoAny || g.fast[d]) && (double)in[d] >= 0.0 && (double)in[d] < g.L[d];
    }
    if (!inb) return false;
    int cell = 0, sc = 0;
#pragma unroll
    for (int d = 0; d < DIM; ++d) {
        int k, kf = 0;
        double xs = 0.0;
        if (f32c) {
            float x = (float)in[d];
            if (kPeriodic) {
                const float y = x + g.Lf[d];
                x = (y == g.twoLf[d]) ? 0.0f : y - g.Lf[d];
                if (!same_bits((PosT)x, in[d])) { row[d] = (PosT)x; *dirty = true; }
            }
            const float q = (GEO != kGeoAny || g.pow2f[d]) ? x * g.invLf[d] : x / g.Lf[d];
            k = (int)((double)q * g.nd[d]);
            if (SIDE == kSideFine) kf = (int)((double)q * fg->nd[d]);
            if (SIDE == kSideHalo) xs = (double)x;
        } else {
            double x = (double)in[d];
            if (kPeriodic) {
                const double y = x + g.L[d];
                const double t = (y == g.twoL[d]) ? 0.0 : y - g.L[d];
                const PosT w = sizeof(PosT) == 4 ? (PosT)(float)t : (PosT)t;
                if (!same_bits(w, in[d])) { row[d] = w; *dirty = true; }
                x = (double)w;
            }
            const double q = (GEO != kGeoAny || g.pow2[d]) ? x * g.invL[d] : x / g.L[d];
            k = (int)(q * g.nd[d]);
            if (SIDE == kSideFine) kf = (int)(q * fg->nd[d]);
            if (SIDE == kSideHalo) xs = x;
        }
        const int n = (int)g.n[d];
        if (k >= n) k -= n;
        if (GEO == kGeoAny && g.fine) k %= (int)g.fmod[d];
        if (SIDE == kSideFine) {
            const int nf = (int)fg->n[d], f = (int)fg->fmod[d];
            if (kf >= nf) kf -= nf;
            int m = kf - f * k;
            if (!(m >= 0 && m < f)) m = kf % f;
            sc += (int)fg->off[d] * m;
        }
        if (SIDE == kSideHalo) {
            const double hi = (double)(k + 1) * hg->cl[d] - hg->ol[d];
            const double lo = (double)k * hg->cl[d] + hg->ol[d];
            sc |= ((xs > hi ? 1 : 0) | (xs < lo ? 2 : 0)) << (2 * d);
        }
        cell += (int)g.off[d] * k;
    }
    *cell_out = cell;
    if (SIDE != kSideNone) *side = sc;
    return true;
}

// DIM > 0: compile-time dimensionality (the common 1-3); 0: runtime g.dim.
// SIDE: *side gets the row's fine cell (row-major over fg->fmod) or its face
// flags (bit 2d: right face of dimension d, bit 2d+1: left face).
template <typename PosT, bool kPeriodic, int DIM = 0, int SIDE = kSideNone, int GEO = kGeoAny>
__device__ __forceinline__ long long bin_row(PosT* row, const Geom& g, long long* idx,
                                             bool* dirty, const FineGeom* fg = nullptr,
                                             const HaloGeom* hg = nullptr,
                                             long long* side = nullptr) {
    if constexpr (DIM > 0 && !kExtPos<PosT>) {
        long long c;
        if (!idx && (GEO != kGeoAny || g.fast32) &&
            bin_row_fast<PosT, kPeriodic, DIM, SIDE, GEO>(row, g, dirty, fg, hg, &c, side))
            return c;
    }
    long long cell = 0, sc = 0;
    const int nd = DIM > 0 ? DIM : g.dim;
#pragma unroll
    for (int d = 0; d < (DIM > 0 ? DIM : MGR_MAX_DIM); ++d) {
        if (DIM == 0 && d >= nd) break;
        long long sd = 0;
        cell += g.off[d] * bin_coord<PosT, kPeriodic, SIDE>(row + d, g, d, idx ? idx + d : nullptr,
                                                            dirty, fg, hg, &sd);
        if (SIDE == kSideFine) sc += (long long)((int)fg->off[d] * (int)sd);   // < 4096 cells
        if (SIDE == kSideHalo) sc |= sd << (2 * d);
    }
    if (SIDE != kSideNone) *side = sc;
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

// match_bin with the bit count at compile time (NBITS > 0: unrolled).
template <int NBITS>
__device__ __forceinline__ unsigned long long match_bin_t(unsigned b, bool valid, int nbits) {
    if constexpr (NBITS == 0) {
        return match_bin(b, valid, nbits);
    } else {
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int i = 0; i < NBITS; ++i) {
            const bool bit = (b >> i) & 1u;
            const unsigned long long m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        return valid ? peers : 0ull;
    }
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

// ------------------------------------------------- one-pass scan words
// Word layout: bits 62-63 status (0 none, 1 aggregate, 2 inclusive prefix),
// bit 61 poison (the value rests on a look-back that timed out), bits 0-60
// the count.  Behind the kScanFlags words the scan keeps its control words
// (ScanCtl), zeroed with them by every count producer.
constexpr uint64_t kScanAgg = 1ull << 62, kScanInc = 2ull << 62, kScanPoison = 1ull << 61,
                   kScanVal = (1ull << 61) - 1;

__device__ __forceinline__ void clear_scan_flags(uint64_t* __restrict__ flags) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kScanFlags + kScanCtlWords;
         i += step)
        flags[i] = 0;
}

__device__ __forceinline__ ScanCtl* scan_ctl(uint64_t* flags) {
    return (ScanCtl*)(flags + kScanFlags);
}

__device__ __forceinline__ void flag_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Poll until the word's status reaches `need`, at most `spins` times (a
// lost producer must not hang the GPU).  On exhaustion the stale word is
// returned with the poison bit set, so everything computed from it is
// marked; spins < 0 gives up at once (test knob scan_spins).
__device__ __forceinline__ uint64_t flag_poll(uint64_t* p, uint64_t need, int spins) {
    uint64_t w = 0;
    for (int spin = 0;; ++spin) {
        if (spins >= 0) w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (spins >= 0 && (w >> 62) >= need) return w;
        if (spin >= spins) return (w & ~(3ull << 62)) | (need << 62) | kScanPoison;
        __builtin_amdgcn_s_sleep(1);
    }
}

// Segment start of bin b's rows of tile `tile` in a pack's output: the
// scan's offset; the redirect bin's rows go to redirect_dst from its row 0
// (minus the bin's start), and the bins after it close the gap it leaves
// (minus its size), so the packed send buffer holds exactly the rows that
// travel (mgr_pack, include/mgr.h).
__device__ __forceinline__ long long seg_start(const int64_t* __restrict__ offsets,
                                               const int64_t* __restrict__ bin_starts, int64_t T,
                                               int64_t tile, int b, int redirect_bin) {
    long long o = offsets[(int64_t)b * T + tile];
    if (redirect_bin >= 0) {
        if (b == redirect_bin) o -= bin_starts[b];
        else if (b > redirect_bin) o -= bin_starts[redirect_bin + 1] - bin_starts[redirect_bin];
    }
    return o;
}

// seg_start for bin min(lane, nb - 1) in two steps: seg_load issues the
// loads unconditionally (no exec mask, no use of their values), seg_value
// combines them -- so a kernel can put its payload loads in between and
// wait for everything once.  Lanes >= nb get a value they must not use.
struct SegLoad {
    long long o, own, gap;
};
__device__ __forceinline__ SegLoad seg_load(const int64_t* __restrict__ offsets,
                                            const int64_t* __restrict__ bin_starts, int64_t T,
                                            int64_t tile, int lane, int nb, int redirect_bin) {
    const int b = min(lane, nb - 1);
    SegLoad s{offsets[(int64_t)b * T + tile], 0, 0};
    if (redirect_bin >= 0) {   // uniform
        s.own = bin_starts[b];
        s.gap = bin_starts[redirect_bin + 1] - bin_starts[redirect_bin];
    }
    return s;
}
__device__ __forceinline__ long long seg_value(const SegLoad& s, int lane, int redirect_bin) {
    if (redirect_bin < 0) return s.o;
    return s.o - (lane == redirect_bin ? s.own : (lane > redirect_bin ? s.gap : 0ll));
}

// A failed scan (ScanCtl::err, mgr_kernels.hip) leaves offsets that must
// not be written through: every pack kernel checks it before its first
// store (the word was written by an earlier kernel, a uniform read).
__device__ __forceinline__ bool scan_failed(const uint32_t* __restrict__ scan_err) {
    return scan_err && *scan_err != 0u;
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

// Clang vector types, not HIP's uint4/uint2: those are union wrappers that
// SROA can leave as an alloca, which the backend then parks in LDS (a
// ds_write/ds_read pair per unit -- measured +15 % on the coop pack).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <int W> struct Unit;
template <> struct Unit<16> { using T = u32x4_t; };
template <> struct Unit<8> { using T = u32x2_t; };
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

// ------------------------------------------------ image stores (packs)
typedef unsigned int u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// Store through an address held as an integer: a global-address-space
// pointer, so the compiler emits global_store (a plain pointer would be flat).
template <typename T>
__device__ __forceinline__ void gstore(unsigned long long a, T v) {
    *(__attribute__((address_space(1))) T*)a = v;
}

// One 16-byte unit (image bytes [x, x + 16)) of a destination-sorted LDS
// image to its output: a bin's rows are one run of the image, and the unit's
// bytes go to gaddr[bin] + x.  A unit inside one run is one 16-byte store;
// a unit straddling two runs goes dword by dword.  For rows wider than 16 B
// a unit covers at most two rows (x / RB and (x + 15) / RB), so both run
// addresses are fetched up front, side by side -- no LDS lookup per dword on
// the straddling path (the lookups were a chain of dependent LDS reads per
// dword).  DROP: a zero address is a dropped bin, not written.
template <int RB, bool DROP, typename BinT>
__device__ __forceinline__ void store_img_unit(const uint8_t* __restrict__ img,
                                               const BinT* ibin,
                                               const unsigned long long* gaddr, int x,
                                               int nbytes) {
    const u32x4_t q = *(const u32x4_t*)(img + x);
    const int r0 = x / RB, r1 = min(x + 15, nbytes - 1) / RB;
    const int bf = ibin[r0], bl = ibin[r1];
    const unsigned long long af = gaddr[bf], al = gaddr[bl];
    if (x + 16 <= nbytes && bf == bl) {
        if (!DROP || af) gstore<u32x4_a4>(af + x, q);
        return;
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int xd = x + 4 * d;
        if (xd >= nbytes) break;
        unsigned long long a;
        if constexpr (RB > 16) a = xd < (r0 + 1) * RB ? af : al;
        else a = gaddr[ibin[xd / RB]];   // narrow rows: up to 4 rows in a unit
        if (!DROP || a) gstore<uint32_t>(a + xd, q[d]);
    }
}

// A wave's 64 * RPW rows of RB bytes (compile time), parked in LDS in row
// order at `rows`, permuted in place into the destination-ordered image (row
// 64 q + lane -> slot[q]), then the image streamed out (store_img_unit,
// gaddr[bin] = the address of the bin's image slot 0 in the output, 0 = not
// written).  The multi-field pack runs it per field, the one-pass partition
// once per wave.  (A/B, round 6: the straddling units deferred to one
// dword-store pass per wave -- 2.3x fewer store instructions in the one-pass
// kernel -- measured 1.22 vs 1.20 ms: store issue is not what bounds it.)
template <int RB, int RPW>
__device__ __forceinline__ void image_pass(uint8_t* rows, const uint8_t* ibin,
                                           const unsigned long long* gaddr, const int* slot,
                                           const bool* valid, int nrows, int lane) {
    constexpr int DW = RB / 4;
    uint32_t* w32 = (uint32_t*)rows;
    uint32_t row[RPW][DW];
#pragma unroll
    for (int q = 0; q < RPW; ++q)
        if (valid[q]) {
#pragma unroll
            for (int p = 0; p < DW; ++p) row[q][p] = w32[(64 * q + lane) * DW + p];
        }
    wave_sync();
#pragma unroll
    for (int q = 0; q < RPW; ++q)
        if (valid[q]) {
#pragma unroll
            for (int p = 0; p < DW; ++p) w32[slot[q] * DW + p] = row[q][p];
        }
    wave_sync();
    const int nbytes = nrows * RB;
    for (int x = 16 * lane; x < nbytes; x += 1024) store_img_unit<RB, true>(rows, ibin, gaddr, x, nbytes);
}

// ------------------------------------------------- flag-set selections
// The halo's selections read 16-bit face flags in chunks of kSelChunk rows:
// lane l holds rows [16 l, 16 l + 16) of a chunk as 8 packed words (two
// 16-byte loads per lane, in flight together), so a set's membership is one
// 16-bit mask per lane and its order is (lane, bit) = row order.  Set k's
// flag bit: nibble k of a 64-bit word (no dynamic indexing into a
// kernel-argument array).
constexpr int kSelChunk = 1024, kSelWords = kSelChunk / 128;

__device__ __forceinline__ void chunk_flags(const uint16_t* __restrict__ flags, int64_t c0,
                                            int crows, int lane, uint32_t (&fw)[kSelWords]) {
    const int r = 16 * lane;
    const uint16_t* p = flags + c0 + r;
    if (crows == kSelChunk && ((uintptr_t)(flags + c0) & 15) == 0) {
        const uint4* q = (const uint4*)p;
        const uint4 a = q[0], b = q[1];
        fw[0] = a.x; fw[1] = a.y; fw[2] = a.z; fw[3] = a.w;
        fw[4] = b.x; fw[5] = b.y; fw[6] = b.z; fw[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < kSelWords; ++i) {
            const uint32_t lo = r + 2 * i < crows ? p[2 * i] : 0u;
            const uint32_t hi = r + 2 * i + 1 < crows ? p[2 * i + 1] : 0u;
            fw[i] = lo | (hi << 16);
        }
    }
}

// bit j of the result: flag bit b of the lane's row j
__device__ __forceinline__ uint32_t set_mask(const uint32_t (&fw)[kSelWords], int b) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < kSelWords; ++i)
        m |= (((fw[i] >> b) & 1u) << (2 * i)) | (((fw[i] >> (16 + b)) & 1u) << (2 * i + 1));
    return m;
}

// Selection sets by flag mask: set k = the rows whose flags hold every bit of
// masks.m[k] (one bit: a face; several: an edge or corner region of the halo).
struct SetMasks {
    uint16_t m[kMaxSets];
};

// The chunk's flag bit-planes (plane b, bit j: the lane's row j has flag bit
// b) for the bits below nbits (the bits any set uses): computed once per
// chunk, every set's membership is then an AND of planes.
struct FlagPlanes {
    uint32_t p[16];
};
__device__ __forceinline__ void flag_planes(const uint32_t (&fw)[kSelWords], int nbits,
                                            FlagPlanes& fp) {
#pragma unroll
    for (int b = 0; b < 16; ++b) fp.p[b] = b < nbits ? set_mask(fw, b) : 0xFFFFu;
}
// bit j of the result: the lane's row j has every flag bit of mask
__device__ __forceinline__ uint32_t set_mask_m(const FlagPlanes& fp, unsigned mask, int nbits) {
    uint32_t r = 0xFFFFu;
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (b < nbits) r &= ((mask >> b) & 1u) ? fp.p[b] : 0xFFFFu;
    return r;
}
// flag_planes / set_mask_m with the flag bits at compile time (NB > 0, NB >=
// every bit a mask uses): the planes unrolled, a set's membership NB ANDs
// with a uniform per-bit fill instead of a run-time loop over 16 bits (the
// loop kept the halo's selection kernels VALU-bound); NB = 0: run time.
template <int NB>
__device__ __forceinline__ void flag_planes_t(const uint32_t (&fw)[kSelWords], int nbits,
                                              FlagPlanes& fp) {
    if constexpr (NB > 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) fp.p[b] = set_mask(fw, b);
    } else {
        flag_planes(fw, nbits, fp);
    }
}
template <int NB>
__device__ __forceinline__ uint32_t set_mask_t(const FlagPlanes& fp, unsigned mask, int nbits) {
    if constexpr (NB > 0) {
        uint32_t r = 0xFFFFu;
#pragma unroll
        for (int b = 0; b < NB; ++b) r &= fp.p[b] | (((mask >> b) & 1u) ? 0u : 0xFFFFu);
        return r;
    } else {
        return set_mask_m(fp, mask, nbits);
    }
}
// The compile-time flag-bit count a launcher instantiates for nbits.
static inline int flag_bits_class(int nbits) {
    return nbits <= 2 ? 2 : nbits <= 4 ? 4 : nbits <= 6 ? 6 : nbits <= 8 ? 8 : 0;
}
__device__ __forceinline__ int mask_bits(const SetMasks& sm, int nsets) {
    unsigned u = 0;
    for (int k = 0; k < nsets; ++k) u |= sm.m[k];
    return u ? 32 - __builtin_clz(u) : 0;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// exclusive prefix over the wave's lanes; *total = the sum
__device__ __forceinline__ int wave_excl(int v, int* total) {
    const int lane = lane_id();
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    *total = __shfl(x, 63, 64);
    return x - v;
}

// inclusive prefix over the wave's 64 lanes by DPP (row shifts inside each
// 16-lane row, then the row broadcasts of lanes 15 and 31): no LDS round
// trips, where __shfl_up lowers to a chain of ds_bpermute_b32.
__device__ __forceinline__ int wave_incl_dpp(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// a 64-bit value of lane l (uniform l), by two readlanes
__device__ __forceinline__ long long readlane64(long long v, int l) {
    const int lo = __builtin_amdgcn_readlane((int)(unsigned long long)v, l);
    const int hi = __builtin_amdgcn_readlane((int)((unsigned long long)v >> 32), l);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
    return (unsigned long long)readlane64((long long)v, l);
}

// exclusive prefix over the wave's lanes of small values (v < 2^BITS), by
// bit-sliced ballots: prefix = sum_i 2^i * (lanes below with bit i) -- BITS
// ballots and lane-mask popcounts (v_mbcnt), no LDS.  wave_excl's __shfl_up
// chain lowers to 7 dependent ds_bpermute_b32 round trips, which made the
// halo's per-set list building latency-bound.
template <int BITS>
__device__ __forceinline__ int wave_excl_small(unsigned v, int* total) {
    int pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < BITS; ++i) {
        const unsigned long long b = __ballot((v >> i) & 1u);
        const unsigned below = __builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u));
        pre += (int)below << i;
        tot += __popcll(b) << i;
    }
    *total = tot;
    return pre;
}

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

// xcd_tile in chunks of C tiles: XCD label x takes chunk x of every group of
// 8 C consecutive tiles, so all XCDs stream through one region of the input
// at a time (C <= 1: xcd_tile's one run per XCD).
__device__ __forceinline__ int64_t xcd_tile_c(int64_t bid, int64_t T, int C) {
    if (C <= 1) return xcd_tile(bid, T);
    const int64_t g = 8 * (int64_t)C;
    if (bid >= (T / g) * g) return bid;
    const int64_t within = bid % g;
    return bid - within + (within & 7) * C + (within >> 3);
}

// Streaming accesses: NT selects the nontemporal (nt) cache policy for data
// that is read or written exactly once.
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


// ----------------------------------------------------------- launch helpers
static inline int grid_for(int64_t n, int per_block_rows = kBlock) {
    int64_t g = (n + per_block_rows - 1) / per_block_rows;
    if (g > 256 * 16) g = 256 * 16;   // grid-stride beyond 16 blocks per CU
    return (int)(g < 1 ? 1 : g);
}

template <typename K>
static void ensure_lds(K kernel, int bytes) {
    if (bytes > 64 * 1024)
        (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// Waves per workgroup for a per-wave LDS footprint: 4 when a 4-wave
// workgroup stays within 64 KiB, fewer otherwise (never above 160 KiB).
static inline int waves_per_block(int per_wave_lds) {
    if (per_wave_lds * kWaves <= 64 * 1024) return kWaves;
    int w = (160 * 1024) / (per_wave_lds > 0 ? per_wave_lds : 1);
    return w < 1 ? 1 : (w > kWaves ? kWaves : w);
}

}  // namespace mgr
