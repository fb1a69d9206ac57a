// fmt.h — exact printf("%g") / iostream default formatting (precision 6) of
// a double, for the device CSV emitter (the reference
// prints hom_conf/het_conf with operator<< on doubles, call.hpp:29-38).
//
// The six significant digits are the exact decimal value of the double
// rounded half-to-even, as glibc does: v = M * 2^E, so
// v * 10^k = (M * 5^k) * 2^(E+k) with M * 5^k an exact multi-limb integer
// (sid_pow5.h); its bits at and below the binary point decide the rounding.
// Integer arithmetic only -- the host and the device produce the same bytes,
// and the host build of the same code is tested against std::to_chars.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sid_pow10.h"
#include "sid_pow5.h"

static __device__ const double sid_p10_d[SID_P10_MAX - SID_P10_MIN + 1] = SID_P10_INIT;
static const double sid_p10_h[SID_P10_MAX - SID_P10_MIN + 1] = SID_P10_INIT;
static __device__ const uint16_t sid_pow5_off_d[SID_POW5_MAX + 2] = SID_POW5_OFF_INIT;
static __device__ const uint64_t sid_pow5_limb_d[SID_POW5_NLIMBS] = SID_POW5_LIMB_INIT;
static const uint16_t sid_pow5_off_h[SID_POW5_MAX + 2] = SID_POW5_OFF_INIT;
static const uint64_t sid_pow5_limb_h[SID_POW5_NLIMBS] = SID_POW5_LIMB_INIT;

#define SID_FMT_MAX 16
#define SID_P10_N (SID_P10_MAX - SID_P10_MIN + 1)   // longest output: "-4.94066e-324" (13 bytes)

// floor(M * 2^E * 10^k) for 0 <= k <= SID_POW5_MAX and where the remainder
// lies against one half: cmp = -1 below (or no remainder), 0 exactly half,
// +1 above.  Returns UINT64_MAX if the quotient does not fit 64 bits.
__host__ __device__ inline uint64_t sid_scale10(uint64_t M, int E, int k, int& cmp)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const uint16_t* off = sid_pow5_off_d;
    const uint64_t* limb = sid_pow5_limb_d;
#else
    const uint16_t* off = sid_pow5_off_h;
    const uint64_t* limb = sid_pow5_limb_h;
#endif
    uint64_t P[16];
    const int n0 = off[k + 1] - off[k];
    uint64_t carry = 0;
    for (int i = 0; i < n0; ++i) {
        const unsigned __int128 t = (unsigned __int128)limb[off[k] + i] * M + carry;
        P[i] = (uint64_t)t;
        carry = (uint64_t)(t >> 64);
    }
    P[n0] = carry;
    const int n = n0 + 1;
    const int sh = -(E + k);   // value = P * 2^-sh
    if (sh <= 0) {
        cmp = -1;
        for (int i = 1; i < n; ++i)
            if (P[i]) return UINT64_MAX;
        if (-sh >= 64 || (sh < 0 && (P[0] >> (64 + sh)) != 0)) return UINT64_MAX;
        return P[0] << -sh;
    }
    const int w = sh >> 6, b = sh & 63;
    for (int i = w + 2; i < n; ++i)
        if (P[i]) return UINT64_MAX;
    const uint64_t lo = w < n ? P[w] : 0, hi = w + 1 < n ? P[w + 1] : 0;
    if (b == 0 && hi) return UINT64_MAX;
    if (b && (hi >> b)) return UINT64_MAX;
    const uint64_t Q = b ? ((lo >> b) | (hi << (64 - b))) : lo;
    const int hb = sh - 1, hw = hb >> 6, hbit = hb & 63;   // the half bit
    const uint64_t hwv = hw < n ? P[hw] : 0;
    const bool half = (hwv >> hbit) & 1;
    bool sticky = (hwv & ((1ull << hbit) - 1)) != 0;      // any bit below it
    for (int i = 0; i < hw && i < n && !sticky; ++i) sticky = P[i] != 0;
    cmp = half ? (sticky ? 1 : 0) : -1;
    return Q;
}

// Fast path of sid_dec6 for normal v: y = fl(v * fl(10^k)) is within
// 2 * 2^-53 * y < 2.3e-10 of the exact v * 10^k (two roundings), so its
// integer part and the side of one half its fraction lies on are exact unless
// the fraction is within 2^-20 of one half, or y within 1e-3 of the 10^5 /
// 10^6 ends of the 6-digit range -- those (a few in 10^6 values) and
// denormals / k outside the table go to the exact multi-limb path.
// p10: the 10^k table (a kernel may pass its LDS copy), null = the global one
__host__ __device__ inline bool sid_dec6_fast(double v, int be, uint32_t& D, int& X, const double* p10)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if (!p10) p10 = sid_p10_d;
#else
    if (!p10) p10 = sid_p10_h;
#endif
    if (be == 0) return false;
    int x = ((be - 1023) * 78913) >> 18;   // floor(e2 * log10(2)): the exponent x or x - 1
    int k = 5 - x;
    if (k - 1 < SID_P10_MIN || k > SID_P10_MAX) return false;
    double y = v * p10[k - SID_P10_MIN];
    if (y >= 1e6) {
        --k;
        ++x;
        y = v * p10[k - SID_P10_MIN];
    }
    if (!(y >= 100000.001) || !(y < 999999.999)) return false;
    const uint32_t Q = (uint32_t)y;
    const double f = y - (double)Q;   // exact (y < 2^20)
    if (f > 0.5 - 0x1p-20 && f < 0.5 + 0x1p-20) return false;
    D = Q + (f > 0.5 ? 1u : 0u);
    X = x;
    if (D == 1000000u) {
        D = 100000u;
        ++X;
    }
    return true;
}

// Six significant digits of v > 0 (finite): D in [100000, 999999], decimal
// exponent X of the leading digit, rounded half-to-even.  false if v is out of
// the supported range (v >= 2^63).
__host__ __device__ inline bool sid_dec6_exact(double v, uint32_t& D, int& X);

// the exact path out of line (its limb array lives in scratch), its results
// returned by value -- (ok << 63) | (X + 1024) << 32 | D -- so that the
// caller's locals never have their address taken (they would live in scratch)
static __host__ __device__ __noinline__ uint64_t sid_dec6_exact_packed(double v)
{
    uint32_t D = 0;
    int X = 0;
    const bool ok = sid_dec6_exact(v, D, X);
    return ((uint64_t)ok << 63) | ((uint64_t)(uint32_t)(X + 1024) << 32) | D;
}

__host__ __device__ inline bool sid_dec6(double v, uint32_t& D, int& X, const double* p10 = nullptr)
{
    const uint64_t bits = __builtin_bit_cast(uint64_t, v);
    const int be = (int)((bits >> 52) & 0x7ff);
    if (be < 1023 + 63 && sid_dec6_fast(v, be, D, X, p10)) return true;
    const uint64_t r = sid_dec6_exact_packed(v);
    D = (uint32_t)r;
    X = (int)((r >> 32) & 0x7FFFFFFFu) - 1024;
    return r >> 63;
}

// the exact multi-limb path
__host__ __device__ inline bool sid_dec6_exact(double v, uint32_t& D, int& X)
{
    const uint64_t bits = __builtin_bit_cast(uint64_t, v);
    const int be = (int)((bits >> 52) & 0x7ff);
    uint64_t M = bits & ((1ull << 52) - 1);
    int E;
    if (be == 0) {
        E = -1074;
    } else {
        M |= 1ull << 52;
        E = be - 1075;
    }
    if (be >= 1023 + 63) return false;
    int x = (int)floor(log10(v));
    for (int iter = 0; iter < 6; ++iter) {
        const int k = 5 - x;
        uint64_t Q;
        int cmp;
        if (k >= 0) {
            if (k > SID_POW5_MAX) {
                x = 5 - SID_POW5_MAX;
                continue;
            }
            Q = sid_scale10(M, E, k, cmp);
        } else {
            // v in [1e6, 2^63): integer part and exact fraction
            const uint64_t I = (E >= 0) ? (M << E) : (M >> -E);
            const double f = (E >= 0) ? 0.0 : v - (double)I;   // exact: the low bits of M
            uint64_t T = 1;
            for (int j = 0; j < -k; ++j) T *= 10;
            Q = I / T;
            const uint64_t R = I % T;
            // compare R + f with T / 2  <=>  2R + 2f with T
            const unsigned __int128 A = (unsigned __int128)R * 2;
            const double F = 2.0 * f;   // in [0, 2)
            if (A >= T) cmp = (A > T || F > 0.0) ? 1 : 0;
            else if (A + 1 == T) cmp = F > 1.0 ? 1 : (F == 1.0 ? 0 : -1);
            else cmp = -1;
        }
        if (Q >= 1000000u) {
            ++x;
            continue;
        }
        if (Q < 100000u) {
            --x;
            continue;
        }
        const bool up = cmp == 1 || (cmp == 0 && (Q & 1));
        D = (uint32_t)Q + (up ? 1u : 0u);
        X = x;
        if (D == 1000000u) {
            D = 100000u;
            ++X;
        }
        return true;
    }
    return false;
}

// "%g" of v decomposed: the six digits D, the exponent X, the digits kept
// after trailing zeros are stripped (nd), or a special form.
enum { SID_G6_NUM = 0, SID_G6_NAN, SID_G6_INF, SID_G6_ZERO, SID_G6_ONE, SID_G6_RANGE };
struct sid_g6 {
    uint32_t D;
    int X, nd, kind, neg;
};

__host__ __device__ inline sid_g6 sid_g6_prep(double v, const double* p10 = nullptr)
{
    const uint64_t bits = __builtin_bit_cast(uint64_t, v);
    const uint64_t mag = bits & 0x7fffffffffffffffull;
    sid_g6 g{0, 0, 0, SID_G6_NUM, (int)(bits >> 63)};
    if (mag > 0x7ff0000000000000ull) g.kind = SID_G6_NAN;
    else if (mag == 0x7ff0000000000000ull) g.kind = SID_G6_INF;
    else if (mag == 0) g.kind = SID_G6_ZERO;
    else if (mag == 0x3ff0000000000000ull) g.kind = SID_G6_ONE;   // 1: the most frequent confidence
    else if (!sid_dec6(__builtin_bit_cast(double, mag), g.D, g.X, p10)) g.kind = SID_G6_RANGE;
    else {
        int nd = 6;
        uint32_t d = g.D;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const bool z = nd > 1 && d % 10u == 0u && nd == 6 - i;
            nd -= z ? 1 : 0;
            d = z ? d / 10u : d;
        }
        g.nd = nd;
    }
    return g;
}

// length of the "%g" text, -1 out of range
__host__ __device__ inline int sid_g6_len(const sid_g6& g)
{
    switch (g.kind) {
    case SID_G6_NAN:
    case SID_G6_INF: return g.neg + 3;
    case SID_G6_ZERO:
    case SID_G6_ONE: return g.neg + 1;
    case SID_G6_RANGE: return -1;
    default: break;
    }
    const int X = g.X, nd = g.nd;
    int n = g.neg;
    if (X < -4 || X >= 6) n += (nd > 1 ? nd + 1 : 1) + 2 + ((X <= -100 || X >= 100) ? 3 : 2);
    else if (X >= 0) n += X + 1 + (nd > X + 1 ? nd - X : 0);
    else n += 2 + (-X - 1) + nd;
    return n;
}

// digit i (0 = leading) of the six-digit D
__host__ __device__ inline char sid_g6_digit(uint32_t D, int i)
{
    const uint32_t P[6] = {100000u, 10000u, 1000u, 100u, 10u, 1u};
    return (char)('0' + (D / P[i]) % 10u);
}

// the text into p (any address space; no private arrays: every loop below is
// unrolled with constant digit indices); returns the length, -1 out of range
__host__ __device__ inline int sid_g6_put(const sid_g6& g, char* p)
{
    int n = 0;
    if (g.neg) p[n++] = '-';
    switch (g.kind) {
    case SID_G6_NAN: p[n] = 'n', p[n + 1] = 'a', p[n + 2] = 'n'; return n + 3;
    case SID_G6_INF: p[n] = 'i', p[n + 1] = 'n', p[n + 2] = 'f'; return n + 3;
    case SID_G6_ZERO: p[n] = '0'; return n + 1;
    case SID_G6_ONE: p[n] = '1'; return n + 1;
    case SID_G6_RANGE: return -1;
    default: break;
    }
    const int X = g.X, nd = g.nd;
    const uint32_t D = g.D;
    if (X < -4 || X >= 6) {
        p[n++] = sid_g6_digit(D, 0);
        if (nd > 1) p[n++] = '.';
#pragma unroll
        for (int i = 1; i < 6; ++i)
            if (i < nd) p[n++] = sid_g6_digit(D, i);
        p[n++] = 'e';
        p[n++] = X < 0 ? '-' : '+';
        int ax = X < 0 ? -X : X;
        if (ax >= 100) {
            p[n++] = (char)('0' + ax / 100);
            ax %= 100;
        }
        p[n++] = (char)('0' + ax / 10);
        p[n++] = (char)('0' + ax % 10);
    } else if (X >= 0) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (i <= X || i < nd) {
                if (i == X + 1) p[n++] = '.';
                p[n++] = sid_g6_digit(D, i);
            }
        }
    } else {
        p[n++] = '0';
        p[n++] = '.';
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if (i < -X - 1) p[n++] = '0';
#pragma unroll
        for (int i = 0; i < 6; ++i)
            if (i < nd) p[n++] = sid_g6_digit(D, i);
    }
    return n;
}

// "%g" of v (precision 6) into p (>= SID_FMT_MAX bytes); returns the length,
// or -1 if v is outside the supported range (|v| >= 2^63, never a confidence).
__host__ __device__ inline int sid_fmt_g6(double v, char* p) { return sid_g6_put(sid_g6_prep(v), p); }

// decimal of an int32 (std::to_chars / operator<<(int)): its length, and the
// text into p (any address space, no private arrays)
__host__ __device__ inline int sid_i32_len(int32_t v)
{
    uint32_t u = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
    int n = v < 0 ? 2 : 1;
    const uint32_t P[9] = {10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u, 1000000000u};
#pragma unroll
    for (int i = 0; i < 9; ++i) n += u >= P[i] ? 1 : 0;
    return n;
}

__host__ __device__ inline int sid_fmt_i32(int32_t v, char* p)
{
    const int n = sid_i32_len(v);
    uint32_t u = v < 0 ? 0u - (uint32_t)v : (uint32_t)v;
    if (v < 0) p[0] = '-';
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        if (k < n - (v < 0 ? 1 : 0)) {
            p[n - 1 - k] = (char)('0' + u % 10u);
            u /= 10u;
        }
    }
    return n;
}
