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

#include "sid_pow5.h"

static __device__ const uint16_t sid_pow5_off_d[SID_POW5_MAX + 2] = SID_POW5_OFF_INIT;
static __device__ const uint64_t sid_pow5_limb_d[SID_POW5_NLIMBS] = SID_POW5_LIMB_INIT;
static const uint16_t sid_pow5_off_h[SID_POW5_MAX + 2] = SID_POW5_OFF_INIT;
static const uint64_t sid_pow5_limb_h[SID_POW5_NLIMBS] = SID_POW5_LIMB_INIT;

#define SID_FMT_MAX 16   // longest output: "-4.94066e-324" (13 bytes)

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

// Six significant digits of v > 0 (finite): D in [100000, 999999], decimal
// exponent X of the leading digit, rounded half-to-even.  false if v is out of
// the supported range (v >= 2^63).
__host__ __device__ inline bool sid_dec6(double v, uint32_t& D, int& X)
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

// "%g" of v (precision 6) into p (>= SID_FMT_MAX bytes); returns the length,
// or -1 if v is outside the supported range (|v| >= 2^63, never a confidence).
__host__ __device__ inline int sid_fmt_g6(double v, char* p)
{
    const uint64_t bits = __builtin_bit_cast(uint64_t, v);
    const uint64_t mag = bits & 0x7fffffffffffffffull;
    int n = 0;
    if (bits >> 63) p[n++] = '-';
    if (mag > 0x7ff0000000000000ull) {
        p[n++] = 'n';
        p[n++] = 'a';
        p[n++] = 'n';
        return n;
    }
    if (mag == 0x7ff0000000000000ull) {
        p[n++] = 'i';
        p[n++] = 'n';
        p[n++] = 'f';
        return n;
    }
    if (mag == 0) {
        p[n++] = '0';
        return n;
    }
    if (mag == 0x3ff0000000000000ull) {   // 1: the most frequent confidence
        p[n++] = '1';
        return n;
    }
    uint32_t D;
    int X;
    if (!sid_dec6(__builtin_bit_cast(double, mag), D, X)) return -1;
    char d[6];
    for (int i = 5; i >= 0; --i) {
        d[i] = (char)('0' + D % 10u);
        D /= 10u;
    }
    int nd = 6;
    while (nd > 1 && d[nd - 1] == '0') --nd;
    if (X < -4 || X >= 6) {
        p[n++] = d[0];
        if (nd > 1) {
            p[n++] = '.';
            for (int i = 1; i < nd; ++i) p[n++] = d[i];
        }
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
        for (int i = 0; i <= X; ++i) p[n++] = d[i];
        if (nd > X + 1) {
            p[n++] = '.';
            for (int i = X + 1; i < nd; ++i) p[n++] = d[i];
        }
    } else {
        p[n++] = '0';
        p[n++] = '.';
        for (int i = 0; i < -X - 1; ++i) p[n++] = '0';
        for (int i = 0; i < nd; ++i) p[n++] = d[i];
    }
    return n;
}

// decimal of an int32 (std::to_chars / operator<<(int)); returns the length
__host__ __device__ inline int sid_fmt_i32(int32_t v, char* p)
{
    int n = 0;
    uint32_t u = (uint32_t)v;
    if (v < 0) {
        p[n++] = '-';
        u = 0u - u;
    }
    char t[10];
    int m = 0;
    do {
        t[m++] = (char)('0' + u % 10u);
        u /= 10u;
    } while (u);
    while (m) p[n++] = t[--m];
    return n;
}
