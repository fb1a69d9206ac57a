// local_site.h — the -m local per-site arithmetic (SURVEY.md §8 rows a5-a8,
// call.cpp:238-273) as device functions, shared by the call kernels
// (local.hip) and the engine's fused -m local formatter (textpath.hip): the
// fast log-domain path, the emulated long-double path, and the class tables
// keyed by (nf, ns, r2) that memoise them per option set.
#pragma once

#include "sid_internal.h"

namespace {

// call.cpp:238-273 for one site; returns the code byte.
__device__ __noinline__ uint32_t local_site_general(uint64_t w, const sid_local_k& K, double& p1,
                                                    double& p2)
{
    uint32_t f, s, nf, ns, cov;
    sid_major(w, f, s, nf, ns, cov);
    const uint32_t r1 = cov - nf, r2 = r1 - ns, m2 = nf + ns;

    sid_ld M;
    M.ln = sid_ln_multinomial(w, cov);
    M.neg = 0;
    M = ld_round(M);

    double e1 = (double)r1 / (double)cov;          // call.cpp:243
    if (e1 > K.E) e1 = K.E;
    sid_ld l1 = ld_mul(ld_mul(M, ld_pow(1 - e1, nf)), ld_pow(e1 / 3., r1));   // lynch.hpp:92-96

    double e2 = 1.5 * (double)r2 / (double)cov;    // call.cpp:250
    if (e2 > K.E) e2 = K.E;
    sid_ld l2 = ld_mul(ld_mul(M, ld_pow((1 - 2. / 3. * e2) / 2., m2)), ld_pow(e2 / 3., r2));

    if (K.prior_on) {                               // call.cpp:256-259
        l1 = ld_mul(l1, ld_from_double(1 - K.prior));
        l2 = ld_mul(l2, ld_from_double(K.prior));
    }
    // near-tie refinement while both are positive normal long doubles
    if (!l1.neg && !l2.neg && l1.ln > SID_LN_LDBL_MIN && l2.ln > SID_LN_LDBL_MIN &&
        l1.ln < SID_LN_LDBL_MAX && l2.ln < SID_LN_LDBL_MAX && fabs(l1.ln - l2.ln) < SID_TIE_BAND &&
        e1 > 0 && e2 >= 0 && !(K.prior_on && K.prior >= 1)) {
        const double d = sid_local_refine_d(nf, ns, r2, K.E, K.prior_on, K.prior);
        l1.ln = l2.ln + d;
    }
    p1 = ld_lrt(l2, l1, K.lg15);
    p2 = ld_lrt(l1, l2, K.lg15);
    const bool het = ld_gt(l2, l1) && p2 < K.sig;   // call.cpp:266
    return f | ((het ? s : f) << 2) | (het ? 0x80u : 0u);
}

// Fast path of call.cpp:238-273 for a site with major counts nf >= ns and
// r2 = coverage - nf - ns other reads.  Depends only on (nf, ns, r2) and the
// options, which is what makes the class table below possible.  Returns
// false when a long double of the reference would leave the normal range
// (then the emulated path must be used).
__host__ __device__ __forceinline__ bool local_fast_p(uint32_t nf, uint32_t ns, uint32_t r2,
                                             const sid_local_k& K, const double* __restrict__ lnt,
                                             double& p1, double& p2, bool& l2_gt_l1)
{
    const uint32_t cov = nf + ns + r2;
    if (cov >= SID_LUTN) return false;
    const uint32_t r1 = cov - nf, m2 = nf + ns;
    // capping decisions on exactly the reference's doubles (call.cpp:243-253)
    const double dc = (double)cov;
    const bool cap1 = (double)r1 / dc > K.E;
    const bool cap2 = 1.5 * (double)r2 / dc > K.E;
    // uncapped bases: 1-e1 = nf/c, e1/3 = r1/(3c), (1-2e2/3)/2 = m2/(2c), e2/3 = r2/(2c)
    const double Lc = lnt[cov];
    const double lA1 = cap1 ? K.cA1 : lnt[nf] - Lc;
    const double lB1 = cap1 ? K.cB1 : lnt[r1] - Lc - SID_LN3;
    const double lA2 = cap2 ? K.cA2 : lnt[m2] - Lc - SID_LN2;
    const double lB2 = cap2 ? K.cB2 : lnt[r2] - Lc - SID_LN2;
    double ln1 = (nf ? (double)nf * lA1 : 0.0) + (r1 ? (double)r1 * lB1 : 0.0);
    double ln2 = (m2 ? (double)m2 * lA2 : 0.0) + (r2 ? (double)r2 * lB2 : 0.0);
    if (K.prior_on) {
        ln1 += K.lp1;
        ln2 += K.lp2;
    }
    const double ninf = -__builtin_inf();
    const bool z1 = ln1 == ninf, z2 = ln2 == ninf;
    // every long double of the reference is a normal number (or an exact 0)?
    if (!((ln1 >= SID_FAST_FLOOR || z1) && (ln2 >= SID_FAST_FLOOR || z2))) return false;
    double d = ln1 - ln2;
    if (!z1 && !z2 && fabs(d) < SID_TIE_BAND) d = sid_local_refine_d(nf, ns, r2, K.E, K.prior_on, K.prior);
    // p1 = LRT(l2, l1), p2 = LRT(l1, l2); at most one chi^2 is non-zero
    const double chi1 = z2 ? 1.7976931348623157e308 : ((!z1 && d > 0.0) ? 2.0 * d : 0.0);
    const double chi2 = z1 ? 1.7976931348623157e308 : ((!z2 && d < 0.0) ? -2.0 * d : 0.0);
    const double chi = fmax(chi1, chi2);
    const double q = sid_chisq_Q(chi, K.lg15);
    p1 = (chi1 == chi) ? q : 1.0;
    p2 = (chi2 == chi) ? q : 1.0;
    l2_gt_l1 = !z2 && (z1 || d < 0.0);
    return true;
}

template <bool GENERAL>
__device__ __forceinline__ uint32_t local_site(uint64_t w, const sid_local_k& K,
                                               const double* __restrict__ lnt, double& p1,
                                               double& p2)
{
    if (GENERAL) return local_site_general(w, K, p1, p2);
    uint32_t f, s, nf, ns, cov;
    sid_major(w, f, s, nf, ns, cov);
    bool gt;
    if (!local_fast_p(nf, ns, cov - nf - ns, K, lnt, p1, p2, gt)) return local_site_general(w, K, p1, p2);
    const bool het = gt && p2 < K.sig;   // call.cpp:266
    return f | ((het ? s : f) << 2) | (het ? 0x80u : 0u);
}


// ------------------------------------------------------ class table ------
// Every fast-path result is a function of (nf, ns, r2) only, so the hot
// kernel reads it from a table built once per option set (the reference's
// per-unique-profile memoisation, call.cpp:217-221, as a dense LDS table):
//   entry (nf < 256, ns < 8, r2 < 4) = one double v
//     v >= +0       p1 = v, p2 = 1            (l2 <= l1)
//     v <= -0       p1 = 1, p2 = -v           (l2 >  l1; het iff p2 < sig)
//     NaN           p1 = p2 = 0               (l1 == l2 == 0)
//     +inf          not tabulated: the fix-up kernel computes the site
// 64 KiB in LDS; sites outside the table (het sites, coverage >= 256 ...)
// are appended to a miss list (one atomic per wave) for the fix-up kernel.
#define SID_TAB_NF 256
#define SID_TAB_NS 8
#define SID_TAB_NR 4
#define SID_TAB_N (SID_TAB_NF * SID_TAB_NS * SID_TAB_NR)

// Second-level table (SID_TAB2_*, sid_internal.h): looked up inline by the
// table kernel for its LDS misses, and by the fix-up.

// LDS slot of (nf, ns, r2): one 256-B bank row per nf (8 ns x 4 r2 entries of
// 8 B), the position in the row XOR-ed with nf.  Linear, every nf's entry of a
// class fell on the same two banks, so a 32-lane half reading the (ns, r2) =
// (0, 0) class at k distinct depths was a k-way conflict (ds_read_b64 banks:
// MI355X_MICROARCH.md §LDS); swizzled, distinct nf mod 32 never collide.
__device__ __forceinline__ uint32_t sid_tab_slot(uint32_t nf, uint32_t ns, uint32_t r2)
{
    return nf * (SID_TAB_NS * SID_TAB_NR) + ((ns * SID_TAB_NR + r2) ^ (nf & (SID_TAB_NS * SID_TAB_NR - 1)));
}

// outputs of a site from its table value v (not +inf); returns the code
__device__ __forceinline__ uint32_t table_decode(double v, uint32_t f, uint32_t s, double sig, double& p1,
                                                 double& p2)
{
    bool het = false;
    if (isnan(v)) {
        p1 = p2 = 0.0;
    } else if (signbit(v)) {
        p1 = 1.0;
        p2 = -v;
        het = p2 < sig;
    } else {
        p1 = v;
        p2 = 1.0;
    }
    return f | ((het ? s : f) << 2) | (het ? 0x80u : 0u);
}

__device__ __forceinline__ uint32_t table_site(uint64_t w, const double* __restrict__ T, double sig,
                                               double& p1, double& p2)
{
    uint32_t f, s, nf, ns, cov;
    sid_major(w, f, s, nf, ns, cov);
    const uint32_t r2 = cov - nf - ns;
    double v = __builtin_inf();
    if (nf < SID_TAB_NF && ns < SID_TAB_NS && r2 < SID_TAB_NR) v = T[sid_tab_slot(nf, ns, r2)];
    if (isinf(v)) {
        p1 = p2 = 0.0;
        return 0xFFu;   // miss marker (not a valid code: bits 4-5 are never set)
    }
    return table_decode(v, f, s, sig, p1, p2);
}

// a site the LDS table missed, through the L2-resident second-level table
// (0xFF: still not covered)
__device__ __forceinline__ uint32_t table2_site(uint64_t w, const double* __restrict__ T2, double sig, double& p1,
                                                double& p2)
{
    uint32_t f, s, nf, ns, cov;
    sid_major(w, f, s, nf, ns, cov);
    const uint32_t r2 = cov - nf - ns;
    double v = __builtin_inf();
    if (nf < SID_TAB2_NF && ns < SID_TAB2_NS && r2 < SID_TAB2_NR) v = T2[(nf * SID_TAB2_NS + ns) * SID_TAB2_NR + r2];
    if (isinf(v)) {
        p1 = p2 = 0.0;
        return 0xFFu;
    }
    return table_decode(v, f, s, sig, p1, p2);
}

// the fix-up of one missed site: the second-level table, else the fast /
// emulated evaluation
__device__ __forceinline__ uint32_t fixup_site(uint64_t w, const double* __restrict__ T2, const sid_local_k& K,
                                               const double* __restrict__ lnt, double& h, double& t)
{
    uint32_t f, s, nf, ns, cov;
    sid_major(w, f, s, nf, ns, cov);
    const uint32_t r2 = cov - nf - ns;
    if (T2 && nf < SID_TAB2_NF && ns < SID_TAB2_NS && r2 < SID_TAB2_NR) {
        const double v = T2[(nf * SID_TAB2_NS + ns) * SID_TAB2_NR + r2];
        if (!isinf(v)) return table_decode(v, f, s, K.sig, h, t);
    }
    return local_site<false>(w, K, lnt, h, t);
}

}  // namespace
