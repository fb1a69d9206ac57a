// sid_math.h — device arithmetic shared by the sid kernels (gfx950).
//
// The reference computes likelihoods in x87 80-bit long double, linear domain
// (lynch.hpp:48-96, call.cpp:247-262); gfx950 has no 80-bit type, so the
// kernels work in the log domain in f64:
//
//   * fast path (every site of the 30x/200x configs): ln l = sum n*ln(base)
//     from an LDS table of ln(k); the multinomial coefficient M cancels in
//     every likelihood ratio, so it is not evaluated.  Valid while every
//     long-double intermediate of the reference stays a normal number; the
//     caller checks the bound and otherwise takes
//   * the emulated path: each long-double value is carried as (ln|v|, sign)
//     and every multiplication is rounded through ld_round(), which applies
//     the x87 format's overflow (-> inf), denormal quantisation (2^-16445
//     steps) and underflow (-> 0), so 0, inf, NaN and the denormal region
//     come out where the reference's long doubles put them.
//
// The chi-square tail (gsl_cdf_chisq_Q(x, 1), stats.cpp:33-35) is
// erfc(sqrt(x/2)) in the normal range; in the denormal range it follows
// GSL 2.7.1's gamma_inc_Q_CF (D * (a/x) * F) so the result rounds like GSL's.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define SID_LUTN 1024               // ln(k) table, k < SID_LUTN  (coverage < 1024 fast path)
#define SID_LN2 0.69314718055994530942
#define SID_LN3 1.09861228866810969140
#define SID_LN_LDBL_MAX 11356.523406294143949      // ln(LDBL_MAX), x87 80-bit
#define SID_LN_LDBL_MIN (-11355.137111933024058)   // ln(LDBL_MIN) = -16382 ln 2
#define SID_LDBL_DENORM_SHIFT 11398.805384308300613 // 16445 ln 2: ln(LDBL_TRUE_MIN) = -shift
#define SID_FAST_FLOOR (-11000.0)                   // fast path while every ln >= this

struct sid_local_k {
    double E;          // site_error_threshold
    double sig;        // significance_level
    double cA1, cB1;   // ln(1-E), ln(E/3.)            capped hom bases
    double cA2, cB2;   // ln((1-2./3.*E)/2.), ln(E/3.) capped het bases
    double lp1, lp2;   // ln|1-prior|, ln(prior)        (prior_on)
    double prior;      // snp_prior
    double lg15;       // GSL lngamma(1.5) (gamma_inc_D)
    int prior_on;      // snp_prior > 0                 call.cpp:256
    int general;       // E < 0 or prior > 1: every site takes the emulated path
};

// Per-(pi, eps) constants of the 10-genotype mixture (lynch.hpp:57-90),
// computed on the host for each objective evaluation.
struct sid_lynch_eval {
    double la;        // ln(1 - e)
    double lb;        // ln(e / 3.)
    double lh;        // ln((1 - 2./3. * e) / 2.)
    double ld[4];     // ln d_i
    double ldd[6];    // ln(d_i * d_j), i < j (double product, lynch.hpp:65)
    double lnorm;     // -ln(1 - sum d_i^2)          (lynch.hpp:70-72)
    double l1p, lp;   // ln(1 - pi), ln(pi)
};

// Up to SID_OBJ_PTS (pi, eps) points per objective launch: Nelder-Mead's
// candidate points of one iteration (and of the next one, lynch_host.cpp) are
// evaluated together.  The dist-only constants are shared; per point only the
// eps- and pi-dependent logs differ (kernel arguments stay small).
#define SID_OBJ_PTS 32
struct sid_lynch_pt {
    double la, lb, lh, l1p, lp;
};
struct sid_lynch_evals {
    double ld[4];
    double ldd[6];
    double lnorm;
    sid_lynch_pt p[SID_OBJ_PTS];
};

// x86 prints NaNs made by invalid operations as "-nan" (default NaN has the
// sign bit set); give every NaN the same sign.
__device__ __forceinline__ double sid_x86_nan(double v) { return isnan(v) ? -__builtin_nan("") : v; }

// ---------------------------------------------------------------- chi^2_1 --
// GSL 2.7.1 gamma_inc_F_CF (modified Lentz), a = 0.5.
__host__ __device__ __forceinline__ double sid_gamma_F_CF(double x)
{
    const double eps = 2.2204460492503131e-16;
    const double small = eps * eps * eps;
    double hn = 1.0, Cn = 1.0 / small, Dn = 1.0;
    for (int n = 2; n < 5000; n++) {
        double an = (n & 1) ? 0.5 * (n - 1) / x : (0.5 * n - 0.5) / x;
        Dn = 1.0 + an * Dn;
        if (fabs(Dn) < small) Dn = small;
        Cn = 1.0 + an / Cn;
        if (fabs(Cn) < small) Cn = small;
        Dn = 1.0 / Dn;
        double delta = Cn * Dn;
        hn *= delta;
        if (fabs(delta - 1.0) < eps) break;
    }
    return hn;
}

// gsl_cdf_chisq_Q(x, 1) (cdf/chisq.c -> cdf/gamma.c gsl_cdf_gamma_Q(x, 0.5, 2))
static __host__ __device__ __noinline__ double sid_chisq_Q_tail(double y, double lg15)
{
    if (__builtin_isinf(y)) return -__builtin_nan("");   // D = exp(inf - inf): default NaN
    if (y > 1.0e6) return 0.0;                          // gamma_inc_Q_large_x: D == 0
    double D = exp(0.5 * log(y) - y - lg15);            // gamma_inc_D, a < 10
    return D * (0.5 / y) * sid_gamma_F_CF(y);
}

__host__ __device__ __forceinline__ double sid_chisq_Q(double x, double lg15)
{
    if (!(x > 0.0)) return (x <= 0.0) ? 1.0 : x;        // x <= 0 -> 1; NaN -> NaN
    double y = x / 2.0;
    if (y <= 700.0) return erfc(sqrt(y));               // Q(1/2, y) = erfc(sqrt(y)), normal range
    return sid_chisq_Q_tail(y, lg15);
}

// ------------------------------------------------------- double-double --
// Near-ties l1 ~ l2 put p = Q(chi^2) on its sqrt(chi^2) branch near 1, where
// a 1e-14 error in ln l becomes a 1e-7 error in p.  There the kernels
// recompute ln l1 - ln l2 from the reference's own double bases with ~1e-30
// accuracy (QD-style double-double exp/log), so exact ties of the reference
// come out as exact ties and near-ties agree to ~1e-16.
struct sid_dd {
    double hi, lo;
};

__host__ __device__ __forceinline__ sid_dd dd_two_sum(double a, double b)
{
    double s = a + b;
    double bb = s - a;
    sid_dd r;
    r.hi = s;
    r.lo = (a - (s - bb)) + (b - bb);
    return r;
}

__host__ __device__ __forceinline__ sid_dd dd_norm(double hi, double lo)
{
    double s = hi + lo;
    sid_dd r;
    r.hi = s;
    r.lo = lo - (s - hi);
    return r;
}

__host__ __device__ __forceinline__ sid_dd dd_add(sid_dd a, sid_dd b)
{
    sid_dd s = dd_two_sum(a.hi, b.hi);
    sid_dd t = dd_two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = dd_norm(s.hi, s.lo);
    s.lo += t.lo;
    return dd_norm(s.hi, s.lo);
}

__host__ __device__ __forceinline__ sid_dd dd_neg(sid_dd a)
{
    a.hi = -a.hi;
    a.lo = -a.lo;
    return a;
}

__host__ __device__ __forceinline__ sid_dd dd_mul(sid_dd a, sid_dd b)
{
    double p = a.hi * b.hi;
    double e = fma(a.hi, b.hi, -p);
    e += a.hi * b.lo + a.lo * b.hi;
    return dd_norm(p, e);
}

__host__ __device__ __forceinline__ sid_dd dd_mul_d(sid_dd a, double b)
{
    double p = a.hi * b;
    double e = fma(a.hi, b, -p);
    e += a.lo * b;
    return dd_norm(p, e);
}

__host__ __device__ __forceinline__ sid_dd dd_div_d(sid_dd a, double b)
{
    const double q1 = a.hi / b;
    const double r = fma(-q1, b, a.hi) + a.lo;   // exact remainder of the hi part
    return dd_norm(q1, r / b);
}

__host__ __device__ __forceinline__ sid_dd dd_ldexp(sid_dd a, int k)
{
    a.hi = ldexp(a.hi, k);
    a.lo = ldexp(a.lo, k);
    return a;
}

// exp of a double-double, |x| < 700
static __host__ __device__ __noinline__ sid_dd dd_exp(sid_dd x)
{
    const sid_dd ln2 = {0.6931471805599452862, 2.319046813846299558e-17};
    const double k = rint(x.hi / ln2.hi);
    sid_dd r = dd_add(x, dd_neg(dd_mul_d(ln2, k)));
    r = dd_ldexp(r, -10);                       // |r| < 3.4e-4
    // e^r - 1 by Taylor to r^9 (error < 1e-36)
    sid_dd term = r, em1 = r;
    for (int i = 2; i <= 9; ++i) {
        term = dd_div_d(dd_mul(term, r), (double)i);
        em1 = dd_add(em1, term);
    }
    // (1 + em1)^(2^10): em1 <- 2 em1 + em1^2
    for (int i = 0; i < 10; ++i) em1 = dd_add(dd_mul_d(em1, 2.0), dd_mul(em1, em1));
    sid_dd one = {1.0, 0.0};
    return dd_ldexp(dd_add(one, em1), (int)k);
}

// ln(b) for a finite double b > 0 (denormals included), as a double-double:
// b = m 2^e, m in [0.5, 1); ln m by one Newton step on a double-double exp.
static __host__ __device__ __noinline__ sid_dd dd_log(double b)
{
    int e;
    const double m = frexp(b, &e);
    const double y = log(m);
    sid_dd E = dd_exp(sid_dd{-y, 0.0});        // ~ 1/m
    sid_dd t = dd_mul_d(E, m);                  // ~ 1
    t = dd_add(t, sid_dd{-1.0, 0.0});           // tiny
    sid_dd t2 = dd_mul(t, t);
    t = dd_add(t, sid_dd{-0.5 * t2.hi, -0.5 * t2.lo});
    const sid_dd ln2 = {0.6931471805599452862, 2.319046813846299558e-17};
    return dd_add(dd_add(sid_dd{y, 0.0}, t), dd_mul_d(ln2, (double)e));
}

// n * ln(b) with powl(b, 0) == 1
__host__ __device__ __forceinline__ sid_dd dd_nlog(double b, uint32_t n)
{
    if (n == 0) return sid_dd{0.0, 0.0};
    return dd_mul_d(dd_log(b), (double)n);
}

// ---------------------------------------------------- near-tie refinement --
// ln l1 - ln l2 of call.cpp:238-262 from the reference's double bases,
// double-double accurate.  Only called when both likelihoods are non-zero.
static __host__ __device__ __noinline__ double sid_local_refine_d(uint32_t nf, uint32_t ns, uint32_t r2, double E,
                                                  int prior_on, double prior)
{
    const uint32_t cov = nf + ns + r2, r1 = cov - nf, m2 = nf + ns;
    double e1 = (double)r1 / (double)cov;
    if (e1 > E) e1 = E;
    double e2 = 1.5 * (double)r2 / (double)cov;
    if (e2 > E) e2 = E;
    sid_dd l1 = dd_add(dd_nlog(1 - e1, nf), dd_nlog(e1 / 3., r1));
    sid_dd l2 = dd_add(dd_nlog((1 - 2. / 3. * e2) / 2., m2), dd_nlog(e2 / 3., r2));
    if (prior_on) {
        l1 = dd_add(l1, dd_log(1 - prior));
        l2 = dd_add(l2, dd_log(prior));
    }
    sid_dd d = dd_add(l1, dd_neg(l2));
    // below the resolution of any evaluation of the reference: an exact tie
    if (fabs(d.hi) <= 1e-28 * (fabs(l1.hi) + fabs(l2.hi))) return 0.0;
    return d.hi + d.lo;
}
#define SID_TIE_BAND 5e-7   // |ln l1 - ln l2| below this is refined

// ------------------------------------------------------ major alleles a5 --
// call.cpp:52-60: stable ascending sort of {0,1,2,3} by count -> first =
// idx[3], second = idx[2].  Equivalent key 4*count+idx (ties -> higher index).
__host__ __device__ __forceinline__ void sid_major(uint64_t w, uint32_t& f, uint32_t& s, uint32_t& nf,
                                          uint32_t& ns, uint32_t& cov)
{
    uint32_t n0 = (uint32_t)(w & 0xffffu), n1 = (uint32_t)((w >> 16) & 0xffffu);
    uint32_t n2 = (uint32_t)((w >> 32) & 0xffffu), n3 = (uint32_t)(w >> 48);
    uint32_t k0 = n0 << 2, k1 = (n1 << 2) | 1u, k2 = (n2 << 2) | 2u, k3 = (n3 << 2) | 3u;
    uint32_t a = max(k0, k1), b = min(k0, k1), c = max(k2, k3), d = min(k2, k3);
    uint32_t kf = max(a, c);
    uint32_t ks = max(min(a, c), max(b, d));
    f = kf & 3u;
    s = ks & 3u;
    nf = kf >> 2;
    ns = ks >> 2;
    cov = n0 + n1 + n2 + n3;
}

// ------------------------------------------- dense profile code (Lynch) --
// A bijection between the "typical" profiles and 14-bit codes, so that the
// histogram (countUniqueProfiles, pileup.cpp:169-196) and the per-site class
// lookup (call.cpp:129-140) index a 16384-entry LDS array instead of hashing.
// m = max count, f = FIRST index holding it, o0..o2 = the other three counts
// in index order.  Typical iff m < 64 and every o <= 3: at 30x that is every
// homozygous site with at most 3 reads of each other base (~99.9% of sites).
// code = f<<12 | m<<6 | o0<<4 | o1<<2 | o2; decode() inverts it exactly.
// profile hash keys (the Lynch histogram and class hash)
#define SID_EMPTY_KEY 0xFFFFFFFFFFFFFFFFull
__device__ __forceinline__ uint64_t sid_hash64(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    k ^= k >> 33;
    return k;
}

// profile_t (A,C,G,T little-endian u16) -> key with lexicographic numeric order
__device__ __forceinline__ uint64_t sid_profile_key(uint64_t w)
{
    return ((w & 0xffffull) << 48) | (((w >> 16) & 0xffffull) << 32) | (((w >> 32) & 0xffffull) << 16) |
           (w >> 48);
}

#define SID_DENSE_N 16384u
#define SID_DENSE_NONE 0xFFFFFFFFu
#define SID_DENSE_ROWS 16   // u64 rows the per-block dense counters are folded into

__host__ __device__ __forceinline__ uint32_t sid_dense_code(uint64_t w)
{
    const uint32_t n0 = (uint32_t)(w & 0xffffu), n1 = (uint32_t)((w >> 16) & 0xffffu);
    const uint32_t n2 = (uint32_t)((w >> 32) & 0xffffu), n3 = (uint32_t)(w >> 48);
    const uint32_t m = max(max(n0, n1), max(n2, n3));
    const uint32_t f = n0 == m ? 0u : n1 == m ? 1u : n2 == m ? 2u : 3u;
    const uint32_t o0 = f == 0 ? n1 : n0, o1 = f <= 1 ? n2 : n1, o2 = f <= 2 ? n3 : n2;
    if (m >= 64u || (o0 | o1 | o2) >= 4u) return SID_DENSE_NONE;
    return (f << 12) | (m << 6) | (o0 << 4) | (o1 << 2) | o2;
}

// LDS slot of a dense code: the low 6 bits XOR-ed with m and f, so that the
// common codes (o = 0, code = f<<12 | m<<6: all in one bank unswizzled) spread
// over the LDS banks.  A bijection on [0, SID_DENSE_N).
__host__ __device__ __forceinline__ uint32_t sid_dense_slot(uint32_t d)
{
    return d ^ (((d >> 6) ^ (d >> 11)) & 63u);
}

// Record code: the dense codes whose three minor counts are all <= 1 (at 30x
// ~98% of sites), 11 bits: f<<9 | m<<3 | o0<<2 | o1<<1 | o2.  The per-site
// lookup keeps one class record (code, p1, p2) per record code in LDS.
#define SID_REC_N 2048u
__host__ __device__ __forceinline__ uint32_t sid_rec_code(uint32_t d)
{
    const uint32_t o = d & 63u;
    if (d == SID_DENSE_NONE || (o & 0x2Au)) return SID_DENSE_NONE;
    return ((d >> 6) << 3) | ((o >> 2) & 4u) | ((o >> 1) & 2u) | (o & 1u);
}
__host__ __device__ __forceinline__ uint32_t sid_rec_dense(uint32_t r)
{
    return ((r >> 3) << 6) | (((r >> 2) & 1u) << 4) | (((r >> 1) & 1u) << 2) | (r & 1u);
}

// profile word (A,C,G,T little-endian u16) of a dense code
__host__ __device__ __forceinline__ uint64_t sid_dense_word(uint32_t code)
{
    const uint32_t f = code >> 12, m = (code >> 6) & 63u;
    const uint32_t o[3] = {(code >> 4) & 3u, (code >> 2) & 3u, code & 3u};
    uint64_t w = 0;
    for (uint32_t i = 0, k = 0; i < 4; ++i) w |= (uint64_t)(i == f ? m : o[k++]) << (16 * i);
    return w;
}

// ------------------------------------------ emulated x87 long double ------
struct sid_ld {
    double ln;   // ln|v|: -inf = 0, +inf = inf, NaN = NaN
    int neg;
};

__device__ __forceinline__ sid_ld ld_round(sid_ld v)
{
    if (v.ln > SID_LN_LDBL_MAX) {
        v.ln = __builtin_inf();
    } else if (v.ln < SID_LN_LDBL_MIN && v.ln != -__builtin_inf()) {
        double q = rint(exp(v.ln + SID_LDBL_DENORM_SHIFT));   // multiples of LDBL_TRUE_MIN
        v.ln = (q == 0.0) ? -__builtin_inf() : log(q) - SID_LDBL_DENORM_SHIFT;
    }
    return v;
}

__device__ __forceinline__ sid_ld ld_mul(sid_ld a, sid_ld b)
{
    sid_ld r;
    r.ln = a.ln + b.ln;   // 0 * inf -> (-inf) + inf = NaN, as in IEEE
    r.neg = a.neg ^ b.neg;
    return ld_round(r);
}

__device__ __forceinline__ sid_ld ld_from_double(double x)
{
    sid_ld r;
    r.ln = (x == 0.0) ? -__builtin_inf() : log(fabs(x));
    r.neg = x < 0.0;
    return r;
}

// powl(b, n) for an integer exponent n >= 0
__device__ __forceinline__ sid_ld ld_pow(double b, uint32_t n)
{
    sid_ld r;
    if (n == 0) {
        r.ln = 0.0;   // powl(x, 0) == 1 for every x, NaN included
        r.neg = 0;
        return r;
    }
    r.ln = (b == 0.0) ? -__builtin_inf() : (double)n * log(fabs(b));
    r.neg = (b < 0.0) && (n & 1u);
    return ld_round(r);
}

__device__ __forceinline__ bool ld_is_zero(sid_ld a) { return a.ln == -__builtin_inf(); }

// a > b on the represented long doubles (false if either is NaN)
__device__ __forceinline__ bool ld_gt(sid_ld a, sid_ld b)
{
    if (isnan(a.ln) || isnan(b.ln)) return false;
    int sa = ld_is_zero(a) ? 0 : (a.neg ? -1 : 1);
    int sb = ld_is_zero(b) ? 0 : (b.neg ? -1 : 1);
    if (sa != sb) return sa > sb;
    if (sa > 0) return a.ln > b.ln;
    if (sa < 0) return a.ln < b.ln;
    return false;
}

// stats.cpp:29-37 likelihoodRatioTest(l_H0, l_H1) on emulated long doubles.
// NaN signs follow the x86-64 reference build: glibc logl() of a negative
// number returns +NaN; an invalid x87/SSE operation (0*inf, inf-inf) gives
// the default NaN, which has the sign bit set; NaN operands propagate.
__device__ __noinline__ double ld_lrt(sid_ld l0, sid_ld l1, double lg15)
{
    if (ld_is_zero(l0)) return 0.0;                           // gsl_cdf_chisq_Q(DBL_MAX, 1)
    if (isnan(l0.ln)) return -__builtin_nan("");              // l0 came from 0*inf
    if (l0.neg) return __builtin_nan("");                     // logl(negative)
    bool take1 = !isnan(l1.ln) && ld_gt(l1, l0);              // fmaxl(l0, l1)
    double mx = take1 ? l1.ln : l0.ln;
    double chisq = -2.0 * (l0.ln - mx);
    if (isnan(chisq)) return -__builtin_nan("");              // inf - inf
    return sid_chisq_Q(chisq, lg15);
}

// multinomialCoefficient, lynch.hpp:48-55: expl of the double lnGamma sum
__device__ __forceinline__ double sid_ln_multinomial(uint64_t w, uint32_t cov)
{
    double v = lgamma((double)cov + 1.0);
    v -= lgamma((double)(w & 0xffffu) + 1.0);
    v -= lgamma((double)((w >> 16) & 0xffffu) + 1.0);
    v -= lgamma((double)((w >> 32) & 0xffffu) + 1.0);
    v -= lgamma((double)(w >> 48) + 1.0);
    return v;
}
