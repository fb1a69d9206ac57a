/*
 * sid_oracle.c — CPU ORACLE for the sid hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * this file (through oracle/_build/liboracle.so or the sid_oracle CLI).  The
 * product never links or calls it.  See sid_oracle.h for what is pinned and
 * what is "parity unpinned".
 *
 * Every function cites the reference file:line it restates
 * (paths relative to EvolBioInf/sid @ v0).
 */
#define _GNU_SOURCE
#include "sid_oracle.h"

#include <ctype.h>
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Parser: pileup.cpp                                                        */
/* ------------------------------------------------------------------------ */

static const char* FIELD_SEPARATORS = " \t"; /* pileup.cpp:11 */

/* pileup.cpp:70-153 parseReadBases (counts only).  The quadratic strlen() in
 * the loop condition (pileup.cpp:76) is kept on purpose so the oracle's cost
 * structure resembles the reference when it is timed as the CPU baseline. */
void oracle_read_bases(const char* read_bases, char reference, uint16_t counts[4])
{
    counts[0] = counts[1] = counts[2] = counts[3] = 0;
    for (size_t i = 0; i < strlen(read_bases); ++i) {
        char base = read_bases[i];
        if (base == '.') {
            base = (char)toupper(reference);
        } else if (base == ',') {
            base = (char)tolower(reference);
        }
        switch (base) {
        case 'a': case 'A': ++counts[0]; break;
        case 'c': case 'C': ++counts[1]; break;
        case 'g': case 'G': ++counts[2]; break;
        case 't': case 'T': ++counts[3]; break;
        case '^': ++i; break; /* skip next char, pileup.cpp:125-127 */
        case '+':
        case '-': {           /* pileup.cpp:128-147 */
            if (!isdigit((unsigned char)read_bases[i + 1])) {
                break;
            }
            char* first_after_number;
            unsigned long length = (unsigned long)strtol(read_bases + i + 1, &first_after_number, 10);
            if (SIZE_MAX - length < i) {
                i = SIZE_MAX;
            } else {
                i = (size_t)(first_after_number - read_bases) + length - 1;
            }
            break;
        }
        default: break;
        }
    }
}

/* pileup.cpp:70-153: the bases vector -- upper-case A/C/G/T in read order,
 * the same walk as oracle_read_bases.  Returns the count; writes up to cap. */
int oracle_read_bases_seq(const char* read_bases, char reference, char* out, int cap)
{
    int n = 0;
    for (size_t i = 0; i < strlen(read_bases); ++i) {
        char base = read_bases[i];
        if (base == '.') {
            base = (char)toupper(reference);
        } else if (base == ',') {
            base = (char)tolower(reference);
        }
        char b = 0;
        switch (base) {
        case 'a': case 'A': b = 'A'; break;
        case 'c': case 'C': b = 'C'; break;
        case 'g': case 'G': b = 'G'; break;
        case 't': case 'T': b = 'T'; break;
        case '^': ++i; break;
        case '+':
        case '-': {
            if (!isdigit((unsigned char)read_bases[i + 1])) break;
            char* first_after_number;
            unsigned long length = (unsigned long)strtol(read_bases + i + 1, &first_after_number, 10);
            if (SIZE_MAX - length < i) i = SIZE_MAX;
            else i = (size_t)(first_after_number - read_bases) + length - 1;
            break;
        }
        default: break;
        }
        if (b) {
            if (out && n < cap) out[n] = b;
            ++n;
        }
    }
    return n;
}

/* pileup.cpp:155-167 parseQualities */
int oracle_parse_qualities(const char* q, uint8_t* out, int cap)
{
    int n = 0;
    for (const char* c = q; *c != '\0' && *c != '\t' && *c != '\n'; ++c) {
        uint8_t quality = (uint8_t)(*c - 33);
        if (quality < 1) quality = 1;
        if (out && n < cap) out[n] = quality;
        ++n;
    }
    return n;
}

/* pileup.cpp:13-68 parsePileupLine */
int oracle_parse_line(char* line, int parse_bq, int parse_mq, oracle_line* out)
{
    char* saveptr = NULL;
    memset(out, 0, sizeof(*out));
    out->position = -1;
    out->reference = 'N';

    char* chromosome_name = strtok_r(line, FIELD_SEPARATORS, &saveptr);
    if (chromosome_name == NULL) {
        return ORACLE_ENULLCHROM; /* std::string(nullptr) throws logic_error */
    }
    out->chrom = chromosome_name;

    char* position = strtok_r(NULL, FIELD_SEPARATORS, &saveptr);
    if (position == NULL) return ORACLE_EMALFORMED;
    out->position = atoi(position);

    char* reference = strtok_r(NULL, FIELD_SEPARATORS, &saveptr);
    if (reference == NULL || strlen(reference) != 1) return ORACLE_EMALFORMED;
    out->reference = reference[0];

    char* coverage_str = strtok_r(NULL, FIELD_SEPARATORS, &saveptr);
    if (coverage_str == NULL) return ORACLE_EMALFORMED;
    out->coverage = atoi(coverage_str);

    char* read_bases = strtok_r(NULL, FIELD_SEPARATORS, &saveptr);
    if (read_bases == NULL) return ORACLE_EMALFORMED;
    oracle_read_bases(read_bases, out->reference, out->counts);

    char* base_qualities = strtok_r(NULL, FIELD_SEPARATORS, &saveptr);
    out->read_bases = read_bases;
    if (parse_bq) {
        /* pileup.cpp:51-54 checks read_bases (never NULL here) and then
         * parseQualities dereferences base_qualities: SIGSEGV when it is NULL. */
        if (base_qualities == NULL) return ORACLE_ENOBQ;
        out->base_qualities = base_qualities;
        out->n_bq = oracle_parse_qualities(base_qualities, NULL, 0);
    }
    if (parse_mq) {
        char* mapping_qualities = strtok_r(NULL, FIELD_SEPARATORS, &saveptr);
        if (mapping_qualities == NULL) return ORACLE_EMISSING_MQ;
        out->mapping_qualities = mapping_qualities;
        out->n_mq = oracle_parse_qualities(mapping_qualities, NULL, 0);
    }
    return ORACLE_OK;
}

/* ------------------------------------------------------------------------ */
/* call.cpp:52-60 getMajorAlleleIndices: std::sort of 4 indices by count.   */
/* libstdc++ sorts 4 elements with its (stable) insertion sort, so ties keep */
/* index order and the last of the tied maxima (highest base index) wins.   */
/* ------------------------------------------------------------------------ */
void oracle_major(const uint16_t p[4], int* first, int* second)
{
    int idx[4] = {0, 1, 2, 3};
    for (int i = 1; i < 4; ++i) {
        int v = idx[i];
        int j = i;
        while (j > 0 && p[v] < p[idx[j - 1]]) {
            idx[j] = idx[j - 1];
            --j;
        }
        idx[j] = v;
    }
    *first = idx[3];
    *second = idx[2];
}

/* ------------------------------------------------------------------------ */
/* GSL 2.7.1 restatements (not vendored in the reference; see header).       */
/* ------------------------------------------------------------------------ */
#define GSL_DBL_EPSILON 2.2204460492503131e-16
#define LogRootTwoPi_ 0.9189385332046727418
#define LANCZOS_7_G 7.0

/* specfunc/gamma.c lanczos_7_c / lngamma_lanczos */
static const double lanczos_7_c[9] = {
    0.99999999999980993227684700473478,   676.520368121885098567009190444019,
    -1259.13921672240287047156078755283,  771.3234287776530788486528258894,
    -176.61502916214059906584551354,      12.507343278686904814458936853,
    -0.13857109526572011689554707,        9.984369578019570859563e-6,
    1.50563273514931155834e-7};

static double lngamma_lanczos(double x)
{
    x -= 1.0; /* Lanczos writes z! instead of Gamma(z) */
    double Ag = lanczos_7_c[0];
    for (int k = 1; k <= 8; k++) Ag += lanczos_7_c[k] / (x + k);
    double term1 = (x + 0.5) * log((x + LANCZOS_7_G + 0.5) / M_E);
    double term2 = LogRootTwoPi_ + log(Ag);
    return term1 + (term2 - LANCZOS_7_G);
}

/* specfunc/gamma.c gsl_sf_lngamma_e.  On this path x is a positive integer
 * (lynch.hpp:48-55) or 1.5 (gamma_inc_D).  The Pade branches around 1 and 2
 * evaluate to exactly 0 at x = 1 and x = 2; other arguments in those bands
 * and x < 0.5 do not occur on the path and fall back to libm lgamma. */
double oracle_gsl_lngamma(double x)
{
    if (fabs(x - 1.0) < 0.01) return x == 1.0 ? 0.0 : lgamma(x);
    if (fabs(x - 2.0) < 0.01) return x == 2.0 ? 0.0 : lgamma(x);
    if (x >= 0.5) return lngamma_lanczos(x);
    return lgamma(x);
}

/* lynch.hpp:11-31 MemoizedLogGamma::operator()(int) (cache is transparent) */
double oracle_log_gamma(int x)
{
    if (x < 0) return oracle_gsl_lngamma(x);
    if (x == 0) return 0;
    return oracle_gsl_lngamma(x);
}

/* specfunc/gamma_inc.c gamma_inc_D, a < 10 branch */
static double gamma_inc_D(double a, double x)
{
    double lg = oracle_gsl_lngamma(a + 1.0);
    double lnr = a * log(x) - x - lg;
    return exp(lnr);
}

/* specfunc/gamma_inc.c gamma_inc_P_series */
static double gamma_inc_P_series(double a, double x)
{
    const int nmax = 10000;
    double D = gamma_inc_D(a, x);
    double sum = 1.0, term = 1.0;
    int n;
    int nlow = (x > a) ? (int)(x - a) : 0;
    for (n = 1; n < nlow; n++) {
        term *= x / (a + n);
        sum += term;
    }
    for (; n < nmax; n++) {
        term *= x / (a + n);
        sum += term;
        if (fabs(term / sum) < GSL_DBL_EPSILON) break;
    }
    return D * sum;
}

/* specfunc/gamma_inc.c gamma_inc_F_CF (modified Lentz) */
static double gamma_inc_F_CF(double a, double x)
{
    const int nmax = 5000;
    const double small = GSL_DBL_EPSILON * GSL_DBL_EPSILON * GSL_DBL_EPSILON;
    double hn = 1.0;
    double Cn = 1.0 / small;
    double Dn = 1.0;
    for (int n = 2; n < nmax; n++) {
        double an;
        if (n & 1)
            an = 0.5 * (n - 1) / x;
        else
            an = (0.5 * n - a) / x;
        Dn = 1.0 + an * Dn;
        if (fabs(Dn) < small) Dn = small;
        Cn = 1.0 + an / Cn;
        if (fabs(Cn) < small) Cn = small;
        Dn = 1.0 / Dn;
        double delta = Cn * Dn;
        hn *= delta;
        if (fabs(delta - 1.0) < GSL_DBL_EPSILON) break;
    }
    return hn;
}

/* specfunc/gamma_inc.c gamma_inc_Q_CF */
static double gamma_inc_Q_CF(double a, double x)
{
    double D = gamma_inc_D(a, x);
    double F = gamma_inc_F_CF(a, x);
    return D * (a / x) * F;
}

/* specfunc/gamma_inc.c gamma_inc_Q_large_x */
static double gamma_inc_Q_large_x(double a, double x)
{
    const int nmax = 5000;
    double D = gamma_inc_D(a, x);
    double sum = 1.0, term = 1.0, last = 1.0;
    for (int n = 1; n < nmax; n++) {
        term *= (a - n) / x;
        if (fabs(term / last) > 1.0) break;
        if (fabs(term / sum) < GSL_DBL_EPSILON) break;
        sum += term;
        last = term;
    }
    return D * (a / x) * sum;
}

/* specfunc/gamma_inc.c gsl_sf_gamma_inc_P_e (branches reachable for a = 0.5) */
static double gamma_inc_P(double a, double x)
{
    if (x == 0.0) return 0.0;
    if (x < 20.0 || x < 0.5 * a) return gamma_inc_P_series(a, x);
    if (a <= x) {
        double Q = (a > 0.2 * x) ? gamma_inc_Q_CF(a, x) : gamma_inc_Q_large_x(a, x);
        return 1.0 - Q;
    }
    if ((x - a) * (x - a) < a) return 1.0 - gamma_inc_Q_CF(a, x);
    return gamma_inc_P_series(a, x);
}

/* specfunc/gamma_inc.c gsl_sf_gamma_inc_Q_e (branches reachable for a = 0.5) */
static double gamma_inc_Q(double a, double x)
{
    if (x == 0.0) return 1.0;
    if (x <= 0.5 * a) return 1.0 - gamma_inc_P_series(a, x);
    if (a < 0.2 && x < 5.0) return 1.0 - gamma_inc_P_series(a, x); /* not reached, a = 0.5 */
    if (a <= x) {
        if (x <= 1.0e+06) return gamma_inc_Q_CF(a, x);
        return gamma_inc_Q_large_x(a, x);
    }
    if (x > a - sqrt(a)) return gamma_inc_Q_CF(a, x);
    return 1.0 - gamma_inc_P_series(a, x);
}

/* cdf/chisq.c gsl_cdf_chisq_Q(x, 1) = cdf/gamma.c gsl_cdf_gamma_Q(x, 0.5, 2) */
double oracle_gsl_chisq_Q(double x)
{
    const double a = 0.5, b = 2.0;
    double y = x / b;
    if (x <= 0.0) return 1.0;
    if (y < a) return 1 - gamma_inc_P(a, y);
    return gamma_inc_Q(a, y);
}

/* ------------------------------------------------------------------------ */
/* stats.cpp:29-37 likelihoodRatioTest                                       */
/* ------------------------------------------------------------------------ */
double oracle_lrt(long double l_H0, long double l_H1)
{
    if (l_H0 != 0) {
        long double chisq = -2 * (logl(l_H0) - logl(fmaxl(l_H0, l_H1)));
        return oracle_gsl_chisq_Q((double)chisq);
    }
    return oracle_gsl_chisq_Q(DBL_MAX);
}

/* ------------------------------------------------------------------------ */
/* lynch.hpp likelihoods                                                     */
/* ------------------------------------------------------------------------ */
static uint32_t coverage_of(const uint16_t p[4])
{
    /* std::accumulate(profile, 0) -> int, stored as uint32 (pileup.hpp:38) */
    return (uint32_t)((int)p[0] + (int)p[1] + (int)p[2] + (int)p[3]);
}

/* lynch.hpp:48-55 */
static long double multinomial_coefficient(const uint16_t p[4], uint32_t coverage)
{
    return expl(oracle_log_gamma((int)(coverage + 1)) - oracle_log_gamma(p[0] + 1) -
                oracle_log_gamma(p[1] + 1) - oracle_log_gamma(p[2] + 1) -
                oracle_log_gamma(p[3] + 1));
}

/* lynch.hpp:92-96 */
static long double hom_lik_ref(const uint16_t p[4], uint32_t cov, double e, int ref)
{
    return multinomial_coefficient(p, cov) * powl(1 - e, p[ref]) *
           powl(e / 3., cov - p[ref]);
}

/* lynch.hpp:76-80 */
static long double het_lik_ref(const uint16_t p[4], uint32_t cov, double e, int r0, int r1)
{
    return multinomial_coefficient(p, cov) * powl((1 - 2. / 3. * e) / 2., p[r0] + p[r1]) *
           powl(e / 3., cov - p[r0] - p[r1]);
}

/* lynch.hpp:82-90 */
long double oracle_hom_lik_dist(const oracle_profile* p, double e, const double d[4])
{
    long double L = 0;
    for (int i = 0; i < 4; ++i) {
        L += d[i] * powl(1 - e, p->profile[i]) * powl(e / 3., p->coverage - p->profile[i]);
    }
    return multinomial_coefficient(p->profile, p->coverage) * L;
}

/* lynch.hpp:57-74 */
long double oracle_het_lik_dist(const oracle_profile* p, double e, const double d[4])
{
    long double L = 0;
    for (int i = 0; i < 4; ++i) {
        for (int j = i + 1; j < 4; ++j) {
            L += d[i] * d[j] * powl((1 - 2. / 3. * e) / 2., p->profile[i] + p->profile[j]) *
                 powl(e / 3., p->coverage - p->profile[i] - p->profile[j]);
        }
    }
    long double s = 0;
    for (int i = 0; i < 4; ++i) s += d[i] * d[i];
    L /= (1 - s);
    return multinomial_coefficient(p->profile, p->coverage) * L;
}

/* ------------------------------------------------------------------------ */
/* call.cpp:238-273: one profile of -m local                                 */
/* ------------------------------------------------------------------------ */
void oracle_local_profile(const uint16_t p[4], double snp_prior, double error_threshold,
                          double significance_level, uint8_t* code, double* hom_conf,
                          double* het_conf)
{
    uint32_t coverage = coverage_of(p);
    int f, s;
    oracle_major(p, &f, &s);

    double error1 = (double)(coverage - p[f]) / (double)coverage;
    if (error1 > error_threshold) error1 = error_threshold;
    long double l1 = hom_lik_ref(p, coverage, error1, f);

    double error2 = 1.5 * (double)(coverage - p[f] - p[s]) / (double)coverage;
    if (error2 > error_threshold) error2 = error_threshold;
    long double l2 = het_lik_ref(p, coverage, error2, f, s);

    if (snp_prior > 0) {
        l1 *= (1 - snp_prior);
        l2 *= snp_prior;
    }
    double p1 = oracle_lrt(l2, l1);
    double p2 = oracle_lrt(l1, l2);

    int het = (l2 > l1 && p2 < significance_level);
    int g1 = het ? s : f;
    *code = (uint8_t)(f | (g1 << 2) | (het ? 0x80 : 0));
    *hom_conf = p1;
    *het_conf = p2;
}

/* ------------------------------------------------------------------------ */
/* pileup.cpp:169-217 unique profiles + distribution                         */
/* ------------------------------------------------------------------------ */
static uint64_t profile_key(const uint16_t p[4])
{
    /* numeric order of this key == lexicographic std::array<uint16_t,4> order */
    return ((uint64_t)p[0] << 48) | ((uint64_t)p[1] << 32) | ((uint64_t)p[2] << 16) | p[3];
}

static int cmp_u64(const void* a, const void* b)
{
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return (x > y) - (x < y);
}

size_t oracle_count_unique(const uint16_t* counts, size_t n, oracle_profile** out)
{
    *out = NULL;
    if (n == 0) return 0;
    uint64_t* keys = (uint64_t*)malloc(n * sizeof(uint64_t));
    for (size_t i = 0; i < n; ++i) keys[i] = profile_key(counts + 4 * i);
    qsort(keys, n, sizeof(uint64_t), cmp_u64);
    size_t u = 0;
    for (size_t i = 0; i < n; ++i)
        if (i == 0 || keys[i] != keys[i - 1]) ++u;
    oracle_profile* prof = (oracle_profile*)calloc(u, sizeof(oracle_profile));
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) {
        if (i == 0 || keys[i] != keys[i - 1]) {
            oracle_profile* q = &prof[k++];
            q->profile[0] = (uint16_t)(keys[i] >> 48);
            q->profile[1] = (uint16_t)(keys[i] >> 32);
            q->profile[2] = (uint16_t)(keys[i] >> 16);
            q->profile[3] = (uint16_t)(keys[i]);
            q->coverage = coverage_of(q->profile);
            q->count = 0;
        }
        prof[k - 1].count += 1; /* uint32, pileup.hpp:34 */
    }
    free(keys);
    *out = prof;
    return u;
}

/* Harness only, not reference behaviour: a unique-profile table given from
 * outside (the whole input's, when this process sees a part of it: the
 * bench's per-rank spot check of the Lynch paths at N ranks, whose estimate
 * and BH run over every rank's profiles, call.cpp:62-143).  While set,
 * oracle_call_method takes it in place of the table of its own sites. */
static oracle_profile* g_table = NULL;
static size_t g_table_u = 0;

static int cmp_key_pair(const void* a, const void* b)
{
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

void oracle_given_profile_table(const uint64_t* key_count_pairs, size_t u)
{
    free(g_table);
    g_table = NULL;
    g_table_u = 0;
    if (!key_count_pairs) return;
    uint64_t* kc = (uint64_t*)malloc((u ? u : 1) * 2 * sizeof(uint64_t));
    if (u) memcpy(kc, key_count_pairs, u * 2 * sizeof(uint64_t));
    qsort(kc, u, 2 * sizeof(uint64_t), cmp_key_pair);   /* key order = the profiles' lexicographic order */
    g_table = (oracle_profile*)calloc(u ? u : 1, sizeof(oracle_profile));
    for (size_t k = 0; k < u; ++k) {
        oracle_profile* q = &g_table[k];
        q->profile[0] = (uint16_t)(kc[2 * k] >> 48);
        q->profile[1] = (uint16_t)(kc[2 * k] >> 32);
        q->profile[2] = (uint16_t)(kc[2 * k] >> 16);
        q->profile[3] = (uint16_t)(kc[2 * k]);
        q->coverage = coverage_of(q->profile);
        q->count = (uint32_t)kc[2 * k + 1];
    }
    free(kc);
    g_table_u = u;
}

/* call.cpp:66-70 remove_if(coverage < 4) */
size_t oracle_filter_min_coverage(oracle_profile* p, size_t u)
{
    size_t k = 0;
    for (size_t i = 0; i < u; ++i)
        if (!(p[i].coverage < 4)) p[k++] = p[i];
    return k;
}

/* pileup.cpp:198-217.  count*coverage and count*profile[i] are 32-bit
 * products (they wrap) before being widened into the 64-bit sums. */
void oracle_nucleotide_distribution(const oracle_profile* p, size_t u, double dist[4])
{
    uint64_t acc[4] = {0, 0, 0, 0};
    uint64_t total = 0;
    for (size_t k = 0; k < u; ++k) {
        total += (uint32_t)(p[k].count * p[k].coverage);
        for (int i = 0; i < 4; ++i) acc[i] += (uint32_t)(p[k].count * p[k].profile[i]);
    }
    if (total != 0) {
        for (int i = 0; i < 4; ++i) dist[i] = (double)acc[i] / (double)total;
    } else {
        for (int i = 0; i < 4; ++i) dist[i] = 0.25;
    }
}

/* ------------------------------------------------------------------------ */
/* lynch.cpp:37-61 compoundLikelihood                                        */
/* ------------------------------------------------------------------------ */
double oracle_compound_likelihood(const oracle_profile* p, size_t u, const double d[4],
                                  double pi, double epsilon)
{
    if (pi < 0 || pi > 1 || epsilon < 0 || epsilon > 1) return DBL_MAX;
    long double logLikelihood = 0;
    for (size_t k = 0; k < u; ++k) {
        long double L = (1. - pi) * oracle_hom_lik_dist(&p[k], epsilon, d) +
                        pi * oracle_het_lik_dist(&p[k], epsilon, d);
        if (L > 0) logLikelihood += logl(L) * p[k].count;
    }
    if (isinf(logLikelihood)) {
        logLikelihood = logLikelihood > 0 ? LDBL_MAX : -LDBL_MAX;
    }
    return (double)(-logLikelihood);
}

/* ------------------------------------------------------------------------ */
/* GSL 2.7.1 multimin/nmsimplex2.c restated for P = n+1 vertices, with the   */
/* gslcblas dscal/daxpy/ddot/dnrm2 kernels it calls.                         */
/* ------------------------------------------------------------------------ */
#define NM_MAXN 4

typedef struct {
    int n;                            /* parameters */
    double x1[NM_MAXN + 1][NM_MAXN];  /* simplex corners */
    double y1[NM_MAXN + 1];
    double ws1[NM_MAXN], ws2[NM_MAXN];
    double center[NM_MAXN], delta[NM_MAXN], xmc[NM_MAXN];
    double S2;
    /* objective */
    const oracle_profile* prof;
    size_t u;
    const double* dist;
    size_t evals;
} nm_state;

static double nm_f(nm_state* s, const double* x)
{
    s->evals++;
    return oracle_compound_likelihood(s->prof, s->u, s->dist, x[0], x[1]);
}

static void b_dscal(int n, double alpha, double* x)
{
    for (int i = 0; i < n; i++) x[i] *= alpha;
}
static void b_daxpy(int n, double alpha, const double* x, double* y)
{
    if (alpha == 0.0) return;
    for (int i = 0; i < n; i++) y[i] += alpha * x[i];
}
static double b_ddot(int n, const double* x, const double* y)
{
    double r = 0.0;
    for (int i = 0; i < n; i++) r += x[i] * y[i];
    return r;
}
static double b_dnrm2(int n, const double* x)
{
    double scale = 0.0, ssq = 1.0;
    if (n <= 0) return 0;
    if (n == 1) return fabs(x[0]);
    for (int i = 0; i < n; i++) {
        const double xi = x[i];
        if (xi != 0.0) {
            const double ax = fabs(xi);
            if (scale < ax) {
                ssq = 1.0 + ssq * (scale / ax) * (scale / ax);
                scale = ax;
            } else {
                ssq += (ax / scale) * (ax / scale);
            }
        }
    }
    return scale * sqrt(ssq);
}

static void nm_compute_center(nm_state* s)
{
    const int P = s->n + 1;
    for (int j = 0; j < s->n; j++) s->center[j] = 0.0;
    for (int i = 0; i < P; i++) b_daxpy(s->n, 1.0, s->x1[i], s->center);
    b_dscal(s->n, 1.0 / P, s->center);
}

static double nm_compute_size(nm_state* s)
{
    const int P = s->n + 1;
    double ss = 0.0;
    for (int i = 0; i < P; i++) {
        memcpy(s->ws1, s->x1[i], sizeof(double) * s->n);
        b_daxpy(s->n, -1.0, s->center, s->ws1);
        double t = b_dnrm2(s->n, s->ws1);
        ss += t * t;
    }
    s->S2 = ss / P;
    return sqrt(ss / P);
}

static double nm_try_corner_move(nm_state* s, double coeff, int corner, double* xc)
{
    const size_t P = (size_t)(s->n + 1);
    double alpha = (1 - coeff) * P / (P - 1.0);
    double beta = (P * coeff - 1.0) / (P - 1.0);
    memcpy(xc, s->center, sizeof(double) * s->n);
    b_dscal(s->n, alpha, xc);
    b_daxpy(s->n, beta, s->x1[corner], xc);
    return nm_f(s, xc);
}

static void nm_update_point(nm_state* s, int i, const double* x, double val)
{
    const size_t P = (size_t)(s->n + 1);
    const double* x_orig = s->x1[i];
    memcpy(s->delta, x, sizeof(double) * s->n);
    b_daxpy(s->n, -1.0, x_orig, s->delta);
    memcpy(s->xmc, x_orig, sizeof(double) * s->n);
    b_daxpy(s->n, -1.0, s->center, s->xmc);
    {
        double d = b_dnrm2(s->n, s->delta);
        double xmcd = b_ddot(s->n, s->xmc, s->delta);
        s->S2 += (2.0 / P) * xmcd + ((P - 1.0) / P) * (d * d / P);
    }
    {
        double alpha = 1.0 / P;
        b_daxpy(s->n, -alpha, x_orig, s->center);
        b_daxpy(s->n, alpha, x, s->center);
    }
    memcpy(s->x1[i], x, sizeof(double) * s->n);
    s->y1[i] = val;
}

static int nm_contract_by_best(nm_state* s, int best, double* xc)
{
    const int P = s->n + 1;
    int status = 0;
    for (int i = 0; i < P; i++) {
        if (i != best) {
            for (int j = 0; j < s->n; j++) s->x1[i][j] = 0.5 * (s->x1[i][j] + s->x1[best][j]);
            memcpy(xc, s->x1[i], sizeof(double) * s->n);
            double newval = nm_f(s, xc);
            s->y1[i] = newval;
            if (!isfinite(newval)) status = 1; /* GSL_EBADFUNC */
        }
    }
    nm_compute_center(s);
    nm_compute_size(s);
    return status;
}

/* nmsimplex_set; returns non-zero where GSL would raise an error */
static int nm_set(nm_state* s, const double* x, const double* step, double* size)
{
    double val = nm_f(s, x);
    if (!isfinite(val)) return 1;
    memcpy(s->x1[0], x, sizeof(double) * s->n);
    s->y1[0] = val;
    for (int i = 0; i < s->n; i++) {
        memcpy(s->ws1, x, sizeof(double) * s->n);
        s->ws1[i] = x[i] + step[i];
        val = nm_f(s, s->ws1);
        if (!isfinite(val)) return 1;
        memcpy(s->x1[i + 1], s->ws1, sizeof(double) * s->n);
        s->y1[i + 1] = val;
    }
    nm_compute_center(s);
    *size = nm_compute_size(s);
    return 0;
}

static int vector_min_index(const double* v, int n)
{
    double min = v[0];
    int imin = 0;
    for (int i = 0; i < n; i++) {
        double x = v[i];
        if (x < min) {
            min = x;
            imin = i;
        }
        if (isnan(x)) return i;
    }
    return imin;
}

/* nmsimplex_iterate; x/fval receive the lowest vertex */
static int nm_iterate(nm_state* s, double* x, double* size, double* fval)
{
    double* xc = s->ws1;
    double* xc2 = s->ws2;
    const int n = s->n + 1;
    int hi, s_hi, lo;
    double dhi, ds_hi, dlo, val, val2;

    dhi = dlo = s->y1[0];
    hi = 0;
    lo = 0;
    ds_hi = s->y1[1];
    s_hi = 1;
    for (int i = 1; i < n; i++) {
        val = s->y1[i];
        if (val < dlo) {
            dlo = val;
            lo = i;
        } else if (val > dhi) {
            ds_hi = dhi;
            s_hi = hi;
            dhi = val;
            hi = i;
        } else if (val > ds_hi) {
            ds_hi = val;
            s_hi = i;
        }
    }

    val = nm_try_corner_move(s, -1.0, hi, xc);
    if (isfinite(val) && val < s->y1[lo]) {
        val2 = nm_try_corner_move(s, -2.0, hi, xc2);
        if (isfinite(val2) && val2 < s->y1[lo]) {
            nm_update_point(s, hi, xc2, val2);
        } else {
            nm_update_point(s, hi, xc, val);
        }
    } else if (!isfinite(val) || val > s->y1[s_hi]) {
        if (isfinite(val) && val <= s->y1[hi]) {
            nm_update_point(s, hi, xc, val);
        }
        val2 = nm_try_corner_move(s, 0.5, hi, xc2);
        if (isfinite(val2) && val2 <= s->y1[hi]) {
            nm_update_point(s, hi, xc2, val2);
        } else {
            if (nm_contract_by_best(s, lo, xc) != 0) return 1; /* "contraction failed" */
        }
    } else {
        nm_update_point(s, hi, xc, val);
    }

    lo = vector_min_index(s->y1, n);
    memcpy(x, s->x1[lo], sizeof(double) * s->n);
    *fval = s->y1[lo];
    if (s->S2 > 0) {
        *size = sqrt(s->S2);
    } else {
        *size = nm_compute_size(s);
    }
    return 0;
}

/* lynch.cpp:17-35 + optimization.hpp:50-89 */
int oracle_estimate(const oracle_profile* p, size_t u, const double dist[4],
                    oracle_est_t* est, long double* lhom, long double* lhet, int verbose)
{
    nm_state s;
    memset(&s, 0, sizeof(s));
    s.n = 2;
    s.prof = p;
    s.u = u;
    s.dist = dist;
    const double x0[2] = {1e-3, 1e-3};   /* DEFAULT_PI, DEFAULT_EPSILON  lynch.cpp:8-10 */
    const double step[2] = {1e-4, 1e-4}; /* DEFAULT_STEPSIZE                          */
    double x[2] = {x0[0], x0[1]};
    double size = 0, fval = 0;
    memset(est, 0, sizeof(*est));
    if (nm_set(&s, x0, step, &size) != 0) {
        est->status = 1;
        return 1;
    }
    int i = 0;
    int status = 0;
    const int GSL_CONTINUE = -2;
    do {
        ++i;
        status = nm_iterate(&s, x, &size, &fval);
        if (status != 0) break;
        status = (size < 1e-5) ? 0 : GSL_CONTINUE;
        if (status == 0 && verbose)
            fprintf(stderr, "# GSL function minimization converged in %d iterations.\n", i);
    } while (status == GSL_CONTINUE && i < 1000);
    int converged = 1;
    if (status == GSL_CONTINUE) {
        converged = 0;
        if (verbose)
            fprintf(stderr, "# Error: GSL function minimization did not converge in %d iterations!\n", i);
    } else if (status != 0) {
        est->status = 1; /* GSL would abort in its error handler */
        return 1;
    }
    est->heterozygosity = x[0];
    est->error_rate = x[1];
    est->fval = fval;
    est->iterations = i;
    est->converged = converged;
    est->evaluations = s.evals;
    if (lhom && lhet) {
        for (size_t k = 0; k < u; ++k) {
            lhom[k] = oracle_hom_lik_dist(&p[k], x[1], dist);
            lhet[k] = oracle_het_lik_dist(&p[k], x[1], dist);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* stats.cpp:58-80 adjustBenjaminiHochberg (tie order provably irrelevant)  */
/* ------------------------------------------------------------------------ */
void oracle_descending_sorted_indices(const double* v, size_t m, size_t* idx);   /* sid_oracle_sort.cpp */

/* stats.cpp:69-80 */
void oracle_bh(const double* p, size_t m, double* adj)
{
    if (m == 0) return;
    size_t* sorted = (size_t*)malloc(m * sizeof(size_t));
    oracle_descending_sorted_indices(p, m, sorted);
    adj[sorted[0]] = p[sorted[0]];
    for (size_t i = 1; i < m; ++i) {
        double cand = p[sorted[i]] * (double)m / (double)(m - i);
        double prev = adj[sorted[i - 1]];
        adj[sorted[i]] = (cand < prev) ? cand : prev; /* std::min(prev, cand) */
    }
    for (size_t i = 0; i < m; ++i)
        if (adj[i] > 1) adj[i] = 1.0;
    free(sorted);
}

/* ------------------------------------------------------------------------ */
/* Method drivers (call.cpp)                                                 */
/* ------------------------------------------------------------------------ */
static long find_profile(const oracle_profile* p, size_t u, const uint16_t q[4])
{
    uint64_t key = profile_key(q);
    size_t lo = 0, hi = u;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        uint64_t k = profile_key(p[mid].profile);
        if (k < key)
            lo = mid + 1;
        else if (k > key)
            hi = mid;
        else
            return (long)mid;
    }
    return -1;
}

int oracle_call_method(int method, int estimate_prior, double snp_prior, double error_threshold,
                       double significance_level, const uint16_t* counts, size_t n,
                       uint8_t* code, double* hom_conf, double* het_conf,
                       oracle_est_t* est_out, size_t* n_unique, int verbose)
{
    oracle_profile* prof = NULL;
    size_t u;
    if (g_table) {   /* (harness: the whole input's table, oracle_given_profile_table) */
        u = g_table_u;
        prof = (oracle_profile*)malloc((u ? u : 1) * sizeof(oracle_profile));
        if (u) memcpy(prof, g_table, u * sizeof(oracle_profile));
    } else {
        u = oracle_count_unique(counts, n, &prof);
    }
    oracle_est_t est;
    memset(&est, 0, sizeof(est));
    int rc = 0;

    if (method == ORACLE_LOCAL) {
        /* call.cpp:213-289 */
        if (estimate_prior) {
            oracle_profile* f = (oracle_profile*)malloc((u ? u : 1) * sizeof(oracle_profile));
            if (u) memcpy(f, prof, u * sizeof(oracle_profile));
            size_t uf = oracle_filter_min_coverage(f, u);
            double dist[4];
            oracle_nucleotide_distribution(f, uf, dist);
            rc = oracle_estimate(f, uf, dist, &est, NULL, NULL, verbose);
            free(f);
            if (rc) goto done;
            snp_prior = est.heterozygosity;
        }
        uint8_t* pc = (uint8_t*)malloc((u ? u : 1));
        double* p1 = (double*)malloc((u ? u : 1) * sizeof(double));
        double* p2 = (double*)malloc((u ? u : 1) * sizeof(double));
        for (size_t k = 0; k < u; ++k)
            oracle_local_profile(prof[k].profile, snp_prior, error_threshold, significance_level,
                                 &pc[k], &p1[k], &p2[k]);
        for (size_t i = 0; i < n; ++i) {
            long k = find_profile(prof, u, counts + 4 * i);
            code[i] = pc[k];
            hom_conf[i] = p1[k];
            het_conf[i] = p2[k];
        }
        free(pc);
        free(p1);
        free(p2);
        if (n_unique) *n_unique = u;
    } else {
        /* call.cpp:62-143 (likelihood_ratio) and call.cpp:145-211 (bayes) */
        u = oracle_filter_min_coverage(prof, u);
        if (verbose) fprintf(stderr, "# unique profiles: %zu\n", u);
        if (n_unique) *n_unique = u;
        double dist[4];
        oracle_nucleotide_distribution(prof, u, dist);
        long double* lhom = (long double*)malloc((u ? u : 1) * sizeof(long double));
        long double* lhet = (long double*)malloc((u ? u : 1) * sizeof(long double));
        rc = oracle_estimate(prof, u, dist, &est, lhom, lhet, verbose);
        if (rc) {
            free(lhom);
            free(lhet);
            goto done;
        }
        if (verbose) {
            fprintf(stderr, "# heterozygosity: %e\n", est.heterozygosity);
            fprintf(stderr, "# error: %e\n", est.error_rate);
        }
        if (u == 0 && method == ORACLE_LIKELIHOOD_RATIO) {
            /* reference: adjustBenjaminiHochberg reads sorted[0] of an empty
               vector (stats.cpp:73); callBayes (call.cpp:145-211) never calls
               it and prints no record */
            free(lhom);
            free(lhet);
            rc = 2;
            goto done;
        }
        uint8_t* pc = (uint8_t*)malloc(u ? u : 1);
        double* c1 = (double*)malloc((u ? u : 1) * sizeof(double));
        double* c2 = (double*)malloc((u ? u : 1) * sizeof(double));
        if (method == ORACLE_LIKELIHOOD_RATIO) {
            double* ph = (double*)malloc(u * sizeof(double));
            double* pt = (double*)malloc(u * sizeof(double));
            for (size_t k = 0; k < u; ++k) {
                long double L_het = lhet[k], L_hom = lhom[k];
                if (estimate_prior) {
                    L_het *= est.heterozygosity;
                    L_hom *= 1 - est.heterozygosity;
                }
                ph[k] = oracle_lrt(L_het, L_hom);
                pt[k] = oracle_lrt(L_hom, L_het);
            }
            oracle_bh(ph, u, c1);
            oracle_bh(pt, u, c2);
            for (size_t k = 0; k < u; ++k) {
                int f, s;
                oracle_major(prof[k].profile, &f, &s);
                int het = c2[k] < significance_level;
                pc[k] = (uint8_t)(f | ((het ? s : f) << 2) | (het ? 0x80 : 0));
            }
            free(ph);
            free(pt);
        } else {
            for (size_t k = 0; k < u; ++k) {
                long double aH = lhom[k] * (1 - est.heterozygosity);
                long double aT = lhet[k] * est.heterozygosity;
                long double PH = aH / (aH + aT);
                long double PT = aT / (aH + aT);
                int f, s;
                oracle_major(prof[k].profile, &f, &s);
                int het = PT > PH;
                pc[k] = (uint8_t)(f | ((het ? s : f) << 2) | (het ? 0x80 : 0));
                c1[k] = (double)PH;
                c2[k] = (double)PT;
            }
        }
        for (size_t i = 0; i < n; ++i) {
            long k = find_profile(prof, u, counts + 4 * i);
            if (k < 0) {
                code[i] = 0x40; /* dropped: profile coverage < 4 */
                hom_conf[i] = het_conf[i] = 0;
            } else {
                code[i] = pc[k];
                hom_conf[i] = c1[k];
                het_conf[i] = c2[k];
            }
        }
        free(pc);
        free(c1);
        free(c2);
        free(lhom);
        free(lhet);
    }
done:
    if (est_out) *est_out = est;
    free(prof);
    return rc;
}

/* Convenience for ctypes: -m local per site directly (no dedupe). */
void oracle_call_local(const uint16_t* counts, size_t n, double snp_prior, double error_threshold,
                       double significance_level, uint8_t* code, double* hom_conf,
                       double* het_conf)
{
    for (size_t i = 0; i < n; ++i)
        oracle_local_profile(counts + 4 * i, snp_prior, error_threshold, significance_level,
                             &code[i], &hom_conf[i], &het_conf[i]);
}

/* ------------------------------------------------------------------------ */
/* call.cpp:311-369 callQualityBasedSimple, one site.  bases / bq / mq as    */
/* pileup.cpp parses them; the j-th counted base pairs with the j-th quality */
/* characters (the reference's index alignment).  Past the end of bq or mq   */
/* the reference reads outside the vectors (undefined); quality 1 is used.   */
/* ------------------------------------------------------------------------ */
void oracle_quality_site(const uint16_t counts[4], const char* bases, int nb, const uint8_t* bq, int nbq,
                         const uint8_t* mq, int nmq, double snp_prior, double significance_level,
                         uint8_t* code, double* p1, double* p2)
{
    static const char ACGT[] = "ACGT";
    int ref0, ref1;
    oracle_major(counts, &ref0, &ref1);
    long double lph = 0, lpt = 0;
    for (int j = 0; j < nb; ++j) {
        const uint8_t b = j < nbq ? bq[j] : 1, m = j < nmq ? mq[j] : 1;
        const double error = pow(10., (b < m ? b : m) / -10.);
        if (bases[j] == ACGT[ref0]) lph += log(1 - error);
        else lph += log(error);
        if (bases[j] == ACGT[ref0] || bases[j] == ACGT[ref1]) lpt += log(1 - 2. / 3. * error);
        else lpt += log(2. / 3. * error);
    }
    const int n = counts[ref0] + counts[ref1];
    const int k = counts[ref1];
    const double logbinom = oracle_log_gamma(n + 1) - oracle_log_gamma(n - k + 1) - oracle_log_gamma(k + 1);
    lpt += logbinom - n * logl(2);
    long double pp1 = expl(lph), pp2 = expl(lpt);
    if (snp_prior > 0) {
        pp1 *= (1 - snp_prior);
        pp2 *= snp_prior;
    }
    *p1 = oracle_lrt(pp2, pp1);
    *p2 = oracle_lrt(pp1, pp2);
    const int het = *p2 < significance_level;
    *code = (uint8_t)(ref0 | ((het ? ref1 : ref0) << 2) | (het ? 0x80 : 0));
}

/* quality method over a whole text (readFile(in, true, true) + the per-site
 * loop); returns ORACLE_* of the first malformed line, or 10 + oracle_call_method's rc */
int oracle_call_quality_text(const char* text, size_t len, int estimate_prior, double snp_prior,
                             double significance_level, uint8_t* code, double* hom, double* het,
                             size_t cap, size_t* n_out, int verbose)
{
    size_t n = 0, ncap = 1024;
    uint16_t* counts = (uint16_t*)malloc(ncap * 8);
    char* line = NULL;
    size_t lcap = 0;
    /* pass 1: parse (errors first, as readFile does), counts */
    const char* p = text;
    const char* end = text + len;
    int rc = ORACLE_OK;
    while (p < end) {
        const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        size_t ll = nl ? (size_t)(nl - p) : (size_t)(end - p);
        if (ll > 0) {
            if (ll + 1 > lcap) {
                lcap = 2 * (ll + 1);
                line = (char*)realloc(line, lcap);
            }
            memcpy(line, p, ll);
            line[ll] = 0;
            oracle_line L;
            rc = oracle_parse_line(line, 1, 1, &L);
            if (rc != ORACLE_OK) break;
            if (n == ncap) {
                ncap *= 2;
                counts = (uint16_t*)realloc(counts, ncap * 8);
            }
            memcpy(counts + 4 * n, L.counts, 8);
            ++n;
        }
        p = nl ? nl + 1 : end;
    }
    if (rc != ORACLE_OK) {
        free(counts);
        free(line);
        return rc;
    }
    *n_out = n;
    if (estimate_prior) {   /* call.cpp:294-305: the -R estimate of the local method */
        uint8_t* c = (uint8_t*)malloc(n ? n : 1);
        double* a = (double*)malloc((n ? n : 1) * 8);
        double* b = (double*)malloc((n ? n : 1) * 8);
        oracle_est_t est;
        int r = oracle_call_method(ORACLE_LOCAL, 1, -1, 0.1, significance_level, counts, n, c, a, b, &est, NULL,
                                   verbose);
        free(c);
        free(a);
        free(b);
        if (r) {
            free(counts);
            free(line);
            return 10 + r;
        }
        snp_prior = est.heterozygosity;
    }
    /* pass 2: per site */
    size_t i = 0;
    char* bases = NULL;
    uint8_t *bq = NULL, *mq = NULL;
    int bcap = 0;
    p = text;
    while (p < end && i < n) {
        const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        size_t ll = nl ? (size_t)(nl - p) : (size_t)(end - p);
        if (ll > 0) {
            memcpy(line, p, ll);
            line[ll] = 0;
            oracle_line L;
            oracle_parse_line(line, 1, 1, &L);
            int nb = oracle_read_bases_seq(L.read_bases, L.reference, NULL, 0);
            int need = nb > L.n_bq ? nb : L.n_bq;
            if (L.n_mq > need) need = L.n_mq;
            if (need + 1 > bcap) {
                bcap = 2 * (need + 1);
                bases = (char*)realloc(bases, bcap);
                bq = (uint8_t*)realloc(bq, bcap);
                mq = (uint8_t*)realloc(mq, bcap);
            }
            oracle_read_bases_seq(L.read_bases, L.reference, bases, bcap);
            oracle_parse_qualities(L.base_qualities, bq, bcap);
            oracle_parse_qualities(L.mapping_qualities, mq, bcap);
            if (i < cap)
                oracle_quality_site(counts + 4 * i, bases, nb, bq, L.n_bq, mq, L.n_mq, snp_prior,
                                    significance_level, &code[i], &hom[i], &het[i]);
            ++i;
        }
        p = nl ? nl + 1 : end;
    }
    free(bases);
    free(bq);
    free(mq);
    free(counts);
    free(line);
    return ORACLE_OK;
}
