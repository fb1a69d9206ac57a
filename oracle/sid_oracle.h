/*
 * sid_oracle.h — CPU ORACLE for the sid hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of EvolBioInf/sid's calling path, used only as
 * the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg.  The product (sid_amd/, libsid.so, the `sid` CLI) never links, loads or
 * calls anything under oracle/.
 *
 * Arithmetic follows the reference line by line, in x87 80-bit long double
 * exactly where the reference uses long double (gcc on x86-64, same libm
 * powl/expl/logl as the reference build would use).
 *
 * Pinning:
 *   - parser / dedupe / nucleotide distribution: pinned against the
 *     reference's own Catch KATs (test/test-*.cpp) and against the
 *     reference's pileup.cpp compiled from /root/reference into oracle/_ref
 *     (tests/test_oracle_ref.py, fuzzed lines);
 *   - the GSL pieces (gsl_sf_lngamma, gsl_cdf_chisq_Q, nmsimplex2) are
 *     restated from GSL 2.7.1's published algorithm (GSL is not vendored in
 *     /root/reference and not installed here; configure.ac:14-16 pins no
 *     version).  chisq_Q is cross-checked against scipy/mpmath; the
 *     nmsimplex2 trajectory is "parity unpinned" against real GSL.
 */
#ifndef SID_ORACLE_H
#define SID_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORACLE_OK = 0,
    ORACLE_EMALFORMED = 1,        /* "Malformed pileup line"                 pileup.cpp:9   */
    ORACLE_EMISSING_MQ = 2,       /* "... or missing mapping qualities"      pileup.cpp:10  */
    ORACLE_ENULLCHROM = 3,        /* std::string = (char*)NULL: SIGSEGV      pileup.cpp:18 */
    ORACLE_ENOBQ = 4,             /* quality mode, no 6th field: parseQualities(NULL)
                                     dereferences NULL: SIGSEGV          pileup.cpp:54,158 */
};

enum { ORACLE_LOCAL = 0, ORACLE_LIKELIHOOD_RATIO = 1, ORACLE_BAYES = 2 };

typedef struct {
    const char* chrom;   /* points into the (mutated) line buffer            */
    int position;        /* atoi()                               pileup.cpp:24 */
    char reference;      /*                                      pileup.cpp:30 */
    int coverage;        /* atoi(), only a reserve() hint         pileup.cpp:36 */
    uint16_t counts[4];  /* profile_t A,C,G,T                     pileup.hpp:7  */
    int n_bq, n_mq;      /* number of parsed quality values (when requested)   */
    const char* read_bases, *base_qualities, *mapping_qualities;   /* tokens */
} oracle_line;

/* pileup.cpp:13-68.  Mutates `line` like strtok_r does.  Returns ORACLE_*. */
int oracle_parse_line(char* line, int parse_bq, int parse_mq, oracle_line* out);
/* pileup.cpp:70-153: counts only (bases/strands are not on the hot path). */
void oracle_read_bases(const char* read_bases, char reference, uint16_t counts[4]);
/* pileup.cpp:155-167. Writes up to `cap` values, returns the count. */
int oracle_parse_qualities(const char* q, uint8_t* out, int cap);
/* pileup.cpp:70-153 bases vector (upper case, read order); returns the count */
int oracle_read_bases_seq(const char* read_bases, char reference, char* out, int cap);
/* call.cpp:311-369, one site */
void oracle_quality_site(const uint16_t counts[4], const char* bases, int nb, const uint8_t* bq, int nbq,
                         const uint8_t* mq, int nmq, double snp_prior, double significance_level,
                         uint8_t* code, double* p1, double* p2);
/* call.cpp:291-372 over a text: ORACLE_* of the first bad line, 10 + rc of the
 * -R estimate on failure, else ORACLE_OK with *n_out sites (results for the
 * first `cap`) */
int oracle_call_quality_text(const char* text, size_t len, int estimate_prior, double snp_prior,
                             double significance_level, uint8_t* code, double* hom, double* het,
                             size_t cap, size_t* n_out, int verbose);

/* call.cpp:52-60 */
void oracle_major(const uint16_t p[4], int* first, int* second);

/* GSL restatements (GSL 2.7.1) */
double oracle_gsl_lngamma(double x);        /* specfunc/gamma.c  gsl_sf_lngamma   */
double oracle_gsl_chisq_Q(double x);        /* cdf/chisq.c       gsl_cdf_chisq_Q(x,1) */
double oracle_log_gamma(int x);             /* lynch.hpp:11-31 memoised wrapper  */

/* stats.cpp:29-37 */
double oracle_lrt(long double l_h0, long double l_h1);

/* One profile through call.cpp:238-273 (-m local).  code: bits0-1 = gt[0],
 * bits2-3 = gt[1], bit7 = het.                                             */
void oracle_local_profile(const uint16_t p[4], double snp_prior, double error_threshold,
                          double significance_level, uint8_t* code, double* hom_conf,
                          double* het_conf);

/* Per-site -m local over n sites (counts n x 4, AoS).  call.cpp:213-289.
 * (Per-profile semantics; the reference's sort/map dedupe does not change
 * per-site results, so the oracle evaluates each site directly.)           */
void oracle_call_local(const uint16_t* counts, size_t n, double snp_prior, double error_threshold,
                       double significance_level, uint8_t* code, double* hom_conf,
                       double* het_conf);

/* ---- unique profiles (pileup.cpp:169-217) ---- */
typedef struct {
    uint16_t profile[4];
    uint32_t count;
    uint32_t coverage;
} oracle_profile;

/* Sorted lexicographically, run-length encoded.  Returns U; *out malloc'd. */
size_t oracle_count_unique(const uint16_t* counts, size_t n, oracle_profile** out);
/* Drops profiles with coverage < 4 in place (call.cpp:66-70). Returns new U. */
size_t oracle_filter_min_coverage(oracle_profile* p, size_t u);
void oracle_nucleotide_distribution(const oracle_profile* p, size_t u, double dist[4]);

/* ---- Lynch path (lynch.hpp:48-96, lynch.cpp:17-61, optimization.hpp) ---- */
long double oracle_hom_lik_dist(const oracle_profile* p, double e, const double dist[4]);
long double oracle_het_lik_dist(const oracle_profile* p, double e, const double dist[4]);
double oracle_compound_likelihood(const oracle_profile* p, size_t u, const double dist[4],
                                  double pi, double eps);

typedef struct {
    double heterozygosity, error_rate, fval;
    int iterations, converged, status;  /* status != 0: GSL would have aborted */
    size_t evaluations;
} oracle_est_t;

/* estimateProfileGenotypeLikelihoods: NM (restated nmsimplex2) then, when
 * lhom/lhet are non-NULL, the per-profile likelihoods at eps-hat.            */
int oracle_estimate(const oracle_profile* p, size_t u, const double dist[4],
                    oracle_est_t* est, long double* lhom, long double* lhet,
                    int verbose /* print "# GSL ..." lines to stderr like the reference */);

/* stats.cpp:58-80 */
void oracle_bh(const double* p, size_t m, double* adj);

/* Harness only: the whole input's unique-profile table (u pairs of u64 key
 * A<<48|C<<32|G<<16|T and count), used by oracle_call_method in place of the
 * table of its own sites until called again with NULL. */
void oracle_given_profile_table(const uint64_t* key_count_pairs, size_t u);

/* ---- whole-method drivers over per-site counts --------------------------
 * Outputs per site: code (bit6 = site dropped, i.e. its profile was filtered
 * out and the reference emits no record), hom_conf, het_conf.  For LR/bayes
 * and -R local the estimate is reported through *est (may be NULL).       */
int oracle_call_method(int method, int estimate_prior, double snp_prior, double error_threshold,
                       double significance_level, const uint16_t* counts, size_t n,
                       uint8_t* code, double* hom_conf, double* het_conf,
                       oracle_est_t* est, size_t* n_unique, int verbose);

#ifdef __cplusplus
}
#endif
#endif
