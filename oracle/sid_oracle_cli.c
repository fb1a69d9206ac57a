/*
 * sid_oracle_cli.c — CPU ORACLE command line.  TEST INFRASTRUCTURE ONLY.
 *
 * Restates sid.cpp:1-110 (option table, method dispatch, CSV output) and
 * call.cpp:11-20 (readFile) on top of sid_oracle.c, so tests can compare the
 * product's `sid` CLI byte for byte against it, and bench.py can time it as
 * the CPU baseline ("port").
 */
#define _GNU_SOURCE
#include <getopt.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sid_oracle.h"

typedef struct {
    const char* method;
    int estimate_prior;
    double snp_prior, significance_level, site_error_threshold;
} opts_t;

/* sid.cpp:26-58, std::map<char,...> iteration order E R h m p r */
static const struct {
    char flag;
    const char* name;
    int has_arg;
    const char* description;
} OPTIONS[] = {
    {'E', "ERROR", 1, "Maximum allowed site error rate for 'local' method. Default: 0.1"},
    {'R', "", 0, "Estimate SNP prior from data, applicable for methods 'likelihood_ratio', 'local', 'quality'. Conflicts -r."},
    {'h', "help", 0, "Print this help message"},
    {'m', "METHOD", 1, "Select the method to use for SNP calling: 'likelihood_ratio' , 'bayes', 'local' or 'quality', default: local"},
    {'p', "LEVEL", 1, "Significance level for statistical tests, only applicable for methods 'likelihood_ratio', 'local'. Default: 0.05"},
    {'r', "PRIOR", 1, "Use the given prior for SNPs, applicable for methods 'local', 'quality'. Conflicts -R. Default: no prior"},
};

static void die_terminate(const char* type, const char* what)
{
    fflush(stdout);
    fprintf(stderr, "terminate called after throwing an instance of '%s'\n  what():  %s\n", type, what);
    abort();
}

typedef struct {
    char** chrom;
    int* pos;
    uint16_t* counts;
    size_t n, cap;
} sites_t;

static void push_site(sites_t* s, const oracle_line* l)
{
    if (s->n == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 4096;
        s->chrom = (char**)realloc(s->chrom, s->cap * sizeof(char*));
        s->pos = (int*)realloc(s->pos, s->cap * sizeof(int));
        s->counts = (uint16_t*)realloc(s->counts, s->cap * 4 * sizeof(uint16_t));
    }
    /* chromosome names repeat; share the previous copy when equal */
    if (s->n > 0 && strcmp(s->chrom[s->n - 1], l->chrom) == 0)
        s->chrom[s->n] = s->chrom[s->n - 1];
    else
        s->chrom[s->n] = strdup(l->chrom);
    s->pos[s->n] = l->position;
    memcpy(s->counts + 4 * s->n, l->counts, 4 * sizeof(uint16_t));
    s->n++;
}

/* call.cpp:11-20 readFile; limit: the bytes to read (harness: ORACLE_RANGE) */
static void read_file(FILE* in, sites_t* s, unsigned long long limit)
{
    char* line = NULL;
    size_t cap = 0;
    ssize_t len;
    unsigned long long used = 0;
    while (used < limit && (len = getline(&line, &cap, in)) >= 0) {
        used += (unsigned long long)len;
        if (len > 0 && line[len - 1] == '\n') line[--len] = '\0';
        if (len > 0) {
            oracle_line l;
            int rc = oracle_parse_line(line, 0, 0, &l);
            if (rc == ORACLE_EMALFORMED) die_terminate("std::invalid_argument", "Malformed pileup line");
            if (rc == ORACLE_EMISSING_MQ)
                die_terminate("std::invalid_argument", "Malformed pileup line or missing mapping qualities");
            if (rc == ORACLE_ENULLCHROM) { /* std::string = (char*)NULL: strlen(NULL) */
                fflush(stdout);
                signal(SIGSEGV, SIG_DFL);
                raise(SIGSEGV);
            }
            push_site(s, &l);
        }
    }
    free(line);
}

int main(int argc, char** argv)
{
    opts_t o = {"local", 0, -1, 0.05, 0.1};
    int flag;
    while ((flag = getopt(argc, argv, "E:Rhm:p:r:")) != -1) {
        switch (flag) {
        case 'E': o.site_error_threshold = atof(optarg); break;
        case 'R': o.estimate_prior = 1; break;
        case 'm': o.method = optarg; break;
        case 'p': o.significance_level = atof(optarg); break;
        case 'r': o.snp_prior = atof(optarg); break;
        case 'h':
            fputs("sid [flags] input_file\n", stdout);
            for (size_t i = 0; i < sizeof(OPTIONS) / sizeof(OPTIONS[0]); ++i) {
                printf("\t-%c", OPTIONS[i].flag);
                if (OPTIONS[i].has_arg > 0) printf(" %s", OPTIONS[i].name);
                printf("\t%s\n", OPTIONS[i].description);
            }
            break;
        default: exit(EXIT_FAILURE);
        }
    }
    if (optind >= argc) {
        fflush(stdout);
        fputs("No file name given!\n", stderr);
        exit(EXIT_FAILURE);
    }
    const char* path = argv[optind];
    FILE* in = fopen(path, "rb");
    if (!in) {
        fflush(stdout);
        fprintf(stderr, "Could not open file: %s\n", path);
        exit(EXIT_FAILURE);
    }
    /* test/bench harness, not a reference option: ORACLE_RANGE=OFF:LEN reads
       only the (line-aligned) bytes [OFF, OFF + LEN) of the file -- the CPU
       baseline's shard processes over one file (bench.py) */
    unsigned long long limit = ~0ull, range_off = 0;
    if (getenv("ORACLE_RANGE")) {
        unsigned long long off = 0, n = 0;
        if (sscanf(getenv("ORACLE_RANGE"), "%llu:%llu", &off, &n) == 2 && fseeko(in, (off_t)off, SEEK_SET) == 0) {
            limit = n;
            range_off = off;
        }
    }
    /* harness, not a reference option: ORACLE_PROFILE_TABLE=FILE (u64 key,
       u64 count pairs) is the whole input's unique-profile table, for a
       process that reads a part of it (bench.py's per-rank spot check of the
       Lynch paths, whose estimate and BH are global: call.cpp:62-143) */
    if (getenv("ORACLE_PROFILE_TABLE")) {
        FILE* tf = fopen(getenv("ORACLE_PROFILE_TABLE"), "rb");
        if (!tf) abort();
        uint64_t* kc = NULL;
        size_t u = 0, ucap = 0;
        uint64_t pair[2];
        while (fread(pair, sizeof pair, 1, tf) == 1) {
            if (u == ucap) {
                ucap = ucap ? 2 * ucap : 4096;
                kc = (uint64_t*)realloc(kc, ucap * sizeof pair);
            }
            kc[2 * u] = pair[0];
            kc[2 * u + 1] = pair[1];
            ++u;
        }
        fclose(tf);
        oracle_given_profile_table(kc, u);
        free(kc);
    }
    int method = -1;
    if (strcmp(o.method, "local") == 0) method = ORACLE_LOCAL;
    else if (strcmp(o.method, "bayes") == 0) method = ORACLE_BAYES;
    else if (strcmp(o.method, "likelihood_ratio") == 0) method = ORACLE_LIKELIHOOD_RATIO;
    else if (strcmp(o.method, "quality") == 0) method = 3;   /* call.cpp:291-372 */

    sites_t s = {0};
    uint8_t* code = NULL;
    double *h = NULL, *t = NULL;
    const char* conf_type = method == ORACLE_BAYES ? "probability" : "p_value";
    if (method == 3) {
        /* readFile(in, true, true): the whole text (the range's bytes with
           ORACLE_RANGE, as read_file below takes them), errors first */
        char* text = NULL;
        size_t len = 0, tcap = 0;
        char buf[1 << 16];
        size_t r;
        while (len < limit &&
               (r = fread(buf, 1, (size_t)(limit - len < sizeof buf ? limit - len : sizeof buf), in)) > 0) {
            if (len + r > tcap) {
                tcap = 2 * (len + r);
                text = (char*)realloc(text, tcap);
            }
            memcpy(text + len, buf, r);
            len += r;
        }
        size_t nq = 0;
        int rc = oracle_call_quality_text(text, len, o.estimate_prior, o.snp_prior, o.significance_level,
                                          NULL, NULL, NULL, 0, &nq, 1);
        if (rc == ORACLE_EMALFORMED) die_terminate("std::invalid_argument", "Malformed pileup line");
        if (rc == ORACLE_EMISSING_MQ)
            die_terminate("std::invalid_argument", "Malformed pileup line or missing mapping qualities");
        if (rc == ORACLE_ENULLCHROM || rc == ORACLE_ENOBQ) {
            fflush(stdout);
            signal(SIGSEGV, SIG_DFL);
            raise(SIGSEGV);
        }
        if (rc == 11) {
            fputs("gsl: nmsimplex2.c: ERROR: non-finite function value encountered\n"
                  "Default GSL error handler invoked.\n", stderr);
            abort();
        }
        code = (uint8_t*)malloc(nq ? nq : 1);
        h = (double*)malloc((nq ? nq : 1) * sizeof(double));
        t = (double*)malloc((nq ? nq : 1) * sizeof(double));
        oracle_call_quality_text(text, len, o.estimate_prior, o.snp_prior, o.significance_level, code, h, t, nq,
                                 &nq, 0);
        if (fseeko(in, (off_t)range_off, SEEK_SET) != 0) abort();
        read_file(in, &s, limit);   /* chrom and pos; cannot fail after the quality parse */
        free(text);
    } else if (method >= 0) {
        read_file(in, &s, limit);
        code = (uint8_t*)malloc(s.n ? s.n : 1);
        h = (double*)malloc((s.n ? s.n : 1) * sizeof(double));
        t = (double*)malloc((s.n ? s.n : 1) * sizeof(double));
        oracle_est_t est;
        int rc = oracle_call_method(method, method == ORACLE_BAYES ? 0 : o.estimate_prior,
                                    o.snp_prior, o.site_error_threshold, o.significance_level,
                                    s.counts, s.n, code, h, t, &est, NULL, 1);
        if (rc == 1) {
            fputs("gsl: nmsimplex2.c: ERROR: non-finite function value encountered\n"
                  "Default GSL error handler invoked.\n", stderr);
            abort();
        }
        if (rc == 2) raise(SIGSEGV); /* reference indexes an empty vector */
    }
    fclose(in);
    printf("chrom,pos,label,gt,hom_conf,het_conf,conf_type\n");
    fflush(stdout);
    static const char ACGT[] = "ACGT";
    for (size_t i = 0; i < s.n; ++i) {
        if (code[i] & 0x40) continue;
        printf("%s,%d,%s,%c%c,%g,%g,%s\n", s.chrom[i], s.pos[i], (code[i] & 0x80) ? "het" : "hom",
               ACGT[code[i] & 3], ACGT[(code[i] >> 2) & 3], h[i], t[i], conf_type);
    }
    return 0;
}
