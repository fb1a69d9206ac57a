// lynch_host.cpp — host side of the Lynch ML path
//
// Owns the device hash histogram, the filtered unique-profile table, the
// Nelder-Mead driver (GSL 2.7.1 nmsimplex2 restated; GSL is not vendored in the
// reference), Benjamini-Hochberg, and the compact class hash used by the
// per-site lookup kernel.  The O(sites) work (histogram, lookup) and the
// O(U) per-profile arithmetic (objective, likelihoods, LRT/posteriors) run on
// the GPU; only O(U) bookkeeping (sort, BH step-up) and the 2-parameter
// simplex stay on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <vector>

#include "sid_internal.h"



extern "C" {
hipError_t sid_launch_hist(const uint16_t* counts, size_t n, unsigned long long* gkeys,
                           unsigned long long* gcnt, uint64_t gmask, unsigned long long* stats,
                           hipStream_t st);
hipError_t sid_launch_rehash(const unsigned long long* okeys, const unsigned long long* ocnt,
                             uint64_t ocap, unsigned long long* gkeys, unsigned long long* gcnt,
                             uint64_t gmask, unsigned long long* distinct, hipStream_t st);
hipError_t sid_launch_compact(const unsigned long long* gkeys, const unsigned long long* gcnt,
                              uint64_t cap, unsigned long long* okeys, unsigned long long* ocnt,
                              unsigned long long* nout, hipStream_t st);
hipError_t sid_launch_objective(const uint64_t* keys, const uint32_t* cnt, const double* lnM, size_t u,
                                const sid_lynch_eval* E, double* partial, int grid, hipStream_t st);
hipError_t sid_launch_profile_lik(const uint64_t* keys, const double* lnM, size_t u,
                                  const sid_lynch_eval* E, double* lhom, double* lhet, hipStream_t st);
hipError_t sid_launch_classify(const uint64_t* keys, const double* lhom, const double* lhet, size_t u,
                               int mode, int use_prior, double pi, double lg15, double* c1, double* c2,
                               uint8_t* code, hipStream_t st);
hipError_t sid_launch_lookup(const uint16_t* counts, size_t n, const unsigned long long* ckeys,
                             const uint32_t* cidx, uint64_t cmask, uint32_t special_idx,
                             const uint8_t* pcode, const double* p1, const double* p2, uint8_t* code,
                             double* hom, double* het, int grid_cap, hipStream_t st);
}

static const uint64_t EMPTY = 0xFFFFFFFFFFFFFFFFull;

static uint64_t host_hash64(uint64_t k)   // == sid_hash64 (lynch.hip)
{
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    k ^= k >> 33;
    return k;
}

template <class T>
static void dfree(T*& p)
{
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

struct sid_lynch_dev {
    // accumulation hash (device)
    unsigned long long* gkeys = nullptr;
    unsigned long long* gcnt = nullptr;
    unsigned long long* stats = nullptr;   // [0] distinct, [1] all-65535 profile count
    uint64_t cap = 0;
    uint64_t distinct = 0;
    bool have_hist = false;
    // explicit (merged) table
    bool loaded = false;
    std::vector<uint64_t> tkeys, tcnt;
    // filtered profiles (host + device)
    bool setup = false;
    std::vector<uint64_t> fkeys;
    std::vector<uint32_t> fcnt;
    double dist[4] = {0.25, 0.25, 0.25, 0.25};
    uint64_t* d_keys = nullptr;
    uint32_t* d_cnt = nullptr;
    double* d_lnM = nullptr;
    double* d_partial = nullptr;
    std::vector<double> h_partial;
    int obj_grid = 0;
    uint64_t evals = 0;
    // class table
    bool prepared = false;
    double* d_lhom = nullptr;
    double* d_lhet = nullptr;
    double* d_c1 = nullptr;
    double* d_c2 = nullptr;
    uint8_t* d_pcode = nullptr;
    unsigned long long* d_ckeys = nullptr;
    uint32_t* d_cidx = nullptr;
    uint64_t cmask = 0;
    uint32_t special_idx = 0xFFFFFFFFu;
};

sid_lynch_dev* sid_lynch_dev_create(int* err)
{
    *err = SID_OK;
    return new sid_lynch_dev();
}

static void free_class(sid_lynch_dev* L)
{
    dfree(L->d_lhom);
    dfree(L->d_lhet);
    dfree(L->d_c1);
    dfree(L->d_c2);
    dfree(L->d_pcode);
    dfree(L->d_ckeys);
    dfree(L->d_cidx);
    L->prepared = false;
}

static void free_setup(sid_lynch_dev* L)
{
    dfree(L->d_keys);
    dfree(L->d_cnt);
    dfree(L->d_lnM);
    dfree(L->d_partial);
    L->setup = false;
    free_class(L);
}

void sid_lynch_dev_destroy(sid_lynch_dev* L)
{
    if (!L) return;
    dfree(L->gkeys);
    dfree(L->gcnt);
    dfree(L->stats);
    free_setup(L);
    delete L;
}

static int lynch_of(sid_ctx* c, sid_lynch_dev** out)
{
    if (!c) return SID_EINVAL;
    if (!c->lynch) {
        int err;
        c->lynch = sid_lynch_dev_create(&err);
        if (err) return err;
    }
    *out = c->lynch;
    return SID_OK;
}

#define HIPCHECK(x)                                              \
    do {                                                         \
        hipError_t e_ = (x);                                     \
        if (e_ != hipSuccess) return sid_set_hip_error(e_);      \
    } while (0)

static int alloc_hash(sid_lynch_dev* L, uint64_t cap, hipStream_t st)
{
    HIPCHECK(hipMalloc(&L->gkeys, cap * sizeof(unsigned long long)));
    HIPCHECK(hipMalloc(&L->gcnt, cap * sizeof(unsigned long long)));
    HIPCHECK(hipMemsetAsync(L->gkeys, 0xFF, cap * sizeof(unsigned long long), st));
    HIPCHECK(hipMemsetAsync(L->gcnt, 0, cap * sizeof(unsigned long long), st));
    L->cap = cap;
    return SID_OK;
}

extern "C" int sid_profile_reset(sid_ctx* c, void* stream)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    dfree(L->gkeys);
    dfree(L->gcnt);
    if (!L->stats) HIPCHECK(hipMalloc(&L->stats, 2 * sizeof(unsigned long long)));
    HIPCHECK(hipMemsetAsync(L->stats, 0, 2 * sizeof(unsigned long long), st));
    rc = alloc_hash(L, 1ull << 16, st);
    if (rc) return rc;
    L->distinct = 0;
    L->have_hist = true;
    L->loaded = false;
    L->tkeys.clear();
    L->tcnt.clear();
    free_setup(L);
    return SID_OK;
}

static int grow_hash(sid_lynch_dev* L, uint64_t need, hipStream_t st)
{
    uint64_t cap = L->cap;
    while (cap < need) cap <<= 1;
    if (cap == L->cap) return SID_OK;
    unsigned long long *ok = L->gkeys, *oc = L->gcnt;
    uint64_t ocap = L->cap;
    L->gkeys = L->gcnt = nullptr;
    int rc = alloc_hash(L, cap, st);
    if (rc) return rc;
    HIPCHECK(hipMemsetAsync(L->stats, 0, sizeof(unsigned long long), st));
    HIPCHECK(sid_launch_rehash(ok, oc, ocap, L->gkeys, L->gcnt, cap - 1, L->stats, st));
    HIPCHECK(hipStreamSynchronize(st));
    (void)hipFree(ok);
    (void)hipFree(oc);
    return SID_OK;
}

extern "C" int sid_profile_accumulate(sid_ctx* c, const uint16_t* counts, size_t n, void* stream)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    if (!L->have_hist) {
        rc = sid_profile_reset(c, stream);
        if (rc) return rc;
    }
    if (n == 0) return SID_OK;
    if (!counts || ((uintptr_t)counts & 7u)) return SID_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    const size_t SUB = 4u << 20;
    for (size_t off = 0; off < n; off += SUB) {
        size_t m = std::min(SUB, n - off);
        rc = grow_hash(L, 2 * (L->distinct + m), st);   // load factor <= 1/2
        if (rc) return rc;
        HIPCHECK(sid_launch_hist(counts + 4 * off, m, L->gkeys, L->gcnt, L->cap - 1, L->stats, st));
        unsigned long long d = 0;
        HIPCHECK(hipMemcpyAsync(&d, L->stats, sizeof(d), hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        L->distinct = d;
    }
    L->setup = false;
    free_class(L);
    return SID_OK;
}

// sorted (key, count) of the accumulated histogram
static int export_hist(sid_lynch_dev* L, std::vector<uint64_t>& keys, std::vector<uint64_t>& cnt)
{
    keys.clear();
    cnt.clear();
    if (!L->have_hist) return SID_OK;
    unsigned long long *ok = nullptr, *oc = nullptr, *nout = nullptr;
    size_t m = std::max<uint64_t>(L->distinct, 1);
    HIPCHECK(hipMalloc(&ok, m * sizeof(unsigned long long)));
    HIPCHECK(hipMalloc(&oc, m * sizeof(unsigned long long)));
    HIPCHECK(hipMalloc(&nout, sizeof(unsigned long long)));
    HIPCHECK(hipMemset(nout, 0, sizeof(unsigned long long)));
    HIPCHECK(sid_launch_compact(L->gkeys, L->gcnt, L->cap, ok, oc, nout, 0));
    unsigned long long nn = 0, stats[2] = {0, 0};
    HIPCHECK(hipMemcpy(&nn, nout, sizeof(nn), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(stats, L->stats, sizeof(stats), hipMemcpyDeviceToHost));
    std::vector<uint64_t> k(nn), v(nn);
    if (nn) {
        HIPCHECK(hipMemcpy(k.data(), ok, nn * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(v.data(), oc, nn * 8, hipMemcpyDeviceToHost));
    }
    (void)hipFree(ok);
    (void)hipFree(oc);
    (void)hipFree(nout);
    std::vector<size_t> ord(nn);
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return k[a] < k[b]; });
    keys.reserve(nn + 1);
    cnt.reserve(nn + 1);
    for (size_t i : ord) {
        keys.push_back(k[i]);
        cnt.push_back(v[i]);
    }
    if (stats[1]) {   // the all-65535 profile sorts last
        keys.push_back(EMPTY);
        cnt.push_back(stats[1]);
    }
    return SID_OK;
}

static int current_table(sid_lynch_dev* L, std::vector<uint64_t>& keys, std::vector<uint64_t>& cnt)
{
    if (L->loaded) {
        keys = L->tkeys;
        cnt = L->tcnt;
        return SID_OK;
    }
    return export_hist(L, keys, cnt);
}

extern "C" int sid_profile_table(sid_ctx* c, uint64_t* keys, uint64_t* counts64, size_t cap, size_t* u)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    if (!u) return SID_EINVAL;
    std::vector<uint64_t> k, v;
    rc = current_table(L, k, v);
    if (rc) return rc;
    *u = k.size();
    if (!keys) return SID_OK;
    if (cap < k.size() || !counts64) return SID_EINVAL;
    std::memcpy(keys, k.data(), k.size() * 8);
    std::memcpy(counts64, v.data(), v.size() * 8);
    return SID_OK;
}

extern "C" int sid_profile_load(sid_ctx* c, const uint64_t* keys, const uint64_t* counts64, size_t u)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    if (u && (!keys || !counts64)) return SID_EINVAL;
    std::vector<size_t> ord(u);
    std::iota(ord.begin(), ord.end(), 0);
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return keys[a] < keys[b]; });
    L->tkeys.clear();
    L->tcnt.clear();
    for (size_t i : ord) {
        if (!L->tkeys.empty() && L->tkeys.back() == keys[i]) {
            L->tcnt.back() += counts64[i];
        } else {
            L->tkeys.push_back(keys[i]);
            L->tcnt.push_back(counts64[i]);
        }
    }
    L->loaded = true;
    free_setup(L);
    return SID_OK;
}

static inline uint32_t key_n(uint64_t key, int i) { return (uint32_t)((key >> (48 - 16 * i)) & 0xffff); }

extern "C" int sid_lynch_setup(sid_ctx* c, sid_estimate* est)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    if (!L->setup) {
        std::vector<uint64_t> k, v;
        rc = current_table(L, k, v);
        if (rc) return rc;
        free_setup(L);
        L->fkeys.clear();
        L->fcnt.clear();
        std::vector<double> lnM;
        // call.cpp:66-70: drop profiles with coverage < 4; UniqueProfile::count
        // is uint32 (pileup.hpp:34)
        for (size_t i = 0; i < k.size(); ++i) {
            uint32_t cov = key_n(k[i], 0) + key_n(k[i], 1) + key_n(k[i], 2) + key_n(k[i], 3);
            if (cov < 4) continue;
            L->fkeys.push_back(k[i]);
            L->fcnt.push_back((uint32_t)v[i]);
            // lynch.hpp:48-55 multinomialCoefficient exponent, double, in order
            double m = sid_gsl_lngamma((double)(cov + 1));
            for (int j = 0; j < 4; ++j) {
                uint32_t nj = key_n(k[i], j);
                m -= sid_gsl_lngamma((double)(nj + 1));
            }
            lnM.push_back(m);
        }
        // pileup.cpp:198-217 (32-bit products, 64-bit sums)
        uint64_t acc[4] = {0, 0, 0, 0}, total = 0;
        for (size_t i = 0; i < L->fkeys.size(); ++i) {
            uint32_t cov = key_n(L->fkeys[i], 0) + key_n(L->fkeys[i], 1) + key_n(L->fkeys[i], 2) +
                           key_n(L->fkeys[i], 3);
            total += (uint32_t)(L->fcnt[i] * cov);
            for (int j = 0; j < 4; ++j) acc[j] += (uint32_t)(L->fcnt[i] * key_n(L->fkeys[i], j));
        }
        for (int j = 0; j < 4; ++j) L->dist[j] = total ? (double)acc[j] / (double)total : 0.25;
        const size_t U = L->fkeys.size();
        const size_t m = std::max<size_t>(U, 1);
        HIPCHECK(hipMalloc(&L->d_keys, m * 8));
        HIPCHECK(hipMalloc(&L->d_cnt, m * 4));
        HIPCHECK(hipMalloc(&L->d_lnM, m * 8));
        if (U) {
            HIPCHECK(hipMemcpy(L->d_keys, L->fkeys.data(), U * 8, hipMemcpyHostToDevice));
            HIPCHECK(hipMemcpy(L->d_cnt, L->fcnt.data(), U * 4, hipMemcpyHostToDevice));
            HIPCHECK(hipMemcpy(L->d_lnM, lnM.data(), U * 8, hipMemcpyHostToDevice));
        }
        L->obj_grid = (int)std::min<size_t>(1024, std::max<size_t>(1, (U + 255) / 256));
        HIPCHECK(hipMalloc(&L->d_partial, 2 * L->obj_grid * sizeof(double)));
        L->h_partial.resize(2 * L->obj_grid);
        L->evals = 0;
        L->setup = true;
    }
    if (est) {
        std::memset(est, 0, sizeof(*est));
        std::memcpy(est->dist, L->dist, sizeof(L->dist));
        est->n_unique = L->fkeys.size();
    }
    return SID_OK;
}

// lynch.hpp:57-90 constants for one (pi, eps)
static void make_eval(const double d[4], double pi, double e, sid_lynch_eval* E)
{
    E->la = std::log(1 - e);
    E->lb = std::log(e / 3.);
    E->lh = std::log((1 - 2. / 3. * e) / 2.);
    int k = 0;
    for (int i = 0; i < 4; ++i) {
        E->ld[i] = std::log(d[i]);
        for (int j = i + 1; j < 4; ++j) E->ldd[k++] = std::log(d[i] * d[j]);
    }
    long double s = 0;
    for (int i = 0; i < 4; ++i) s += d[i] * d[i];
    E->lnorm = -(double)logl(1 - s);
    E->l1p = std::log(1. - pi);
    E->lp = std::log(pi);
}

// lynch.cpp:37-61
static int objective(sid_ctx* c, double pi, double eps, double* out)
{
    sid_lynch_dev* L = c->lynch;
    L->evals++;
    if (pi < 0 || pi > 1 || eps < 0 || eps > 1) {
        *out = DBL_MAX;
        return SID_OK;
    }
    const size_t U = L->fkeys.size();
    if (U == 0) {
        *out = -0.0;   // static_cast<double>(-0.0L)
        return SID_OK;
    }
    sid_lynch_eval E;
    make_eval(L->dist, pi, eps, &E);
    HIPCHECK(sid_launch_objective(L->d_keys, L->d_cnt, L->d_lnM, U, &E, L->d_partial, L->obj_grid, 0));
    HIPCHECK(hipMemcpy(L->h_partial.data(), L->d_partial, 2 * L->obj_grid * sizeof(double),
                       hipMemcpyDeviceToHost));
    long double sum = 0;
    for (int b = 0; b < L->obj_grid; ++b) sum += (long double)L->h_partial[2 * b];
    for (int b = 0; b < L->obj_grid; ++b) sum += (long double)L->h_partial[2 * b + 1];
    if (std::isinf((double)sum)) sum = sum > 0 ? LDBL_MAX : -LDBL_MAX;
    *out = (double)(-sum);
    return SID_OK;
}

extern "C" int sid_lynch_objective(sid_ctx* c, double pi, double eps, double* out)
{
    if (!c || !out) return SID_EINVAL;
    int rc = sid_lynch_setup(c, nullptr);
    if (rc) return rc;
    return objective(c, pi, eps, out);
}

// ---------------------------------------------------------------------------
// Nelder-Mead: GSL 2.7.1 multimin/nmsimplex2.c for 2 parameters, with the
// gslcblas kernels it uses (dnrm2 with scale/ssq).  The vertex arithmetic
// depends only on the sequence of comparisons between objective values, so
// agreeing comparisons give bit-identical (pi, eps).
// ---------------------------------------------------------------------------
namespace {
struct Simplex {
    static const int N = 2, P = 3;
    double x1[P][N];
    double y1[P];
    double center[N];
    double S2 = 0;
    sid_ctx* ctx;
    int err = SID_OK;

    double f(const double* x)
    {
        double v = 0;
        int rc = objective(ctx, x[0], x[1], &v);
        if (rc && !err) err = rc;
        return v;
    }
    static double nrm2(const double* x)
    {
        double scale = 0.0, ssq = 1.0;
        for (int i = 0; i < N; ++i) {
            if (x[i] != 0.0) {
                double ax = std::fabs(x[i]);
                if (scale < ax) {
                    ssq = 1.0 + ssq * (scale / ax) * (scale / ax);
                    scale = ax;
                } else {
                    ssq += (ax / scale) * (ax / scale);
                }
            }
        }
        return scale * std::sqrt(ssq);
    }
    static void axpy(double a, const double* x, double* y)
    {
        if (a == 0.0) return;
        for (int i = 0; i < N; ++i) y[i] += a * x[i];
    }
    void compute_center()
    {
        for (int j = 0; j < N; ++j) center[j] = 0.0;
        for (int i = 0; i < P; ++i) axpy(1.0, x1[i], center);
        for (int j = 0; j < N; ++j) center[j] *= 1.0 / P;
    }
    double compute_size()
    {
        double ss = 0.0;
        for (int i = 0; i < P; ++i) {
            double s[N];
            for (int j = 0; j < N; ++j) s[j] = x1[i][j];
            axpy(-1.0, center, s);
            double t = nrm2(s);
            ss += t * t;
        }
        S2 = ss / P;
        return std::sqrt(ss / P);
    }
    double corner_move(double coeff, int corner, double* xc)
    {
        const size_t p = P;
        double alpha = (1 - coeff) * p / (p - 1.0);
        double beta = (p * coeff - 1.0) / (p - 1.0);
        for (int j = 0; j < N; ++j) xc[j] = center[j] * alpha;
        axpy(beta, x1[corner], xc);
        return f(xc);
    }
    void update_point(int i, const double* x, double val)
    {
        const size_t p = P;
        double delta[N], xmc[N];
        for (int j = 0; j < N; ++j) delta[j] = x[j];
        axpy(-1.0, x1[i], delta);
        for (int j = 0; j < N; ++j) xmc[j] = x1[i][j];
        axpy(-1.0, center, xmc);
        double d = nrm2(delta);
        double xmcd = 0.0;
        for (int j = 0; j < N; ++j) xmcd += xmc[j] * delta[j];
        S2 += (2.0 / p) * xmcd + ((p - 1.0) / p) * (d * d / p);
        axpy(-1.0 / p, x1[i], center);
        axpy(1.0 / p, x, center);
        for (int j = 0; j < N; ++j) x1[i][j] = x[j];
        y1[i] = val;
    }
    bool contract_by_best(int best)
    {
        bool ok = true;
        for (int i = 0; i < P; ++i) {
            if (i == best) continue;
            for (int j = 0; j < N; ++j) x1[i][j] = 0.5 * (x1[i][j] + x1[best][j]);
            double xc[N] = {x1[i][0], x1[i][1]};
            y1[i] = f(xc);
            if (!std::isfinite(y1[i])) ok = false;
        }
        compute_center();
        compute_size();
        return ok;
    }
    bool set(const double* x, const double* step, double* size)
    {
        double v = f(x);
        if (!std::isfinite(v)) return false;
        x1[0][0] = x[0];
        x1[0][1] = x[1];
        y1[0] = v;
        for (int i = 0; i < N; ++i) {
            double xt[N] = {x[0], x[1]};
            xt[i] = x[i] + step[i];
            v = f(xt);
            if (!std::isfinite(v)) return false;
            x1[i + 1][0] = xt[0];
            x1[i + 1][1] = xt[1];
            y1[i + 1] = v;
        }
        compute_center();
        *size = compute_size();
        return true;
    }
    bool iterate(double* x, double* size, double* fval)
    {
        double xc[N], xc2[N];
        int hi = 0, lo = 0, s_hi = 1;
        double dhi = y1[0], dlo = y1[0], ds_hi = y1[1];
        for (int i = 1; i < P; ++i) {
            double v = y1[i];
            if (v < dlo) {
                dlo = v;
                lo = i;
            } else if (v > dhi) {
                ds_hi = dhi;
                s_hi = hi;
                dhi = v;
                hi = i;
            } else if (v > ds_hi) {
                ds_hi = v;
                s_hi = i;
            }
        }
        double val = corner_move(-1.0, hi, xc);
        if (std::isfinite(val) && val < y1[lo]) {
            double val2 = corner_move(-2.0, hi, xc2);
            if (std::isfinite(val2) && val2 < y1[lo])
                update_point(hi, xc2, val2);
            else
                update_point(hi, xc, val);
        } else if (!std::isfinite(val) || val > y1[s_hi]) {
            if (std::isfinite(val) && val <= y1[hi]) update_point(hi, xc, val);
            double val2 = corner_move(0.5, hi, xc2);
            if (std::isfinite(val2) && val2 <= y1[hi]) {
                update_point(hi, xc2, val2);
            } else if (!contract_by_best(lo)) {
                return false;
            }
        } else {
            update_point(hi, xc, val);
        }
        // gsl_vector_min_index
        int imin = 0;
        double mn = y1[0];
        for (int i = 0; i < P; ++i) {
            if (y1[i] < mn) {
                mn = y1[i];
                imin = i;
            }
            if (std::isnan(y1[i])) {
                imin = i;
                break;
            }
        }
        x[0] = x1[imin][0];
        x[1] = x1[imin][1];
        *fval = y1[imin];
        *size = S2 > 0 ? std::sqrt(S2) : compute_size();
        return true;
    }
};
}  // namespace

// lynch.cpp:17-35 + optimization.hpp:50-89
static int run_estimate(sid_ctx* c, int verbose, sid_estimate* est)
{
    sid_lynch_dev* L = c->lynch;
    Simplex S;
    S.ctx = c;
    const double x0[2] = {1e-3, 1e-3};   // DEFAULT_PI, DEFAULT_EPSILON  lynch.cpp:8-10
    const double step[2] = {1e-4, 1e-4}; // DEFAULT_STEPSIZE
    double x[2] = {x0[0], x0[1]}, size = 0, fval = 0;
    L->evals = 0;
    if (!S.set(x0, step, &size)) return S.err ? S.err : SID_EBADFUNC;
    if (S.err) return S.err;
    int i = 0, status = 0;
    const int CONTINUE = -2;
    do {
        ++i;
        if (!S.iterate(x, &size, &fval)) return S.err ? S.err : SID_EBADFUNC;   // "contraction failed"
        if (S.err) return S.err;
        status = size < 1e-5 ? 0 : CONTINUE;
        if (status == 0 && verbose)
            std::fprintf(stderr, "# GSL function minimization converged in %d iterations.\n", i);
    } while (status == CONTINUE && i < 1000);
    int converged = 1;
    if (status == CONTINUE) {
        converged = 0;
        if (verbose)
            std::fprintf(stderr, "# Error: GSL function minimization did not converge in %d iterations!\n", i);
    }
    est->heterozygosity = x[0];
    est->error_rate = x[1];
    est->fval = fval;
    est->iterations = i;
    est->converged = converged;
    est->evaluations = L->evals;
    return SID_OK;
}

extern "C" int sid_lynch_prepare(sid_ctx* c, int verbose, sid_estimate* est_out)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    sid_estimate est;
    rc = sid_lynch_setup(c, &est);
    if (rc) return rc;
    const int method = c->opts.method;
    const size_t U = L->fkeys.size();
    if (verbose && method != SID_METHOD_LOCAL) std::fprintf(stderr, "# unique profiles: %zu\n", U);
    rc = run_estimate(c, verbose, &est);
    if (rc) return rc;
    if (est_out) *est_out = est;
    if (method == SID_METHOD_LOCAL) return SID_OK;   // -R local: caller applies the prior
    if (verbose) {
        std::fprintf(stderr, "# heterozygosity: %e\n", est.heterozygosity);
        std::fprintf(stderr, "# error: %e\n", est.error_rate);
    }
    if (U == 0) return SID_EEMPTY;

    free_class(L);
    HIPCHECK(hipMalloc(&L->d_lhom, U * 8));
    HIPCHECK(hipMalloc(&L->d_lhet, U * 8));
    HIPCHECK(hipMalloc(&L->d_c1, U * 8));
    HIPCHECK(hipMalloc(&L->d_c2, U * 8));
    HIPCHECK(hipMalloc(&L->d_pcode, U));
    sid_lynch_eval E;
    make_eval(L->dist, est.heterozygosity, est.error_rate, &E);
    HIPCHECK(sid_launch_profile_lik(L->d_keys, L->d_lnM, U, &E, L->d_lhom, L->d_lhet, 0));
    const int mode = method == SID_METHOD_BAYES ? 1 : 0;
    HIPCHECK(sid_launch_classify(L->d_keys, L->d_lhom, L->d_lhet, U, mode,
                                 method == SID_METHOD_LIKELIHOOD_RATIO && c->opts.estimate_prior,
                                 est.heterozygosity, c->K.lg15, L->d_c1, L->d_c2, L->d_pcode, 0));
    if (mode == 0) {
        // stats.cpp:58-80 Benjamini-Hochberg over the U p-values, then
        // call.cpp:113-127 labels from the adjusted p_het
        std::vector<double> ph(U), pt(U);
        std::vector<uint8_t> code(U);
        HIPCHECK(hipMemcpy(ph.data(), L->d_c1, U * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(pt.data(), L->d_c2, U * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(code.data(), L->d_pcode, U, hipMemcpyDeviceToHost));
        auto bh = [U](const std::vector<double>& p) {
            std::vector<size_t> idx(U);
            std::iota(idx.begin(), idx.end(), 0);
            std::sort(idx.begin(), idx.end(), [&p](size_t i, size_t j) { return p[i] > p[j]; });
            std::vector<double> adj(U);
            adj[idx[0]] = p[idx[0]];
            for (size_t i = 1; i < U; ++i)
                adj[idx[i]] = std::min(adj[idx[i - 1]], p[idx[i]] * double(U) / double(U - i));
            for (auto& a : adj)
                if (a > 1) a = 1.0;
            return adj;
        };
        std::vector<double> ah = bh(ph), at = bh(pt);
        for (size_t i = 0; i < U; ++i) {
            uint8_t f = code[i] & 3, s = (code[i] >> 2) & 3;
            bool het = at[i] < c->opts.significance_level;
            code[i] = (uint8_t)(f | ((het ? s : f) << 2) | (het ? 0x80 : 0));
        }
        HIPCHECK(hipMemcpy(L->d_c1, ah.data(), U * 8, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(L->d_c2, at.data(), U * 8, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(L->d_pcode, code.data(), U, hipMemcpyHostToDevice));
    }
    // compact class hash over the U filtered profiles
    uint64_t cap = 16;
    while (cap < 2 * U) cap <<= 1;
    std::vector<uint64_t> ck(cap, EMPTY);
    std::vector<uint32_t> ci(cap, 0xFFFFFFFFu);
    L->special_idx = 0xFFFFFFFFu;
    for (size_t i = 0; i < U; ++i) {
        uint64_t key = L->fkeys[i];
        if (key == EMPTY) {
            L->special_idx = (uint32_t)i;
            continue;
        }
        uint64_t h = host_hash64(key) & (cap - 1);
        while (ck[h] != EMPTY) h = (h + 1) & (cap - 1);
        ck[h] = key;
        ci[h] = (uint32_t)i;
    }
    HIPCHECK(hipMalloc(&L->d_ckeys, cap * 8));
    HIPCHECK(hipMalloc(&L->d_cidx, cap * 4));
    HIPCHECK(hipMemcpy(L->d_ckeys, ck.data(), cap * 8, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(L->d_cidx, ci.data(), cap * 4, hipMemcpyHostToDevice));
    L->cmask = cap - 1;
    HIPCHECK(hipDeviceSynchronize());
    L->prepared = true;
    return SID_OK;
}

extern "C" int sid_lookup_sites(sid_ctx* c, const uint16_t* counts, size_t n, uint8_t* code,
                                double* hom_conf, double* het_conf, void* stream)
{
    if (!c) return SID_EINVAL;
    sid_lynch_dev* L = c->lynch;
    if (!L || !L->prepared) return SID_ESTATE;
    if (n == 0) return SID_OK;
    if (!counts || !code || !hom_conf || !het_conf || ((uintptr_t)counts & 7u)) return SID_EINVAL;
    HIPCHECK(sid_launch_lookup(counts, n, L->d_ckeys, L->d_cidx, L->cmask, L->special_idx, L->d_pcode,
                               L->d_c1, L->d_c2, code, hom_conf, het_conf, c->grid_cap,
                               (hipStream_t)stream));
    return SID_OK;
}
