// lynch_host.cpp — host side of the Lynch ML path
//
// Owns the device hash histogram, the filtered unique-profile table, the
// Nelder-Mead driver (GSL 2.7.1 nmsimplex2 restated; GSL is not vendored in the
// reference), Benjamini-Hochberg, and the compact class hash used by the
// per-site lookup kernel.  The O(sites) work (histogram, lookup) and the
// O(U) work (table sort and filter, lnM, objective, likelihoods,
// LRT/posteriors, BH, class tables) run on the GPU; the host drives the
// 2-parameter simplex, computes the lnGamma table once per context, and
// takes BH over only when NaN / -0 p-values occur.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "sid_internal.h"
#include "sid_nm.h"



extern "C" {
hipError_t sid_launch_hist(const uint16_t* counts, size_t n, unsigned long long* gkeys,
                           unsigned long long* gcnt, uint64_t gmask, unsigned long long* stats,
                           int skip_dense, hipStream_t st);
hipError_t sid_launch_hist_dense(const uint16_t* counts, size_t n, uint32_t* part, unsigned long long* dense,
                                 unsigned long long* list, uint64_t cap, unsigned long long* ctr, int grid_max,
                                 hipStream_t st);
hipError_t sid_launch_hist_list(const unsigned long long* list, uint64_t m, unsigned long long* gkeys,
                                unsigned long long* gcnt, uint64_t gmask, unsigned long long* stats, hipStream_t st);
hipError_t sid_launch_dense_compact(const unsigned long long* dense, unsigned long long* okeys,
                                    unsigned long long* ocnt, unsigned long long* nout, hipStream_t st);
hipError_t sid_launch_pack_class(const double* p1, const double* p2, size_t u, double* cc, hipStream_t st);
hipError_t sid_launch_rehash(const unsigned long long* okeys, const unsigned long long* ocnt,
                             uint64_t ocap, unsigned long long* gkeys, unsigned long long* gcnt,
                             uint64_t gmask, unsigned long long* distinct, hipStream_t st);
hipError_t sid_launch_compact(const unsigned long long* gkeys, const unsigned long long* gcnt,
                              uint64_t cap, unsigned long long* okeys, unsigned long long* ocnt,
                              unsigned long long* nout, hipStream_t st);
hipError_t sid_launch_objective(const uint64_t* keys, const uint32_t* cnt, const double* lnM, size_t u,
                                const sid_lynch_evals* EV, int npts, double* partial, double* out,
                                unsigned int* seq_out, unsigned int seq, int grid, hipStream_t st);
hipError_t sid_launch_nm(const uint64_t* keys, const uint32_t* cnt, const double* lnM, size_t u, int nb,
                         const sid_nm_dist* D, const double* x0, const double* step, int lookahead,
                         double* partial, unsigned int* bar, int grid, long long timeout, sid_nm_result* res,
                         hipStream_t st);
hipError_t sid_launch_profile_lik(const uint64_t* keys, const double* lnM, size_t u,
                                  const sid_lynch_eval* E, double* lhom, double* lhet, hipStream_t st);
hipError_t sid_launch_classify(const uint64_t* keys, const double* lhom, const double* lhet, size_t u,
                               int mode, int use_prior, double pi, double lg15, double* c1, double* c2,
                               uint8_t* code, hipStream_t st);
hipError_t sid_launch_lookup(const uint16_t* counts, size_t n, const unsigned long long* ckeys,
                             const uint32_t* cidx, uint64_t cmask, uint32_t special_idx,
                             const uint8_t* pcode, const double* p1, const double* p2, const double* rec,
                             const uint8_t* rcode, const double* cc, uint8_t* code,
                             double* hom, double* het, int grid_cap, hipStream_t st);
hipError_t sid_launch_rec_build(const uint32_t* dense_cidx, const uint8_t* pcode, const double* cc, double* rec,
                                uint8_t* rcode, hipStream_t st);
size_t sid_bh_ws_bytes(size_t m);
hipError_t sid_launch_bh(const double* p1, const double* p2, size_t m, double* adj1, double* adj2, void* ws,
                         size_t ws_bytes, int* odd, hipStream_t st);
hipError_t sid_launch_bh_label(const double* adj_het, size_t m, double sig, uint8_t* code, hipStream_t st);
size_t sid_setup_ws_bytes(size_t n);
hipError_t sid_launch_setup_select(const unsigned long long* keys, const unsigned long long* cnts, size_t n, bool sort,
                                   unsigned long long* skeys, unsigned long long* scnts, void* ws, size_t ws_bytes,
                                   uint32_t* nsel, uint32_t* maxcov, hipStream_t st);
hipError_t sid_launch_setup_gather(const unsigned long long* skeys, const unsigned long long* scnts, size_t n,
                                   const void* ws, const uint32_t* nsel, const double* lgk, uint64_t* okeys,
                                   uint32_t* ocnt, double* olnM, unsigned long long* sums, hipStream_t st);
hipError_t sid_launch_class_tables(const uint64_t* keys, uint32_t U, uint32_t* dense_cidx, unsigned long long* ckeys,
                                   uint32_t* cidx, uint64_t cmask, hipStream_t st);
}

static const uint64_t EMPTY = 0xFFFFFFFFFFFFFFFFull;

template <class T>
static void dfree(T*& p)
{
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

// SID_LYNCH_TIMING=1: the estimate's phase times (ms) on stderr, measurement only
static bool lynch_timing()
{
    static const bool on = std::getenv("SID_LYNCH_TIMING") != nullptr;
    return on;
}

struct sid_lynch_dev {
    // accumulation hash (device)
    unsigned long long* gkeys = nullptr;
    unsigned long long* gcnt = nullptr;
    unsigned long long* stats = nullptr;   // [0] distinct, [1] all-65535 profile count, [2] fallback sites
    uint64_t cap = 0;
    uint64_t distinct = 0;                 // upper bound of stats[0]
    // dense-coded profiles (sid_math.h): one u64 counter per code; the other
    // profiles' keys go through the fallback list into the hash
    unsigned long long* dense = nullptr;   // [SID_DENSE_ROWS][SID_DENSE_N]
    uint32_t* part = nullptr;              // per-block rows of the dense pass
    int hist_grid = 256;                   // blocks of the dense pass: 89 us vs 95 us at 512 (hist_probe)
    unsigned long long* list = nullptr;
    uint64_t list_cap = 0;
    hipStream_t acc_stream = nullptr;      // stream of the last accumulate
    bool have_hist = false;
    // explicit (merged) table
    bool loaded = false;
    std::vector<uint64_t> tkeys, tcnt;
    // exported table of the current histogram (sid_profile_table), valid until
    // the next reset / accumulate / load
    bool export_valid = false;
    std::vector<uint64_t> ekeys, ecnt;
    // no profile survived the coverage filter under -m bayes: every site is
    // dropped (callBayes prints the header only, call.cpp:145-211)
    bool empty_classes = false;
    // filtered profiles (device): U of them, sorted by key
    bool setup = false;
    size_t nU = 0;
    bool has_special = false;              // the all-65535 profile is the last one
    double dist[4] = {0.25, 0.25, 0.25, 0.25};
    uint64_t* d_keys = nullptr;
    uint32_t* d_cnt = nullptr;
    double* d_lnM = nullptr;
    int obj_grid = 0;
    bool lookahead = false;                // NM prefetches two iterations' candidates
    uint64_t evals = 0;
    uint64_t launches = 0;
    double* d_partial = nullptr;           // [SID_OBJ_PTS][obj_grid][2]
    // objective results land in host-mapped memory (no copy): {hi, lo} per
    // point and the launch's sequence number per point
    double* h_out = nullptr;
    unsigned int* h_seq = nullptr;
    double* d_out = nullptr;
    unsigned int* d_seq = nullptr;
    unsigned int seq = 0;
    // device-resident estimate (sid_nm_kernel), SID_NM_DEVICE=1; off by
    // default: measured 1.0 ms per estimate vs 0.44 ms host-driven (C3,
    // U = 12k), its rounds bound by cross-XCD synchronisation (barrier
    // 8 us, fold after the L2 invalidate 7 us, simplex step 8 us per round)
    bool nm_device = false;
    int nm_grid = 0;                       // co-resident blocks (one per CU)
    long long nm_timeout = 0;              // wall-clock ticks
    double* d_nmpart = nullptr;            // [2][SID_OBJ_PTS][1024][2]
    unsigned int* d_nmbar = nullptr;       // barrier counter, abort flag
    sid_nm_result* d_nmres = nullptr;
    sid_nm_result* h_nmres = nullptr;      // pinned
    uint64_t nm_rounds = 0, nm_points = 0, nm_fallbacks = 0;
    // class table
    bool prepared = false;
    double* d_lhom = nullptr;
    double* d_lhet = nullptr;
    double* d_c1 = nullptr;
    double* d_c2 = nullptr;
    uint8_t* d_pcode = nullptr;
    unsigned long long* d_ckeys = nullptr;
    uint32_t* d_cidx = nullptr;
    uint32_t* d_dense_cidx = nullptr;      // dense code -> class index (SID_DENSE_NONE: none)
    // grow-only capacities of the buffers above (no hipMalloc/hipFree per call)
    size_t cap_u = 0;                      // U-sized arrays
    size_t cap_c = 0;                      // class hash
    size_t cap_x = 0;                      // export buffer (keys, counts)
    unsigned long long* d_exp = nullptr;   // [cap_x keys][cap_x counts][1 count]
    unsigned long long* d_sexp = nullptr;  // sorted table: [cap_x keys][cap_x counts]
    void* d_setws = nullptr;               // setup scratch (sort, select)
    size_t setws_bytes = 0;
    uint32_t* d_setsc = nullptr;           // {nsel, maxcov} + 5 u64 sums (8-aligned at +8)
    std::vector<double> lg;                // lg[k] = GSL lngamma(k + 1), grown on demand
    double* d_lg = nullptr;                // device copy of lg
    size_t d_lg_n = 0;
    double* d_cc = nullptr;                // {p1, p2} per class, packed for the gather
    double* d_rec = nullptr;               // {p1, p2} per record code (sid_math.h), SID_REC_N, then per dense code
    uint8_t* d_rcode = nullptr;            // code per record code, then per dense code
    void* d_bhws = nullptr;                // device BH scratch (radix sort)
    size_t bhws_bytes = 0;
    int* d_odd = nullptr;                  // BH saw NaN / -0 p-values: host BH instead
    uint64_t cmask = 0;
    uint32_t special_idx = 0xFFFFFFFFu;
    // record tails per class for the engine's fused formatter (sid_lynch_fmt)
    char* d_lstr = nullptr;                // [cap_s][SID_LSTR_BYTES]
    uint8_t* d_dlen = nullptr;             // SID_DENSE_N
    uint32_t* d_strbad = nullptr;          // a confidence the %g cannot print (never a p-value)
    size_t cap_s = 0;
    bool have_str = false;
};

sid_lynch_dev* sid_lynch_dev_create(int* err)
{
    *err = SID_OK;
    return new sid_lynch_dev();
}

static void free_class(sid_lynch_dev* L)
{
    L->prepared = false;
    L->have_str = false;
}

static void free_setup(sid_lynch_dev* L)
{
    L->setup = false;
    free_class(L);
}

static void release_buffers(sid_lynch_dev* L)
{
    dfree(L->d_keys);
    dfree(L->d_cnt);
    dfree(L->d_lnM);
    dfree(L->d_lhom);
    dfree(L->d_lhet);
    dfree(L->d_c1);
    dfree(L->d_c2);
    dfree(L->d_pcode);
    dfree(L->d_cc);
    dfree(L->d_partial);
    dfree(L->d_nmpart);
    dfree(L->d_nmbar);
    dfree(L->d_nmres);
    dfree(L->d_ckeys);
    dfree(L->d_cidx);
    dfree(L->d_dense_cidx);
    dfree(L->d_rec);
    dfree(L->d_rcode);
    dfree(L->d_bhws);
    dfree(L->d_odd);
    dfree(L->d_lstr);
    dfree(L->d_dlen);
    dfree(L->d_strbad);
    L->cap_s = 0;
    L->bhws_bytes = 0;
    dfree(L->d_exp);
    dfree(L->d_sexp);
    dfree(L->d_setws);
    dfree(L->d_setsc);
    dfree(L->d_lg);
    L->setws_bytes = L->d_lg_n = 0;
    L->cap_u = L->cap_c = L->cap_x = 0;
}

void sid_lynch_dev_destroy(sid_lynch_dev* L)
{
    if (!L) return;
    dfree(L->gkeys);
    dfree(L->gcnt);
    dfree(L->stats);
    dfree(L->dense);
    dfree(L->part);
    dfree(L->list);
    if (L->h_out) (void)hipHostFree(L->h_out);
    if (L->h_seq) (void)hipHostFree(L->h_seq);
    if (L->h_nmres) (void)hipHostFree(L->h_nmres);
    release_buffers(L);
    delete L;
}

static int lynch_of(sid_ctx* c, sid_lynch_dev** out)
{
    if (!c) return SID_EINVAL;
    // every Lynch entry point works on the context's device, whichever
    // device the calling thread had current
    if (hipSetDevice(c->device) != hipSuccess) return SID_EHIP;
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
    if (!L->stats) HIPCHECK(hipMalloc(&L->stats, 3 * sizeof(unsigned long long)));
    if (!L->dense) {
        HIPCHECK(hipMalloc(&L->dense, SID_DENSE_ROWS * SID_DENSE_N * sizeof(unsigned long long)));
        HIPCHECK(hipMalloc(&L->part, (size_t)L->hist_grid * SID_DENSE_N * sizeof(uint32_t)));
    }
    HIPCHECK(hipMemsetAsync(L->stats, 0, 3 * sizeof(unsigned long long), st));
    HIPCHECK(hipMemsetAsync(L->dense, 0, SID_DENSE_ROWS * SID_DENSE_N * sizeof(unsigned long long), st));
    if (L->gkeys) {   // keep the allocation, clear it
        HIPCHECK(hipMemsetAsync(L->gkeys, 0xFF, L->cap * sizeof(unsigned long long), st));
        HIPCHECK(hipMemsetAsync(L->gcnt, 0, L->cap * sizeof(unsigned long long), st));
    } else {
        rc = alloc_hash(L, 1ull << 16, st);
        if (rc) return rc;
    }
    L->acc_stream = st;
    L->distinct = 0;
    L->have_hist = true;
    L->loaded = false;
    L->tkeys.clear();
    L->tcnt.clear();
    L->export_valid = false;
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

// countUniqueProfiles (pileup.cpp:169-196), accumulated on the device: the
// dense pass counts the typical profiles and lists the others; the list is
// hashed after growing the hash for it (load factor <= 1/2).  One host sync
// per call (the fallback count).
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
    if (L->acc_stream != st) {   // ordered after work queued on another stream
        HIPCHECK(hipStreamSynchronize(L->acc_stream));
        L->acc_stream = st;
    }
    if (!L->list) {
        L->list_cap = std::min<uint64_t>(std::max<uint64_t>(n / 64, 1u << 16), 1u << 22);
        if (const char* e = std::getenv("SID_HIST_LIST_CAP")) L->list_cap = std::max(1ull, std::strtoull(e, nullptr, 10));
        HIPCHECK(hipMalloc(&L->list, L->list_cap * sizeof(unsigned long long)));
    }
    HIPCHECK(hipMemsetAsync(L->stats + 2, 0, sizeof(unsigned long long), st));
    HIPCHECK(sid_launch_hist_dense(counts, n, L->part, L->dense, L->list, L->list_cap, L->stats + 2, L->hist_grid,
                                   st));
    unsigned long long sv[3] = {0, 0, 0};
    HIPCHECK(hipMemcpyAsync(sv, L->stats, sizeof(sv), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    const uint64_t F = sv[2];
    L->distinct = sv[0];
    if (F) {
        rc = grow_hash(L, 2 * (L->distinct + F), st);
        if (rc) return rc;
        if (F <= L->list_cap) {
            HIPCHECK(sid_launch_hist_list(L->list, F, L->gkeys, L->gcnt, L->cap - 1, L->stats, st));
        } else {   // list overflowed: hash the non-dense sites straight from the counts
            HIPCHECK(sid_launch_hist(counts, n, L->gkeys, L->gcnt, L->cap - 1, L->stats, 1, st));
            HIPCHECK(hipStreamSynchronize(st));
            dfree(L->list);
            L->list_cap = std::min<uint64_t>(F + F / 4, 1ull << 28);
            HIPCHECK(hipMalloc(&L->list, L->list_cap * sizeof(unsigned long long)));
        }
        L->distinct += F;   // upper bound until the next read of stats[0]
    }
    L->export_valid = false;
    free_setup(L);
    return SID_OK;
}

// The current profile table, sorted by key, on the device: *n entries at
// *keys / *cnts (inside d_sexp or d_exp), with the coverage >= 4 selection
// (call.cpp:66-70) left in d_setws and {nsel, maxcov} in d_setsc.  The
// accumulated histogram is compacted (dense codes, then the hash), the
// all-65535 profile appended (it sorts last), and radix-sorted; a loaded
// table is uploaded already sorted.  Two host syncs (the compacted count,
// then nsel/maxcov).
static int device_table(sid_lynch_dev* L, size_t* n, const unsigned long long** keys,
                        const unsigned long long** cnts, uint32_t* nsel, uint32_t* maxcov)
{
    *n = 0;
    *nsel = *maxcov = 0;
    size_t m = 1;
    if (L->loaded) m = std::max<size_t>(L->tkeys.size(), 1);
    else if (L->have_hist) m = L->distinct + SID_DENSE_N + 1;
    if (m > L->cap_x) {
        dfree(L->d_exp);
        dfree(L->d_sexp);
        L->cap_x = std::max(m, 2 * L->cap_x);
        HIPCHECK(hipMalloc(&L->d_exp, (2 * L->cap_x + 1) * sizeof(unsigned long long)));
        HIPCHECK(hipMalloc(&L->d_sexp, 2 * L->cap_x * sizeof(unsigned long long)));
    }
    if (!L->d_setsc) HIPCHECK(hipMalloc(&L->d_setsc, 8 + 5 * sizeof(unsigned long long)));
    unsigned long long *ek = L->d_exp, *ec = L->d_exp + L->cap_x, *nout = L->d_exp + 2 * L->cap_x;
    unsigned long long *sk = L->d_sexp, *sc = L->d_sexp + L->cap_x;
    size_t nn = 0;
    bool sort = true;
    if (L->loaded) {
        nn = L->tkeys.size();
        if (nn) {
            HIPCHECK(hipMemcpyAsync(sk, L->tkeys.data(), nn * 8, hipMemcpyHostToDevice, 0));
            HIPCHECK(hipMemcpyAsync(sc, L->tcnt.data(), nn * 8, hipMemcpyHostToDevice, 0));
        }
        sort = false;
        ek = sk;
        ec = sc;
    } else if (L->have_hist) {
        if (L->acc_stream) HIPCHECK(hipStreamSynchronize(L->acc_stream));
        HIPCHECK(hipMemsetAsync(nout, 0, sizeof(unsigned long long), 0));
        HIPCHECK(sid_launch_dense_compact(L->dense, ek, ec, nout, 0));
        HIPCHECK(sid_launch_compact(L->gkeys, L->gcnt, L->cap, ek, ec, nout, 0));
        unsigned long long hv[3] = {0, 0, 0};   // nout, distinct, special count
        HIPCHECK(hipMemcpyAsync(&hv[0], nout, 8, hipMemcpyDeviceToHost, 0));
        HIPCHECK(hipMemcpyAsync(&hv[1], L->stats, 16, hipMemcpyDeviceToHost, 0));
        HIPCHECK(hipStreamSynchronize(0));
        nn = hv[0];
        if (hv[2]) {
            const unsigned long long sp[2] = {EMPTY, hv[2]};
            HIPCHECK(hipMemcpyAsync(ek + nn, &sp[0], 8, hipMemcpyHostToDevice, 0));
            HIPCHECK(hipMemcpyAsync(ec + nn, &sp[1], 8, hipMemcpyHostToDevice, 0));
            ++nn;
        }
    }
    if (nn == 0) return SID_OK;
    const size_t need = sid_setup_ws_bytes(nn);
    if (need > L->setws_bytes) {
        dfree(L->d_setws);
        L->setws_bytes = 0;
        const size_t sz = std::max(need, 2 * L->setws_bytes);
        L->setws_bytes = 0;
        HIPCHECK(hipMalloc(&L->d_setws, sz));
        L->setws_bytes = sz;
    }
    HIPCHECK(sid_launch_setup_select(ek, ec, nn, sort, sk, sc, L->d_setws, L->setws_bytes, L->d_setsc,
                                     L->d_setsc + 1, 0));
    uint32_t hs[2] = {0, 0};
    HIPCHECK(hipMemcpyAsync(hs, L->d_setsc, 8, hipMemcpyDeviceToHost, 0));
    HIPCHECK(hipStreamSynchronize(0));   // also orders the pageable uploads above
    *n = nn;
    *keys = sk;
    *cnts = sc;
    *nsel = hs[0];
    *maxcov = hs[1];
    return SID_OK;
}

static int current_table(sid_lynch_dev* L, std::vector<uint64_t>& keys, std::vector<uint64_t>& cnt)
{
    keys.clear();
    cnt.clear();
    if (L->loaded) {
        keys = L->tkeys;
        cnt = L->tcnt;
        return SID_OK;
    }
    if (!L->have_hist) return SID_OK;
    if (!L->export_valid) {   // one export per histogram (compaction, sort, syncs)
        size_t n;
        const unsigned long long *k, *v;
        uint32_t ns, mc;
        int rc = device_table(L, &n, &k, &v, &ns, &mc);
        if (rc) return rc;
        L->ekeys.resize(n);
        L->ecnt.resize(n);
        if (n) {
            HIPCHECK(hipMemcpyAsync(L->ekeys.data(), k, n * 8, hipMemcpyDeviceToHost, 0));
            HIPCHECK(hipMemcpyAsync(L->ecnt.data(), v, n * 8, hipMemcpyDeviceToHost, 0));
            HIPCHECK(hipStreamSynchronize(0));
        }
        L->export_valid = true;   // until the histogram changes
    }
    keys = L->ekeys;
    cnt = L->ecnt;
    return SID_OK;
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
    L->export_valid = false;
    free_setup(L);
    return SID_OK;
}

extern "C" int sid_lynch_setup(sid_ctx* c, sid_estimate* est)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    if (!L->setup) {
        free_setup(L);
        size_t n = 0;
        const unsigned long long *k = nullptr, *v = nullptr;
        uint32_t U32 = 0, maxcov = 0;
        rc = device_table(L, &n, &k, &v, &U32, &maxcov);
        if (rc) return rc;
        const size_t U = U32;
        // GSL lngamma(k + 1) for every count that occurs (the coverages bound
        // them), computed once per context on the host and kept on the device
        if (U && maxcov >= L->lg.size()) {
            size_t n0 = L->lg.size(), n1 = std::max<size_t>(maxcov + 1, 2 * n0);
            L->lg.resize(n1);
            for (size_t i = n0; i < n1; ++i) L->lg[i] = sid_gsl_lngamma((double)(i + 1));
        }
        if (U && L->lg.size() > L->d_lg_n) {
            dfree(L->d_lg);
            L->d_lg_n = 0;
            HIPCHECK(hipMalloc(&L->d_lg, L->lg.size() * 8));
            HIPCHECK(hipMemcpy(L->d_lg, L->lg.data(), L->lg.size() * 8, hipMemcpyHostToDevice));
            L->d_lg_n = L->lg.size();
        }
        if (U > L->cap_u || !L->d_keys) {   // every U-sized array, grow-only
            const size_t m = std::max<size_t>({U, 2 * L->cap_u, 1024});
            dfree(L->d_keys);
            dfree(L->d_cnt);
            dfree(L->d_lnM);
            dfree(L->d_lhom);
            dfree(L->d_lhet);
            dfree(L->d_c1);
            dfree(L->d_c2);
            dfree(L->d_pcode);
            dfree(L->d_cc);
            HIPCHECK(hipMalloc(&L->d_keys, m * 8));
            HIPCHECK(hipMalloc(&L->d_cnt, m * 4));
            HIPCHECK(hipMalloc(&L->d_lnM, m * 8));
            HIPCHECK(hipMalloc(&L->d_lhom, m * 8));
            HIPCHECK(hipMalloc(&L->d_lhet, m * 8));
            HIPCHECK(hipMalloc(&L->d_c1, m * 8));
            HIPCHECK(hipMalloc(&L->d_c2, m * 8));
            HIPCHECK(hipMalloc(&L->d_pcode, m));
            HIPCHECK(hipMalloc(&L->d_cc, m * 16));
            L->cap_u = m;
        }
        // pileup.cpp:198-217 distribution (32-bit products, 64-bit sums) and
        // lynch.hpp:48-55 lnM per profile, gathered in key order
        unsigned long long acc[5] = {0, 0, 0, 0, 0};
        bool special = false;
        if (U) {
            unsigned long long* sums = (unsigned long long*)(L->d_setsc + 2);
            HIPCHECK(sid_launch_setup_gather(k, v, n, L->d_setws, L->d_setsc, L->d_lg, L->d_keys, L->d_cnt,
                                             L->d_lnM, sums, 0));
            uint64_t last = 0;
            HIPCHECK(hipMemcpyAsync(acc, sums, sizeof(acc), hipMemcpyDeviceToHost, 0));
            HIPCHECK(hipMemcpyAsync(&last, L->d_keys + (U - 1), 8, hipMemcpyDeviceToHost, 0));
            HIPCHECK(hipStreamSynchronize(0));
            special = last == EMPTY;
        }
        for (int j = 0; j < 4; ++j) L->dist[j] = acc[4] ? (double)acc[j] / (double)acc[4] : 0.25;
        L->nU = U;
        L->has_special = special;
        L->obj_grid = (int)std::min<size_t>(1024, std::max<size_t>(1, (U + 255) / 256));
        // two-iteration prefetch (up to 28 points per launch) while the points
        // still fit the chip alongside each other (U x 28 profile-points);
        // SID_NM_LOOKAHEAD=0/1 overrides (measurement)
        L->lookahead = U <= 32768;
        if (const char* e = std::getenv("SID_NM_LOOKAHEAD")) L->lookahead = std::atoi(e) != 0;
        if (const char* e = std::getenv("SID_NM_DEVICE")) L->nm_device = std::atoi(e) != 0;
        if (!L->d_partial) HIPCHECK(hipMalloc(&L->d_partial, SID_OBJ_PTS * 2 * 1024 * sizeof(double)));
        if (!L->h_out) {
            HIPCHECK(hipHostMalloc((void**)&L->h_out, 2 * SID_OBJ_PTS * sizeof(double),
                                   hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHECK(hipHostMalloc((void**)&L->h_seq, SID_OBJ_PTS * sizeof(unsigned int),
                                   hipHostMallocMapped | hipHostMallocCoherent));
            std::memset(L->h_seq, 0, SID_OBJ_PTS * sizeof(unsigned int));
            HIPCHECK(hipHostGetDevicePointer((void**)&L->d_out, L->h_out, 0));
            HIPCHECK(hipHostGetDevicePointer((void**)&L->d_seq, L->h_seq, 0));
        }
        L->evals = 0;
        L->setup = true;
    }
    if (est) {
        std::memset(est, 0, sizeof(*est));
        std::memcpy(est->dist, L->dist, sizeof(L->dist));
        est->n_unique = L->nU;
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

// lynch.cpp:37-61 at k <= SID_OBJ_PTS points in one launch.  Out-of-range
// points return DBL_MAX without evaluation (lynch.cpp:40-42).
static int objective_batch(sid_ctx* c, const double (*x)[2], int k, double* out)
{
    sid_lynch_dev* L = c->lynch;
    const size_t U = L->nU;
    sid_lynch_evals EV;
    int idx[SID_OBJ_PTS];
    int m = 0;
    if (k > SID_OBJ_PTS) return SID_EINVAL;
    for (int i = 0; i < k; ++i) {
        const double pi = x[i][0], eps = x[i][1];
        if (pi < 0 || pi > 1 || eps < 0 || eps > 1) {
            out[i] = DBL_MAX;
        } else if (U == 0) {
            out[i] = -0.0;   // static_cast<double>(-0.0L)
        } else {
            sid_lynch_eval E;
            make_eval(L->dist, pi, eps, &E);
            if (m == 0) {
                std::memcpy(EV.ld, E.ld, sizeof(EV.ld));
                std::memcpy(EV.ldd, E.ldd, sizeof(EV.ldd));
                EV.lnorm = E.lnorm;
            }
            EV.p[m] = {E.la, E.lb, E.lh, E.l1p, E.lp};
            idx[m++] = i;
        }
    }
    if (m == 0) return SID_OK;
    const unsigned int seq = ++L->seq;
    L->launches++;
    HIPCHECK(sid_launch_objective(L->d_keys, L->d_cnt, L->d_lnM, U, &EV, m, L->d_partial, L->d_out, L->d_seq, seq,
                                  L->obj_grid, 0));
    // poll the mapped sequence numbers; the stream status is the backstop
    auto ready = [&] {
        for (int j = 0; j < m; ++j)
            if (__atomic_load_n(&L->h_seq[j], __ATOMIC_ACQUIRE) != seq) return false;
        return true;
    };
    for (uint64_t spin = 0; !ready(); ++spin) {
        if ((spin & 255) != 255) continue;
        const hipError_t q = hipStreamQuery(0);
        if (q == hipErrorNotReady) continue;
        if (q != hipSuccess) return sid_set_hip_error(q);
        if (!ready()) return sid_set_hip_error(hipErrorUnknown);   // finished without its result
        break;
    }
    for (int j = 0; j < m; ++j) {
        long double sum = (long double)L->h_out[2 * j] + (long double)L->h_out[2 * j + 1];
        if (std::isinf((double)sum)) sum = sum > 0 ? LDBL_MAX : -LDBL_MAX;
        out[idx[j]] = (double)(-sum);
    }
    return SID_OK;
}

static int objective(sid_ctx* c, double pi, double eps, double* out)
{
    const double x[1][2] = {{pi, eps}};
    return objective_batch(c, x, 1, out);
}

extern "C" int sid_lynch_objective(sid_ctx* c, double pi, double eps, double* out)
{
    if (!c || !out) return SID_EINVAL;
    int rc = sid_lynch_setup(c, nullptr);
    if (rc) return rc;
    return objective(c, pi, eps, out);
}

// ---------------------------------------------------------------------------
// Nelder-Mead driven from the host: GSL 2.7.1 multimin/nmsimplex2.c for 2
// parameters, vertex arithmetic from sid_nm.h (shared with the device-resident
// estimate, sid_nm_kernel), one objective launch per prefetch.
// ---------------------------------------------------------------------------
namespace {
struct Simplex {
    static const int N = SID_NM_N, P = SID_NM_P;
    sid_nm_simplex s;
    sid_ctx* ctx;
    int err = SID_OK;

    // Objective values of the points the next step may ask for, evaluated in
    // one launch (prefetch).  The objective is a pure function of the point,
    // so f() returning a prefetched value changes nothing in the trajectory.
    double cx[SID_OBJ_PTS][N], cv[SID_OBJ_PTS];
    int cn = 0;

    void prefetch(const double (*pts)[N], int k)
    {
        cn = 0;
        if (err) return;
        k = std::min(k, (int)SID_OBJ_PTS);
        int rc = objective_batch(ctx, pts, k, cv);
        if (rc) {
            err = rc;
            return;
        }
        for (int i = 0; i < k; ++i) {
            cx[i][0] = pts[i][0];
            cx[i][1] = pts[i][1];
        }
        cn = k;
    }
    bool cached(const double* x) const
    {
        for (int i = 0; i < cn; ++i)
            if (cx[i][0] == x[0] && cx[i][1] == x[1]) return true;
        return false;
    }
    double f(const double* x)
    {
        ctx->lynch->evals++;
        for (int i = 0; i < cn; ++i)
            if (cx[i][0] == x[0] && cx[i][1] == x[1]) return cv[i];
        double v = 0;
        int rc = objective(ctx, x[0], x[1], &v);
        if (rc && !err) err = rc;
        return v;
    }
    double corner_move(double coeff, int corner, double* xc)
    {
        sid_nm_corner_point(s, coeff, corner, xc);
        return f(xc);
    }
    bool contract_by_best(int best)
    {
        double pts[P][N];
        int k = 0;
        for (int i = 0; i < P; ++i) {
            if (i == best) continue;
            for (int j = 0; j < N; ++j) pts[k][j] = 0.5 * (s.x1[i][j] + s.x1[best][j]);
            ++k;
        }
        prefetch(pts, k);
        bool ok = true;
        for (int i = 0; i < P; ++i) {
            if (i == best) continue;
            for (int j = 0; j < N; ++j) s.x1[i][j] = 0.5 * (s.x1[i][j] + s.x1[best][j]);
            double xc[N] = {s.x1[i][0], s.x1[i][1]};
            s.y1[i] = f(xc);
            if (!std::isfinite(s.y1[i])) ok = false;
        }
        sid_nm_compute_center(s);
        sid_nm_compute_size(s);
        return ok;
    }
    bool set(const double* x, const double* step, double* size)
    {
        double pts[P][N] = {{x[0], x[1]}, {x[0] + step[0], x[1]}, {x[0], x[1] + step[1]}};
        prefetch(pts, P);
        double v = f(x);
        if (!std::isfinite(v)) return false;
        s.x1[0][0] = x[0];
        s.x1[0][1] = x[1];
        s.y1[0] = v;
        for (int i = 0; i < N; ++i) {
            double xt[N] = {x[0], x[1]};
            xt[i] = x[i] + step[i];
            v = f(xt);
            if (!std::isfinite(v)) return false;
            s.x1[i + 1][0] = xt[0];
            s.x1[i + 1][1] = xt[1];
            s.y1[i + 1] = v;
        }
        sid_nm_compute_center(s);
        *size = sid_nm_compute_size(s);
        return true;
    }
    bool iterate(double* x, double* size, double* fval)
    {
        double xc[N], xc2[N];
        int hi, s_hi, lo;
        sid_nm_order(s, hi, s_hi, lo);
        {
            double c1[4][N];
            sid_nm_candidates(s, hi, c1);
            if (!(cached(c1[0]) && cached(c1[1]) && cached(c1[2]) && cached(c1[3]))) {
                double pts[SID_OBJ_PTS][N];
                int k = sid_nm_request(s, ctx->lynch->lookahead, pts, SID_OBJ_PTS);
                prefetch(pts, k);
            }
        }
        double val = corner_move(-1.0, hi, xc);
        if (std::isfinite(val) && val < s.y1[lo]) {
            double val2 = corner_move(-2.0, hi, xc2);
            if (std::isfinite(val2) && val2 < s.y1[lo])
                sid_nm_update_point(s, hi, xc2, val2);
            else
                sid_nm_update_point(s, hi, xc, val);
        } else if (!std::isfinite(val) || val > s.y1[s_hi]) {
            if (std::isfinite(val) && val <= s.y1[hi]) sid_nm_update_point(s, hi, xc, val);
            double val2 = corner_move(0.5, hi, xc2);
            if (std::isfinite(val2) && val2 <= s.y1[hi]) {
                sid_nm_update_point(s, hi, xc2, val2);
            } else if (!contract_by_best(lo)) {
                return false;
            }
        } else {
            sid_nm_update_point(s, hi, xc, val);
        }
        const int imin = sid_nm_min_index(s);
        x[0] = s.x1[imin][0];
        x[1] = s.x1[imin][1];
        *fval = s.y1[imin];
        *size = s.S2 > 0 ? std::sqrt(s.S2) : sid_nm_compute_size(s);
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
    L->launches = 0;
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

// lynch.cpp:17-35 + optimization.hpp:50-89 in one cooperative launch
// (lynch.hip sid_nm_kernel).  Returns SID_OK with *done = false when the
// device estimate is unavailable (cooperative launch refused, deadline):
// the caller then runs the host driver.
static int run_estimate_device(sid_ctx* c, int verbose, sid_estimate* est, bool* done)
{
    sid_lynch_dev* L = c->lynch;
    *done = false;
    if (!L->d_nmpart) {
        int ncu = 0, coop = 0, khz = 0;
        HIPCHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
        HIPCHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, c->device));
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0)
            khz = 100000;
        if (!coop || ncu < 1) {
            L->nm_device = false;
            return SID_OK;
        }
        L->nm_grid = ncu;
        L->nm_timeout = (long long)khz * 1000 * 5;   // 5 s: the estimate takes < 1 ms
        HIPCHECK(hipMalloc(&L->d_nmpart, (size_t)2 * SID_OBJ_PTS * 1024 * 2 * sizeof(double)));
        HIPCHECK(hipMalloc(&L->d_nmbar, 2 * sizeof(unsigned int)));
        HIPCHECK(hipMalloc(&L->d_nmres, sizeof(sid_nm_result)));
        HIPCHECK(hipHostMalloc((void**)&L->h_nmres, sizeof(sid_nm_result), hipHostMallocDefault));
    }
    sid_lynch_eval E;
    make_eval(L->dist, 0.5, 0.5, &E);   // only the dist-only constants are used
    sid_nm_dist D;
    std::memcpy(D.ld, E.ld, sizeof(D.ld));
    std::memcpy(D.ldd, E.ldd, sizeof(D.ldd));
    D.lnorm = E.lnorm;
    const double x0[2] = {1e-3, 1e-3};   // DEFAULT_PI, DEFAULT_EPSILON  lynch.cpp:8-10
    const double step[2] = {1e-4, 1e-4}; // DEFAULT_STEPSIZE
    hipError_t e = sid_launch_nm(L->d_keys, L->d_cnt, L->d_lnM, L->nU, L->obj_grid, &D, x0, step, L->lookahead ? 1 : 0,
                                 L->d_nmpart, L->d_nmbar, L->nm_grid, L->nm_timeout, L->d_nmres, 0);
    if (e == hipErrorCooperativeLaunchTooLarge || e == hipErrorNotSupported) {
        (void)hipGetLastError();
        L->nm_device = false;
        return SID_OK;
    }
    HIPCHECK(e);
    HIPCHECK(hipMemcpyAsync(L->h_nmres, L->d_nmres, sizeof(sid_nm_result), hipMemcpyDeviceToHost, 0));
    HIPCHECK(hipStreamSynchronize(0));
    const sid_nm_result r = *L->h_nmres;
    L->nm_rounds = (uint64_t)r.rounds;
    L->nm_points = r.points;
    if (lynch_timing())
        std::fprintf(stderr, "{\"nm_ticks\": [%lld, %lld, %lld, %lld]}\n", r.ticks[0], r.ticks[1], r.ticks[2],
                     r.ticks[3]);
    L->launches = 1;
    if (r.status >= 2) {   // deadline, round cap, internal: the host driver decides
        L->nm_fallbacks++;
        return SID_OK;
    }
    L->evals = r.evals;
    if (r.status == 1) return SID_EBADFUNC;   // non-finite at the start, or "contraction failed"
    *done = true;
    const int i = r.iterations;
    if (verbose) {
        if (r.converged)
            std::fprintf(stderr, "# GSL function minimization converged in %d iterations.\n", i);
        else
            std::fprintf(stderr, "# Error: GSL function minimization did not converge in %d iterations!\n", i);
    }
    est->heterozygosity = r.x[0];
    est->error_rate = r.x[1];
    est->fval = r.fval;
    est->iterations = i;
    est->converged = r.converged;
    est->evaluations = r.evals;
    return SID_OK;
}

extern "C" int sid_lynch_prepare(sid_ctx* c, int verbose, sid_estimate* est_out)
{
    return sid_lynch_prepare_given(c, verbose, nullptr, est_out);
}

// The estimate (pi-hat, eps-hat) may come from another device or rank that ran
// the Nelder-Mead on the same merged table (one
// estimate, broadcast): then only the per-profile classification runs here.
extern "C" int sid_lynch_prepare_given(sid_ctx* c, int verbose, const sid_estimate* given, sid_estimate* est_out)
{
    sid_lynch_dev* L;
    int rc = lynch_of(c, &L);
    if (rc) return rc;
    const bool timing = lynch_timing();
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = now();
    sid_estimate est;
    rc = sid_lynch_setup(c, &est);
    if (rc) return rc;
    const auto t1 = now();
    const int method = c->opts.method;
    const size_t U = L->nU;
    // the -R estimate of local and quality prints only the minimiser's line
    const bool local_like = method == SID_METHOD_LOCAL || method == SID_METHOD_QUALITY;
    if (verbose && !local_like) std::fprintf(stderr, "# unique profiles: %zu\n", U);
    bool done = false;
    if (given) {
        const uint64_t nu = est.n_unique;
        double dist[4];
        std::memcpy(dist, est.dist, sizeof dist);
        est = *given;
        est.n_unique = nu;
        std::memcpy(est.dist, dist, sizeof dist);
        done = true;
    }
    if (!done && L->nm_device && U > 0) {
        rc = run_estimate_device(c, verbose, &est, &done);
        if (rc) return rc;
    }
    if (!done) {
        rc = run_estimate(c, verbose, &est);
        if (rc) return rc;
    }
    const auto t2 = now();
    if (est_out) *est_out = est;
    if (local_like) return SID_OK;   // -R local / quality: the caller applies the prior
    if (verbose) {
        std::fprintf(stderr, "# heterozygosity: %e\n", est.heterozygosity);
        std::fprintf(stderr, "# error: %e\n", est.error_rate);
    }
    free_class(L);
    L->empty_classes = false;
    if (U == 0) {
        // likelihood_ratio: adjustBenjaminiHochberg reads sorted[0] of an
        // empty vector (stats.cpp:73) and the reference crashes; bayes never
        // adjusts and prints no record at all (call.cpp:145-211)
        if (method == SID_METHOD_LIKELIHOOD_RATIO) return SID_EEMPTY;
        L->empty_classes = true;
        L->prepared = true;
        return SID_OK;
    }
    sid_lynch_eval E;
    make_eval(L->dist, est.heterozygosity, est.error_rate, &E);
    HIPCHECK(sid_launch_profile_lik(L->d_keys, L->d_lnM, U, &E, L->d_lhom, L->d_lhet, 0));
    const int mode = method == SID_METHOD_BAYES ? 1 : 0;
    HIPCHECK(sid_launch_classify(L->d_keys, L->d_lhom, L->d_lhet, U, mode,
                                 method == SID_METHOD_LIKELIHOOD_RATIO && c->opts.estimate_prior,
                                 est.heterozygosity, c->K.lg15, L->d_c1, L->d_c2, L->d_pcode, 0));
    bool host_bh = mode == 0;
    if (mode == 0) {
        // stats.cpp:58-80 on the device (radix sort + min-scan), adjusted
        // values into the likelihood arrays (no longer needed), then swapped in
        const size_t need = sid_bh_ws_bytes(U);
        if (need > L->bhws_bytes) {
            dfree(L->d_bhws);
            L->bhws_bytes = 0;
            HIPCHECK(hipMalloc(&L->d_bhws, need));
            L->bhws_bytes = need;
        }
        if (!L->d_odd) HIPCHECK(hipMalloc(&L->d_odd, sizeof(int)));
        HIPCHECK(hipMemsetAsync(L->d_odd, 0, sizeof(int), 0));
        HIPCHECK(sid_launch_bh(L->d_c1, L->d_c2, U, L->d_lhom, L->d_lhet, L->d_bhws, L->bhws_bytes, L->d_odd, 0));
        int odd = 0;
        HIPCHECK(hipMemcpyAsync(&odd, L->d_odd, sizeof(int), hipMemcpyDeviceToHost, 0));
        HIPCHECK(hipStreamSynchronize(0));
        if (!odd) {
            HIPCHECK(sid_launch_bh_label(L->d_lhet, U, c->opts.significance_level, L->d_pcode, 0));
            std::swap(L->d_c1, L->d_lhom);
            std::swap(L->d_c2, L->d_lhet);
            host_bh = false;
        }
    }
    if (host_bh) {
        // stats.cpp:58-80 Benjamini-Hochberg over the U p-values, then
        // call.cpp:113-127 labels from the adjusted p_het
        std::vector<double> ph(U), pt(U);
        std::vector<uint8_t> code(U);
        HIPCHECK(hipMemcpyAsync(ph.data(), L->d_c1, U * 8, hipMemcpyDeviceToHost, 0));
        HIPCHECK(hipMemcpyAsync(pt.data(), L->d_c2, U * 8, hipMemcpyDeviceToHost, 0));
        HIPCHECK(hipMemcpyAsync(code.data(), L->d_pcode, U, hipMemcpyDeviceToHost, 0));
        HIPCHECK(hipStreamSynchronize(0));
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
        HIPCHECK(hipMemcpyAsync(L->d_c1, ah.data(), U * 8, hipMemcpyHostToDevice, 0));
        HIPCHECK(hipMemcpyAsync(L->d_c2, at.data(), U * 8, hipMemcpyHostToDevice, 0));
        HIPCHECK(hipMemcpyAsync(L->d_pcode, code.data(), U, hipMemcpyHostToDevice, 0));
        HIPCHECK(hipStreamSynchronize(0));   // the host vectors go out of scope
    }
    const auto t3 = now();
    // compact class hash over the U filtered profiles (the all-65535 one is
    // special_idx) and dense code -> class index for the lookup fast path
    uint64_t cap = 16;
    while (cap < 2 * U) cap <<= 1;
    if (cap > L->cap_c) {
        dfree(L->d_ckeys);
        dfree(L->d_cidx);
        L->cap_c = 0;
        HIPCHECK(hipMalloc(&L->d_ckeys, cap * 8));
        HIPCHECK(hipMalloc(&L->d_cidx, cap * 4));
        L->cap_c = cap;
    }
    if (!L->d_dense_cidx) HIPCHECK(hipMalloc(&L->d_dense_cidx, SID_DENSE_N * 4));
    L->cmask = cap - 1;
    L->special_idx = L->has_special ? (uint32_t)(U - 1) : 0xFFFFFFFFu;
    HIPCHECK(sid_launch_class_tables(L->d_keys, (uint32_t)U, L->d_dense_cidx, L->d_ckeys, L->d_cidx, L->cmask, 0));
    HIPCHECK(sid_launch_pack_class(L->d_c1, L->d_c2, U, L->d_cc, 0));
    if (!L->d_rec) {
        HIPCHECK(hipMalloc(&L->d_rec, (SID_REC_N + SID_DENSE_N) * 16));
        HIPCHECK(hipMalloc(&L->d_rcode, SID_REC_N + SID_DENSE_N));
    }
    HIPCHECK(sid_launch_rec_build(L->d_dense_cidx, L->d_pcode, L->d_cc, L->d_rec, L->d_rcode, 0));
    // the classes' record tails for the engine's fused formatter
    if (U > L->cap_s) {
        dfree(L->d_lstr);
        L->cap_s = 0;
        HIPCHECK(hipMalloc(&L->d_lstr, U * SID_LSTR_BYTES));
        L->cap_s = U;
    }
    if (!L->d_dlen) HIPCHECK(hipMalloc(&L->d_dlen, SID_DENSE_N));
    if (!L->d_strbad) HIPCHECK(hipMalloc(&L->d_strbad, 4));
    HIPCHECK(hipMemsetAsync(L->d_strbad, 0, 4, 0));
    HIPCHECK(sid_launch_lynch_str_build(L->d_pcode, L->d_cc, (uint32_t)U, mode == 1 ? "probability" : "p_value",
                                        L->d_dense_cidx, L->d_lstr, L->d_dlen, L->d_strbad, 0));
    uint32_t strbad = 0;
    HIPCHECK(hipMemcpyAsync(&strbad, L->d_strbad, 4, hipMemcpyDeviceToHost, 0));
    HIPCHECK(hipStreamSynchronize(0));
    L->have_str = strbad == 0;
    L->prepared = true;
    if (timing)
        std::fprintf(stderr,
                     "{\"lynch_prepare_ms\": {\"setup\": %.3f, \"estimate\": %.3f, \"evaluations\": %llu, "
                     "\"launches\": %llu, \"nm_device\": %d, \"nm_rounds\": %llu, \"nm_points\": %llu, "
                     "\"classify_bh\": %.3f, \"class_tables\": %.3f}}\n",
                     ms(t0, t1), ms(t1, t2), (unsigned long long)est.evaluations, (unsigned long long)L->launches,
                     (int)L->nm_device, (unsigned long long)L->nm_rounds, (unsigned long long)L->nm_points,
                     ms(t2, t3), ms(t3, now()));
    return SID_OK;
}

int sid_lynch_fmt_view(const sid_ctx* c, sid_lynch_fmt* v)
{
    const sid_lynch_dev* L = c ? c->lynch : nullptr;
    if (!L || !L->prepared || !v) return SID_ESTATE;
    const int m = c->opts.method;
    if (m != SID_METHOD_LIKELIHOOD_RATIO && m != SID_METHOD_BAYES) return SID_ESTATE;
    if (!L->empty_classes && !L->have_str) return SID_ESTATE;
    v->dense_cidx = L->d_dense_cidx;
    v->ckeys = L->d_ckeys;
    v->cidx = L->d_cidx;
    v->cmask = L->cmask;
    v->special_idx = L->special_idx;
    v->lstr = L->d_lstr;
    v->dlen = L->d_dlen;
    v->empty = L->empty_classes ? 1 : 0;
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
    if (hipSetDevice(c->device) != hipSuccess) return SID_EHIP;
    if (L->empty_classes) {   // no class: every site dropped (code bit 6)
        HIPCHECK(hipMemsetAsync(code, SID_CODE_DROPPED, n, (hipStream_t)stream));
        return SID_OK;
    }
    HIPCHECK(sid_launch_lookup(counts, n, L->d_ckeys, L->d_cidx, L->cmask, L->special_idx, L->d_pcode,
                               L->d_c1, L->d_c2, L->d_rec, L->d_rcode, L->d_cc, code, hom_conf, het_conf, c->grid_cap,
                               (hipStream_t)stream));
    return SID_OK;
}
