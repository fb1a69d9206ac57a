// capi.cpp — C ABI of libsid.so: status, options, contexts, -m local,
// synthetic input.  The Lynch-path entry points live in lynch_host.cpp, the
// parser in parse.cpp, the CSV emitter in emit.cpp.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sid_internal.h"
#include "synth.h"

// process-wide: the streaming engine's worker threads report through it
static std::atomic<int> g_last_hip_error{0};

int sid_set_hip_error(hipError_t e)
{
    g_last_hip_error.store((int)e);
    return e == hipErrorOutOfMemory ? SID_ENOMEM : SID_EHIP;
}

extern "C" int sid_last_hip_error(void) { return g_last_hip_error.load(); }

extern "C" const char* sid_strerror(int status)
{
    switch (status) {
    case SID_OK: return "ok";
    case SID_EINVAL: return "invalid argument";
    case SID_EHIP: return "HIP runtime error";
    case SID_ENOMEM: return "out of memory";
    case SID_EMALFORMED: return "Malformed pileup line";
    case SID_EMISSING_MQ: return "Malformed pileup line or missing mapping qualities";
    case SID_ENULLCHROM: return "line without a chromosome field";
    case SID_ESTATE: return "call order violated";
    case SID_EBADFUNC: return "non-finite function value encountered";
    case SID_EEMPTY: return "no profile with coverage >= 4";
    case SID_EIO: return "output write failed";
    case SID_ERANGE: return "value outside the device formatter's range";
    case SID_ENOBQ: return "no base-quality field";
    case SID_ELINE: return "a pileup line too long for one chunk (4 GiB)";
    default: return "unknown status";
    }
}

extern "C" const char* sid_version(void) { return "sid-mi355x 0.1.0 (gfx950)"; }

// sid.cpp:11-17 defaults
extern "C" void sid_opts_default(sid_opts* o)
{
    if (!o) return;
    o->method = SID_METHOD_LOCAL;
    o->estimate_prior = 0;
    o->snp_prior = -1;
    o->significance_level = 0.05;
    o->site_error_threshold = 0.1;
}

// GSL 2.7.1 specfunc/gamma.c lngamma_lanczos (x >= 0.5, away from 1 and 2,
// where the Pade branches return exactly 0 at the integers).
double sid_gsl_lngamma(double x)
{
    if (x == 1.0 || x == 2.0) return 0.0;
    static const double c[9] = {
        0.99999999999980993227684700473478,  676.520368121885098567009190444019,
        -1259.13921672240287047156078755283, 771.3234287776530788486528258894,
        -176.61502916214059906584551354,     12.507343278686904814458936853,
        -0.13857109526572011689554707,       9.984369578019570859563e-6,
        1.50563273514931155834e-7};
    x -= 1.0;
    double Ag = c[0];
    for (int k = 1; k <= 8; k++) Ag += c[k] / (x + k);
    double term1 = (x + 0.5) * std::log((x + 7.0 + 0.5) / M_E);
    double term2 = 0.9189385332046727418 + std::log(Ag);
    return term1 + (term2 - 7.0);
}

void sid_build_local_k(const sid_opts& o, sid_local_k* K)
{
    const double E = o.site_error_threshold;
    K->E = E;
    K->sig = o.significance_level;
    // capped bases, computed from the same doubles the reference feeds powl
    K->cA1 = std::log(1 - E);
    K->cB1 = std::log(E / 3.);
    K->cA2 = std::log((1 - 2. / 3. * E) / 2.);
    K->cB2 = K->cB1;
    K->prior = o.snp_prior;
    K->prior_on = o.snp_prior > 0;
    K->lp1 = K->prior_on ? std::log(std::fabs(1 - o.snp_prior)) : 0.0;
    K->lp2 = K->prior_on ? std::log(o.snp_prior) : 0.0;
    K->lg15 = sid_gsl_lngamma(1.5);
    // negative bases (E < 0) or a negative prior factor need signed long
    // double emulation on every site
    K->general = (E < 0) || (K->prior_on && (1 - o.snp_prior) < 0);
}

extern "C" int sid_device_count(int* n)
{
    if (!n) return SID_EINVAL;
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) {
        *n = 0;
        return sid_set_hip_error(e);
    }
    return SID_OK;
}

// class table of the -m local fast path for the context's options
static hipError_t sid_build_table(sid_ctx* c)
{
    if (c->K.general) return hipSuccess;
    hipError_t e = sid_launch_local_table_build(&c->K, c->d_lnt, c->ws.table, c->ws.table2, nullptr);
    if (e == hipSuccess) e = sid_launch_local_str_build(&c->K, c->ws.table, c->ws.table2, &c->ws, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e;
}

extern "C" int sid_create(int device, const sid_opts* opts, sid_ctx** out)
{
    if (!out) return SID_EINVAL;
    *out = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return sid_set_hip_error(e);
    sid_ctx* c = new sid_ctx();
    c->device = device;
    if (opts) c->opts = *opts; else sid_opts_default(&c->opts);
    sid_build_local_k(c->opts, &c->K);
    // SID_TABLE_TAIL=0: the second-level class table off, its sites through
    // the fix-up (tests/test_local_gpu.py covers both)
    if (const char* g = std::getenv("SID_TABLE_TAIL")) c->ws.tail = std::atoi(g) != 0;

    std::vector<double> lnt(SID_LUTN);
    lnt[0] = -INFINITY;
    for (int k = 1; k < SID_LUTN; ++k) lnt[k] = std::log((double)k);
    const size_t tab = 8192;   // SID_TAB_N (local.hip)
    c->ws.cap = 4u << 20;
    e = hipMalloc(&c->d_lnt, SID_LUTN * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(c->d_lnt, lnt.data(), SID_LUTN * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&c->ws.table, tab * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&c->ws.table2, SID_TAB2_N * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&c->ws.str1, tab * SID_STR_BYTES);
    if (e == hipSuccess) e = hipMalloc(&c->ws.len1, tab);
    if (e == hipSuccess) e = hipMalloc(&c->ws.str2, (size_t)SID_TAB2_N * SID_STR_BYTES);
    if (e == hipSuccess) e = hipMalloc(&c->ws.len2, SID_TAB2_N);
    if (e == hipSuccess) e = hipMalloc(&c->ws.miss, (size_t)c->ws.cap * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&c->ws.ctr, 2 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(c->ws.ctr, 0, 2 * sizeof(uint32_t));
    if (e == hipSuccess) e = sid_build_table(c);
    if (e != hipSuccess) {
        int rc = sid_set_hip_error(e);
        sid_destroy(c);
        return rc;
    }
    *out = c;
    return SID_OK;
}

extern "C" int sid_destroy(sid_ctx* c)
{
    if (!c) return SID_OK;
    (void)hipSetDevice(c->device);
    if (c->d_lnt) (void)hipFree(c->d_lnt);
    if (c->d_cdf) (void)hipFree(c->d_cdf);
    if (c->ws.table) (void)hipFree(c->ws.table);
    if (c->ws.table2) (void)hipFree(c->ws.table2);
    for (void* p : {(void*)c->ws.str1, (void*)c->ws.len1, (void*)c->ws.str2, (void*)c->ws.len2})
        if (p) (void)hipFree(p);
    if (c->ws.miss) (void)hipFree(c->ws.miss);
    if (c->ws.ctr) (void)hipFree(c->ws.ctr);
    if (c->lynch) sid_lynch_dev_destroy(c->lynch);
    for (int b = 0; b < 2; ++b) {
        if (c->fmt_d[b]) (void)hipFree(c->fmt_d[b]);
        if (c->fmt_h[b]) (void)hipHostFree(c->fmt_h[b]);
    }
    for (char* p : c->in_h)
        if (p) (void)hipHostFree(p);
    for (void* p : {(void*)c->d_qtab, (void*)c->d_lg, (void*)c->d_scratch, (void*)c->d_qlo})
        if (p) (void)hipFree(p);
    for (auto& v : {c->ev_pool, c->ev_pending})
        for (auto& ev : v) {
            (void)hipEventDestroy(ev.start);
            (void)hipEventDestroy(ev.mid);
            (void)hipEventDestroy(ev.end);
        }
    delete c;
    return SID_OK;
}

extern "C" int sid_set_prior(sid_ctx* c, double snp_prior)
{
    if (!c) return SID_EINVAL;
    c->opts.snp_prior = snp_prior;
    sid_build_local_k(c->opts, &c->K);
    (void)hipSetDevice(c->device);
    hipError_t e = sid_build_table(c);
    return e == hipSuccess ? SID_OK : sid_set_hip_error(e);
}

extern "C" int sid_call_local(sid_ctx* c, const uint16_t* counts, size_t n, uint8_t* code,
                              double* hom_conf, double* het_conf, void* stream)
{
    if (!c) return SID_EINVAL;
    if (n == 0) return SID_OK;
    if (!counts || !code || !hom_conf || !het_conf) return SID_EINVAL;
    if (((uintptr_t)counts & 7u) || ((uintptr_t)hom_conf & 7u) || ((uintptr_t)het_conf & 7u))
        return SID_EINVAL;
    sid_timing_ev ev{nullptr, nullptr, nullptr};
    if (c->timing) {
        if (c->ev_pool.empty()) {
            sid_timing_ev x;
            if (hipEventCreate(&x.start) != hipSuccess || hipEventCreate(&x.mid) != hipSuccess ||
                hipEventCreate(&x.end) != hipSuccess)
                return SID_EHIP;
            c->ev_pool.push_back(x);
        }
        ev = c->ev_pool.back();
        c->ev_pool.pop_back();
        (void)hipEventRecord(ev.start, (hipStream_t)stream);
        c->ws.ev_mid = ev.mid;
    }
    hipError_t e = sid_launch_local(counts, n, code, hom_conf, het_conf, &c->K, c->d_lnt, &c->ws,
                                    c->grid_cap, (hipStream_t)stream);
    c->ws.parity ^= 1;   // the fix-up kernel zeroed the other counter
    if (c->timing) {
        c->ws.ev_mid = nullptr;
        (void)hipEventRecord(ev.end, (hipStream_t)stream);
        c->ev_pending.push_back(ev);
    }
    return e == hipSuccess ? SID_OK : sid_set_hip_error(e);
}

// ----------------------------------------------------------- measurement --
extern "C" int sid_timing_enable(sid_ctx* c, int enable)
{
    if (!c) return SID_EINVAL;
    c->timing = enable != 0;
    return SID_OK;
}

extern "C" int sid_timing_read(sid_ctx* c, uint64_t* calls, double* main_ms, double* fixup_ms)
{
    if (!c) return SID_EINVAL;
    double m = 0, f = 0;
    uint64_t k = 0;
    for (auto& ev : c->ev_pending) {
        hipError_t e = hipEventSynchronize(ev.end);
        if (e != hipSuccess) return sid_set_hip_error(e);
        float a = 0, b = 0;
        // the general-option path records no mid event: all time is "main"
        if (hipEventElapsedTime(&a, ev.start, ev.mid) == hipSuccess &&
            hipEventElapsedTime(&b, ev.mid, ev.end) == hipSuccess) {
            m += a;
            f += b;
        } else {
            (void)hipEventElapsedTime(&a, ev.start, ev.end);
            m += a;
        }
        ++k;
        c->ev_pool.push_back(ev);
    }
    c->ev_pending.clear();
    if (calls) *calls = k;
    if (main_ms) *main_ms = k ? m / k : 0.0;
    if (fixup_ms) *fixup_ms = k ? f / k : 0.0;
    return SID_OK;
}

// ------------------------------------------------------------- synthetic --
uint32_t sid_poisson_cdf(double mean, std::vector<uint64_t>& cdf)
{
    cdf.clear();
    double p = std::exp(-mean), cum = 0.0;
    for (uint32_t k = 0; k < SID_SYNTH_MAX_DEPTH_TABLE; ++k) {
        if (k > 0) p = p * mean / k;
        cum += p;
        double t = std::ldexp(cum, 64);
        uint64_t T = (t >= 18446744073709551615.0) ? UINT64_MAX : (uint64_t)t;
        cdf.push_back(T);
        if (T == UINT64_MAX || (k > mean && p < 1e-20)) break;
    }
    cdf.back() = UINT64_MAX;
    return (uint32_t)cdf.size();
}

// the context's device copy of the Poisson CDF for mean_depth
static int ctx_cdf(sid_ctx* c, double mean_depth)
{
    if (mean_depth != c->cdf_mean) {
        std::vector<uint64_t> cdf;
        uint32_t k = sid_poisson_cdf(mean_depth, cdf);
        if (c->d_cdf) (void)hipFree(c->d_cdf);
        c->d_cdf = nullptr;
        hipError_t e = hipMalloc(&c->d_cdf, k * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMemcpy(c->d_cdf, cdf.data(), k * sizeof(uint64_t), hipMemcpyHostToDevice);
        if (e != hipSuccess) return sid_set_hip_error(e);
        c->cdf_k = k;
        c->cdf_mean = mean_depth;
    }
    return SID_OK;
}

extern "C" int sid_synth_counts(sid_ctx* c, uint64_t seed, double mean_depth, uint64_t first_site,
                                size_t n, uint16_t* counts, void* stream)
{
    if (!c || (!counts && n) || !(mean_depth >= 0) || mean_depth > 600) return SID_EINVAL;
    if (n == 0) return SID_OK;
    if ((uintptr_t)counts & 7u) return SID_EINVAL;
    (void)hipSetDevice(c->device);
    int rc = ctx_cdf(c, mean_depth);
    if (rc != SID_OK) return rc;
    hipError_t e = sid_launch_synth(seed, first_site, n, c->d_cdf, c->cdf_k, counts, (hipStream_t)stream);
    return e == hipSuccess ? SID_OK : sid_set_hip_error(e);
}

extern "C" int sid_synth_text_device(sid_ctx* c, uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                                     uint64_t sites_per_chrom, char* out, size_t cap, size_t* len, void* stream)
{
    if (!c || !len || (!out && cap) || !(mean_depth >= 0) || mean_depth > 600) return SID_EINVAL;
    (void)hipSetDevice(c->device);
    int rc = ctx_cdf(c, mean_depth);
    if (rc != SID_OK) return rc;
    sid_synth_gen_ws ws;
    const hipStream_t st = (hipStream_t)stream;
    uint64_t res[2] = {0, 0};
    hipError_t e = sid_launch_synth_text(seed, c->d_cdf, c->cdf_k, first_site, n, sites_per_chrom, &ws, out, cap, st,
                                         mean_depth);
    if (e == hipSuccess) e = hipMemcpyAsync(res, ws.res, sizeof res, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    sid_synth_gen_release(&ws);
    if (e != hipSuccess) return sid_set_hip_error(e);
    *len = res[0];
    return res[1] ? SID_ERANGE : SID_OK;
}

extern "C" int sid_synth_counts_host(uint64_t seed, double mean_depth, uint64_t first_site,
                                     size_t n, uint16_t* counts)
{
    if ((!counts && n) || !(mean_depth >= 0) || mean_depth > 600) return SID_EINVAL;
    std::vector<uint64_t> cdf;
    uint32_t k = sid_poisson_cdf(mean_depth, cdf);
    uint64_t* out = (uint64_t*)counts;
    for (size_t i = 0; i < n; ++i) {
        uint64_t w = sid_synth_counts(seed, first_site + i, cdf.data(), k);
        std::memcpy(out + i, &w, 8);
    }
    return SID_OK;
}

static void synth_text_range(uint64_t seed, const std::vector<uint64_t>& cdf, uint64_t first,
                             size_t n, uint64_t spc, bool mq, std::string& out)
{
    static const char UP[] = "ACGT", LO[] = "acgt";
    out.clear();
    out.reserve(n * 96);
    char num[32];
    std::string bases, quals, mquals;
    const uint32_t k = (uint32_t)cdf.size();
    for (size_t i = 0; i < n; ++i) {
        const uint64_t site = first + i;
        uint64_t chrom = spc ? site / spc + 1 : 1;
        uint64_t pos = spc ? site % spc + 1 : site + 1;
        sid_synth_site s = sid_synth_site_header(seed, site, cdf.data(), k);
        out += "chr";
        out.append(num, (size_t)std::snprintf(num, sizeof num, "%llu", (unsigned long long)chrom));
        out += '\t';
        out.append(num, (size_t)std::snprintf(num, sizeof num, "%llu", (unsigned long long)pos));
        out += '\t';
        out += UP[s.ref];
        out += '\t';
        out.append(num, (size_t)std::snprintf(num, sizeof num, "%u", s.depth));
        out += '\t';
        if (s.depth == 0) {
            out += mq ? "*\t*\t*\n" : "*\t*\n";
            continue;
        }
        bases.clear();
        quals.clear();
        mquals.clear();
        for (uint32_t r = 0; r < s.depth; ++r) {
            uint32_t strand;
            uint32_t b = sid_synth_read_base(&s, r, &strand);
            int st, en;
            uint32_t q;
            sid_synth_read_marks(&s, r, &st, &en, &q);
            if (st) bases += "^]";
            if (b == s.ref)
                bases += strand ? '.' : ',';
            else
                bases += strand ? UP[b] : LO[b];
            if (en) bases += '$';
            quals += (char)('!' + q);
            if (mq) mquals += (char)('!' + sid_synth_read_mapq(&s, r));
        }
        out += bases;
        out += '\t';
        out += quals;
        if (mq) {
            out += '\t';
            out += mquals;
        }
        out += '\n';
    }
}

static int synth_text(uint64_t seed, double mean_depth, uint64_t first_site, size_t n, uint64_t sites_per_chrom,
                      bool mq, char* buf, size_t cap, size_t* len);

extern "C" int sid_synth_text(uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                              uint64_t sites_per_chrom, char* buf, size_t cap, size_t* len)
{
    return synth_text(seed, mean_depth, first_site, n, sites_per_chrom, false, buf, cap, len);
}

extern "C" int sid_synth_text_mq(uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                                 uint64_t sites_per_chrom, char* buf, size_t cap, size_t* len)
{
    return synth_text(seed, mean_depth, first_site, n, sites_per_chrom, true, buf, cap, len);
}

static int synth_text(uint64_t seed, double mean_depth, uint64_t first_site, size_t n, uint64_t sites_per_chrom,
                      bool mq, char* buf, size_t cap, size_t* len)
{
    if (!len || !(mean_depth >= 0) || mean_depth > 600) return SID_EINVAL;
    std::vector<uint64_t> cdf;
    sid_poisson_cdf(mean_depth, cdf);
    unsigned T = std::thread::hardware_concurrency();
    if (T == 0) T = 1;
    if (T > 16) T = 16;
    if (n < 100000) T = 1;
    std::vector<std::string> parts(T);
    std::vector<std::thread> th;
    size_t per = (n + T - 1) / T;
    for (unsigned t = 0; t < T; ++t) {
        size_t b = t * per, e = std::min(n, b + per);
        if (b >= e) continue;
        th.emplace_back([&, t, b, e] { synth_text_range(seed, cdf, first_site + b, e - b, sites_per_chrom, mq, parts[t]); });
    }
    for (auto& x : th) x.join();
    size_t total = 0;
    for (auto& p : parts) total += p.size();
    *len = total;
    if (!buf) return SID_OK;
    if (cap < total) return SID_ENOMEM;
    size_t off = 0;
    for (auto& p : parts) {
        std::memcpy(buf + off, p.data(), p.size());
        off += p.size();
    }
    return SID_OK;
}
