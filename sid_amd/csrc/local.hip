// local.hip — `-m local` per-site kernel.
//
// Replaces call.cpp:213-289 (callSiteMLError): the reference dedupes the
// sites into unique profiles, classifies each profile in long double and
// gathers the result back per site through a std::map.  The result is a pure
// function of the 4 counts + options, so here one lane classifies one site
// directly: no dedupe, no map, one streaming pass
//
//   HBM read  8 B/site  (profile_t: 4 x u16 A,C,G,T)
//   HBM write 17 B/site (u8 code + f64 hom_conf + f64 het_conf)
//
// Each thread owns 4 consecutive sites: two 16-B loads, one 4-B code store,
// two 16-B stores per confidence column, so every wave instruction moves
// whole 64-B segments.  The ln(k) table lives in LDS (8 KiB per block).
#include "fmt.h"
#include "local_site.h"

namespace {

template <bool GENERAL>
__global__ __launch_bounds__(256) void sid_local_kernel_x4(const ulonglong2* __restrict__ counts,
                                                          size_t ngroups,
                                                          uint32_t* __restrict__ code4,
                                                          double2* __restrict__ hom,
                                                          double2* __restrict__ het,
                                                          sid_local_k K,
                                                          const double* __restrict__ g_lnt)
{
    __shared__ double lnt[SID_LUTN];
    if (!GENERAL) {
        for (int i = threadIdx.x; i < SID_LUTN; i += blockDim.x) lnt[i] = g_lnt[i];
        __syncthreads();
    }
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += stride) {
        const ulonglong2 a = counts[2 * g];
        const ulonglong2 b = counts[2 * g + 1];
        double h0, h1, h2, h3, t0, t1, t2, t3;
        uint32_t c0 = local_site<GENERAL>(a.x, K, lnt, h0, t0);
        uint32_t c1 = local_site<GENERAL>(a.y, K, lnt, h1, t1);
        uint32_t c2 = local_site<GENERAL>(b.x, K, lnt, h2, t2);
        uint32_t c3 = local_site<GENERAL>(b.y, K, lnt, h3, t3);
        code4[g] = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
        hom[2 * g] = make_double2(h0, h1);
        hom[2 * g + 1] = make_double2(h2, h3);
        het[2 * g] = make_double2(t0, t1);
        het[2 * g + 1] = make_double2(t2, t3);
    }
}

// Any alignment, one site per thread (ragged tails, sub-array pointers).
template <bool GENERAL>
__global__ __launch_bounds__(256) void sid_local_kernel_x1(const uint64_t* __restrict__ counts,
                                                          size_t n, uint8_t* __restrict__ code,
                                                          double* __restrict__ hom,
                                                          double* __restrict__ het, sid_local_k K,
                                                          const double* __restrict__ g_lnt)
{
    __shared__ double lnt[SID_LUTN];
    if (!GENERAL) {
        for (int i = threadIdx.x; i < SID_LUTN; i += blockDim.x) lnt[i] = g_lnt[i];
        __syncthreads();
    }
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        double h, t;
        code[i] = (uint8_t)local_site<GENERAL>(counts[i], K, lnt, h, t);
        hom[i] = h;
        het[i] = t;
    }
}

// Table entry for (nf, ns, r2): v >= +0 -> p1 = v, p2 = 1; v <= -0 -> p1 = 1,
// p2 = -v; NaN -> both 0 (NaN-free: the reference's 0/0 never reaches here);
// +inf -> not covered (the site needs the fast or emulated path).
__global__ __launch_bounds__(256) void sid_local_table_build(sid_local_k K, const double* __restrict__ lnt,
                                                            double* __restrict__ table, uint32_t NF, uint32_t NS,
                                                            uint32_t NR, bool swz)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NF * NS * NR) return;
    const uint32_t r2 = i % NR, ns = (i / NR) % NS, nf = i / (NR * NS);
    double v = __builtin_inf();
    double p1, p2;
    bool gt;
    // a profile with these majors exists iff nf >= ns and both minor counts <= ns
    if (nf >= ns && r2 <= 2 * ns && local_fast_p(nf, ns, r2, K, lnt, p1, p2, gt)) {
        if (p1 == 0.0 && p2 == 0.0) v = __builtin_nan("");
        else if (gt) v = -p2;       // p1 == 1
        else v = p1;                // p2 == 1
    }
    table[swz ? sid_tab_slot(nf, ns, r2) : i] = v;
}

// Sites are processed in pairs (one 16-B profile_t load per lane), blocks
// striding over 1024-pair tiles, lanes contiguous in every wave instruction:
// loads and the 16-B conf stores move 1 KiB per instruction, the 2-B code
// stores 128 B (one full L2 line).  Misses go to an LDS list (one LDS atomic
// per missed site), flushed with one global atomic per block.  (Measured and
// not kept: 2 or 4 pairs per thread, non-temporal stores, one contiguous tile
// range per block)
#define SID_LMISS 2048

typedef double sid_dvec2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(1024) void sid_local_table_p2(const ulonglong2* __restrict__ pairs, size_t npairs,
                                                           uint16_t* __restrict__ code2, sid_dvec2* __restrict__ hom,
                                                           sid_dvec2* __restrict__ het,
                                                           const double* __restrict__ g_table, double sig,
                                                           const double* __restrict__ T2,
                                                           uint32_t* __restrict__ miss, uint32_t cap,
                                                           uint32_t* __restrict__ ctr)
{
    __shared__ double T[SID_TAB_N];
    __shared__ uint32_t lmiss[SID_LMISS];
    __shared__ uint32_t lcnt, gbase;
    {
        const double2* src = (const double2*)g_table;
        double2* dst = (double2*)T;
        for (int i = threadIdx.x; i < SID_TAB_N / 2; i += blockDim.x) dst[i] = src[i];
    }
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += stride) {
        const ulonglong2 c = pairs[p];
        double h0, h1, t0, t1;
        uint32_t a = table_site(c.x, T, sig, h0, t0);
        uint32_t b = table_site(c.y, T, sig, h1, t1);
        // LDS misses (30x het sites, 200x sites with r2 >= 4) through the
        // second-level table before the stores: an L2 hit the other waves
        // hide, instead of a scattered rewrite later
        if (T2 && (a == 0xFFu || b == 0xFFu)) {
            if (a == 0xFFu) a = table2_site(c.x, T2, sig, h0, t0);
            if (b == 0xFFu) b = table2_site(c.y, T2, sig, h1, t1);
        }
        code2[p] = (uint16_t)(a | (b << 8));
        hom[p] = sid_dvec2{h0, h1};
        het[p] = sid_dvec2{t0, t1};
        if (a == 0xFFu || b == 0xFFu) {
            for (int k = 0; k < 2; ++k) {
                if ((k ? b : a) != 0xFFu) continue;
                const uint32_t idx = (uint32_t)(2 * p + k);
                const uint32_t slot = atomicAdd(&lcnt, 1u);
                if (slot < SID_LMISS) {
                    lmiss[slot] = idx;
                } else {
                    const uint32_t g = atomicAdd(ctr, 1u);
                    if (g < cap) miss[g] = idx;
                }
            }
        }
    }
    __syncthreads();
    const uint32_t nl = lcnt < SID_LMISS ? lcnt : SID_LMISS;
    if (nl == 0) return;
    if (threadIdx.x == 0) gbase = atomicAdd(ctr, nl);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
        if (gbase + i < cap) miss[gbase + i] = lmiss[i];
}

__global__ __launch_bounds__(1024) void sid_local_table_x1(const uint64_t* __restrict__ counts, size_t n,
                                                           uint8_t* __restrict__ code, double* __restrict__ hom,
                                                           double* __restrict__ het,
                                                           const double* __restrict__ g_table, double sig,
                                                           uint32_t* __restrict__ miss, uint32_t cap,
                                                           uint32_t* __restrict__ ctr, size_t base)
{
    __shared__ double T[SID_TAB_N];
    for (int i = threadIdx.x; i < SID_TAB_N; i += blockDim.x) T[i] = g_table[i];
    __syncthreads();
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        double h, t;
        const uint32_t c = table_site(counts[i], T, sig, h, t);
        code[i] = (uint8_t)c;
        hom[i] = h;
        het[i] = t;
        if (c == 0xFFu) {   // ragged / unaligned remainder only: plain global append
            const uint32_t g = atomicAdd(ctr, 1u);
            if (g < cap) miss[g] = (uint32_t)(base + i);
        }
    }
}

// Sites the table does not cover: the miss list (or, if it overflowed, a
// scan for the 0xFF marker).  Resets the other parity's counter for the next
// call on this stream.
__global__ __launch_bounds__(256) void sid_local_fixup(const uint64_t* __restrict__ counts, size_t n,
                                                       uint8_t* __restrict__ code, double* __restrict__ hom,
                                                       double* __restrict__ het, sid_local_k K,
                                                       const double* __restrict__ lnt,
                                                       const double* __restrict__ T2,
                                                       const uint32_t* __restrict__ miss, uint32_t cap,
                                                       uint32_t* __restrict__ ctr, int parity)
{
    const uint32_t m = ctr[parity];
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr[parity ^ 1] = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const size_t t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (m <= cap) {
        for (size_t j = t0; j < m; j += stride) {
            const uint32_t i = miss[j];
            double h, t;
            code[i] = (uint8_t)fixup_site(counts[i], T2, K, lnt, h, t);
            hom[i] = h;
            het[i] = t;
        }
    } else {
        for (size_t i = t0; i < n; i += stride) {
            if (code[i] != 0xFFu) continue;
            double h, t;
            code[i] = (uint8_t)fixup_site(counts[i], T2, K, lnt, h, t);
            hom[i] = h;
            het[i] = t;
        }
    }
}

}  // namespace

// The engine's -m local formatter (textpath.hip) memoises the record tails
// per class as well: entry k of a string table (SID_STR_BYTES) holds, for
// class-table entry k, byte 0 the tail's length (0xFF: not tabulated, as the
// +inf entries), byte 1 bit 0 the het label, and from byte SID_STR_TEXT the
// tail "hom_conf,het_conf,p_value\n" (%g, call.hpp:29-38; -m local's
// conf_type), zero-padded to the end of the entry; len[k] = byte 0 again.
__global__ __launch_bounds__(256) void sid_local_str_build(const double* __restrict__ table, uint32_t N, double sig,
                                                          char* __restrict__ str, uint8_t* __restrict__ len)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double v = table[i];
    char* e = str + (size_t)i * SID_STR_BYTES;
    char buf[2 * SID_FMT_MAX + 16];   // the text, then copied when it fits
    for (int k = 0; k < SID_STR_BYTES; ++k) e[k] = 0;
    if (isinf(v)) {
        len[i] = 0xFF;
        e[0] = (char)0xFF;
        return;
    }
    double p1, p2;
    const uint32_t c = table_decode(v, 0, 0, sig, p1, p2);
    char* t = buf;
    int n = sid_g6_put(sid_g6_prep(p1), t);
    t[n++] = ',';
    n += sid_g6_put(sid_g6_prep(p2), t + n);
    if (n + 9 > SID_STR_BYTES - SID_STR_TEXT) {   // (one of p1, p2 is 1 or both are 0: at most 12 + 1 + 1)
        for (int k = 0; k < SID_STR_BYTES; ++k) e[k] = 0;
        len[i] = 0xFF;
        e[0] = (char)0xFF;
        return;
    }
    const char tail[] = ",p_value\n";
    for (int k = 0; k < 9; ++k) t[n++] = tail[k];
    for (int k = 0; k < n; ++k) e[SID_STR_TEXT + k] = buf[k];
    e[0] = (char)n;
    e[1] = (char)((c & 0x80u) ? 1 : 0);
    len[i] = (uint8_t)n;
}

// ------------------------------------------------------------- launcher --
// Called by the C ABI (capi.cpp).  counts must be at least 8-byte aligned
// (profile_t is 8 bytes).  Non-general option sets: table kernel (x4 when the
// arrays allow 16-B accesses, x1 otherwise) + fix-up kernel.  General option
// sets (E < 0, prior > 1): the direct kernels with the emulated path.
extern "C" hipError_t sid_launch_local_table_build(const sid_local_k* K, const double* d_lnt, double* d_table,
                                                   double* d_table2, hipStream_t stream)
{
    sid_local_table_build<<<SID_TAB_N / 256, 256, 0, stream>>>(*K, d_lnt, d_table, SID_TAB_NF, SID_TAB_NS,
                                                               SID_TAB_NR, true);
    if (d_table2)
        sid_local_table_build<<<SID_TAB2_N / 256, 256, 0, stream>>>(*K, d_lnt, d_table2, SID_TAB2_NF, SID_TAB2_NS,
                                                                    SID_TAB2_NR, false);
    return hipGetLastError();
}

extern "C" hipError_t sid_launch_local_str_build(const sid_local_k* K, const double* d_table, const double* d_table2,
                                                 const sid_local_ws* ws, hipStream_t stream)
{
    sid_local_str_build<<<SID_TAB_N / 256, 256, 0, stream>>>(d_table, SID_TAB_N, K->sig, ws->str1, ws->len1);
    sid_local_str_build<<<SID_TAB2_N / 256, 256, 0, stream>>>(d_table2, SID_TAB2_N, K->sig, ws->str2, ws->len2);
    return hipGetLastError();
}

extern "C" hipError_t sid_launch_local(const uint16_t* counts, size_t n, uint8_t* code,
                                       double* hom, double* het, const sid_local_k* K,
                                       const double* d_lnt, const sid_local_ws* ws, int grid_cap,
                                       hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    const bool aligned = (((uintptr_t)counts | (uintptr_t)hom | (uintptr_t)het) & 15u) == 0 &&
                         (((uintptr_t)code) & 3u) == 0;
    if (!K->general && ws && ws->table) {
        const uint32_t cap = n < 0xFFFFFFFFull ? ws->cap : 0u;   // u32 site indices
        uint32_t* ctr = ws->ctr + ws->parity;
        const int tb = 1024;
        size_t done = 0;
        const bool aligned2 = (((uintptr_t)counts | (uintptr_t)hom | (uintptr_t)het) & 15u) == 0 &&
                              (((uintptr_t)code) & 1u) == 0;
        if (aligned2 && n >= 2) {
            const size_t npairs = n / 2;
            size_t want = (npairs + (size_t)tb - 1) / (size_t)tb;
            int grid = (int)(want < (size_t)ws->table_grid ? want : (size_t)ws->table_grid);
            const double* T2 = ws->tail ? ws->table2 : nullptr;
            sid_local_table_p2<<<grid, tb, 0, stream>>>((const ulonglong2*)counts, npairs, (uint16_t*)code,
                                                        (sid_dvec2*)hom, (sid_dvec2*)het, ws->table, K->sig, T2,
                                                        ws->miss, cap, ctr);
            done = npairs * 2;
        }
        if (done < n) {
            const size_t rest = n - done;
            size_t want = (rest + tb - 1) / tb;
            int grid = (int)(want < (size_t)ws->table_grid ? want : (size_t)ws->table_grid);
            // miss indices are recorded relative to `counts` (base = done)
            sid_local_table_x1<<<grid, tb, 0, stream>>>((const uint64_t*)counts + done, rest, code + done,
                                                        hom + done, het + done, ws->table, K->sig,
                                                        ws->miss, cap, ctr, done);
        }
        if (ws->ev_mid) (void)hipEventRecord(ws->ev_mid, stream);   // measurement: main | fix-up
        sid_local_fixup<<<256, 256, 0, stream>>>((const uint64_t*)counts, n, code, hom, het, *K, d_lnt, ws->table2,
                                                 ws->miss, cap, ws->ctr, ws->parity);
        return hipGetLastError();
    }
    const int block = 256;
    size_t done = 0;
    if (aligned && n >= 4) {
        const size_t ngroups = n / 4;
        size_t want = (ngroups + block - 1) / block;
        int grid = (int)(want < (size_t)grid_cap ? want : (size_t)grid_cap);
        if (K->general)
            sid_local_kernel_x4<true><<<grid, block, 0, stream>>>(
                (const ulonglong2*)counts, ngroups, (uint32_t*)code, (double2*)hom, (double2*)het,
                *K, d_lnt);
        else
            sid_local_kernel_x4<false><<<grid, block, 0, stream>>>(
                (const ulonglong2*)counts, ngroups, (uint32_t*)code, (double2*)hom, (double2*)het,
                *K, d_lnt);
        done = ngroups * 4;
    }
    if (done < n) {
        const size_t rest = n - done;
        size_t want = (rest + block - 1) / block;
        int grid = (int)(want < (size_t)grid_cap ? want : (size_t)grid_cap);
        const uint64_t* c = (const uint64_t*)counts + done;
        if (K->general)
            sid_local_kernel_x1<true><<<grid, block, 0, stream>>>(c, rest, code + done, hom + done,
                                                                  het + done, *K, d_lnt);
        else
            sid_local_kernel_x1<false><<<grid, block, 0, stream>>>(c, rest, code + done, hom + done,
                                                                   het + done, *K, d_lnt);
    }
    return hipGetLastError();
}
