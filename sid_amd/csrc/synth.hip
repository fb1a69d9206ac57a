// synth.hip — device side of the counter-based synthetic pileup (synth.h).
// Fills profile_t counts for sites [first, first+n) directly in HBM, so the
// bench's inputs are resident before the timed region starts.
#include <hip/hip_runtime.h>

#include "synth.h"

namespace {
__global__ __launch_bounds__(256) void sid_synth_kernel(uint64_t seed, uint64_t first, size_t n,
                                                        const uint64_t* __restrict__ cdf,
                                                        uint32_t kmax, uint64_t* __restrict__ out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = sid_synth_counts(seed, first + i, cdf, kmax);
}
}  // namespace

extern "C" hipError_t sid_launch_synth(uint64_t seed, uint64_t first, size_t n,
                                       const uint64_t* d_cdf, uint32_t kmax, uint16_t* counts,
                                       hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    size_t want = (n + 255) / 256;
    int grid = (int)(want < 8192 ? want : 8192);
    sid_synth_kernel<<<grid, 256, 0, stream>>>(seed, first, n, d_cdf, kmax, (uint64_t*)counts);
    return hipGetLastError();
}

// ------------------------------------------------------- synthetic text --
// The generator's text (sid_synth_text, capi.cpp) produced on the device, one
// lane per site: a length pass (only the read marks are drawn), a scan, and a
// write pass.  Used to stream the C4/C5 configs (3G / 500M sites) through the
// engine without ever storing them.
#include <algorithm>

#include "sid_internal.h"

namespace {

__device__ __forceinline__ uint32_t dec_len(uint64_t v)
{
    uint32_t n = 1;
    while (v >= 10) {
        v /= 10;
        ++n;
    }
    return n;
}

__device__ __forceinline__ char* put_dec(char* o, uint64_t v)
{
    const uint32_t n = dec_len(v);
    for (uint32_t k = n; k-- > 0;) {
        o[k] = (char)('0' + v % 10);
        v /= 10;
    }
    return o + n;
}

struct SynthLine {
    uint64_t chrom, pos;
    sid_synth_site s;
};

__device__ __forceinline__ SynthLine synth_line(uint64_t seed, uint64_t site, uint64_t spc,
                                                const uint64_t* __restrict__ cdf, uint32_t kmax)
{
    SynthLine L;
    L.chrom = spc ? site / spc + 1 : 1;
    L.pos = spc ? site % spc + 1 : site + 1;
    L.s = sid_synth_site_header(seed, site, cdf, kmax);
    return L;
}

__global__ __launch_bounds__(256) void sid_synth_len_kernel(uint64_t seed, uint64_t first, uint64_t n,
                                                            uint64_t spc, const uint64_t* __restrict__ cdf,
                                                            uint32_t kmax, uint32_t* __restrict__ len)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const SynthLine L = synth_line(seed, first + i, spc, cdf, kmax);
    // "chr" chrom \t pos \t ref \t depth \t
    uint32_t l = 3 + dec_len(L.chrom) + 1 + dec_len(L.pos) + 1 + 1 + 1 + dec_len(L.s.depth) + 1;
    if (L.s.depth == 0) {
        l += 4;   // "*\t*\n"
    } else {
        uint32_t b = 0;
        for (uint32_t r = 0; r < L.s.depth; ++r) {
            int st, en;
            uint32_t q;
            sid_synth_read_marks(&L.s, r, &st, &en, &q);
            b += 1 + 2 * st + en;
        }
        l += b + 1 + L.s.depth + 1;   // bases \t quals \n
    }
    len[i] = l;
}

// The line of site i (l bytes) into o (any address space): one walk over the
// reads writes each base with its marks and its quality character (the
// qualities are the depth bytes before the final '\n').
__device__ __forceinline__ void synth_write_line(const SynthLine& L, uint32_t l, char* o)
{
    const char UP[4] = {'A', 'C', 'G', 'T'}, LO[4] = {'a', 'c', 'g', 't'};
    char* const o0 = o;
    *o++ = 'c';
    *o++ = 'h';
    *o++ = 'r';
    o = put_dec(o, L.chrom);
    *o++ = '\t';
    o = put_dec(o, L.pos);
    *o++ = '\t';
    *o++ = UP[L.s.ref];
    *o++ = '\t';
    o = put_dec(o, L.s.depth);
    *o++ = '\t';
    if (L.s.depth == 0) {
        *o++ = '*';
        *o++ = '\t';
        *o++ = '*';
        *o = '\n';
        return;
    }
    char* q = o0 + l - 1 - L.s.depth;
    for (uint32_t r = 0; r < L.s.depth; ++r) {
        uint32_t strand;
        const uint32_t b = sid_synth_read_base(&L.s, r, &strand);
        int st, en;
        uint32_t ql;
        sid_synth_read_marks(&L.s, r, &st, &en, &ql);
        if (st) {
            *o++ = '^';
            *o++ = ']';
        }
        *o++ = b == L.s.ref ? (strand ? '.' : ',') : (strand ? UP[b] : LO[b]);
        if (en) *o++ = '$';
        *q++ = (char)('!' + ql);
    }
    *o = '\t';
    *q = '\n';
}

__global__ void sid_synth_write_kernel(uint64_t seed, uint64_t first, uint64_t n, uint64_t spc,
                                       const uint64_t* __restrict__ cdf, uint32_t kmax,
                                       const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                       uint64_t cap, char* __restrict__ out, uint32_t lds_cap)
{
    extern __shared__ __attribute__((aligned(16))) char buf[];
    const uint32_t B = blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * B, i = i0 + threadIdx.x;
    const uint64_t i1 = i0 + B < n ? i0 + B : n;
    const uint64_t b0 = off[i0], b1 = off[i1 - 1] + len[i1 - 1];   // the block's bytes [b0, b1)
    const bool staged = b1 <= cap && b1 - b0 + 16 <= lds_cap;
    const uint32_t phase = (uint32_t)((uintptr_t)(out + b0) & 15u);
    if (i < n && off[i] + len[i] <= cap) {
        const SynthLine L = synth_line(seed, first + i, spc, cdf, kmax);
        char* o = staged ? buf + phase + (off[i] - b0) : out + off[i];
        synth_write_line(L, len[i], o);
    }
    if (!staged) return;
    __syncthreads();
    char* dst = out + b0 - phase;   // 16-B aligned
    const uint32_t span = phase + (uint32_t)(b1 - b0);
    for (uint32_t k = threadIdx.x * 16; k < span; k += B * 16) {
        if (k >= phase && k + 16 <= span) {
            *(uint4*)(dst + k) = *(const uint4*)(buf + k);
        } else {
            for (uint32_t j = k; j < k + 16 && j < span; ++j)
                if (j >= phase) dst[j] = buf[j];
        }
    }
}

__global__ void sid_synth_check_kernel(uint64_t* res, uint64_t cap)
{
    res[1] = res[0] > cap ? 1 : 0;
}

}  // namespace

void sid_synth_gen_release(sid_synth_gen_ws* ws)
{
    for (void* p : {(void*)ws->len, (void*)ws->off, (void*)ws->res})
        if (p) (void)hipFree(p);
    *ws = sid_synth_gen_ws{};
}

hipError_t sid_launch_synth_text(uint64_t seed, const uint64_t* d_cdf, uint32_t kmax, uint64_t first, uint64_t n,
                                 uint64_t spc, sid_synth_gen_ws* ws, char* out, uint64_t cap, hipStream_t st,
                                 double mean_depth)
{
    hipError_t e = hipSuccess;
    if (!ws->res && (e = hipMalloc(&ws->res, 2 * sizeof(uint64_t))) != hipSuccess) return e;
    if (n > ws->cap) {
        if (ws->len) (void)hipFree(ws->len);
        if (ws->off) (void)hipFree(ws->off);
        ws->len = nullptr;
        ws->off = nullptr;
        ws->cap = 0;
        if ((e = hipMalloc(&ws->len, ((n * 4 + 7) & ~(uint64_t)7) + sid_scan_ws_bytes(n))) != hipSuccess) return e;
        if ((e = hipMalloc(&ws->off, n * 8)) != hipSuccess) return e;
        ws->cap = n;
    }
    if ((e = hipMemsetAsync(ws->res, 0, 2 * sizeof(uint64_t), st)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)((n + 255) / 256);
    sid_synth_len_kernel<<<g, 256, 0, st>>>(seed, first, n, spc, d_cdf, kmax, ws->len);
    e = sid_scan_u32(ws->len, n, ws->off, ws->res, (uint64_t*)((char*)ws->len + ((n * 4 + 7) & ~(uint64_t)7)), st);
    if (e != hipSuccess) return e;
    sid_synth_check_kernel<<<1, 1, 0, st>>>(ws->res, cap);
    // no host sync between the passes: a line is written only when it ends
    // within cap, and res[1] tells the caller the text is incomplete
    // lines assembled in LDS, stored 16 B at a time: 256 sites a block up to a
    // mean depth of ~60 (about 20 KiB), 64 beyond (a 200x block is ~27 KiB);
    // a block whose lines do not fit stores them byte by byte
    const uint32_t B = mean_depth > 60.0 ? 64u : 256u;
    const uint32_t lds = std::min<uint32_t>(64u << 10, (uint32_t)(B * (40.0 + 4.2 * mean_depth)) + 64u);
    const unsigned gw = (unsigned)((n + B - 1) / B);
    sid_synth_write_kernel<<<gw, B, lds, st>>>(seed, first, n, spc, d_cdf, kmax, ws->off, ws->len, cap, out, lds);
    return hipGetLastError();
}
