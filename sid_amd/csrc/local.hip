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
#include "sid_math.h"

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
    p1 = sid_x86_nan(ld_lrt(l2, l1, K.lg15));
    p2 = sid_x86_nan(ld_lrt(l1, l2, K.lg15));
    const bool het = ld_gt(l2, l1) && p2 < K.sig;   // call.cpp:266
    return f | ((het ? s : f) << 2) | (het ? 0x80u : 0u);
}

template <bool GENERAL>
__device__ __forceinline__ uint32_t local_site(uint64_t w, const sid_local_k& K,
                                               const double* __restrict__ lnt, double& p1,
                                               double& p2)
{
    if (GENERAL) return local_site_general(w, K, p1, p2);
    uint32_t f, s, nf, ns, cov;
    sid_major(w, f, s, nf, ns, cov);
    if (cov >= SID_LUTN) return local_site_general(w, K, p1, p2);
    const uint32_t r1 = cov - nf, r2 = r1 - ns, m2 = nf + ns;

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
    if (!((ln1 >= SID_FAST_FLOOR || z1) && (ln2 >= SID_FAST_FLOOR || z2)))
        return local_site_general(w, K, p1, p2);

    const double d = ln1 - ln2;
    // p1 = LRT(l2, l1), p2 = LRT(l1, l2); at most one chi^2 is non-zero
    const double chi1 = z2 ? 1.7976931348623157e308 : ((!z1 && d > 0.0) ? 2.0 * d : 0.0);
    const double chi2 = z1 ? 1.7976931348623157e308 : ((!z2 && d < 0.0) ? -2.0 * d : 0.0);
    const double chi = fmax(chi1, chi2);
    const double q = sid_chisq_Q(chi, K.lg15);
    p1 = (chi1 == chi) ? q : 1.0;
    p2 = (chi2 == chi) ? q : 1.0;
    const bool het = !z2 && (z1 || d < 0.0) && p2 < K.sig;
    return f | ((het ? s : f) << 2) | (het ? 0x80u : 0u);
}

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

}  // namespace

// ------------------------------------------------------------- launcher --
// Called by the C ABI (capi.cpp).  counts must be at least 8-byte aligned
// (profile_t is 8 bytes); the x4 kernel is used when the arrays allow 16-B
// accesses, the x1 kernel for the rest.
extern "C" hipError_t sid_launch_local(const uint16_t* counts, size_t n, uint8_t* code,
                                       double* hom, double* het, const sid_local_k* K,
                                       const double* d_lnt, int grid_cap, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    const int block = 256;
    const bool aligned = (((uintptr_t)counts | (uintptr_t)hom | (uintptr_t)het) & 15u) == 0 &&
                         (((uintptr_t)code) & 3u) == 0;
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
