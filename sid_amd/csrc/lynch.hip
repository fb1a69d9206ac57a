// lynch.hip — Lynch ML path kernels.
//
//   sid_hist_kernel      countUniqueProfiles (pileup.cpp:169-196) as a hash
//                        histogram: per-block LDS pre-aggregation, then one
//                        global atomic per (block, distinct profile).
//   sid_objective_kernel compoundLikelihood (lynch.cpp:37-61) over the
//                        filtered unique profiles: one lane per profile,
//                        10-genotype mixture in the log domain
//                        (lynch.hpp:57-74,82-90), count*ln L reduced per
//                        block in double-double.
//   sid_profile_lik_kernel  per-profile (L_hom, L_het) at eps-hat
//                        (lynch.cpp:28-33) as emulated long doubles.
//   sid_classify_kernel  LRT (call.cpp:93-104) or bayes posteriors
//                        (call.cpp:170-194) per profile.
//   sid_lookup_kernel    per-site gather of the class table
//                        (call.cpp:129-140) through a compact,
//                        L2/MALL-resident hash of the U profiles.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cstdlib>

#include "sid_math.h"
#include "sid_nm.h"

#define SID_LN_LDBL_TRUE_MIN (-SID_LDBL_DENORM_SHIFT)

__device__ __forceinline__ void sid_global_insert(unsigned long long* gkeys, unsigned long long* gcnt,
                                                  uint64_t gmask, unsigned long long* distinct,
                                                  uint64_t key, unsigned long long add)
{
    uint64_t h = sid_hash64(key) & gmask;
    for (uint64_t probe = 0; probe <= gmask; ++probe) {
        unsigned long long prev = atomicCAS(&gkeys[h], SID_EMPTY_KEY, (unsigned long long)key);
        if (prev == SID_EMPTY_KEY || prev == key) {
            atomicAdd(&gcnt[h], add);
            if (prev == SID_EMPTY_KEY) atomicAdd(distinct, 1ull);
            return;
        }
        h = (h + 1) & gmask;
    }
}

// as sid_global_insert, returning 1 if the key was new instead of counting it
__device__ __forceinline__ unsigned sid_global_insert_new(unsigned long long* gkeys, unsigned long long* gcnt,
                                                          uint64_t gmask, uint64_t key, unsigned long long add)
{
    uint64_t h = sid_hash64(key) & gmask;
    for (uint64_t probe = 0; probe <= gmask; ++probe) {
        unsigned long long prev = atomicCAS(&gkeys[h], SID_EMPTY_KEY, (unsigned long long)key);
        if (prev == SID_EMPTY_KEY || prev == key) {
            atomicAdd(&gcnt[h], add);
            return prev == SID_EMPTY_KEY;
        }
        h = (h + 1) & gmask;
    }
    return 0;
}

#define SID_HIST_LCAP 4096
#define SID_HIST_PROBES 32

// counts: n sites; keys of value SID_EMPTY_KEY (all four counts 65535) go to
// stats[1].  stats[0] = distinct keys inserted in the global table.  With
// SKIP_DENSE the dense-coded profiles are left out (they were counted by
// sid_hist_dense_kernel): the overflow path of the fallback list.
template <bool SKIP_DENSE>
__global__ __launch_bounds__(256) void sid_hist_kernel(const uint64_t* __restrict__ counts, size_t n,
                                                       size_t per_block, unsigned long long* gkeys,
                                                       unsigned long long* gcnt, uint64_t gmask,
                                                       unsigned long long* stats)
{
    __shared__ unsigned long long lkeys[SID_HIST_LCAP];
    __shared__ unsigned int lcnt[SID_HIST_LCAP];
    for (int i = threadIdx.x; i < SID_HIST_LCAP; i += blockDim.x) {
        lkeys[i] = SID_EMPTY_KEY;
        lcnt[i] = 0;
    }
    __syncthreads();
    const size_t begin = (size_t)blockIdx.x * per_block;
    const size_t end = begin + per_block < n ? begin + per_block : n;
    for (size_t i = begin + threadIdx.x; i < end; i += blockDim.x) {
        const uint64_t w = counts[i];
        if (SKIP_DENSE && sid_dense_code(w) != SID_DENSE_NONE) continue;
        const uint64_t key = sid_profile_key(w);
        if (key == SID_EMPTY_KEY) {
            atomicAdd(&stats[1], 1ull);
            continue;
        }
        uint32_t h = (uint32_t)(sid_hash64(key) & (SID_HIST_LCAP - 1));
        bool done = false;
        for (int p = 0; p < SID_HIST_PROBES; ++p) {
            unsigned long long prev = atomicCAS(&lkeys[h], SID_EMPTY_KEY, (unsigned long long)key);
            if (prev == SID_EMPTY_KEY || prev == key) {
                atomicAdd(&lcnt[h], 1u);
                done = true;
                break;
            }
            h = (h + 1) & (SID_HIST_LCAP - 1);
        }
        if (!done) sid_global_insert(gkeys, gcnt, gmask, &stats[0], key, 1ull);
    }
    __syncthreads();
    for (int s = threadIdx.x; s < SID_HIST_LCAP; s += blockDim.x) {
        if (lkeys[s] != SID_EMPTY_KEY)
            sid_global_insert(gkeys, gcnt, gmask, &stats[0], lkeys[s], lcnt[s]);
    }
}

__global__ void sid_hist_rehash_kernel(const unsigned long long* okeys, const unsigned long long* ocnt,
                                       uint64_t ocap, unsigned long long* gkeys,
                                       unsigned long long* gcnt, uint64_t gmask,
                                       unsigned long long* distinct)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ocap;
         i += (uint64_t)gridDim.x * blockDim.x)
        if (okeys[i] != SID_EMPTY_KEY) sid_global_insert(gkeys, gcnt, gmask, distinct, okeys[i], ocnt[i]);
}

// output slot of this lane in an append to *ctr by the lanes with take set:
// one atomic per wave (same-address atomics serialise at the memory side)
__device__ __forceinline__ unsigned long long sid_wave_append(bool take, unsigned long long* ctr)
{
    const unsigned long long mask = __ballot(take);
    if (mask == 0) return 0;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)mask) - 1u;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(mask));
    base = (unsigned long long)__shfl((long long)base, (int)leader);
    return base + (unsigned long long)__popcll(mask & ((1ull << lane) - 1ull));
}

// Compaction of a table into (key, count) pairs after *nout: each block owns a
// contiguous range, counts its entries, takes its output range with ONE
// global atomic (same-address device atomics cost ~13 ns each, serialised:
// one per wave was 27 us for a 128k-slot hash) and writes them in order.
// SRC::at(i, key, cnt) -> whether slot i holds an entry.
struct sid_hash_src {
    const unsigned long long* keys;
    const unsigned long long* cnt;
    __device__ bool at(uint64_t i, unsigned long long& k, unsigned long long& c) const
    {
        k = keys[i];
        if (k == SID_EMPTY_KEY) return false;
        c = cnt[i];
        return true;
    }
};

template <class SRC>
__global__ __launch_bounds__(256) void sid_compact_kernel(SRC src, uint64_t n, unsigned long long* __restrict__ okeys,
                                                          unsigned long long* __restrict__ ocnt,
                                                          unsigned long long* nout)
{
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    __shared__ uint32_t wc[4];
    __shared__ unsigned long long base;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t c = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 256) {
        unsigned long long k, v;
        c += src.at(i, k, v) ? 1u : 0u;
    }
    for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_down((int)c, off, 64);
    if (lane == 0) wc[wid] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = wc[0] + wc[1] + wc[2] + wc[3];
        base = t ? atomicAdd(nout, (unsigned long long)t) : 0ull;
    }
    __syncthreads();
    unsigned long long off0 = base;
    for (uint64_t b = lo; b < hi; b += 256) {
        const uint64_t i = b + threadIdx.x;
        unsigned long long k = 0, v = 0;
        const bool take = i < hi && src.at(i, k, v);
        const unsigned long long mask = __ballot(take);
        __syncthreads();   // wc of the previous tile consumed
        if (lane == 0) wc[wid] = (uint32_t)__popcll(mask);
        __syncthreads();
        uint32_t before = 0;
        for (int w = 0; w < wid; ++w) before += wc[w];
        if (take) {
            const unsigned long long o = off0 + before + (unsigned long long)__popcll(mask & ((1ull << lane) - 1ull));
            okeys[o] = k;
            ocnt[o] = v;
        }
        off0 += wc[0] + wc[1] + wc[2] + wc[3];
    }
}

// ------------------------------------------------ dense histogram ---------
// countUniqueProfiles (pileup.cpp:169-196) for the dense-coded profiles
// (sid_math.h): one LDS u32 counter per code, one ds_add per site, no probing.
// Each block writes its 64 KiB of counters to its own row of `part`
// (coalesced, no atomics: cross-block atomics on the hot codes serialise at
// the memory side), and sid_hist_reduce_kernel folds the rows into
// SID_DENSE_ROWS u64 rows.  Every other profile (het sites, deep or noisy
// columns; ~0.1% at 30x) is appended, as its key, to a global fallback list
// with one atomic per wave, and hashed by sid_hist_list_kernel.  16-B loads
// of site pairs, lanes contiguous.
typedef double sid_dvec2 __attribute__((ext_vector_type(2)));

// Fallback keys are collected in a per-block LDS list (one LDS atomic per
// key) and flushed with one global atomic per block: a global atomic per
// wave on the single list counter serialises at the memory side (measured:
// 8x the kernel's streaming time, tools/debug/hist_probe.hip).  Keys beyond
// the LDS capacity take the global counter directly.
#define SID_HIST_LLIST 1024

__device__ __forceinline__ void sid_fallback_append(bool fb, uint64_t key, unsigned long long* llist,
                                                    uint32_t* lcnt, unsigned long long* __restrict__ list,
                                                    uint64_t cap, unsigned long long* __restrict__ ctr)
{
    if (!fb) return;
    const uint32_t slot = atomicAdd(lcnt, 1u);
    if (slot < SID_HIST_LLIST) {
        llist[slot] = key;
        return;
    }
    const unsigned long long off = atomicAdd(ctr, 1ull);
    if (off < cap) list[off] = key;
}

constexpr int SID_HIST_PAIRS = 4;   // site pairs a lane keeps in flight (16 B each)
template <bool PAIRS>
__global__ __launch_bounds__(1024) void sid_hist_dense_kernel(const uint64_t* __restrict__ counts, size_t n,
                                                              uint32_t* __restrict__ part,
                                                              unsigned long long* __restrict__ list,
                                                              uint64_t cap, unsigned long long* __restrict__ ctr)
{
    __shared__ uint32_t H[SID_DENSE_N];
    __shared__ unsigned long long llist[SID_HIST_LLIST];
    __shared__ uint32_t lcnt;
    __shared__ unsigned long long lbase;
    for (uint32_t i = threadIdx.x; i < SID_DENSE_N; i += blockDim.x) H[i] = 0;
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
    if (PAIRS) {
        // SID_HIST_PAIRS site pairs per lane in flight (16 B each): one block of
        // 16 waves per CU (the 64 KiB table) is too few waves to cover the
        // HBM latency with two
        const ulonglong2* pairs = (const ulonglong2*)counts;
        const size_t npairs = n / 2;
        const size_t stride = (size_t)gridDim.x * blockDim.x;
        for (size_t base = (size_t)blockIdx.x * blockDim.x; base < npairs; base += SID_HIST_PAIRS * stride) {
            ulonglong2 c[SID_HIST_PAIRS];
            bool v[SID_HIST_PAIRS];
#pragma unroll
            for (int u = 0; u < SID_HIST_PAIRS; ++u) {
                const size_t p = base + threadIdx.x + u * stride;
                v[u] = p < npairs;
                c[u] = v[u] ? pairs[p] : make_ulonglong2(0, 0);
            }
#pragma unroll
            for (int k = 0; k < 2 * SID_HIST_PAIRS; ++k) {
                const uint64_t w = (k & 1) ? c[k >> 1].y : c[k >> 1].x;
                const bool vk = v[k >> 1];
                const uint32_t d = sid_dense_code(w);
                const bool fb = vk && d == SID_DENSE_NONE;
                if (vk && !fb) atomicAdd(&H[sid_dense_slot(d)], 1u);
                sid_fallback_append(fb, sid_profile_key(w), llist, &lcnt, list, cap, ctr);
            }
        }
        // odd last site
        if ((n & 1) && blockIdx.x == 0 && threadIdx.x < 64) {
            const bool mine = threadIdx.x == 0;
            const uint64_t w = mine ? counts[n - 1] : 0;
            const uint32_t d = sid_dense_code(w);
            const bool fb = mine && d == SID_DENSE_NONE;
            if (mine && !fb) atomicAdd(&H[sid_dense_slot(d)], 1u);
            sid_fallback_append(fb, sid_profile_key(w), llist, &lcnt, list, cap, ctr);
        }
    } else {
        for (size_t base = (size_t)blockIdx.x * blockDim.x; base < n; base += (size_t)gridDim.x * blockDim.x) {
            const size_t i = base + threadIdx.x;
            const bool v = i < n;
            const uint64_t w = v ? counts[i] : 0;
            const uint32_t d = sid_dense_code(w);
            const bool fb = v && d == SID_DENSE_NONE;
            if (v && !fb) atomicAdd(&H[sid_dense_slot(d)], 1u);
            sid_fallback_append(fb, sid_profile_key(w), llist, &lcnt, list, cap, ctr);
        }
    }
    __syncthreads();
    uint32_t* row = part + (size_t)blockIdx.x * SID_DENSE_N;
    for (uint32_t i = threadIdx.x; i < SID_DENSE_N; i += blockDim.x) row[i] = H[sid_dense_slot(i)];
    const uint32_t nl = lcnt < SID_HIST_LLIST ? lcnt : SID_HIST_LLIST;
    if (nl == 0) return;
    if (threadIdx.x == 0) lbase = atomicAdd(ctr, (unsigned long long)nl);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
        if (lbase + i < cap) list[lbase + i] = llist[i];
}

// dense[g][code] += sum of the block rows of row group g (one thread per code
// and group; no atomics)
__global__ __launch_bounds__(256) void sid_hist_reduce_kernel(const uint32_t* __restrict__ part, uint32_t nrows,
                                                              unsigned long long* __restrict__ dense)
{
    const uint32_t code = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t g = blockIdx.y;
    const uint32_t r0 = (uint32_t)((uint64_t)nrows * g / SID_DENSE_ROWS);
    const uint32_t r1 = (uint32_t)((uint64_t)nrows * (g + 1) / SID_DENSE_ROWS);
    unsigned long long a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint32_t r = r0;
    for (; r + 4 <= r1; r += 4) {
        a0 += part[(size_t)r * SID_DENSE_N + code];
        a1 += part[(size_t)(r + 1) * SID_DENSE_N + code];
        a2 += part[(size_t)(r + 2) * SID_DENSE_N + code];
        a3 += part[(size_t)(r + 3) * SID_DENSE_N + code];
    }
    for (; r < r1; ++r) a0 += part[(size_t)r * SID_DENSE_N + code];
    dense[(size_t)g * SID_DENSE_N + code] += a0 + a1 + a2 + a3;
}

// the fallback list into the global hash (the all-65535 key to stats[1])
// The fallback keys: each block pre-aggregates its contiguous range (at most
// SID_LIST_PER keys) in an LDS table, so hot keys (common het profiles) reach
// the global hash once per block, and the new-key / special counts take one
// atomic per block.
#define SID_LIST_PER 1024
#define SID_LIST_LDS 2048
__global__ __launch_bounds__(256) void sid_hist_list_kernel(const unsigned long long* __restrict__ list, uint64_t m,
                                                            unsigned long long* gkeys, unsigned long long* gcnt,
                                                            uint64_t gmask, unsigned long long* stats)
{
    __shared__ unsigned long long lk[SID_LIST_LDS];
    __shared__ uint32_t lc[SID_LIST_LDS];
    __shared__ unsigned long long red[2][4];
    for (int i = threadIdx.x; i < SID_LIST_LDS; i += blockDim.x) {
        lk[i] = SID_EMPTY_KEY;
        lc[i] = 0;
    }
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * SID_LIST_PER;
    const uint64_t hi = lo + SID_LIST_PER < m ? lo + SID_LIST_PER : m;
    unsigned long long nnew = 0, nspecial = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const uint64_t key = list[i];
        if (key == SID_EMPTY_KEY) {
            ++nspecial;
            continue;
        }
        // at most SID_LIST_PER distinct keys in 2x as many slots: always lands
        uint32_t h = (uint32_t)sid_hash64(key) & (SID_LIST_LDS - 1);
        for (;;) {
            const unsigned long long prev = atomicCAS(&lk[h], SID_EMPTY_KEY, (unsigned long long)key);
            if (prev == SID_EMPTY_KEY || prev == key) {
                atomicAdd(&lc[h], 1u);
                break;
            }
            h = (h + 1) & (SID_LIST_LDS - 1);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < SID_LIST_LDS; i += blockDim.x)
        if (lk[i] != SID_EMPTY_KEY) nnew += sid_global_insert_new(gkeys, gcnt, gmask, lk[i], lc[i]);
    for (int off = 32; off > 0; off >>= 1) {
        nnew += __shfl_down(nnew, off, 64);
        nspecial += __shfl_down(nspecial, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = nnew;
        red[1][threadIdx.x >> 6] = nspecial;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] +
                                     red[threadIdx.x][3];
        if (v) atomicAdd(&stats[threadIdx.x], v);
    }
}

// non-zero dense counters (summed over the SID_DENSE_ROWS rows) -> (key, count)
struct sid_dense_src {
    const unsigned long long* dense;
    __device__ bool at(uint64_t i, unsigned long long& k, unsigned long long& c) const
    {
        unsigned long long v = 0;
        for (int g = 0; g < SID_DENSE_ROWS; ++g) v += dense[(size_t)g * SID_DENSE_N + i];
        if (!v) return false;
        k = sid_profile_key(sid_dense_word((uint32_t)i));
        c = v;
        return true;
    }
};

// ------------------------------------------------ 10-genotype mixture -----
// sid_lynch_eval: sid_math.h

__device__ __forceinline__ double sid_lse2(double a, double b)
{
    if (isnan(a) || isnan(b)) return a + b;   // NaN operands propagate (fmax would drop them)
    double m = fmax(a, b);
    if (m == -__builtin_inf()) return m;
    return m + log1p(exp(fmin(a, b) - m));
}

// one powl factor n*ln(base); 0 when n == 0; underflow of the long double -> 0
__device__ __forceinline__ double sid_pow_ln(double lbase, uint32_t n)
{
    if (n == 0) return 0.0;
    double v = (double)n * lbase;
    return v < SID_LN_LDBL_TRUE_MIN ? -__builtin_inf() : v;
}

// ln of d * powl(x, a) * powl(y, b) with the reference's underflow points
__device__ __forceinline__ double sid_term(double ld, double pa, double pb)
{
    double t = ld + pa;
    if (t < SID_LN_LDBL_TRUE_MIN) return -__builtin_inf();
    t += pb;
    return t < SID_LN_LDBL_TRUE_MIN ? -__builtin_inf() : t;
}

// ln of the pre-M sums of lynch.hpp:82-90 (hom) and :57-74 (het)
__device__ __forceinline__ void sid_mixture(uint64_t key, const sid_lynch_eval& E, double& s_hom,
                                            double& s_het)
{
    uint32_t n[4] = {(uint32_t)(key >> 48), (uint32_t)((key >> 32) & 0xffff),
                     (uint32_t)((key >> 16) & 0xffff), (uint32_t)(key & 0xffff)};
    const uint32_t c = n[0] + n[1] + n[2] + n[3];
    double m = -__builtin_inf();
    double t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        t[i] = sid_term(E.ld[i], sid_pow_ln(E.la, n[i]), sid_pow_ln(E.lb, c - n[i]));
        m = fmax(m, t[i]);
    }
    double acc = 0.0;
    if (m != -__builtin_inf()) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += exp(t[i] - m);
        s_hom = m + log(acc);
    } else {
        s_hom = m;
    }
    double u[6];
    double mu = -__builtin_inf();
    int k = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = i + 1; j < 4; ++j) {
            u[k] = sid_term(E.ldd[k], sid_pow_ln(E.lh, n[i] + n[j]), sid_pow_ln(E.lb, c - n[i] - n[j]));
            mu = fmax(mu, u[k]);
            ++k;
        }
    if (E.lnorm == __builtin_inf()) {
        // one base only in the distribution: every d_i d_j is 0 and so is
        // 1 - sum d^2, so the reference's het likelihood is 0/0 = -nan
        // (lynch.hpp:70-72), and so is every L that contains it
        s_het = -__builtin_nan("");
    } else if (mu != -__builtin_inf()) {
        double a2 = 0.0;
#pragma unroll
        for (int q = 0; q < 6; ++q) a2 += exp(u[q] - mu);
        s_het = mu + log(a2) + E.lnorm;
    } else {
        s_het = mu;
    }
}

// ---- the mixture as the reference's long doubles, every operation rounded
// (ld_round: x87 overflow, denormal steps, underflow), in its order of
// evaluation (lynch.hpp:48-96): for the profiles whose likelihoods leave the
// normal long double range (coverage in the thousands), where the log-domain
// sums above lose the reference's denormal quantisation, a 0 * inf = NaN or an
// inf (multinomialCoefficient over LDBL_MAX).
__device__ __forceinline__ sid_ld ld_ln(double ln)
{
    sid_ld r;
    r.ln = ln;
    r.neg = 0;
    return r;
}
// a + b, both >= 0 (NaN propagates)
__device__ __forceinline__ sid_ld ld_add_pos(sid_ld a, sid_ld b)
{
    if (isnan(a.ln) || isnan(b.ln)) return ld_ln(a.ln + b.ln);
    const double m = fmax(a.ln, b.ln);
    if (m == -__builtin_inf() || m == __builtin_inf()) return ld_ln(m);
    return ld_round(ld_ln(m + log1p(exp(fmin(a.ln, b.ln) - m))));
}
// d * powl(x, a) * powl(y, b) (lynch.hpp:65-66, :85-86): ld = ln d (a double),
// lx, ly the bases' logs
__device__ __forceinline__ sid_ld ld_term(double ld, double lx, uint32_t a, double ly, uint32_t b)
{
    const sid_ld px = a ? ld_round(ld_ln((double)a * lx)) : ld_ln(0.0);
    const sid_ld py = b ? ld_round(ld_ln((double)b * ly)) : ld_ln(0.0);
    return ld_mul(ld_mul(ld_ln(ld), px), py);
}
// homozygousLikelihood / heterozygousLikelihood (lynch.hpp:57-74, :82-90)
__device__ __noinline__ void sid_mixture_ld(uint64_t key, const sid_lynch_eval& E, double lnM, sid_ld* hom,
                                            sid_ld* het)
{
    const uint32_t n[4] = {(uint32_t)(key >> 48), (uint32_t)((key >> 32) & 0xffff),
                           (uint32_t)((key >> 16) & 0xffff), (uint32_t)(key & 0xffff)};
    const uint32_t c = n[0] + n[1] + n[2] + n[3];
    const sid_ld M = ld_round(ld_ln(lnM));   // expl of the double lnGamma sum
    sid_ld L = ld_ln(-__builtin_inf());
    for (int i = 0; i < 4; ++i) L = ld_add_pos(L, ld_term(E.ld[i], E.la, n[i], E.lb, c - n[i]));
    *hom = ld_mul(M, L);
    sid_ld H = ld_ln(-__builtin_inf());
    int k = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = i + 1; j < 4; ++j, ++k) H = ld_add_pos(H, ld_term(E.ldd[k], E.lh, n[i] + n[j], E.lb, c - n[i] - n[j]));
    H = ld_round(ld_ln(H.ln + E.lnorm));     // L /= (1 - s): 0 / 0 = NaN when 1 - s is 0
    *het = ld_mul(M, H);
}
// the log-domain path is exact (to double rounding) while every intermediate
// of the reference is a normal long double with 64 bits to spare: the sums
// (the smallest partial result feeding a later operation) above LDBL_MIN *
// 2^64 and M below LDBL_MAX.  A sum the log-domain path finds empty is not
// taken as 0: its terms are cut at LDBL_TRUE_MIN, the reference's round to
// the nearest multiple of it (a term of 0.55 units is 1 unit there).
__device__ __forceinline__ bool sid_mixture_normal(double sh, double st, double lnM)
{
    constexpr double lo = SID_LN_LDBL_MIN + 64.0 * SID_LN2;
    return lnM < SID_LN_LDBL_MAX - 1.0 && sh > lo && (isnan(st) || st > lo);
}

__device__ __forceinline__ void sid_two_sum(double a, double b, double& s, double& e)
{
    s = a + b;
    double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}

// One (pi, eps) point per blockIdx.y.  Each block reduces its share of
// sum count*ln L in double-double into partial[point][block]; a second kernel
// (sid_objective_fold_kernel) adds the block partials in block order.  Two
// launches cost less than a last-block ticket (per-block device-scope fence +
// same-address atomic: +7 us per launch at 188 blocks) and than block
// partials written straight to host-mapped memory and folded by the host
// (+1.7 us per round trip) (tools/debug/obj_probe.hip).
// sum count * ln L over one slice of the profiles (i = slice*256 + tid +
// j*nslices*256) reduced over the block in double-double; the result is in
// thread 0.  blockDim.x == 256.
__device__ __forceinline__ void sid_objective_slice(const uint64_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ cnt,
                                                    const double* __restrict__ lnM, size_t u, size_t slice,
                                                    size_t nslices, const sid_lynch_eval& E, double& H,
                                                    double& Lo)
{
    double hi = 0.0, lo = 0.0;
    for (size_t i = slice * blockDim.x + threadIdx.x; i < u; i += nslices * blockDim.x) {
        double sh, st;
        sid_mixture(keys[i], E, sh, st);
        // L = (1-pi) M S_hom + pi M S_het  (lynch.cpp:46-47); M multiplies last
        double lhom = sh == -__builtin_inf() ? sh : lnM[i] + sh;
        double lhet = st == -__builtin_inf() ? st : lnM[i] + st;
        double lL = sid_lse2(E.l1p + lhom, E.lp + lhet);
        constexpr double nlo = SID_LN_LDBL_MIN + 64.0 * SID_LN2;
        if (!sid_mixture_normal(sh, st, lnM[i]) || (E.l1p + lhom < nlo && lhom != -__builtin_inf()) ||
            (E.lp + lhet < nlo && lhet != -__builtin_inf())) {
            sid_ld hm, ht;
            sid_mixture_ld(keys[i], E, lnM[i], &hm, &ht);
            lL = ld_add_pos(ld_mul(ld_ln(E.l1p), hm), ld_mul(ld_ln(E.lp), ht)).ln;
        }
        if (lL > -__builtin_inf() && !isnan(lL)) {   // if (L > 0)
            double v = lL * (double)cnt[i];          // logl(L) * p.count
            double p = fma(lL, (double)cnt[i], -v);  // exact product error
            double s, e;
            sid_two_sum(hi, v, s, e);
            hi = s;
            lo += e + p;
        }
    }
    // wave64 then block reduction, double-double
    __shared__ double sh_hi[4], sh_lo[4];
    for (int off = 32; off > 0; off >>= 1) {
        double ohi = __shfl_down(hi, off, 64);
        double olo = __shfl_down(lo, off, 64);
        double s, e;
        sid_two_sum(hi, ohi, s, e);
        hi = s;
        lo += olo + e;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        sh_hi[wid] = hi;
        sh_lo[wid] = lo;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        H = 0.0;
        Lo = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            double s, e;
            sid_two_sum(H, sh_hi[w], s, e);
            H = s;
            Lo += sh_lo[w] + e;
        }
    }
    __syncthreads();   // sh_hi/sh_lo reusable
}

__global__ __launch_bounds__(256) void sid_objective_kernel(const uint64_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ cnt,
                                                            const double* __restrict__ lnM, size_t u,
                                                            sid_lynch_evals EV, double* __restrict__ partial)
{
    const int pt = blockIdx.y;
    sid_lynch_eval E;
    E.la = EV.p[pt].la;
    E.lb = EV.p[pt].lb;
    E.lh = EV.p[pt].lh;
    E.l1p = EV.p[pt].l1p;
    E.lp = EV.p[pt].lp;
#pragma unroll
    for (int i = 0; i < 4; ++i) E.ld[i] = EV.ld[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) E.ldd[i] = EV.ldd[i];
    E.lnorm = EV.lnorm;
    double H, Lo;
    sid_objective_slice(keys, cnt, lnM, u, blockIdx.x, gridDim.x, E, H, Lo);
    if (threadIdx.x == 0) {
        double* part = partial + ((size_t)pt * gridDim.x + blockIdx.x) * 2;
        part[0] = H;
        part[1] = Lo;
    }
}

// One block per point: the nb block partials (in parallel, then a fixed
// tree), {hi, lo} and the call's sequence number into host-mapped memory, so
// the host reads the result without a copy.
__global__ __launch_bounds__(256) void sid_objective_fold_kernel(const double* __restrict__ partial, int nb,
                                                                 double* out, volatile unsigned int* seq_out,
                                                                 unsigned int seq)
{
    const int pt = blockIdx.x;
    const double* part = partial + (size_t)pt * nb * 2;
    double bh = 0.0, bl = 0.0;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        double s, e;
        sid_two_sum(bh, part[2 * b], s, e);
        bh = s;
        bl += part[2 * b + 1] + e;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ohi = __shfl_down(bh, off, 64);
        const double olo = __shfl_down(bl, off, 64);
        double s, e;
        sid_two_sum(bh, ohi, s, e);
        bh = s;
        bl += olo + e;
    }
    __shared__ double sh_hi[4], sh_lo[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        sh_hi[wid] = bh;
        sh_lo[wid] = bl;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double H = 0.0, Lo = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        double s, e;
        sid_two_sum(H, sh_hi[w], s, e);
        H = s;
        Lo += sh_lo[w] + e;
    }
    double s, e;
    sid_two_sum(H, Lo, s, e);   // normalise
    out[2 * pt] = s;
    out[2 * pt + 1] = e;
    __threadfence_system();
    seq_out[pt] = seq;
}

// ------------------------------------------------ device-resident estimate --
// estimateProfileGenotypeLikelihoods (lynch.cpp:17-35) + FunctionMinimizer
// (optimization.hpp:50-89) in one cooperative launch: G co-resident blocks
// evaluate the objective for the points Nelder-Mead asks for (work items =
// point x 256-profile slice, the slices of sid_objective_kernel), meet at a
// grid barrier, and every block folds the partials and advances its own copy
// of the simplex (sid_nm.h arithmetic) — the same values in every block, so
// they all request the same points next and stop together: one barrier per
// round and no host round trip.
//
// The simplex is advanced by wave 0 of each block with all 64 lanes running
// the same (uniform) code on register-resident state; the value cache is
// lane-distributed (lane i holds entry i), so a lookup is one compare and a
// ballot instead of a serial scan.  An iteration whose candidate values are
// not all known is undone and its candidates (with lookahead: also the next
// iteration's) become the next round's points; earlier values stay cached,
// so the replay after the round takes the exact path the host driver takes.
// Every wait is bounded by a wall-clock deadline: on expiry the kernel sets
// an abort flag that every block polls, all blocks leave, and the host falls
// back to the host driver.
#define SID_NM_MAX_ROUNDS 4096
#define SID_NM_ITER_MAX 1000   // optimization.hpp:79 (i < 1000)

// wave-0 controller state: uniform across the wave except the cache
struct sid_nmw {
    sid_nm_simplex S;
    int phase;   // 0: simplex not set, 1: iterating
    int iter;
    int state;   // 0 running, else 16 + sid_nm_result.status
    int converged;
    unsigned long long evals;
    double x[2], fval, size;
    double cx, cy, cv;   // this lane's cache entry
    int cn, chead;
    double rx, ry;       // this lane's point of the next round
    int npts;
};

// what wave 0 posts for a round (LDS)
struct sid_nm_round {
    int go;
    int npts, ne;
    double pts[SID_OBJ_PTS][2];
    double val[SID_OBJ_PTS];
    int evl[SID_OBJ_PTS];
    sid_lynch_pt prm[SID_OBJ_PTS];
};

__device__ __forceinline__ int sid_lane() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ bool sid_nmw_get(const sid_nmw& w, const double* x, double& v)
{
    const bool hit = sid_lane() < w.cn && w.cx == x[0] && w.cy == x[1];
    const unsigned long long m = __ballot(hit);
    if (!m) return false;
    v = __shfl(w.cv, __ffsll((unsigned long long)m) - 1, 64);
    return true;
}

__device__ __forceinline__ void sid_nmw_put(sid_nmw& w, double x0, double x1, double v)
{
    if (sid_lane() == w.chead) {
        w.cx = x0;
        w.cy = x1;
        w.cv = v;
    }
    w.chead = (w.chead + 1) & 63;
    if (w.cn < 64) ++w.cn;
}

// appends x to the lane-held point list unless present or full
__device__ __forceinline__ void sid_nmw_add(sid_nmw& w, const double* x)
{
    const bool dup = sid_lane() < w.npts && w.rx == x[0] && w.ry == x[1];
    if (__ballot(dup)) return;
    if (w.npts >= SID_OBJ_PTS) return;
    if (sid_lane() == w.npts) {
        w.rx = x[0];
        w.ry = x[1];
    }
    ++w.npts;
}

// the points of the next round: the iteration's candidates (+ lookahead, as
// sid_nm_request) that are not cached
__device__ __forceinline__ void sid_nmw_request(sid_nmw& w, bool lookahead)
{
    w.npts = 0;
    int hi, s_hi, lo;
    sid_nm_order(w.S, hi, s_hi, lo);
    double c1[4][SID_NM_N];
    sid_nm_candidates(w.S, hi, c1);
    double t;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (!sid_nmw_get(w, c1[i], t)) sid_nmw_add(w, c1[i]);
    if (!lookahead) return;
    for (int o = 0; o < 4; ++o) {
        sid_nm_simplex s = w.S;
        if (o == 0) sid_nm_update_point(s, hi, c1[0], 0.0);   // reflection accepted
        if (o == 1) sid_nm_update_point(s, hi, c1[1], 0.0);   // expansion accepted
        if (o == 2) {                                         // outside contraction
            sid_nm_update_point(s, hi, c1[0], 0.0);
            sid_nm_update_point(s, hi, c1[3], 0.0);
        }
        if (o == 3) sid_nm_update_point(s, hi, c1[2], 0.0);   // inside contraction
        for (int q = 0; q < 2; ++q) {
            const int h2 = q == 0 ? s_hi : hi;
            if (h2 == hi && o < 2) continue;
            double c2[4][SID_NM_N];
            sid_nm_candidates(s, h2, c2);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (!sid_nmw_get(w, c2[i], t)) sid_nmw_add(w, c2[i]);
        }
    }
}

// nmsimplex2_set with the three start values known; 1: need, -1: non-finite
__device__ __forceinline__ int sid_nmw_try_set(sid_nmw& w, const double* x, const double* step)
{
    const double p0[2] = {x[0], x[1]}, p1[2] = {x[0] + step[0], x[1]}, p2[2] = {x[0], x[1] + step[1]};
    double v0, v1, v2;
    const bool h0 = sid_nmw_get(w, p0, v0), h1 = sid_nmw_get(w, p1, v1), h2 = sid_nmw_get(w, p2, v2);
    if (!(h0 && h1 && h2)) {
        w.npts = 0;
        if (!h0) sid_nmw_add(w, p0);
        if (!h1) sid_nmw_add(w, p1);
        if (!h2) sid_nmw_add(w, p2);
        return 1;
    }
    // f(x), then f(x + step_i e_i) in order, stopping at the first non-finite
    ++w.evals;
    if (!isfinite(v0)) return -1;
    ++w.evals;
    if (!isfinite(v1)) return -1;
    ++w.evals;
    if (!isfinite(v2)) return -1;
    w.S.x1[0][0] = p0[0];
    w.S.x1[0][1] = p0[1];
    w.S.x1[1][0] = p1[0];
    w.S.x1[1][1] = p1[1];
    w.S.x1[2][0] = p2[0];
    w.S.x1[2][1] = p2[1];
    w.S.y1[0] = v0;
    w.S.y1[1] = v1;
    w.S.y1[2] = v2;
    sid_nm_compute_center(w.S);
    w.size = sid_nm_compute_size(w.S);
    return 0;
}

// nmsimplex2_iterate on a copy of the simplex, committed only when every value
// it asks for is known.  0: done, 1: need (points listed), -1: contraction failed
__device__ __forceinline__ int sid_nmw_try_iterate(sid_nmw& w, bool lookahead)
{
    sid_nm_simplex t = w.S;
    unsigned long long ev = 0;
    int hi, s_hi, lo;
    sid_nm_order(t, hi, s_hi, lo);
    double xc[2], xc2[2], val, val2;
    bool miss = false;
    sid_nm_corner_point(t, -1.0, hi, xc);
    ++ev;
    if (!sid_nmw_get(w, xc, val)) miss = true;
    if (!miss) {
        if (isfinite(val) && val < t.y1[lo]) {
            sid_nm_corner_point(t, -2.0, hi, xc2);
            ++ev;
            if (!sid_nmw_get(w, xc2, val2)) {
                miss = true;
            } else if (isfinite(val2) && val2 < t.y1[lo]) {
                sid_nm_update_point(t, hi, xc2, val2);
            } else {
                sid_nm_update_point(t, hi, xc, val);
            }
        } else if (!isfinite(val) || val > t.y1[s_hi]) {
            if (isfinite(val) && val <= t.y1[hi]) sid_nm_update_point(t, hi, xc, val);
            sid_nm_corner_point(t, 0.5, hi, xc2);
            ++ev;
            if (!sid_nmw_get(w, xc2, val2)) {
                miss = true;
            } else if (isfinite(val2) && val2 <= t.y1[hi]) {
                sid_nm_update_point(t, hi, xc2, val2);
            } else {
                // contract_by_best(lo): the two other vertices move halfway
                // to the best one (x1[lo] itself does not move)
                const int a = lo == 0 ? 1 : 0, b = lo == 2 ? 1 : 2;
                double pa[2], pb[2], va, vb;
                for (int j = 0; j < SID_NM_N; ++j) {
                    pa[j] = 0.5 * (t.x1[a][j] + t.x1[lo][j]);
                    pb[j] = 0.5 * (t.x1[b][j] + t.x1[lo][j]);
                }
                const bool ha = sid_nmw_get(w, pa, va), hb = sid_nmw_get(w, pb, vb);
                if (!(ha && hb)) {
                    w.npts = 0;
                    if (!ha) sid_nmw_add(w, pa);
                    if (!hb) sid_nmw_add(w, pb);
                    return 1;
                }
                for (int j = 0; j < SID_NM_N; ++j) {
                    t.x1[a][j] = pa[j];
                    t.x1[b][j] = pb[j];
                }
                ev += 2;
                t.y1[a] = va;
                t.y1[b] = vb;
                const bool ok = isfinite(va) && isfinite(vb);
                sid_nm_compute_center(t);
                sid_nm_compute_size(t);
                if (!ok) return -1;
            }
        } else {
            sid_nm_update_point(t, hi, xc, val);
        }
    }
    if (miss) {
        sid_nmw_request(w, lookahead);
        return 1;
    }
    w.S = t;
    w.evals += ev;
    const int imin = sid_nm_min_index(w.S);
    w.x[0] = w.S.x1[imin][0];
    w.x[1] = w.S.x1[imin][1];
    w.fval = w.S.y1[imin];
    w.size = w.S.S2 > 0 ? sqrt(w.S.S2) : sid_nm_compute_size(w.S);
    return 0;
}

// runs the algorithm as far as the known values allow (wave 0, uniform)
__device__ __forceinline__ void sid_nmw_advance(sid_nmw& w, const double* x0, const double* step, bool lookahead)
{
    w.npts = 0;
    while (w.state == 0) {
        if (w.phase == 0) {
            const int r = sid_nmw_try_set(w, x0, step);
            if (r == 1) break;
            if (r < 0) {
                w.state = 16 + 1;
                break;
            }
            w.phase = 1;
            continue;
        }
        const int r = sid_nmw_try_iterate(w, lookahead);
        if (r == 1) break;
        ++w.iter;
        if (r < 0) {
            w.state = 16 + 1;   // "contraction failed"
            break;
        }
        if (w.size < 1e-5) {
            w.state = 16;
            w.converged = 1;
        } else if (w.iter >= SID_NM_ITER_MAX) {
            w.state = 16;
            w.converged = 0;
        }
    }
    if (w.state == 0 && w.npts == 0) w.state = 16 + 4;   // no progress possible: never expected
}

// wave 0: the round's points into LDS; out of [0,1]^2 -> DBL_MAX without
// evaluation (lynch.cpp:40-42), an empty table -> -0.0
// (static_cast<double>(-0.0L)); lynch.hpp:57-90 constants of the others
__device__ __forceinline__ void sid_nmw_post(const sid_nmw& w, size_t u, sid_nm_round& R)
{
    const int lane = sid_lane();
    const bool mine = lane < w.npts;
    const double pi = w.rx, e = w.ry;
    const bool out = mine && (pi < 0 || pi > 1 || e < 0 || e > 1);
    const bool ev = mine && !out && u != 0;
    const unsigned long long em = __ballot(ev);
    if (mine) {
        R.pts[lane][0] = pi;
        R.pts[lane][1] = e;
        if (!ev) R.val[lane] = out ? DBL_MAX : -0.0;
    }
    if (ev) {
        const int q = __popcll(em & ((1ull << lane) - 1ull));
        R.evl[q] = lane;
        R.prm[q] = {log(1 - e), log(e / 3.), log((1 - 2. / 3. * e) / 2.), log(1. - pi), log(pi)};
    }
    if (lane == 0) {
        R.npts = w.npts;
        R.ne = __popcll(em);
        R.go = w.state == 0;
    }
}

// thread 0: arrive at the round's barrier and wait for every block; false on
// abort (another block gave up) or when this block's deadline passes
__device__ bool sid_nm_barrier(unsigned int* bar, unsigned int target, int* abort_flag, long long deadline)
{
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    // relaxed polls (an acquire load would invalidate this XCD's L2 on every
    // poll, under the blocks still evaluating); the caller fences once
    unsigned int spins = 0;
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if ((++spins & 31) == 0) {
            if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
            if (wall_clock64() > deadline) {
                __hip_atomic_store(abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
    return true;
}

__global__ __launch_bounds__(256) void sid_nm_kernel(const uint64_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ cnt,
                                                     const double* __restrict__ lnM, size_t u, int nb,
                                                     sid_nm_dist D, double x00, double x01, double st0,
                                                     double st1, int lookahead, double* partial,
                                                     unsigned int* bar, int* abort_flag, long long timeout,
                                                     sid_nm_result* res)
{
    __shared__ sid_nm_round R;
    __shared__ int alive;
    const double x0[2] = {x00, x01}, step[2] = {st0, st1};
    const long long deadline = wall_clock64() + timeout;
    const unsigned int G = gridDim.x;
    const bool w0 = threadIdx.x < 64;
    sid_nmw w;
    if (w0) {
        w.cn = w.chead = 0;
        w.cx = w.cy = w.cv = 0.0;
        w.rx = w.ry = 0.0;
        w.phase = w.iter = w.state = w.converged = 0;
        w.evals = 0;
        w.x[0] = x0[0];
        w.x[1] = x0[1];
        w.fval = w.size = 0.0;
        sid_nmw_advance(w, x0, step, lookahead != 0);
        sid_nmw_post(w, u, R);
    }
    if (threadIdx.x == 0) alive = 1;
    __syncthreads();
    int round = 0;
    unsigned long long points = 0;
    long long tk[4] = {0, 0, 0, 0}, t0 = wall_clock64(), t1;
    for (;;) {
        if (!R.go || !alive || round >= SID_NM_MAX_ROUNDS) break;
        const int ne = R.ne;
        double* part = partial + (size_t)(round & 1) * SID_OBJ_PTS * nb * 2;
        for (int it = blockIdx.x; it < ne * nb; it += G) {
            const int q = it / nb, s = it - q * nb;
            sid_lynch_eval E;
            E.la = R.prm[q].la;
            E.lb = R.prm[q].lb;
            E.lh = R.prm[q].lh;
            E.l1p = R.prm[q].l1p;
            E.lp = R.prm[q].lp;
#pragma unroll
            for (int i = 0; i < 4; ++i) E.ld[i] = D.ld[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) E.ldd[i] = D.ldd[i];
            E.lnorm = D.lnorm;
            double H, Lo;
            sid_objective_slice(keys, cnt, lnM, u, s, nb, E, H, Lo);
            if (threadIdx.x == 0) {
                part[((size_t)q * nb + s) * 2] = H;
                part[((size_t)q * nb + s) * 2 + 1] = Lo;
            }
        }
        t1 = wall_clock64();
        tk[0] += t1 - t0;
        t0 = t1;
        if (threadIdx.x == 0) alive = sid_nm_barrier(bar, G * (unsigned)(round + 1), abort_flag, deadline);
        __syncthreads();
        if (!alive) break;
        t1 = wall_clock64();
        tk[1] += t1 - t0;
        t0 = t1;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // fold: one wave per point, lanes over the slices, double-double
        const int lane = sid_lane(), wid = threadIdx.x >> 6;
        for (int q = wid; q < ne; q += (int)(blockDim.x >> 6)) {
            double bh = 0.0, bl = 0.0;
            for (int b = lane; b < nb; b += 64) {
                double s, e;
                sid_two_sum(bh, part[((size_t)q * nb + b) * 2], s, e);
                bh = s;
                bl += part[((size_t)q * nb + b) * 2 + 1] + e;
            }
            for (int off = 32; off > 0; off >>= 1) {
                const double ohi = __shfl_down(bh, off, 64);
                const double olo = __shfl_down(bl, off, 64);
                double s, e;
                sid_two_sum(bh, ohi, s, e);
                bh = s;
                bl += olo + e;
            }
            if (lane == 0) {
                double s, e;
                sid_two_sum(bh, bl, s, e);
                R.val[R.evl[q]] = -s;   // -(sum) (lynch.cpp:59-60); an infinite sum stays infinite
            }
        }
        __syncthreads();
        t1 = wall_clock64();
        tk[2] += t1 - t0;
        t0 = t1;
        if (w0) {
            points += ne;
            const int np = R.npts;
            for (int i = 0; i < np; ++i) sid_nmw_put(w, R.pts[i][0], R.pts[i][1], R.val[i]);
            sid_nmw_advance(w, x0, step, lookahead != 0);
        }
        __syncthreads();   // R read by every wave above
        if (w0) {
            if (w.state == 0 && round + 1 >= SID_NM_MAX_ROUNDS) w.state = 16 + 3;
            sid_nmw_post(w, u, R);
        }
        __syncthreads();
        t1 = wall_clock64();
        tk[3] += t1 - t0;
        t0 = t1;
        ++round;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        res->x[0] = w.x[0];
        res->x[1] = w.x[1];
        res->fval = w.fval;
        res->size = w.size;
        res->iterations = w.iter;
        res->converged = w.converged;
        res->status = !alive ? 2 : (w.state >= 16 ? w.state - 16 : 4);
        res->rounds = round;
        res->evals = w.evals;
        res->points = points;
        for (int i = 0; i < 4; ++i) res->ticks[i] = tk[i];
    }
}

// Per-profile L_hom, L_het at eps-hat as emulated long doubles (ln, sign=+).
__global__ __launch_bounds__(256) void sid_profile_lik_kernel(const uint64_t* __restrict__ keys,
                                                              const double* __restrict__ lnM,
                                                              size_t u, sid_lynch_eval E,
                                                              double* __restrict__ lhom,
                                                              double* __restrict__ lhet)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < u;
         i += (size_t)gridDim.x * blockDim.x) {
        double sh, st;
        sid_mixture(keys[i], E, sh, st);
        if (!sid_mixture_normal(sh, st, lnM[i])) {
            sid_ld hm, ht;
            sid_mixture_ld(keys[i], E, lnM[i], &hm, &ht);
            lhom[i] = hm.ln;
            lhet[i] = ht.ln;
            continue;
        }
        sid_ld M;
        M.ln = lnM[i];
        M.neg = 0;
        M = ld_round(M);
        sid_ld H, T;
        H.ln = sh;
        H.neg = 0;
        T.ln = st;
        T.neg = 0;
        lhom[i] = ld_mul(M, ld_round(H)).ln;
        lhet[i] = ld_mul(M, ld_round(T)).ln;
    }
}

// mode 0: likelihood_ratio p-values (before BH); mode 1: bayes posteriors.
__global__ __launch_bounds__(256) void sid_classify_kernel(const uint64_t* __restrict__ keys,
                                                           const double* __restrict__ lhom,
                                                           const double* __restrict__ lhet, size_t u,
                                                           int mode, int use_prior, double pi,
                                                           double lg15, double* __restrict__ c1,
                                                           double* __restrict__ c2,
                                                           uint8_t* __restrict__ code)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < u;
         i += (size_t)gridDim.x * blockDim.x) {
        sid_ld H, T;
        H.ln = lhom[i];
        H.neg = 0;
        T.ln = lhet[i];
        T.neg = 0;
        // profile_t from the key, then majors (call.cpp:52-60)
        const uint64_t k = keys[i];
        const uint64_t w = (k >> 48) | (((k >> 32) & 0xffff) << 16) | (((k >> 16) & 0xffff) << 32) |
                           ((k & 0xffff) << 48);
        uint32_t f, s, nf, ns, cov;
        sid_major(w, f, s, nf, ns, cov);
        if (mode == 0) {
            if (use_prior) {                                  // call.cpp:94-97
                T = ld_mul(T, ld_from_double(pi));
                H = ld_mul(H, ld_from_double(1 - pi));
            }
            c1[i] = ld_lrt(T, H, lg15);                       // p_hom
            c2[i] = ld_lrt(H, T, lg15);                       // p_het
            code[i] = (uint8_t)(f | (s << 2));                // label decided after BH (host)
        } else {
            sid_ld aH = ld_mul(H, ld_from_double(1 - pi));    // call.cpp:177-178
            sid_ld aT = ld_mul(T, ld_from_double(pi));
            sid_ld sum;
            sum.ln = sid_lse2(aH.ln, aT.ln);
            sum.neg = 0;
            sum = ld_round(sum);
            double ph, pt;
            if (ld_is_zero(sum) || isnan(sum.ln) || isinf(sum.ln)) {
                ph = (ld_is_zero(aH) && !ld_is_zero(sum)) ? 0.0 : -__builtin_nan("");
                pt = (ld_is_zero(aT) && !ld_is_zero(sum)) ? 0.0 : -__builtin_nan("");
            } else {
                ph = exp(aH.ln - sum.ln);
                pt = exp(aT.ln - sum.ln);
            }
            c1[i] = sid_x86_nan(ph);
            c2[i] = sid_x86_nan(pt);
            const bool het = ld_gt(aT, aH) && !isnan(ph) && !isnan(pt);   // P_het > P_hom
            code[i] = (uint8_t)(f | ((het ? s : f) << 2) | (het ? 0x80u : 0u));
        }
    }
}

// Compact class hash: slot -> profile index (or ~0u); open addressing.
__global__ __launch_bounds__(256) void sid_lookup_kernel(const uint64_t* __restrict__ counts, size_t n,
                                                         const unsigned long long* __restrict__ ckeys,
                                                         const uint32_t* __restrict__ cidx,
                                                         uint64_t cmask, uint32_t special_idx,
                                                         const uint8_t* __restrict__ pcode,
                                                         const double* __restrict__ p1,
                                                         const double* __restrict__ p2,
                                                         uint8_t* __restrict__ code,
                                                         double* __restrict__ hom,
                                                         double* __restrict__ het)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t key = sid_profile_key(counts[i]);
        uint64_t h = sid_hash64(key) & cmask;
        uint32_t idx = 0xFFFFFFFFu;
        if (key == SID_EMPTY_KEY) {        // the all-65535 profile is kept out of the table
            idx = special_idx;
        } else {
            for (uint64_t probe = 0; probe <= cmask; ++probe) {
                const unsigned long long k = ckeys[h];
                if (k == key) {
                    idx = cidx[h];
                    break;
                }
                if (k == SID_EMPTY_KEY) break;
                h = (h + 1) & cmask;
            }
        }
        if (idx == 0xFFFFFFFFu) {          // profile filtered (coverage < 4): no record
            code[i] = 0x40;
            hom[i] = 0.0;
            het[i] = 0.0;
        } else {
            code[i] = pcode[idx];
            hom[i] = p1[idx];
            het[i] = p2[idx];
        }
    }
}

// The same lookup with the class records of the record codes (sid_math.h,
// ~98% of 30x sites) in LDS: such a site costs one LDS read of its
// (code, {p1, p2}); the others probe the L2-resident class hash and gather.
// Pairs of sites per lane (16-B count loads, 2-B code and 16-B conf stores,
// lanes contiguous).
__device__ __forceinline__ uint32_t sid_class_hash(uint64_t w, const unsigned long long* __restrict__ ckeys,
                                                   const uint32_t* __restrict__ cidx, uint64_t cmask,
                                                   uint32_t special_idx)
{
    const uint64_t key = sid_profile_key(w);
    if (key == SID_EMPTY_KEY) return special_idx;
    uint64_t h = sid_hash64(key) & cmask;
    for (uint64_t probe = 0; probe <= cmask; ++probe) {
        const unsigned long long k = ckeys[h];
        if (k == key) return cidx[h];
        if (k == SID_EMPTY_KEY) break;
        h = (h + 1) & cmask;
    }
    return 0xFFFFFFFFu;
}

// Sites without a record code are deferred to an LDS list and resolved after
// the block's streaming loop, all lanes together: inline, every wave holding
// one such site (~86% of waves at 30x) would stall on the dependent
// hash-probe and gather loads inside the streaming loop.
#define SID_LOOKUP_LMISS 2048

// record table (LDS) first; a dense-coded site that is not a record site
// through the dense table (L2-resident, SID_DENSE_N entries) inline, before
// the stores (an L2 hit the other waves hide; deferring it meant scattered
// rewrites of stored lines); 0xFF: deferred to the class hash
__device__ __forceinline__ uint32_t sid_lookup_rec(uint64_t w, const sid_dvec2* R, const uint8_t* C,
                                                   const sid_dvec2* __restrict__ D, const uint8_t* __restrict__ DC,
                                                   sid_dvec2& conf)
{
    const uint32_t d = sid_dense_code(w);
    const uint32_t r = sid_rec_code(d);
    if (r != SID_DENSE_NONE) {
        conf = R[r];
        return C[r];
    }
    if (D && d != SID_DENSE_NONE) {
        conf = D[d];
        return DC[d];
    }
    conf = sid_dvec2{0.0, 0.0};
    return 0xFFu;   // deferred
}

template <int U>
__global__ __launch_bounds__(1024) void sid_lookup_rec_kernel(const ulonglong2* __restrict__ pairs, size_t npairs,
                                                              const sid_dvec2* __restrict__ g_rec,
                                                              const uint8_t* __restrict__ g_rcode,
                                                              const unsigned long long* __restrict__ ckeys,
                                                              const uint32_t* __restrict__ cidx, uint64_t cmask,
                                                              uint32_t special_idx,
                                                              const uint8_t* __restrict__ pcode,
                                                              const sid_dvec2* __restrict__ cc,
                                                              uint16_t* __restrict__ code2,
                                                              sid_dvec2* __restrict__ hom,
                                                              sid_dvec2* __restrict__ het, bool dense_inline)
{
    const sid_dvec2* D = dense_inline ? g_rec + SID_REC_N : nullptr;
    const uint8_t* DC = g_rcode + SID_REC_N;
    __shared__ sid_dvec2 R[SID_REC_N];
    __shared__ uint8_t C[SID_REC_N];
    __shared__ unsigned long long lmiss[SID_LOOKUP_LMISS];
    __shared__ uint32_t lcnt;
    for (uint32_t i = threadIdx.x; i < SID_REC_N; i += blockDim.x) {
        R[i] = g_rec[i];
        C[i] = g_rcode[i];
    }
    if (threadIdx.x == 0) lcnt = 0;
    __syncthreads();
    const uint64_t* counts = (const uint64_t*)pairs;
    uint8_t* code = (uint8_t*)code2;
    double* homd = (double*)hom;
    double* hetd = (double*)het;
    auto resolve = [&](size_t i) {   // the general path for site i
        sid_dvec2 cf;
        const uint64_t w = counts[i];
        const uint32_t idx = sid_class_hash(w, ckeys, cidx, cmask, special_idx);
        uint32_t k = 0x40u;   // profile filtered (coverage < 4): no record
        cf = sid_dvec2{0.0, 0.0};
        if (idx != 0xFFFFFFFFu) {
            cf = cc[idx];
            k = pcode[idx];
        }
        code[i] = (uint8_t)k;
        homd[i] = cf.x;
        hetd[i] = cf.y;
    };
    const size_t tile = (size_t)blockDim.x * U;
    for (size_t base = (size_t)blockIdx.x * tile; base < npairs; base += (size_t)gridDim.x * tile) {
        ulonglong2 c[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const size_t p = base + (size_t)j * blockDim.x + threadIdx.x;
            if (p < npairs) c[j] = pairs[p];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const size_t p = base + (size_t)j * blockDim.x + threadIdx.x;
            if (p < npairs) {
                sid_dvec2 ca, cb;
                const uint32_t ka = sid_lookup_rec(c[j].x, R, C, D, DC, ca);
                const uint32_t kb = sid_lookup_rec(c[j].y, R, C, D, DC, cb);
                code2[p] = (uint16_t)(ka | (kb << 8));
                hom[p] = sid_dvec2{ca.x, cb.x};
                het[p] = sid_dvec2{ca.y, cb.y};
                if (ka == 0xFFu || kb == 0xFFu) {
                    for (int q = 0; q < 2; ++q) {
                        if ((q ? kb : ka) != 0xFFu) continue;
                        const size_t i = 2 * p + q;
                        const uint32_t slot = atomicAdd(&lcnt, 1u);
                        if (slot < SID_LOOKUP_LMISS) lmiss[slot] = i;
                        else resolve(i);   // list full: inline
                    }
                }
            }
        }
    }
    __syncthreads();   // orders the placeholder stores before the resolved ones
    const uint32_t nl = lcnt < SID_LOOKUP_LMISS ? lcnt : SID_LOOKUP_LMISS;
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x) resolve(lmiss[i]);
}

// record tables from the dense class index: rec[r] = {p1, p2}, rcode[r] =
// code of the class of record code r (0x40 / zeros: no class); then, at
// SID_REC_N + d, the same for every dense code d
__global__ __launch_bounds__(256) void sid_rec_build_kernel(const uint32_t* __restrict__ dense_cidx,
                                                            const uint8_t* __restrict__ pcode,
                                                            const sid_dvec2* __restrict__ cc,
                                                            sid_dvec2* __restrict__ rec, uint8_t* __restrict__ rcode)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= SID_REC_N + SID_DENSE_N) return;
    const uint32_t idx = dense_cidx[r < SID_REC_N ? sid_rec_dense(r) : r - SID_REC_N];
    rec[r] = idx == SID_DENSE_NONE ? sid_dvec2{0.0, 0.0} : cc[idx];
    rcode[r] = idx == SID_DENSE_NONE ? (uint8_t)0x40 : pcode[idx];
}

// class records packed for the gather: cc[i] = {p1[i], p2[i]}
__global__ __launch_bounds__(256) void sid_pack_class_kernel(const double* __restrict__ p1,
                                                             const double* __restrict__ p2, size_t u,
                                                             sid_dvec2* __restrict__ cc)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < u; i += (size_t)gridDim.x * blockDim.x)
        cc[i] = sid_dvec2{p1[i], p2[i]};
}

// ------------------------------------------------ setup on the device -----
// call.cpp:66-70 + pileup.cpp:198-217 + lynch.hpp:48-55 over the sorted
// (key, count) table: keep coverage >= 4 (flag + select), count as uint32
// (UniqueProfile::count), lnM from the host's GSL lnGamma table in the
// reference's order, and the nucleotide-distribution sums with 32-bit products
// (integer sums: order-free).  sums: [0..3] per base, [4] total.
__device__ __forceinline__ uint32_t sid_key_n(uint64_t key, int i) { return (uint32_t)((key >> (48 - 16 * i)) & 0xffff); }

__global__ __launch_bounds__(256) void sid_setup_flag_kernel(const unsigned long long* __restrict__ keys, size_t n,
                                                             uint8_t* __restrict__ flags, uint32_t* __restrict__ maxcov)
{
    uint32_t mx = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        const uint32_t cov = sid_key_n(k, 0) + sid_key_n(k, 1) + sid_key_n(k, 2) + sid_key_n(k, 3);
        flags[i] = cov >= 4;
        mx = cov > mx ? cov : mx;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_down((int)mx, off, 64);
        mx = o > mx ? o : mx;
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(maxcov, mx);
}

__global__ __launch_bounds__(256) void sid_setup_gather_kernel(const unsigned long long* __restrict__ keys,
                                                               const unsigned long long* __restrict__ cnts,
                                                               const uint32_t* __restrict__ sel,
                                                               const uint32_t* __restrict__ nsel,
                                                               const double* __restrict__ lgk,
                                                               uint64_t* __restrict__ okeys, uint32_t* __restrict__ ocnt,
                                                               double* __restrict__ olnM,
                                                               unsigned long long* __restrict__ sums)
{
    const uint32_t U = *nsel;
    unsigned long long acc[5] = {0, 0, 0, 0, 0};
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < U; j += gridDim.x * blockDim.x) {
        const uint32_t i = sel[j];
        const uint64_t k = keys[i];
        const uint32_t c = (uint32_t)cnts[i];
        const uint32_t n0 = sid_key_n(k, 0), n1 = sid_key_n(k, 1), n2 = sid_key_n(k, 2), n3 = sid_key_n(k, 3);
        const uint32_t cov = n0 + n1 + n2 + n3;
        okeys[j] = k;
        ocnt[j] = c;
        double m = lgk[cov];   // lgk[x] = GSL lngamma(x + 1)
        m -= lgk[n0];
        m -= lgk[n1];
        m -= lgk[n2];
        m -= lgk[n3];
        olnM[j] = m;
        acc[0] += (uint32_t)(c * n0);
        acc[1] += (uint32_t)(c * n1);
        acc[2] += (uint32_t)(c * n2);
        acc[3] += (uint32_t)(c * n3);
        acc[4] += (uint32_t)(c * cov);
    }
    __shared__ unsigned long long red[4][5];
    for (int q = 0; q < 5; ++q) {
        unsigned long long v = acc[q];
        for (int off = 32; off > 0; off >>= 1) v += (unsigned long long)__shfl_down((long long)v, off, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][q] = v;
    }
    __syncthreads();
    if (threadIdx.x < 5) {   // one atomic per (block, sum)
        const unsigned long long v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                     red[3][threadIdx.x];
        if (v) atomicAdd(&sums[threadIdx.x], v);
    }
}

// class tables of the lookup: dense code -> class index, and the compact
// class hash (any insertion order: lookups match whole keys)
__global__ __launch_bounds__(256) void sid_class_tables_kernel(const uint64_t* __restrict__ keys, uint32_t U,
                                                               uint32_t* __restrict__ dense_cidx,
                                                               unsigned long long* __restrict__ ckeys,
                                                               uint32_t* __restrict__ cidx, uint64_t cmask)
{
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < U; j += gridDim.x * blockDim.x) {
        const uint64_t key = keys[j];
        if (key == SID_EMPTY_KEY) continue;   // the all-65535 profile: special_idx
        const uint64_t w = (key >> 48) | (((key >> 32) & 0xffff) << 16) | (((key >> 16) & 0xffff) << 32) |
                           ((key & 0xffff) << 48);
        const uint32_t d = sid_dense_code(w);
        if (d != SID_DENSE_NONE) dense_cidx[d] = j;
        uint64_t h = sid_hash64(key) & cmask;
        for (uint64_t probe = 0; probe <= cmask; ++probe) {
            const unsigned long long prev = atomicCAS(&ckeys[h], SID_EMPTY_KEY, (unsigned long long)key);
            if (prev == SID_EMPTY_KEY) {
                cidx[h] = j;
                break;
            }
            h = (h + 1) & cmask;
        }
    }
}

// ------------------------------------------------ Benjamini-Hochberg ------
// stats.cpp:58-80 on the device: p sorted descending (radix sort, with the
// original indices), adj[0] = p[0], adj[i] = min(adj[i-1], p[i] * m / (m - i)),
// capped at 1, scattered back.  The tie order is irrelevant (equal p get equal
// adj), so any sort gives the reference's values.  NaN or -0 p-values (their
// order or sign could differ from std::sort's) flag `odd`; the host then
// takes its own BH.
// Both p arrays in one sort: key = the p's bit pattern (monotonic for
// p >= +0) with bit 63 marking the second array, so a descending sort gives
// array 2 then array 1, each descending in p.
__global__ __launch_bounds__(256) void sid_bh_key_kernel(const double* __restrict__ p1, const double* __restrict__ p2,
                                                         size_t m, unsigned long long* __restrict__ keys,
                                                         uint32_t* __restrict__ idx, int* __restrict__ odd)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * m; i += (size_t)gridDim.x * blockDim.x) {
        const bool second = i >= m;
        const double v = second ? p2[i - m] : p1[i];
        if (isnan(v) || signbit(v)) atomicExch(odd, 1);   // NaN, -0 or < 0: host BH
        keys[i] = (unsigned long long)__double_as_longlong(v) | (second ? 1ull << 63 : 0ull);
        idx[i] = (uint32_t)(second ? i - m : i);
    }
}

// One block per array (blockIdx.x 0: array 2, sorted first; 1: array 1).
// Per-thread chunk minima, a parallel exclusive min-scan of them (fmin is
// exact, so any scan order gives the serial result), then the chunk walk.
#define SID_BH_TB 1024
__global__ __launch_bounds__(SID_BH_TB) void sid_bh_scan_kernel(const unsigned long long* __restrict__ ks,
                                                                const uint32_t* __restrict__ is, size_t m,
                                                                double* __restrict__ adj1, double* __restrict__ adj2)
{
    const unsigned long long* k = ks + (size_t)blockIdx.x * m;
    const uint32_t* ix = is + (size_t)blockIdx.x * m;
    double* adj = blockIdx.x == 0 ? adj2 : adj1;
    __shared__ double wmin[SID_BH_TB / 64];
    const size_t per = (m + SID_BH_TB - 1) / SID_BH_TB;
    const size_t lo = threadIdx.x * per, hi = lo + per < m ? lo + per : m;
    const double dm = (double)m;
    auto val = [&](size_t i) {
        const double p = __longlong_as_double((long long)(k[i] & ~(1ull << 63)));
        return i == 0 ? p : p * dm / (double)(m - i);   // stats.cpp:74-76
    };
    // up to 16 per thread: every load issued at once into registers (a
    // chunk walk of dependent trips was latency-bound)
    constexpr int R = 16;
    double rv[R];
    uint32_t ri[R];
    const bool regs = per <= R;
    double mn = __builtin_inf();
    if (regs) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const size_t i = lo + r;
            rv[r] = i < hi ? val(i) : __builtin_inf();
            ri[r] = i < hi ? ix[i] : 0u;
            mn = fmin(mn, rv[r]);
        }
    } else {
        for (size_t i = lo; i < hi; ++i) mn = fmin(mn, val(i));
    }
    // inclusive min-scan in the wave, then over the wave totals
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double v = mn;
    for (int off = 1; off < 64; off <<= 1) {
        const double t = __shfl_up(v, off, 64);
        if (lane >= off) v = fmin(v, t);
    }
    if (lane == 63) wmin[wid] = v;
    __syncthreads();
    double before = __builtin_inf();
    for (int w = 0; w < wid; ++w) before = fmin(before, wmin[w]);
    double excl = __shfl_up(v, 1, 64);
    excl = lane == 0 ? before : fmin(before, excl);
    double acc = excl;
    if (regs) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc = fmin(acc, rv[r]);
            if (lo + r < hi) adj[ri[r]] = acc > 1 ? 1.0 : acc;   // stats.cpp:77-79
        }
    } else {
        for (size_t i = lo; i < hi; ++i) {
            acc = fmin(acc, val(i));
            adj[ix[i]] = acc > 1 ? 1.0 : acc;
        }
    }
}

// call.cpp:113-127: the label from the adjusted p_het
__global__ __launch_bounds__(256) void sid_bh_label_kernel(const double* __restrict__ adj_het, size_t m, double sig,
                                                           uint8_t* __restrict__ code)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t c = code[i], f = c & 3u, s = (c >> 2) & 3u;
        const bool het = adj_het[i] < sig;
        code[i] = (uint8_t)(f | ((het ? s : f) << 2) | (het ? 0x80u : 0u));
    }
}

// ------------------------------------------------------------ launchers --
extern "C" {

hipError_t sid_launch_hist(const uint16_t* counts, size_t n, unsigned long long* gkeys,
                           unsigned long long* gcnt, uint64_t gmask, unsigned long long* stats,
                           int skip_dense, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const size_t per_block = 16384;
    const size_t grid = (n + per_block - 1) / per_block;
    if (skip_dense)
        sid_hist_kernel<true><<<(unsigned)grid, 256, 0, st>>>((const uint64_t*)counts, n, per_block, gkeys, gcnt,
                                                              gmask, stats);
    else
        sid_hist_kernel<false><<<(unsigned)grid, 256, 0, st>>>((const uint64_t*)counts, n, per_block, gkeys, gcnt,
                                                               gmask, stats);
    return hipGetLastError();
}

// dense histogram pass; *ctr (fallback count) must be zero on entry.  part
// holds SID_HIST_GRID_MAX rows of SID_DENSE_N u32.
#define SID_HIST_GRID_MAX 512
hipError_t sid_launch_hist_dense(const uint16_t* counts, size_t n, uint32_t* part, unsigned long long* dense,
                                 unsigned long long* list, uint64_t cap, unsigned long long* ctr, int grid_max,
                                 hipStream_t st)
{
    if (n == 0) return hipSuccess;
    const bool pairs = ((uintptr_t)counts & 15u) == 0 && n >= 2;
    const size_t units = pairs ? (n / 2 + 1) : n;
    const size_t gm = (size_t)(grid_max > 0 && grid_max < SID_HIST_GRID_MAX ? grid_max : SID_HIST_GRID_MAX);
    size_t want = (units + 8 * 1024 - 1) / (8 * 1024);   // >= 8 units per lane
    const unsigned grid = (unsigned)(want < gm ? (want ? want : 1) : gm);
    if (pairs)
        sid_hist_dense_kernel<true><<<grid, 1024, 0, st>>>((const uint64_t*)counts, n, part, list, cap, ctr);
    else
        sid_hist_dense_kernel<false><<<grid, 1024, 0, st>>>((const uint64_t*)counts, n, part, list, cap, ctr);
    sid_hist_reduce_kernel<<<dim3(SID_DENSE_N / 256, SID_DENSE_ROWS), 256, 0, st>>>(part, grid, dense);
    return hipGetLastError();
}

hipError_t sid_launch_hist_list(const unsigned long long* list, uint64_t m, unsigned long long* gkeys,
                                unsigned long long* gcnt, uint64_t gmask, unsigned long long* stats, hipStream_t st)
{
    if (m == 0) return hipSuccess;
    const uint64_t g = (m + SID_LIST_PER - 1) / SID_LIST_PER;
    if (g > 0x7fffffffull) return hipErrorInvalidValue;
    sid_hist_list_kernel<<<(unsigned)g, 256, 0, st>>>(list, m, gkeys, gcnt, gmask, stats);
    return hipGetLastError();
}

hipError_t sid_launch_dense_compact(const unsigned long long* dense, unsigned long long* okeys,
                                    unsigned long long* ocnt, unsigned long long* nout, hipStream_t st)
{
    sid_compact_kernel<<<32, 256, 0, st>>>(sid_dense_src{dense}, SID_DENSE_N, okeys, ocnt, nout);
    return hipGetLastError();
}

hipError_t sid_launch_pack_class(const double* p1, const double* p2, size_t u, double* cc, hipStream_t st)
{
    if (u == 0) return hipSuccess;
    uint64_t g = (u + 255) / 256;
    sid_pack_class_kernel<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, st>>>(p1, p2, u, (sid_dvec2*)cc);
    return hipGetLastError();
}

// record tables of the lookup (after pack_class); rec: SID_REC_N x 16 B, rcode: SID_REC_N B
// setup: sort the exported table, select coverage >= 4, gather.  ws: scratch of
// sid_setup_ws_bytes(n); keys/cnts (n entries) are sorted into skeys/scnts.
size_t sid_setup_ws_bytes(size_t n)
{
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (const unsigned long long*)nullptr, (unsigned long long*)nullptr, (int)n);
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0), (const uint8_t*)nullptr,
                                        (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    return ((std::max(a, b) + 255) & ~(size_t)255) + n * (1 + 4) + 520;
}

static size_t setup_sel_offset(size_t n)
{
    size_t a = 0, b = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (const unsigned long long*)nullptr, (unsigned long long*)nullptr, (int)n);
    (void)hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0), (const uint8_t*)nullptr,
                                        (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    const size_t tb = (std::max(a, b) + 255) & ~(size_t)255;
    return (tb + n + 3) & ~(size_t)3;
}

// phase 1: sort (unless already sorted), flag coverage >= 4 (and the largest
// coverage, for the lnGamma table), select the indices; the table stays in
// skeys/scnts and the selection in ws for phase 2
hipError_t sid_launch_setup_select(const unsigned long long* keys, const unsigned long long* cnts, size_t n, bool sort,
                                   unsigned long long* skeys, unsigned long long* scnts, void* ws, size_t ws_bytes,
                                   uint32_t* nsel, uint32_t* maxcov, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(maxcov, 0, 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(nsel, 0, 4, st);
    if (e != hipSuccess || n == 0) return e;
    size_t a = 0, b = 0;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, a, keys, skeys, cnts, scnts, (int)n, 0, 64, st);
    if (e == hipSuccess)
        e = hipcub::DeviceSelect::Flagged(nullptr, b, hipcub::CountingInputIterator<uint32_t>(0), (const uint8_t*)nullptr,
                                          (uint32_t*)nullptr, nsel, (int)n, st);
    if (e != hipSuccess) return e;
    char* w = (char*)ws;
    const size_t tb = (std::max(a, b) + 255) & ~(size_t)255;
    if (setup_sel_offset(n) + n * 4 > ws_bytes) return hipErrorInvalidValue;
    uint8_t* flags = (uint8_t*)(w + tb);
    uint32_t* sel = (uint32_t*)(w + setup_sel_offset(n));
    if (sort) {
        e = hipcub::DeviceRadixSort::SortPairs(w, a, keys, skeys, cnts, scnts, (int)n, 0, 64, st);
        if (e != hipSuccess) return e;
    }
    const unsigned long long* k = sort ? skeys : keys;
    uint64_t g = (n + 255) / 256;
    sid_setup_flag_kernel<<<(unsigned)(g < 1024 ? g : 1024), 256, 0, st>>>(k, n, flags, maxcov);
    e = hipcub::DeviceSelect::Flagged(w, b, hipcub::CountingInputIterator<uint32_t>(0), flags, sel, nsel, (int)n, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

// phase 2: gather the selected profiles (lnM from lgk, distribution sums)
hipError_t sid_launch_setup_gather(const unsigned long long* skeys, const unsigned long long* scnts, size_t n,
                                   const void* ws, const uint32_t* nsel, const double* lgk, uint64_t* okeys,
                                   uint32_t* ocnt, double* olnM, unsigned long long* sums, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(sums, 0, 5 * sizeof(unsigned long long), st);
    if (e != hipSuccess || n == 0) return e;
    const uint32_t* sel = (const uint32_t*)((const char*)ws + setup_sel_offset(n));
    uint64_t g = (n + 255) / 256;
    sid_setup_gather_kernel<<<(unsigned)(g < 1024 ? g : 1024), 256, 0, st>>>(skeys, scnts, sel, nsel, lgk, okeys, ocnt,
                                                                              olnM, sums);
    return hipGetLastError();
}

hipError_t sid_launch_class_tables(const uint64_t* keys, uint32_t U, uint32_t* dense_cidx, unsigned long long* ckeys,
                                   uint32_t* cidx, uint64_t cmask, hipStream_t st)
{
    hipError_t e = hipMemsetAsync(dense_cidx, 0xFF, SID_DENSE_N * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(ckeys, 0xFF, (cmask + 1) * 8, st);
    if (e != hipSuccess || U == 0) return e;
    uint64_t g = (U + 255) / 256;
    sid_class_tables_kernel<<<(unsigned)(g < 1024 ? g : 1024), 256, 0, st>>>(keys, U, dense_cidx, ckeys, cidx, cmask);
    return hipGetLastError();
}

// BH of p1[0..m) into adj1 and of p2 into adj2 (p untouched); ws: device
// scratch of sid_bh_ws_bytes(m); *odd must be zero on entry
size_t sid_bh_ws_bytes(size_t m)
{
    size_t t = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, t, (const unsigned long long*)nullptr,
                                                       (unsigned long long*)nullptr, (const uint32_t*)nullptr,
                                                       (uint32_t*)nullptr, (int)(2 * m));
    return ((t + 255) & ~(size_t)255) + 2 * m * (8 + 8 + 4 + 4) + 256;
}

hipError_t sid_launch_bh(const double* p1, const double* p2, size_t m, double* adj1, double* adj2, void* ws,
                         size_t ws_bytes, int* odd, hipStream_t st)
{
    if (m == 0) return hipSuccess;
    const int n = (int)(2 * m);
    size_t t = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, t, (const unsigned long long*)nullptr,
                                                                (unsigned long long*)nullptr, (const uint32_t*)nullptr,
                                                                (uint32_t*)nullptr, n, 0, 64, st);
    if (e != hipSuccess) return e;
    char* w = (char*)ws;
    const size_t tb = (t + 255) & ~(size_t)255;
    if (tb + 2 * m * 24 > ws_bytes) return hipErrorInvalidValue;
    unsigned long long* keys = (unsigned long long*)(w + tb);
    unsigned long long* ks = keys + 2 * m;
    uint32_t* idx = (uint32_t*)(ks + 2 * m);
    uint32_t* is = idx + 2 * m;
    uint64_t g = (2 * m + 255) / 256;
    sid_bh_key_kernel<<<(unsigned)(g < 1024 ? g : 1024), 256, 0, st>>>(p1, p2, m, keys, idx, odd);
    e = hipcub::DeviceRadixSort::SortPairsDescending(w, t, keys, ks, idx, is, n, 0, 64, st);
    if (e != hipSuccess) return e;
    sid_bh_scan_kernel<<<2, SID_BH_TB, 0, st>>>(ks, is, m, adj1, adj2);
    return hipGetLastError();
}

hipError_t sid_launch_bh_label(const double* adj_het, size_t m, double sig, uint8_t* code, hipStream_t st)
{
    if (m == 0) return hipSuccess;
    uint64_t g = (m + 255) / 256;
    sid_bh_label_kernel<<<(unsigned)(g < 1024 ? g : 1024), 256, 0, st>>>(adj_het, m, sig, code);
    return hipGetLastError();
}

hipError_t sid_launch_rec_build(const uint32_t* dense_cidx, const uint8_t* pcode, const double* cc, double* rec,
                                uint8_t* rcode, hipStream_t st)
{
    sid_rec_build_kernel<<<(SID_REC_N + SID_DENSE_N) / 256, 256, 0, st>>>(dense_cidx, pcode, (const sid_dvec2*)cc,
                                                                          (sid_dvec2*)rec, rcode);
    return hipGetLastError();
}

hipError_t sid_launch_rehash(const unsigned long long* okeys, const unsigned long long* ocnt,
                             uint64_t ocap, unsigned long long* gkeys, unsigned long long* gcnt,
                             uint64_t gmask, unsigned long long* distinct, hipStream_t st)
{
    uint64_t g = (ocap + 255) / 256;
    sid_hist_rehash_kernel<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, st>>>(okeys, ocnt, ocap, gkeys,
                                                                            gcnt, gmask, distinct);
    return hipGetLastError();
}

hipError_t sid_launch_compact(const unsigned long long* gkeys, const unsigned long long* gcnt,
                              uint64_t cap, unsigned long long* okeys, unsigned long long* ocnt,
                              unsigned long long* nout, hipStream_t st)
{
    const uint64_t g = (cap + 2047) / 2048;   // >= 8 tiles per block, one atomic per block
    sid_compact_kernel<<<(unsigned)(g < 256 ? (g ? g : 1) : 256), 256, 0, st>>>(sid_hash_src{gkeys, gcnt}, cap, okeys,
                                                                                ocnt, nout);
    return hipGetLastError();
}

hipError_t sid_launch_objective(const uint64_t* keys, const uint32_t* cnt, const double* lnM, size_t u,
                                const sid_lynch_evals* EV, int npts, double* partial, double* out,
                                unsigned int* seq_out, unsigned int seq, int grid, hipStream_t st)
{
    if (npts < 1 || npts > SID_OBJ_PTS || grid < 1 || grid > 1024) return hipErrorInvalidValue;
    sid_objective_kernel<<<dim3(grid, npts), 256, 0, st>>>(keys, cnt, lnM, u, *EV, partial);
    sid_objective_fold_kernel<<<npts, 256, 0, st>>>(partial, grid, out, seq_out, seq);
    return hipGetLastError();
}

hipError_t sid_launch_nm(const uint64_t* keys, const uint32_t* cnt, const double* lnM, size_t u, int nb,
                         const sid_nm_dist* D, const double* x0, const double* step, int lookahead,
                         double* partial, unsigned int* bar, int grid, long long timeout, sid_nm_result* res,
                         hipStream_t st)
{
    if (nb < 1 || nb > 1024 || grid < 1) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(bar, 0, 2 * sizeof(unsigned int), st);
    if (e != hipSuccess) return e;
    sid_nm_dist d = *D;
    double x00 = x0[0], x01 = x0[1], st0 = step[0], st1 = step[1];
    int* abort_flag = (int*)(bar + 1);
    void* args[] = {(void*)&keys, (void*)&cnt,   (void*)&lnM, (void*)&u,          (void*)&nb,
                    (void*)&d,    (void*)&x00,   (void*)&x01, (void*)&st0,        (void*)&st1,
                    (void*)&lookahead, (void*)&partial, (void*)&bar, (void*)&abort_flag, (void*)&timeout,
                    (void*)&res};
    return hipLaunchCooperativeKernel((const void*)sid_nm_kernel, dim3(grid), dim3(256), args, 0, st);
}

hipError_t sid_launch_profile_lik(const uint64_t* keys, const double* lnM, size_t u,
                                  const sid_lynch_eval* E, double* lhom, double* lhet, hipStream_t st)
{
    if (u == 0) return hipSuccess;
    uint64_t g = (u + 255) / 256;
    sid_profile_lik_kernel<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, st>>>(keys, lnM, u, *E, lhom, lhet);
    return hipGetLastError();
}

hipError_t sid_launch_classify(const uint64_t* keys, const double* lhom, const double* lhet, size_t u,
                               int mode, int use_prior, double pi, double lg15, double* c1, double* c2,
                               uint8_t* code, hipStream_t st)
{
    if (u == 0) return hipSuccess;
    uint64_t g = (u + 255) / 256;
    sid_classify_kernel<<<(unsigned)(g < 4096 ? g : 4096), 256, 0, st>>>(keys, lhom, lhet, u, mode,
                                                                         use_prior, pi, lg15, c1, c2, code);
    return hipGetLastError();
}

hipError_t sid_launch_lookup(const uint16_t* counts, size_t n, const unsigned long long* ckeys,
                             const uint32_t* cidx, uint64_t cmask, uint32_t special_idx,
                             const uint8_t* pcode,
                             const double* p1, const double* p2, const double* rec, const uint8_t* rcode,
                             const double* cc, uint8_t* code, double* hom,
                             double* het, int grid_cap, hipStream_t st)
{
    if (n == 0) return hipSuccess;
    size_t done = 0;
    const bool aligned = (((uintptr_t)counts | (uintptr_t)hom | (uintptr_t)het) & 15u) == 0 &&
                         (((uintptr_t)code) & 1u) == 0;
    if (rec && rcode && cc && aligned && n >= 2) {
        const size_t npairs = n / 2;
        // one pair per thread, at most 1024 blocks, the dense profiles' records
        // looked up inline (measured best: C3 246 us vs 257 us with two pairs
        // per thread)
        size_t want = (npairs + (size_t)1024 - 1) / (size_t)1024;
        const unsigned grid = (unsigned)(want < 1024 ? want : 1024);
        sid_lookup_rec_kernel<1><<<grid, 1024, 0, st>>>((const ulonglong2*)counts, npairs, (const sid_dvec2*)rec,
                                                        rcode, ckeys, cidx, cmask, special_idx, pcode,
                                                        (const sid_dvec2*)cc, (uint16_t*)code, (sid_dvec2*)hom,
                                                        (sid_dvec2*)het, true);
        done = 2 * npairs;
    }
    if (done < n) {
        const size_t rest = n - done;
        uint64_t g = (rest + 255) / 256;
        unsigned grid = (unsigned)(g < (uint64_t)grid_cap ? g : (uint64_t)grid_cap);
        sid_lookup_kernel<<<grid, 256, 0, st>>>((const uint64_t*)counts + done, rest, ckeys, cidx, cmask,
                                                special_idx, pcode, p1, p2, code + done, hom + done, het + done);
    }
    return hipGetLastError();
}

}  // extern "C"
