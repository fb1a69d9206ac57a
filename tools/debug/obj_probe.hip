// obj_probe.hip — where the time of the Nelder-Mead objective launch goes
// (not part of libsid).  U synthetic 30x-like profiles, 4 points per launch:
//   prod      sid_launch_objective as shipped (block partials, then a fold
//             kernel writing host-mapped memory)
//   hostmap   plain, with the partials written straight into host-mapped
//             memory and polled by the host (no fold kernel)
//   plain     same per-profile work, block partials only (no ticket/fence)
//   trivial   plain with the 10-genotype mixture replaced by two FMAs
//   split<P>  16 lanes per profile (4 hom + 6 het terms on their own lanes,
//             sums gathered in the reference order), P profiles per group,
//             ticket + last-block reduction like prod
// Kernel time from events over back-to-back launches; "rt" = launch + host
// poll round trip per launch, as the host NM sees it.
#include "../../sid_amd/csrc/lynch.hip"

struct Ev4 {
    sid_lynch_eval e[4];
};
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <set>
#include <vector>

template <bool TRIVIAL>
__global__ __launch_bounds__(256) void plain_kernel(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
                                                     const double* __restrict__ lnM, size_t u, Ev4 EV,
                                                     double* partial)
{
    const int pt = blockIdx.y;
    const sid_lynch_eval& E = EV.e[pt];
    double hi = 0.0, lo = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < u; i += (size_t)gridDim.x * blockDim.x) {
        double sh, st;
        if (TRIVIAL) {
            sh = E.la * (double)(keys[i] >> 48);
            st = E.lb * (double)(keys[i] & 0xffff);
        } else {
            sid_mixture(keys[i], E, sh, st);
        }
        double lhom = lnM[i] + sh, lhet = lnM[i] + st;
        double lL = TRIVIAL ? fmax(E.l1p + lhom, E.lp + lhet) : sid_lse2(E.l1p + lhom, E.lp + lhet);
        double v = lL * (double)cnt[i];
        double p = fma(lL, (double)cnt[i], -v);
        double s, e;
        sid_two_sum(hi, v, s, e);
        hi = s;
        lo += e + p;
    }
    for (int off = 32; off > 0; off >>= 1) {
        double ohi = __shfl_down(hi, off, 64), olo = __shfl_down(lo, off, 64), s, e;
        sid_two_sum(hi, ohi, s, e);
        hi = s;
        lo += olo + e;
    }
    if ((threadIdx.x & 63) == 0) {
        double* part = partial + ((size_t)pt * gridDim.x + blockIdx.x) * 8 + (threadIdx.x >> 6) * 2;
        part[0] = hi;
        part[1] = lo;
    }
}

__device__ __forceinline__ double pick4(const double* a, int i)
{
    double r = a[0];
    r = i == 1 ? a[1] : r;
    r = i == 2 ? a[2] : r;
    r = i == 3 ? a[3] : r;
    return r;
}

template <int PPG>
__global__ __launch_bounds__(256) void split_kernel(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
                                                     const double* __restrict__ lnM, size_t u, Ev4 EV,
                                                     double* partial, unsigned int* ticket, double* out)
{
    const int pt = blockIdx.y;
    const sid_lynch_eval& E = EV.e[pt];
    const int sub = threadIdx.x & 15;
    const size_t g0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const size_t ng = ((size_t)gridDim.x * blockDim.x) >> 4;
    // this lane's term: sub 0-3 hom i=sub; 8-13 het pair k=sub-8; others none
    const bool hom = sub < 4, het = sub >= 8 && sub < 14;
    const int k = sub - 8;
    const int pi_ = k < 3 ? 0 : (k < 5 ? 1 : 2);
    const int pj_ = k == 0 ? 1 : (k == 1 || k == 3) ? 2 : 3;
    double ldk = 0.0;
    if (hom) ldk = pick4(E.ld, sub);
    if (het) {
        ldk = E.ldd[0];
        ldk = k == 1 ? E.ldd[1] : ldk;
        ldk = k == 2 ? E.ldd[2] : ldk;
        ldk = k == 3 ? E.ldd[3] : ldk;
        ldk = k == 4 ? E.ldd[4] : ldk;
        ldk = k == 5 ? E.ldd[5] : ldk;
    }
    const double lx = hom ? E.la : E.lh;
    double hi = 0.0, lo = 0.0;
    const int base = (threadIdx.x & 63) & ~15;
    for (int r = 0; r < PPG; ++r) {
        const size_t i = g0 + (size_t)r * ng;
        const bool valid = i < u;
        const uint64_t key = valid ? keys[i] : 0;
        const uint32_t n0 = (uint32_t)(key >> 48), n1 = (uint32_t)((key >> 32) & 0xffff),
                       n2 = (uint32_t)((key >> 16) & 0xffff), n3 = (uint32_t)(key & 0xffff);
        const uint32_t c = n0 + n1 + n2 + n3;
        uint32_t nn[4] = {n0, n1, n2, n3};
        uint32_t a = 0;
        if (hom) a = sub == 0 ? n0 : sub == 1 ? n1 : sub == 2 ? n2 : n3;
        if (het) {
            uint32_t x = pi_ == 0 ? n0 : pi_ == 1 ? n1 : n2;
            uint32_t y = pj_ == 1 ? n1 : pj_ == 2 ? n2 : n3;
            a = x + y;
        }
        (void)nn;
        double t = -__builtin_inf();
        if (hom || het) t = sid_term(ldk, sid_pow_ln(lx, a), sid_pow_ln(E.lb, c - a));
        double m = t;
        m = fmax(m, __shfl_xor(m, 1, 64));
        m = fmax(m, __shfl_xor(m, 2, 64));
        m = fmax(m, __shfl_xor(m, 4, 64));
        const double ex = m == -__builtin_inf() ? 0.0 : exp(t - m);
        // ordered sums as in sid_mixture: lane sub 0 (hom), sub 8 (het)
        const int lead = (threadIdx.x & 63) & ~7;
        double acc = 0.0;
        const int cntk = (sub & 8) ? 6 : 4;
        for (int q = 0; q < 6; ++q) {
            const double v = __shfl(ex, lead + q, 64);
            if (q < cntk) acc += v;
        }
        double s = m == -__builtin_inf() ? m : m + log(acc);
        if ((sub & 8) && m != -__builtin_inf()) s += E.lnorm;
        const double s_het = __shfl(s, base + 8, 64);
        if (sub == 0 && valid) {
            const double sh = s, st = s_het;
            double lhom = sh == -__builtin_inf() ? sh : lnM[i] + sh;
            double lhet = st == -__builtin_inf() ? st : lnM[i] + st;
            double lL = sid_lse2(E.l1p + lhom, E.lp + lhet);
            if (lL > -__builtin_inf() && !isnan(lL)) {
                double v = lL * (double)cnt[i];
                double p = fma(lL, (double)cnt[i], -v);
                double s2, e;
                sid_two_sum(hi, v, s2, e);
                hi = s2;
                lo += e + p;
            }
        }
    }
    __shared__ double sh_hi[4], sh_lo[4];
    __shared__ bool last;
    for (int off = 32; off > 0; off >>= 1) {
        double ohi = __shfl_down(hi, off, 64), olo = __shfl_down(lo, off, 64), s, e;
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
    double* part = partial + (size_t)pt * 2 * gridDim.x;
    if (threadIdx.x == 0) {
        double H = 0.0, Lo = 0.0;
        for (int w = 0; w < 4; ++w) {
            double s, e;
            sid_two_sum(H, sh_hi[w], s, e);
            H = s;
            Lo += sh_lo[w] + e;
        }
        part[2 * blockIdx.x] = H;
        part[2 * blockIdx.x + 1] = Lo;
        __threadfence();
        last = atomicAdd(&ticket[pt], 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    double bh = 0.0, bl = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
        const double x = ((volatile double*)part)[2 * b], y = ((volatile double*)part)[2 * b + 1];
        double s, e;
        sid_two_sum(bh, x, s, e);
        bh = s;
        bl += y + e;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ohi = __shfl_down(bh, off, 64), olo = __shfl_down(bl, off, 64);
        double s, e;
        sid_two_sum(bh, ohi, s, e);
        bh = s;
        bl += olo + e;
    }
    __syncthreads();
    if (lane == 0) {
        sh_hi[wid] = bh;
        sh_lo[wid] = bl;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double H = 0.0, Lo = 0.0;
    for (int w = 0; w < 4; ++w) {
        double s, e;
        sid_two_sum(H, sh_hi[w], s, e);
        H = s;
        Lo += sh_lo[w] + e;
    }
    ticket[pt] = 0;
    double s, e;
    sid_two_sum(H, Lo, s, e);
    out[2 * pt] = s;
    out[2 * pt + 1] = e;
}

// second kernel of the two-kernel variant: one block per point folds the
// per-wave partials of plain_kernel (nw of them) and writes host-mapped memory
__global__ __launch_bounds__(256) void fold_kernel(const double* partial, int nw, double* out, volatile unsigned* seq_out,
                                                   unsigned seq)
{
    const int pt = blockIdx.x;
    const double* part = partial + (size_t)pt * nw * 2;
    double bh = 0.0, bl = 0.0;
    for (int b = threadIdx.x; b < nw; b += blockDim.x) {
        double s, e;
        sid_two_sum(bh, part[2 * b], s, e);
        bh = s;
        bl += part[2 * b + 1] + e;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double ohi = __shfl_down(bh, off, 64), olo = __shfl_down(bl, off, 64);
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
    for (int w = 0; w < 4; ++w) {
        double s, e;
        sid_two_sum(H, sh_hi[w], s, e);
        H = s;
        Lo += sh_lo[w] + e;
    }
    double s, e;
    sid_two_sum(H, Lo, s, e);
    out[2 * pt] = s;
    out[2 * pt + 1] = e;
    __threadfence_system();
    seq_out[pt] = seq;
}

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

static void make_eval(double pi, double e, sid_lynch_eval* E)
{
    const double d[4] = {0.3, 0.2, 0.2, 0.3};
    E->la = std::log(1 - e);
    E->lb = std::log(e / 3.);
    E->lh = std::log((1 - 2. / 3. * e) / 2.);
    int k = 0;
    double s2 = 0;
    for (int i = 0; i < 4; ++i) {
        E->ld[i] = std::log(d[i]);
        s2 += d[i] * d[i];
        for (int j = i + 1; j < 4; ++j) E->ldd[k++] = std::log(d[i] * d[j]);
    }
    E->lnorm = -std::log(1 - s2);
    E->l1p = std::log(1. - pi);
    E->lp = std::log(pi);
}

int main(int argc, char** argv)
{
    const size_t U = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 12000;
    const int reps = 200;
    std::set<uint64_t> ks;
    uint64_t s = 12345;
    auto rnd = [&s] {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    };
    while (ks.size() < U) {
        uint32_t n[4] = {(uint32_t)(rnd() % 4), (uint32_t)(rnd() % 4), (uint32_t)(rnd() % 4), (uint32_t)(rnd() % 4)};
        n[rnd() % 4] = 4 + (uint32_t)(rnd() % 60);
        if (rnd() % 8 == 0) n[rnd() % 4] = 4 + (uint32_t)(rnd() % 40);
        ks.insert(((uint64_t)n[0] << 48) | ((uint64_t)n[1] << 32) | ((uint64_t)n[2] << 16) | n[3]);
    }
    std::vector<uint64_t> hk(ks.begin(), ks.end());
    std::vector<uint32_t> hc(U);
    std::vector<double> hl(U);
    for (size_t i = 0; i < U; ++i) {
        hc[i] = 1 + (uint32_t)(rnd() % 100000);
        hl[i] = -(double)(rnd() % 100) * 0.1;
    }
    uint64_t* dk;
    uint32_t* dc;
    double *dl, *part, *dout;
    unsigned int *ticket, *hseq, *dseq;
    double* hout;
    CK(hipMalloc(&dk, U * 8));
    CK(hipMalloc(&dc, U * 4));
    CK(hipMalloc(&dl, U * 8));
    CK(hipMalloc(&part, 4 * 2 * 65536 * 8));
    CK(hipMalloc(&ticket, 16));
    CK(hipMemset(ticket, 0, 16));
    CK(hipHostMalloc((void**)&hout, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&hseq, 16, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(hseq, 0, 16);
    CK(hipHostGetDevicePointer((void**)&dout, hout, 0));
    CK(hipHostGetDevicePointer((void**)&dseq, hseq, 0));
    double* ddout;
    CK(hipMalloc(&ddout, 64));
    double *hpart, *dpart;
    CK(hipHostMalloc((void**)&hpart, 4 * 2 * 1024 * 8, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void**)&dpart, hpart, 0));
    CK(hipMemcpy(dk, hk.data(), U * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, hc.data(), U * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dl, hl.data(), U * 8, hipMemcpyHostToDevice));
    sid_lynch_evals EV;
    sid_lynch_eval EE[4];
    for (int p = 0; p < 4; ++p) make_eval(1e-3 * (1 + p), 1e-2 * (1 + 0.1 * p), &EE[p]);
    Ev4 EV4;
    for (int p = 0; p < 4; ++p) {
        EV4.e[p] = EE[p];
        EV.p[p] = {EE[p].la, EE[p].lb, EE[p].lh, EE[p].l1p, EE[p].lp};
    }
    std::memcpy(EV.ld, EE[0].ld, sizeof EV.ld);
    std::memcpy(EV.ldd, EE[0].ldd, sizeof EV.ldd);
    EV.lnorm = EE[0].lnorm;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = (int)std::min<size_t>(1024, (U + 255) / 256);
    unsigned int seq = 0;
    auto timed = [&](const char* name, auto launch) {
        for (int i = 0; i < 10; ++i) launch();
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(a, st));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            launch();
            CK(hipStreamSynchronize(st));
        }
        double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        std::printf("{\"variant\": \"%s\", \"U\": %zu, \"us_per_launch_b2b\": %.2f, \"us_round_trip_sync\": %.2f}\n",
                    name, U, ms * 1000 / reps, rt);
    };
    timed("prod", [&] {
        CK(sid_launch_objective(dk, dc, dl, U, &EV, 4, part, dout, dseq, ++seq, grid, st));
    });
    // prod with host polling of the mapped sequence (as lynch_host.cpp does)
    {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            const unsigned q = ++seq;
            CK(sid_launch_objective(dk, dc, dl, U, &EV, 4, part, dout, dseq, q, grid, st));
            while (__atomic_load_n(&hseq[3], __ATOMIC_ACQUIRE) != q) {
            }
        }
        double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        std::printf("{\"variant\": \"prod_poll\", \"U\": %zu, \"us_round_trip_poll\": %.2f}\n", U, rt);
        CK(hipStreamSynchronize(st));
    }
    {   // hostmap: per-wave partials into host-mapped memory, polled against a sentinel
        uint64_t* raw = (uint64_t*)hpart;
        const size_t slots = (size_t)8 * grid * 4;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            for (size_t j = 0; j < slots; ++j) __atomic_store_n(&raw[j], 0x7FF4D1B5E0C0FFEEull, __ATOMIC_RELAXED);
            std::atomic_thread_fence(std::memory_order_seq_cst);
            plain_kernel<false><<<dim3(grid, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, dpart);
            for (size_t j = 0; j < slots; ++j)
                while (__atomic_load_n(&raw[j], __ATOMIC_ACQUIRE) == 0x7FF4D1B5E0C0FFEEull) {
                }
        }
        double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        std::printf("{\"variant\": \"hostmap_poll\", \"U\": %zu, \"us_round_trip_poll\": %.2f}\n", U, rt);
        CK(hipStreamSynchronize(st));
    }
    auto two = [&](int g, const char* name) {
        timed(name, [&] {
            plain_kernel<false><<<dim3(g, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, part);
            fold_kernel<<<4, 256, 0, st>>>(part, g * 4, dout, dseq, ++seq);
        });
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            const unsigned q = ++seq;
            plain_kernel<false><<<dim3(g, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, part);
            fold_kernel<<<4, 256, 0, st>>>(part, g * 4, dout, dseq, q);
            while (__atomic_load_n(&hseq[3], __ATOMIC_ACQUIRE) != q) {
            }
        }
        double rt = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
        std::printf("{\"variant\": \"%s_poll\", \"U\": %zu, \"us_round_trip_poll\": %.2f, \"value\": %.17g}\n", name, U,
                    rt, hout[6] + hout[7]);
        CK(hipStreamSynchronize(st));
    };
    two(grid, "two");
    two((grid + 1) / 2, "two_half");
    two((grid + 3) / 4, "two_quarter");
    for (int g : {grid / 2, grid / 4, 8}) {
        if (g < 1) continue;
        char nm[32];
        std::snprintf(nm, sizeof nm, "prod_grid%d", g);
        timed(nm, [&] { CK(sid_launch_objective(dk, dc, dl, U, &EV, 4, part, dout, dseq, ++seq, g, st)); });
    }
    timed("plain", [&] { plain_kernel<false><<<dim3(grid, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, part); });
    timed("trivial", [&] { plain_kernel<true><<<dim3(grid, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, part); });
    auto split = [&](auto P, const char* name) {
        constexpr int PP = decltype(P)::value;
        const size_t groups = (U + PP - 1) / PP;
        const int g = (int)((groups * 16 + 255) / 256);
        timed(name, [&] { split_kernel<PP><<<dim3(g, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, part, ticket, ddout); });
        double o[8];
        CK(hipMemcpy(o, ddout, 64, hipMemcpyDeviceToHost));
        plain_kernel<false><<<dim3(grid, 4), 256, 0, st>>>(dk, dc, dl, U, EV4, part);
        fold_kernel<<<4, 256, 0, st>>>(part, grid * 4, dout, dseq, ++seq);
        CK(hipStreamSynchronize(st));
        for (int p = 0; p < 4; ++p)
            std::printf("  pt %d split %.17g prod %.17g\n", p, o[2 * p] + o[2 * p + 1], hout[2 * p] + hout[2 * p + 1]);
    };
    split(std::integral_constant<int, 1>(), "split1");
    split(std::integral_constant<int, 2>(), "split2");
    split(std::integral_constant<int, 4>(), "split4");
    return 0;
}
