// hist_probe.hip — where the time of the dense histogram pass goes (not part
// of libsid).  Same grid/loop shape as sid_hist_dense_kernel over the C3
// synthetic counts, with pieces switched on one at a time:
//   loads   16-B pair loads + dense code, folded into a register
//   lds     + one ds_add per site (swizzled slot)
//   lds_raw + one ds_add per site (unswizzled code)
//   fb      + fallback-list append (ballot, one global atomic per wave)
//   full    lds + fb + per-block row flush (the product kernel's work)
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../include/sid.h"
#include "../../sid_amd/csrc/sid_math.h"

enum { LOADS = 0, LDS = 1, LDS_RAW = 2, FB = 3, FULL = 4, WAVEAGG = 5, LDSROW = 6, LDSLIST = 7 };

extern "C" hipError_t sid_launch_hist_dense(const uint16_t* counts, size_t n, uint32_t* part, unsigned long long* dense,
                                            unsigned long long* list, uint64_t cap, unsigned long long* ctr,
                                            int grid_max, hipStream_t st);

__device__ __forceinline__ uint64_t key_of(uint64_t w)
{
    return ((w & 0xffffull) << 48) | (((w >> 16) & 0xffffull) << 32) | (((w >> 32) & 0xffffull) << 16) | (w >> 48);
}

__device__ __forceinline__ void fb_append(bool fb, uint64_t key, unsigned long long* list, uint64_t cap,
                                          unsigned long long* ctr)
{
    const unsigned long long mask = __ballot(fb);
    if (mask == 0) return;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)mask) - 1u;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(mask));
    base = (unsigned long long)__shfl((long long)base, (int)leader);
    if (fb) {
        const unsigned long long off = base + (unsigned long long)__popcll(mask & ((1ull << lane) - 1ull));
        if (off < cap) list[off] = key;
    }
}

template <int MODE, int U = 2>
__global__ __launch_bounds__(1024) void probe(const ulonglong2* __restrict__ pairs, size_t npairs, uint32_t* part,
                                              unsigned long long* list, uint64_t cap, unsigned long long* ctr,
                                              uint32_t* sink)
{
    __shared__ uint32_t H[SID_DENSE_N];
    __shared__ unsigned long long llist[1024];
    __shared__ uint32_t lcnt;
    if (threadIdx.x == 0) lcnt = 0;
    for (uint32_t i = threadIdx.x; i < SID_DENSE_N; i += blockDim.x) H[i] = 0;
    __syncthreads();
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t base = (size_t)blockIdx.x * blockDim.x; base < npairs; base += U * stride) {
        ulonglong2 c[U];
        bool vv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const size_t pj = base + threadIdx.x + j * stride;
            vv[j] = pj < npairs;
            c[j] = vv[j] ? pairs[pj] : ulonglong2{0, 0};
        }
        uint64_t w[2 * U];
        bool v[2 * U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            w[2 * j] = c[j].x;
            w[2 * j + 1] = c[j].y;
            v[2 * j] = v[2 * j + 1] = vv[j];
        }
        if (MODE == WAVEAGG) {
            // one LDS add per distinct code of the wave's 64 lanes (leader loop)
#pragma unroll
            for (int k = 0; k < 2 * U; ++k) {
                const uint32_t d = sid_dense_code(w[k]);
                bool pending = v[k] && d != SID_DENSE_NONE;
                unsigned long long rem = __ballot(pending);
                while (rem) {
                    const uint32_t leader = (uint32_t)__ffsll((long long)rem) - 1u;
                    const uint32_t dl = __shfl((int)d, (int)leader);
                    const unsigned long long same = __ballot(pending && d == dl);
                    if (__lane_id() == leader) atomicAdd(&H[sid_dense_slot(dl)], (uint32_t)__popcll(same));
                    if (d == dl) pending = false;
                    rem &= ~same;
                }
            }
            continue;
        }
#pragma unroll
        for (int k = 0; k < 2 * U; ++k) {
            const uint32_t d = sid_dense_code(w[k]);
            const bool fb = v[k] && d == SID_DENSE_NONE;
            if (MODE == LOADS) acc += d;
            if (MODE == LDS || MODE == FB || MODE == FULL || MODE == LDSROW || MODE == LDSLIST)
                if (v[k] && !fb) atomicAdd(&H[sid_dense_slot(d)], 1u);
            if (MODE == LDSLIST && fb) {
                const uint32_t slot = atomicAdd(&lcnt, 1u);
                if (slot < 1024) llist[slot] = key_of(w[k]);
            }
            if (MODE == LDS_RAW)
                if (v[k] && !fb) atomicAdd(&H[d], 1u);
            if (MODE == FB || MODE == FULL) fb_append(fb, key_of(w[k]), list, cap, ctr);
        }
    }
    __syncthreads();
    if (MODE == LDSLIST && threadIdx.x < (lcnt < 1024 ? lcnt : 1024)) list[blockIdx.x * 1024 + threadIdx.x] = llist[threadIdx.x];
    if (MODE == FULL || MODE == WAVEAGG || MODE == LDSROW || MODE == LDSLIST) {
        uint32_t* row = part + (size_t)blockIdx.x * SID_DENSE_N;
        for (uint32_t i = threadIdx.x; i < SID_DENSE_N; i += blockDim.x) row[i] = H[sid_dense_slot(i)];
    } else {
        acc += H[threadIdx.x];
        if (acc == 0x12345678u) sink[0] = acc;
    }
}

int main()
{
    const size_t n = 50000000, npairs = n / 2;
    sid_opts o;
    sid_opts_default(&o);
    sid_ctx* ctx = nullptr;
    if (sid_create(0, &o, &ctx)) return 1;
    uint16_t* counts;
    uint32_t *part, *sink;
    unsigned long long *list, *ctr;
    hipMalloc(&counts, n * 8);
    hipMalloc(&part, 512ull * SID_DENSE_N * 4);
    hipMalloc(&list, (1ull << 22) * 8);
    hipMalloc(&ctr, 8);
    hipMalloc(&sink, 4);
    unsigned long long* dense;
    hipMalloc(&dense, 16ull * SID_DENSE_N * 8);
    hipMemset(dense, 0, 16ull * SID_DENSE_N * 8);
    sid_synth_counts(ctx, 3, 30.0, 0, n, counts, nullptr);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](auto launch, const char* name, int grid) {
        for (int w = 0; w < 2; ++w) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 10;
        for (int r = 0; r < reps; ++r) {
            hipMemsetAsync(ctr, 0, 8);
            launch();
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("{\"probe\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps_in\": %.1f}\n", name, grid, ms,
               8.0 * n / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const ulonglong2* P = (const ulonglong2*)counts;
    for (int grid : {256, 512}) {
        timeit([&] { probe<LOADS><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "loads", grid);
        timeit([&] { probe<LDS><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds", grid);
        timeit([&] { probe<LDS_RAW><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds_raw", grid);
        timeit([&] { probe<FB><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "fb", grid);
        timeit([&] { probe<FULL><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "full", grid);
        timeit([&] { probe<LDSROW><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds+row", grid);
        timeit([&] { probe<LDSLIST><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds+row+llist", grid);
        timeit([&] { probe<LOADS, 4><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "loads_u4", grid);
        timeit([&] { probe<LOADS, 8><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "loads_u8", grid);
        timeit([&] { probe<LOADS, 1><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "loads_u1", grid);
        timeit([&] { probe<LDS, 4><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds_u4", grid);
        timeit([&] { probe<LDSLIST, 4><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds+row+llist_u4", grid);
        timeit([&] { probe<LDSLIST, 8><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "lds+row+llist_u8", grid);
        timeit([&] { probe<WAVEAGG, 2><<<grid, 1024>>>(P, npairs, part, list, 1 << 22, ctr, sink); }, "waveagg", grid);
        timeit([&] { (void)sid_launch_hist_dense(counts, n, part, dense, list, 1 << 22, ctr, grid, nullptr); },
               "product(dense+reduce)", grid);
    }
    sid_destroy(ctx);
    return 0;
}
