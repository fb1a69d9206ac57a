// write_probe.hip — is HBM write bandwidth on this GPU bounded by the store
// pattern?  (not part of libsid).  The -m local mix is 68% stores, and a
// plain float4 store stream measured 4.56 TB/s (stream_probe.hip) against
// 6.49 TB/s for reads.  Variants: grid / block size, stores in flight per
// thread, grid-stride vs block-contiguous, nontemporal stores, and the local
// mix with nontemporal conf stores.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double dvec2 __attribute__((ext_vector_type(2)));
typedef float fvec4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void wr_stride(fvec4* __restrict__ b, size_t n)
{
    const size_t step = (size_t)gridDim.x * blockDim.x;
    const fvec4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * step < n; i += U * step) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            if (NT)
                __builtin_nontemporal_store(v, b + i + j * step);
            else
                b[i + j * step] = v;
        }
    }
    for (; i < n; i += step) b[i] = v;
}

// each block owns one contiguous range, U stores per thread per tile
template <int U, bool NT>
__global__ void wr_chunk(fvec4* __restrict__ b, size_t n)
{
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    const fvec4 v = {1.f, 2.f, 3.f, (float)threadIdx.x};
    for (size_t base = lo; base < hi; base += (size_t)blockDim.x * U) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            size_t i = base + (size_t)j * blockDim.x + threadIdx.x;
            if (i < hi) {
                if (NT)
                    __builtin_nontemporal_store(v, b + i);
                else
                    b[i] = v;
            }
        }
    }
}

template <bool NT>
__global__ void copy_stride(const fvec4* __restrict__ a, fvec4* __restrict__ b, size_t n)
{
    const size_t step = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        fvec4 v = NT ? __builtin_nontemporal_load(a + i) : a[i];
        if (NT)
            __builtin_nontemporal_store(v, b + i);
        else
            b[i] = v;
    }
}

// the local kernel's traffic mix (8 B in, 1 + 16 B out per site), conf
// stores optionally nontemporal
template <int U, bool NT>
__global__ __launch_bounds__(1024) void mix(const ulonglong2* __restrict__ in, size_t npairs,
                                            uint16_t* __restrict__ code, dvec2* __restrict__ hom,
                                            dvec2* __restrict__ het)
{
    const size_t tile = (size_t)blockDim.x * U;
    for (size_t base = (size_t)blockIdx.x * tile; base < npairs; base += (size_t)gridDim.x * tile) {
        ulonglong2 c[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            size_t p = base + (size_t)j * blockDim.x + threadIdx.x;
            if (p < npairs) c[j] = in[p];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            size_t p = base + (size_t)j * blockDim.x + threadIdx.x;
            if (p < npairs) {
                code[p] = (uint16_t)(c[j].x ^ c[j].y);
                dvec2 h = {(double)(c[j].x & 0xff), 1.0}, t = {1.0, (double)(c[j].y & 0xff)};
                if (NT) {
                    __builtin_nontemporal_store(h, hom + p);
                    __builtin_nontemporal_store(t, het + p);
                } else {
                    hom[p] = h;
                    het[p] = t;
                }
            }
        }
    }
}

// the mix over block-contiguous ranges of tiles
template <int U, bool NT>
__global__ void mix_chunk(const ulonglong2* __restrict__ in, size_t npairs, uint16_t* __restrict__ code,
                          dvec2* __restrict__ hom, dvec2* __restrict__ het)
{
    const size_t tile = (size_t)blockDim.x * U;
    const size_t ntiles = (npairs + tile - 1) / tile;
    const size_t t0 = ntiles * blockIdx.x / gridDim.x, t1 = ntiles * (blockIdx.x + 1) / gridDim.x;
    for (size_t t = t0; t < t1; ++t) {
        const size_t base = t * tile;
        ulonglong2 c[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            size_t p = base + (size_t)j * blockDim.x + threadIdx.x;
            if (p < npairs) c[j] = in[p];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            size_t p = base + (size_t)j * blockDim.x + threadIdx.x;
            if (p < npairs) {
                code[p] = (uint16_t)(c[j].x ^ c[j].y);
                dvec2 h = {(double)(c[j].x & 0xff), 1.0}, t2 = {1.0, (double)(c[j].y & 0xff)};
                if (NT) {
                    __builtin_nontemporal_store(h, hom + p);
                    __builtin_nontemporal_store(t2, het + p);
                } else {
                    hom[p] = h;
                    het[p] = t2;
                }
            }
        }
    }
}

__global__ void copy_chunk(const fvec4* __restrict__ a, fvec4* __restrict__ b, size_t n)
{
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    for (size_t base = lo; base < hi; base += (size_t)blockDim.x * 4) {
        fvec4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            size_t i = base + (size_t)j * blockDim.x + threadIdx.x;
            if (i < hi) v[j] = a[i];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            size_t i = base + (size_t)j * blockDim.x + threadIdx.x;
            if (i < hi) b[i] = v[j];
        }
    }
}

int main()
{
    void* big;
    const size_t bytes = 2ull << 30;
    if (hipMalloc(&big, bytes) != hipSuccess) return 1;
    const size_t n = 50000000, npairs = n / 2;
    void *cnt, *code, *hom, *het;
    hipMalloc(&cnt, n * 8);
    hipMalloc(&code, n);
    hipMalloc(&hom, n * 8);
    hipMalloc(&het, n * 8);
    hipMemset(cnt, 1, n * 8);
    hipMemset(big, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](auto launch, double nbytes, const char* name) {
        for (int w = 0; w < 3; ++w) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, nbytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    fvec4* b = (fvec4*)big;
    const size_t n4 = bytes / 16;
    const size_t h4 = n4 / 2;
    char nm[96];
    for (int grid : {1024, 4096, 8192}) {
        snprintf(nm, sizeof nm, "copy_chunk_tb256_g%d", grid);
        timeit([&] { copy_chunk<<<grid, 256>>>(b, b + h4, h4); }, bytes, nm);
    }
    for (int grid : {1024, 2048}) {
        snprintf(nm, sizeof nm, "mix25_U2_g%d", grid);
        timeit([&] { mix<2, false><<<grid, 1024>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
               25.0 * n, nm);
    }
    for (int tb : {256, 512, 1024})
        for (int grid : {256, 512, 1024, 2048, 4096, 8192}) {
            if ((size_t)tb * grid > 4u << 20) continue;
            snprintf(nm, sizeof nm, "mixc_U1_tb%d_g%d", tb, grid);
            timeit([&] { mix_chunk<1, false><<<grid, tb>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
                   25.0 * n, nm);
            snprintf(nm, sizeof nm, "mixc_U2_tb%d_g%d", tb, grid);
            timeit([&] { mix_chunk<2, false><<<grid, tb>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
                   25.0 * n, nm);
            snprintf(nm, sizeof nm, "mixc_U4_tb%d_g%d", tb, grid);
            timeit([&] { mix_chunk<4, false><<<grid, tb>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
                   25.0 * n, nm);
            snprintf(nm, sizeof nm, "mixc_U2nt_tb%d_g%d", tb, grid);
            timeit([&] { mix_chunk<2, true><<<grid, tb>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
                   25.0 * n, nm);
        }
    return 0;
}
