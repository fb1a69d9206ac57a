// stream_probe.hip — speed-of-light probe for the -m local traffic mix on this
// GPU (not part of libsid).  Same grid/tile shape as sid_local_table_p2, no
// arithmetic: what HBM gives for 8 B read + 17 B written per site, next to a
// float4 copy and pure read / pure write streams.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double dvec2 __attribute__((ext_vector_type(2)));

template <int U>
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
                hom[p] = dvec2{(double)(c[j].x & 0xff), 1.0};
                het[p] = dvec2{1.0, (double)(c[j].y & 0xff)};
            }
        }
    }
}

__global__ __launch_bounds__(1024) void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__global__ __launch_bounds__(1024) void readonly(const float4* __restrict__ a, size_t n, float* out)
{
    float s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}

__global__ __launch_bounds__(1024) void writeonly(float4* __restrict__ b, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = make_float4(1, 2, 3, 4);
}

int main()
{
    const size_t n = 50000000, npairs = n / 2;
    void *cnt, *code, *hom, *het, *big;
    hipMalloc(&cnt, n * 8);
    hipMalloc(&code, n);
    hipMalloc(&hom, n * 8);
    hipMalloc(&het, n * 8);
    hipMalloc(&big, 1ull << 31);
    hipMemset(cnt, 1, n * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](auto launch, double bytes, const char* name) {
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
        printf("{\"probe\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    for (int grid : {512, 1024, 2048}) {
        char nm[64];
        snprintf(nm, sizeof nm, "mix25_U2_grid%d", grid);
        timeit([&] { mix<2><<<grid, 1024>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
               25.0 * n, nm);
        snprintf(nm, sizeof nm, "mix25_U4_grid%d", grid);
        timeit([&] { mix<4><<<grid, 1024>>>((const ulonglong2*)cnt, npairs, (uint16_t*)code, (dvec2*)hom, (dvec2*)het); },
               25.0 * n, nm);
    }
    const size_t n4 = (1ull << 30) / 16;   // 1 GiB each way
    timeit([&] { copy4<<<2048, 1024>>>((const float4*)big, (float4*)((char*)big + (1ull << 30)), n4); },
           2.0 * n4 * 16, "copy_float4_1GiB");
    timeit([&] { readonly<<<2048, 1024>>>((const float4*)big, 2 * n4, (float*)code); }, 2.0 * n4 * 16,
           "read_2GiB");
    timeit([&] { writeonly<<<2048, 1024>>>((float4*)big, 2 * n4); }, 2.0 * n4 * 16, "write_2GiB");
    return 0;
}
