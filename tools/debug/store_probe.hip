// store_probe.hip — pure-store HBM bandwidth on this GPU, in the shape
// MI355X_MICROARCH.md quotes 6.0-6.2 TB/s for ("plain stores ... one dword per
// lane, 256 B per wave-instruction, random 2,304-B rows of a 75 MB or 302 MB
// table, 8 waves per CU") and in the streaming shapes the engine's kernels
// use (16 B per lane = 1 KiB per wave-instruction, contiguous), with default
// and nontemporal cache policy, over tables of 75 MB, 302 MB and 4 GB.  Not
// part of libsid.  Build: hipcc -O3 --offload-arch=gfx950 -o store_probe store_probe.hip
// Prints one JSON line per variant.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float fvec4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

// the guide's shape: each wave sweeps rows of 2304 B (576 dwords) in random
// order, one dword per lane per instruction (9 instructions per row)
template <bool NT>
__global__ __launch_bounds__(256) void rows_dword(float* __restrict__ t, uint32_t nrows, uint32_t rows_per_wave,
                                                  uint32_t seed)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint32_t h = wave * 2654435761u ^ seed;
    for (uint32_t k = 0; k < rows_per_wave; ++k) {
        h = h * 1664525u + 1013904223u;
        float* row = t + (size_t)(h % nrows) * 576;
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            if (NT) __builtin_nontemporal_store((float)k, row + j * 64 + lane);
            else row[j * 64 + lane] = (float)k;
        }
    }
}

// contiguous stream, V dwords per lane per instruction (1 or 4), grid-stride
template <int V, bool NT>
__global__ __launch_bounds__(256) void stream(float* __restrict__ t, size_t n_vec)
{
    const size_t step = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += step) {
        if (V == 4) {
            const fvec4 v = {1.f, 2.f, 3.f, (float)i};
            if (NT) __builtin_nontemporal_store(v, (fvec4*)t + i);
            else ((fvec4*)t)[i] = v;
        } else {
            if (NT) __builtin_nontemporal_store((float)i, t + i);
            else t[i] = (float)i;
        }
    }
}

int main()
{
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const size_t sizes[3] = {75ull << 20, 302ull << 20, 4ull << 30};
    float* t = nullptr;
    CK(hipMalloc(&t, sizes[2]));
    CK(hipMemset(t, 0, sizes[2]));
    for (size_t bytes : sizes) {
        // rows: 8 waves per CU (2 blocks of 256), each sweeping enough rows to
        // write the table's bytes ~4 times over
        const uint32_t nrows = (uint32_t)(bytes / 2304);
        const uint32_t waves = (uint32_t)cus * 8;
        const uint32_t rpw = (uint32_t)((4 * bytes / 2304 + waves - 1) / waves);
        for (int nt = 0; nt < 2; ++nt) {
            auto run = [&]() {
                if (nt) rows_dword<true><<<cus * 2, 256>>>(t, nrows, rpw, 7u);
                else rows_dword<false><<<cus * 2, 256>>>(t, nrows, rpw, 7u);
            };
            run();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) run();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            const double by = 5.0 * (double)waves * rpw * 2304.0;
            std::printf("{\"shape\": \"rows_2304B_dword\", \"table_bytes\": %zu, \"nt\": %d, \"waves_per_cu\": 8, "
                        "\"TBps\": %.3f}\n", bytes, nt, by / (ms * 1e-3) / 1e12);
        }
        for (int v = 0; v < 2; ++v)
            for (int nt = 0; nt < 2; ++nt)
                for (int wpc : {8, 16, 32}) {
                    const int grid = cus * wpc / 4;
                    const size_t nvec = v ? bytes / 16 : bytes / 4;
                    auto run = [&]() {
                        if (v && nt) stream<4, true><<<grid, 256>>>(t, nvec);
                        else if (v) stream<4, false><<<grid, 256>>>(t, nvec);
                        else if (nt) stream<1, true><<<grid, 256>>>(t, nvec);
                        else stream<1, false><<<grid, 256>>>(t, nvec);
                    };
                    run();
                    CK(hipDeviceSynchronize());
                    const int reps = bytes < (1ull << 30) ? 50 : 5;
                    CK(hipEventRecord(a));
                    for (int r = 0; r < reps; ++r) run();
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    std::printf("{\"shape\": \"stream_%s\", \"table_bytes\": %zu, \"nt\": %d, \"waves_per_cu\": %d, "
                                "\"TBps\": %.3f}\n", v ? "16B_per_lane" : "dword_per_lane", bytes, nt, wpc,
                                (double)reps * bytes / (ms * 1e-3) / 1e12);
                }
    }
    CK(hipFree(t));
    return 0;
}
