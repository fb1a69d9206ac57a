// pcie_probe.cpp — the PCIe ceiling the engine's PCIe path runs against (not
// part of libsid): pinned host -> HBM as one 4 GiB copy, as 32 x 128 MiB
// copies back to back, and the same H2D with 2 GiB of HBM -> pinned D2H on a
// second stream at the same time (full duplex).  Run it under different
// HSA_ENABLE_SDMA settings to compare the copy engines with blit kernels.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const size_t N = 4ull << 30, M = 2ull << 30, P = 128ull << 20;
    char *h, *hd, *d, *dd;
    if (hipHostMalloc((void**)&h, N, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipHostMalloc((void**)&hd, M, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipMalloc(&d, N) != hipSuccess || hipMalloc(&dd, M) != hipSuccess) return 1;
    std::memset(h, 'A', N);
    std::memset(hd, 0, M);
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    auto rep = [](const char* name, double bytes, double s) {
        printf("{\"probe\": \"%s\", \"GBps\": %.2f, \"ms\": %.2f}\n", name, bytes / s / 1e9, s * 1e3);
        fflush(stdout);
    };
    for (int r = 0; r < 3; ++r) {
        double t0 = now();
        hipMemcpyAsync(d, h, N, hipMemcpyHostToDevice, s1);
        hipStreamSynchronize(s1);
        rep("h2d_one_4GiB", N, now() - t0);
        t0 = now();
        for (size_t o = 0; o < N; o += P) hipMemcpyAsync(d + o, h + o, P, hipMemcpyHostToDevice, s1);
        hipStreamSynchronize(s1);
        rep("h2d_128MiB_pieces", N, now() - t0);
        t0 = now();
        hipMemcpyAsync(hd, dd, M, hipMemcpyDeviceToHost, s2);
        hipStreamSynchronize(s2);
        rep("d2h_one_2GiB", M, now() - t0);
        t0 = now();
        for (size_t o = 0; o < N; o += P) hipMemcpyAsync(d + o, h + o, P, hipMemcpyHostToDevice, s1);
        for (size_t o = 0; o < M; o += P / 2) hipMemcpyAsync(hd + o, dd + o, P / 2, hipMemcpyDeviceToHost, s2);
        hipStreamSynchronize(s1);
        const double t1 = now();
        hipStreamSynchronize(s2);
        rep("duplex_h2d_part", N, t1 - t0);
        rep("duplex_both_done", N + M, now() - t0);
    }
    return 0;
}
