// h2d_probe.cpp — host->device transfer options for the text path (not part
// of libsid): 2 GiB of pageable text (as mmap'ed page cache is) to HBM by
//   pageable   hipMemcpyAsync straight from pageable memory
//   register   hipHostRegister of the pageable range, then DMA
//   staged     T host threads memcpy into two pinned 64 MiB buffers, DMA
//              overlapped (double buffering)
// and device->host of 1 GiB into pinned and pageable memory.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const size_t N = 2ull << 30;
    char* src = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    for (size_t i = 0; i < N; i += 4096) src[i] = (char)i;   // fault in
    std::memset(src, 'A', N);
    char* dst;
    hipMalloc(&dst, N);
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    auto report = [](const char* name, size_t bytes, double s) {
        printf("{\"probe\": \"%s\", \"GBps\": %.2f, \"ms\": %.2f}\n", name, bytes / s / 1e9, s * 1e3);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        double t0 = now();
        hipMemcpyAsync(dst, src, N, hipMemcpyHostToDevice, st);
        hipStreamSynchronize(st);
        report("pageable_h2d", N, now() - t0);
    }
    {
        double t0 = now();
        hipError_t e = hipHostRegister(src, N, hipHostRegisterDefault);
        double t1 = now();
        if (e == hipSuccess) {
            report("register_cost", N, t1 - t0);
            for (int rep = 0; rep < 2; ++rep) {
                double t2 = now();
                hipMemcpyAsync(dst, src, N, hipMemcpyHostToDevice, st);
                hipStreamSynchronize(st);
                report("registered_h2d", N, now() - t2);
            }
            hipHostUnregister(src);
        } else {
            printf("{\"probe\": \"register\", \"error\": %d}\n", (int)e);
        }
    }
    const size_t B = 64ull << 20;
    char* pin[2];
    hipHostMalloc((void**)&pin[0], B, hipHostMallocDefault);
    hipHostMalloc((void**)&pin[1], B, hipHostMallocDefault);
    hipEvent_t done[2];
    hipEventCreate(&done[0]);
    hipEventCreate(&done[1]);
    for (int T : {1, 4, 8, 16}) {
        double t0 = now();
        for (size_t off = 0, k = 0; off < N; off += B, ++k) {
            const int b = (int)(k & 1);
            hipEventSynchronize(done[b]);
            const size_t len = std::min(B, N - off);
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    size_t lo = len * t / T, hi = len * (t + 1) / T;
                    std::memcpy(pin[b] + lo, src + off + lo, hi - lo);
                });
            for (auto& x : th) x.join();
            hipMemcpyAsync(dst + off, pin[b], len, hipMemcpyHostToDevice, st);
            hipEventRecord(done[b], st);
        }
        hipStreamSynchronize(st);
        char nm[64];
        snprintf(nm, sizeof nm, "staged_h2d_T%d", T);
        report(nm, N, now() - t0);
    }
    {
        char* hp;
        hipHostMalloc((void**)&hp, N / 2, hipHostMallocDefault);
        for (int rep = 0; rep < 2; ++rep) {
            double t0 = now();
            hipMemcpyAsync(hp, dst, N / 2, hipMemcpyDeviceToHost, st);
            hipStreamSynchronize(st);
            report("pinned_d2h", N / 2, now() - t0);
        }
        double t0 = now();
        hipMemcpyAsync(src, dst, N / 2, hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        report("pageable_d2h", N / 2, now() - t0);
    }
    return 0;
}
