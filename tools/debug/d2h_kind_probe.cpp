// Which device->pinned-host copies the runtime carries out with a copy engine
// and which with a blit kernel: sizes with and without a multiple of 4 bytes,
// run under rocprofv3 --kernel-trace --memory-copy-trace (a blit shows up as
// __amd_rocclr_copyBuffer in the kernel trace, a copy-engine copy in the
// memory-copy trace).  Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/d2hk d2h_kind_probe.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

int main()
{
    const size_t M = 96ull << 20;
    char *dd = nullptr, *hd = nullptr, *d2 = nullptr, *h2 = nullptr;
    if (hipMalloc(&d2, M) != hipSuccess || hipHostMalloc((void**)&h2, M, hipHostMallocDefault) != hipSuccess) return 1;
    hipStream_t s, s2;
    hipEvent_t a, b;
    if (hipMalloc(&dd, M) != hipSuccess || hipHostMalloc((void**)&hd, M, hipHostMallocDefault) != hipSuccess ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&a) != hipSuccess ||
        hipEventCreate(&b) != hipSuccess)
        return 1;
    (void)hipMemset(dd, 1, M);
    const size_t sizes[] = {64ull << 20, (64ull << 20) + 3, (64ull << 20) + 4, (64ull << 20) + 2, 70000001, 70000000};
    hipEvent_t w;
    if (hipEventCreateWithFlags(&w, hipEventDisableTiming) != hipSuccess) return 1;
    // rep 2, 3: the copy's stream first waits for an event of another stream
    // (recorded after a fill there; done or not yet); rep 4: a host->device
    // copy runs on the other stream meanwhile
    // rep 5: into a large pinned arena (8 GiB, as the engine's host arena)
    char* big = nullptr;
    if (hipHostMalloc((void**)&big, 8ull << 30, hipHostMallocDefault) != hipSuccess) return 3;
    for (int rep = 0; rep < 6; ++rep)
        for (size_t n : sizes) {
            if (rep == 4) (void)hipMemcpyAsync(d2, h2, M, hipMemcpyHostToDevice, s2);
            if (rep == 2 || rep == 3) {
                (void)hipMemsetAsync(dd + M - 4096, 0, 4096, s2);
                (void)hipEventRecord(w, s2);
                if (rep == 3) (void)hipEventSynchronize(w);
                (void)hipStreamWaitEvent(s, w, 0);
            }
            (void)hipEventRecord(a, s);
            (void)hipMemcpyAsync(rep == 5 ? big + (5ull << 30) : hd, dd, n, hipMemcpyDeviceToHost, s);
            (void)hipEventRecord(b, s);
            if (hipStreamSynchronize(s) != hipSuccess || hipStreamSynchronize(s2) != hipSuccess) return 2;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("rep %d D2H %zu bytes (mod 4 = %zu): %.3f ms, %.1f GB/s\n", rep, n, n % 4, ms, n / (ms * 1e6));
        }
    return 0;
}
