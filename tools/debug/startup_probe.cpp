// The CLI's start-up, piece by piece (measurement only): HIP runtime init
// (hipInit, then hipGetDeviceCount), the device's context (hipSetDevice +
// hipFree(0)), the first and a second sid_create (class tables, lazy
// code-object loads), the engine's pieces (streams, events, a pinned word),
// sid_engine_create, and a hipMalloc / hipFree pair.
// Build: hipcc -O2 -Iinclude tools/debug/startup_probe.cpp -Lbuild -lsid -Wl,-rpath,$PWD/build -o build/startup_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "../../include/sid.h"

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double t_last;
static void step(const char* name, int rc = 0)
{
    const double t = now();
    std::printf("{\"step\": \"%s\", \"ms\": %.2f, \"rc\": %d}\n", name, (t - t_last) * 1e3, rc);
    std::fflush(stdout);
    t_last = now();
}

int main()
{
    const double t0 = now();
    t_last = t0;
    int rc = (int)hipInit(0);
    step("hipInit", rc);
    int n = 0;
    rc = sid_device_count(&n);
    step("hipGetDeviceCount", rc);
    rc = (int)hipSetDevice(0);
    step("hipSetDevice", rc);
    rc = (int)hipFree(nullptr);
    step("hipFree(0) (context)", rc);
    sid_opts o;
    sid_opts_default(&o);
    for (int k = 0; k < 2; ++k) {
        sid_ctx* c = nullptr;
        rc = sid_create(0, &o, &c);
        step(k ? "sid_create 1" : "sid_create 0", rc);
    }
    hipStream_t s[3];
    for (int k = 0; k < 3; ++k) {
        rc = (int)hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking);
        step("hipStreamCreateWithFlags", rc);
    }
    hipEvent_t ev[8];
    for (auto& e : ev) rc |= (int)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    step("8 x hipEventCreateWithFlags", rc);
    void* h = nullptr;
    rc = (int)hipHostMalloc(&h, 128, hipHostMallocDefault);
    step("hipHostMalloc 128 B", rc);
    void* p = nullptr;
    rc = (int)hipMalloc(&p, 1ull << 30);
    rc |= (int)hipFree(p);
    step("hipMalloc+hipFree 1 GiB", rc);
    sid_engine_cfg cfg;
    sid_engine_cfg_default(&cfg);
    cfg.devices = 1;
    sid_engine* e = nullptr;
    rc = sid_engine_create(&o, &cfg, &e);
    step("sid_engine_create", rc);
    std::printf("{\"step\": \"total\", \"ms\": %.2f}\n", (now() - t0) * 1e3);
    return 0;
}
