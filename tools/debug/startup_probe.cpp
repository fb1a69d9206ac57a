// The CLI's start-up, piece by piece (measurement only): HIP runtime init
// (hipGetDeviceCount), the first and a second sid_create (class tables, lazy
// code-object loads), sid_engine_create, and a hipMalloc / hipFree pair.
// Build: hipcc -O2 -Iinclude tools/debug/startup_probe.cpp -Lbuild -lsid -Wl,-rpath,$PWD/build -o build/startup_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "../../include/sid.h"

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    double t = now();
    int n = 0;
    sid_device_count(&n);
    double t1 = now();
    std::printf("{\"step\": \"hipGetDeviceCount\", \"ms\": %.2f, \"devices\": %d}\n", (t1 - t) * 1e3, n);
    sid_opts o;
    sid_opts_default(&o);
    for (int k = 0; k < 2; ++k) {
        t = now();
        sid_ctx* c = nullptr;
        int rc = sid_create(0, &o, &c);
        t1 = now();
        std::printf("{\"step\": \"sid_create %d\", \"ms\": %.2f, \"rc\": %d}\n", k, (t1 - t) * 1e3, rc);
    }
    t = now();
    void* p = nullptr;
    (void)hipMalloc(&p, 1ull << 30);
    (void)hipFree(p);
    t1 = now();
    std::printf("{\"step\": \"hipMalloc+hipFree 1 GiB\", \"ms\": %.2f}\n", (t1 - t) * 1e3);
    sid_engine_cfg cfg;
    sid_engine_cfg_default(&cfg);
    cfg.devices = 1;
    t = now();
    sid_engine* e = nullptr;
    int rc = sid_engine_create(&o, &cfg, &e);
    t1 = now();
    std::printf("{\"step\": \"sid_engine_create\", \"ms\": %.2f, \"rc\": %d}\n", (t1 - t) * 1e3, rc);
    return 0;
}
