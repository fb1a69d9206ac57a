// How long a process that used the GPU takes to go away after its last
// instruction (measurement only): the mode picks what it set up before
// _exit(0); it prints its exit time (unix seconds) and exit_probe.py measures
// from there to the parent's wait returning.
//   init    hipInit + the device's context (hipFree(0))
//   streams + 3 non-blocking streams and a kernel-free copy on each
//   hbm     + 4 GiB of HBM written (hipMemset)
//   pinned  + 64 MiB of pinned host memory
//   engine  sid_engine_create (one device), nothing run
// Build: hipcc -O2 -Iinclude tools/debug/exit_probe.cpp -Lbuild -lsid -Wl,-rpath,$PWD/build -o build/exit_probe
#include <hip/hip_runtime.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

#include "../../include/sid.h"

static double unix_now()
{
    timeval tv;
    gettimeofday(&tv, nullptr);
    return tv.tv_sec + tv.tv_usec * 1e-6;
}

int main(int argc, char** argv)
{
    const char* mode = argc > 1 ? argv[1] : "init";
    const bool streams = !std::strcmp(mode, "streams") || !std::strcmp(mode, "hbm") || !std::strcmp(mode, "pinned");
    const bool hbm = !std::strcmp(mode, "hbm") || !std::strcmp(mode, "pinned");
    const bool pinned = !std::strcmp(mode, "pinned");
    int rc = 0;
    if (!std::strcmp(mode, "engine")) {
        sid_opts o;
        sid_opts_default(&o);
        sid_engine_cfg cfg;
        sid_engine_cfg_default(&cfg);
        cfg.devices = 1;
        sid_engine* e = nullptr;
        rc = sid_engine_create(&o, &cfg, &e);
    } else {
        rc |= (int)hipInit(0);
        rc |= (int)hipSetDevice(0);
        rc |= (int)hipFree(nullptr);
        void* d = nullptr;
        if (streams) {
            rc |= (int)hipMalloc(&d, hbm ? (4ull << 30) : (1ull << 20));
            for (int k = 0; k < 3; ++k) {
                hipStream_t s;
                rc |= (int)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
                rc |= (int)hipMemsetAsync(d, k, hbm ? (4ull << 30) : (1ull << 20), s);
                rc |= (int)hipStreamSynchronize(s);
            }
        }
        if (pinned) {
            void* h = nullptr;
            rc |= (int)hipHostMalloc(&h, 64ull << 20, hipHostMallocDefault);
            rc |= (int)hipMemcpy(h, d, 64ull << 20, hipMemcpyDeviceToHost);
        }
    }
    std::printf("{\"mode\": \"%s\", \"rc\": %d, \"main_exit_unix\": %.6f}\n", mode, rc, unix_now());
    std::fflush(stdout);
    _exit(0);
}
