// host_bw_probe.cpp — what the host memory gives the whole node's PCIe path
// (not part of libsid).  At N GPUs the C2 step moves, per GPU,
// 4.07 GB of pinned text to the device and 2.13 GB of records back: 8 GPUs
// draw ~0.66 TB/s from host DRAM through their DMA engines.  One GPU box
// cannot run 8 DMA streams, so this probe measures the two sides it can:
//
//   cpu_read   N threads (spread over the NUMA nodes this process may use,
//              each pinned to one CPU) each stream their own pinned buffer
//              (hipHostMalloc, first touched by that thread: node-local), R
//              passes of 64-bit loads: the aggregate read bandwidth host DRAM
//              sustains for N concurrent streams
//   dma_h2d    the GPU's H2D of its pinned buffer (copy engine) alone and
//              while N - 1 CPU threads stream theirs: the DMA under host-
//              memory contention
//
// Output: one JSON object per line; plus the NUMA layout (nodes, CPUs, the
// GPU's node).  Build: hipcc -O3 -march=x86-64-v3 -o host_bw_probe
// host_bw_probe.cpp -lpthread (tools/debug, gitignored binary).
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::vector<int> parse_cpulist(const std::string& s)
{
    std::vector<int> out;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        const std::string part = s.substr(i, j - i);
        const size_t d = part.find('-');
        if (!part.empty()) {
            const int lo = std::atoi(part.c_str());
            const int hi = d == std::string::npos ? lo : std::atoi(part.c_str() + d + 1);
            for (int c = lo; c <= hi; ++c) out.push_back(c);
        }
        i = j + 1;
    }
    return out;
}

static std::string read_line(const std::string& path)
{
    std::ifstream f(path);
    std::string s;
    std::getline(f, s);
    return s;
}

// the CPUs this process may use, grouped by NUMA node
static std::vector<std::vector<int>> node_cpus()
{
    cpu_set_t set;
    CPU_ZERO(&set);
    sched_getaffinity(0, sizeof set, &set);
    std::vector<std::vector<int>> nodes;
    for (int n = 0; n < 64; ++n) {
        const std::string s = read_line("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
        if (s.empty()) continue;
        std::vector<int> mine;
        for (int c : parse_cpulist(s))
            if (CPU_ISSET(c, &set)) mine.push_back(c);
        if (!mine.empty()) nodes.push_back(mine);
    }
    if (nodes.empty()) {
        std::vector<int> all;
        for (int c = 0; c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &set)) all.push_back(c);
        nodes.push_back(all);
    }
    return nodes;
}

static void pin(int cpu)
{
    cpu_set_t s;
    CPU_ZERO(&s);
    CPU_SET(cpu, &s);
    pthread_setaffinity_np(pthread_self(), sizeof s, &s);
}

static uint64_t stream_read(const uint64_t* p, size_t n)
{
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (size_t i = 0; i + 4 <= n; i += 4) {
        a0 += p[i];
        a1 += p[i + 1];
        a2 += p[i + 2];
        a3 += p[i + 3];
    }
    return a0 ^ a1 ^ a2 ^ a3;
}

int main(int argc, char** argv)
{
    const size_t B = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024) << 20;   // MiB per buffer
    const int R = argc > 2 ? std::atoi(argv[2]) : 4;                                  // passes
    const int maxT = argc > 3 ? std::atoi(argv[3]) : 16;
    auto nodes = node_cpus();
    std::vector<int> order;   // CPUs dealt round robin over the nodes
    for (size_t k = 0;; ++k) {
        bool any = false;
        for (auto& nd : nodes)
            if (k < nd.size()) order.push_back(nd[k]), any = true;
        if (!any) break;
    }
    int gpu_node = -1;
    {
        int dev = 0;
        char bdf[64] = {0};
        if (hipDeviceGetPCIBusId(bdf, sizeof bdf, dev) == hipSuccess) {
            std::string b(bdf);
            for (auto& ch : b) ch = (char)std::tolower(ch);
            const std::string s = read_line("/sys/bus/pci/devices/" + b + "/numa_node");
            if (!s.empty()) gpu_node = std::atoi(s.c_str());
        }
    }
    std::printf("{\"probe\": \"layout\", \"numa_nodes_usable\": %zu, \"cpus_usable\": %zu, \"gpu_numa_node\": %d, "
                "\"buffer_MiB\": %zu, \"passes\": %d}\n",
                nodes.size(), order.size(), gpu_node, B >> 20, R);
    std::fflush(stdout);
    const int T = std::min<int>(maxT, (int)order.size());
    std::vector<uint64_t*> buf(T, nullptr);
    // each buffer pinned and first touched by the thread (CPU) that reads it
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                pin(order[t]);
                if (hipHostMalloc((void**)&buf[t], B, hipHostMallocDefault) != hipSuccess) buf[t] = nullptr;
                if (buf[t]) std::memset(buf[t], t + 1, B);
            });
        for (auto& x : th) x.join();
    }
    for (auto* p : buf)
        if (!p) {
            std::fprintf(stderr, "host_bw_probe: hipHostMalloc failed\n");
            return 1;
        }
    // the NUMA node of each buffer's first page (move_pages with no target
    // nodes reports where a page lives)
    {
        std::string nodes_of = "[";
        for (int t = 0; t < T; ++t) {
            void* pg = buf[t];
            int status = -1;
            if (syscall(SYS_move_pages, 0, 1UL, &pg, nullptr, &status, 0) != 0) status = -1;
            nodes_of += (t ? ", " : "") + std::to_string(status);
        }
        std::printf("{\"probe\": \"buffer_nodes\", \"first_page_node\": %s], \"reader_cpus\": [", nodes_of.c_str());
        for (int t = 0; t < T; ++t) std::printf("%s%d", t ? ", " : "", order[t]);
        std::printf("]}\n");
        std::fflush(stdout);
    }
    std::atomic<uint64_t> sink{0};
    auto cpu_read = [&](int n, double* secs) {
        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        std::vector<std::thread> th;
        std::vector<double> dt(n, 0);
        for (int t = 0; t < n; ++t)
            th.emplace_back([&, t] {
                pin(order[t]);
                ready++;
                while (!go.load()) {
                }
                const double a = now();
                uint64_t x = 0;
                for (int r = 0; r < R; ++r) x ^= stream_read(buf[t], B / 8);
                dt[t] = now() - a;
                sink ^= x;
            });
        while (ready.load() < n) {
        }
        const double a = now();
        go = true;
        for (auto& x : th) x.join();
        *secs = now() - a;
        return (double)n * R * B / *secs / 1e9;
    };
    for (int n = 1; n <= T; n *= 2) {
        double s = 0;
        const double gbs = cpu_read(n, &s);
        std::printf("{\"probe\": \"cpu_read\", \"threads\": %d, \"GBps\": %.1f, \"s\": %.3f}\n", n, gbs, s);
        std::fflush(stdout);
    }
    if (T != 1 && (T & (T - 1))) {
        double s = 0;
        std::printf("{\"probe\": \"cpu_read\", \"threads\": %d, \"GBps\": %.1f, \"s\": %.3f}\n", T, cpu_read(T, &s), s);
    }
    // the GPU's DMA from buffer 0 (CPU 0's node), alone and beside n readers
    char* d = nullptr;
    hipStream_t st;
    if (hipMalloc(&d, B) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    auto dma = [&](int reps) {
        const double a = now();
        for (int r = 0; r < reps; ++r) (void)hipMemcpyAsync(d, buf[0], B, hipMemcpyHostToDevice, st);
        (void)hipStreamSynchronize(st);
        return (double)reps * B / (now() - a) / 1e9;
    };
    dma(1);
    std::printf("{\"probe\": \"dma_h2d\", \"cpu_readers\": 0, \"GBps\": %.1f}\n", dma(2 * R));
    std::fflush(stdout);
    for (int n = 1; n < T; n = n * 2 + 1) {
        std::atomic<bool> stop{false};
        std::vector<std::thread> th;
        std::atomic<uint64_t> bytes{0};
        // the readers' bytes between the DMA's start and end: each reader
        // times its passes; a pass counts by the part of it inside the window
        std::vector<std::vector<std::pair<double, double>>> passes(n + 1);
        for (int t = 1; t <= n; ++t)
            th.emplace_back([&, t] {
                pin(order[t]);
                while (!stop.load()) {
                    const double p0 = now();
                    sink ^= stream_read(buf[t], B / 8);
                    passes[t].emplace_back(p0, now());
                }
            });
        const double a = now();
        const double g = dma(2 * R);
        const double b = now();
        stop = true;
        for (auto& x : th) x.join();
        double in = 0;
        for (auto& v : passes)
            for (auto& pr : v) {
                const double lo = std::max(pr.first, a), hi = std::min(pr.second, b);
                if (hi > lo) in += (double)B * (hi - lo) / (pr.second - pr.first);
            }
        (void)bytes;
        std::printf("{\"probe\": \"dma_h2d\", \"cpu_readers\": %d, \"GBps\": %.1f, \"cpu_GBps_beside\": %.1f}\n", n, g,
                    in / (b - a) / 1e9);
        std::fflush(stdout);
    }
    std::fprintf(stderr, "(sink %llu)\n", (unsigned long long)sink.load());
    return 0;
}
