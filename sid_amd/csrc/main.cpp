// main.cpp — the `sid` command line on MI355X.
//
// Same surface as sid.cpp:1-110: getopt flags -h -m -r -R -p -E with the
// reference's defaults, help text, error messages and exit codes; CSV on
// stdout, "# ..." diagnostics on stderr.  Behind it, by default, the
// streaming engine (run.cpp, sid_engine_*): the input file in line-aligned
// chunks -> device text buffers -> parse -> call / Lynch -> records formatted
// on the device -> stdout in file order, every visible GPU taking chunks in
// turn, with bounded host memory (C4's 3G sites stream through).
//
// Extra long options (no short letter, so they cannot collide with the
// reference's flags): --devices N, --threads N, --stats, --host-parse,
// --chunk-bytes N, --hold-bytes N, --retain-bytes N, --host-hold N.
//
// --host-parse keeps the round-1 path instead: the whole input parsed on the
// host (sid_parse_text), counts to the devices, records formatted on the host
// (sid_format_csv).
//
// As in the reference, the whole input is parsed before anything is written
// to stdout, so a malformed line aborts with no CSV output (call.cpp:11-20
// reads the file before sid.cpp:102 prints the header).
#include <fcntl.h>
#include <getopt.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <csignal>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sid.h"

namespace {

struct Options {
    std::string method = "local";
    sid_opts o;
    int devices = 0;   // 0: every visible device
    int threads = 0;
    bool stats = false;
    bool host_parse = false;   // parse and format on the host (sid_parse_text / sid_format_csv)
    uint64_t chunk_bytes = 0;  // engine knobs (0 = defaults)
    uint64_t hold_bytes = 0;
    uint64_t host_hold = 0;   // --host-hold: sid_engine_cfg.host_hold_bytes
    uint64_t retain_bytes = 0;
};

// sid.cpp:26-58; std::map<char,...> iterates E R h m p r
const struct {
    char flag;
    const char* name;
    int has_arg;
    const char* description;
} OPTIONS[] = {
    {'E', "ERROR", 1, "Maximum allowed site error rate for 'local' method. Default: 0.1"},
    {'R', "", 0, "Estimate SNP prior from data, applicable for methods 'likelihood_ratio', 'local', 'quality'. Conflicts -r."},
    {'h', "help", 0, "Print this help message"},
    {'m', "METHOD", 1, "Select the method to use for SNP calling: 'likelihood_ratio' , 'bayes', 'local' or 'quality', default: local"},
    {'p', "LEVEL", 1, "Significance level for statistical tests, only applicable for methods 'likelihood_ratio', 'local'. Default: 0.05"},
    {'r', "PRIOR", 1, "Use the given prior for SNPs, applicable for methods 'local', 'quality'. Conflicts -R. Default: no prior"},
};

[[noreturn]] void terminate_like(const char* type, const char* what)
{
    std::fflush(stdout);
    std::fprintf(stderr, "terminate called after throwing an instance of '%s'\n  what():  %s\n", type, what);
    std::abort();
}

[[noreturn]] void fail(const char* what, int rc)
{
    std::fflush(stdout);
    if (rc == SID_EHIP)
        std::fprintf(stderr, "sid: %s: %s (hip error %d)\n", what, sid_strerror(rc), sid_last_hip_error());
    else
        std::fprintf(stderr, "sid: %s: %s\n", what, sid_strerror(rc));
    std::exit(EXIT_FAILURE);
}

#define CHECK(call, what)                 \
    do {                                  \
        int rc_ = (call);                 \
        if (rc_ != SID_OK) fail(what, rc_); \
    } while (0)

#define HCHECK(call, what)                                                              \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "sid: %s: %s\n", what, hipGetErrorString(e_));         \
            std::exit(EXIT_FAILURE);                                                    \
        }                                                                               \
    } while (0)

double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// wall-clock seconds (--stats: main's entry and exit, so a caller timing the
// process can split off the start-up and the teardown)
double unix_now()
{
    return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

// The end of a successful run: stdout and stderr flushed, then the process
// ends without the HIP runtime's teardown (the kernel driver releases the
// HBM, the pinned pages and the mapping with the process either way).
// (exit() with the runtime's static destructors measured 0.06-0.18 s slower;
// DESIGN.md §6.)  Under the profiler (ROCPROF* / ROCP_* in the environment: rocprofv3 sets
// them for its preloaded tool, which writes its buffers from atexit
// handlers) exit() is used too, so traces of this binary are complete.
bool tool_attached()
{
    for (char** e = environ; e && *e; ++e)
        if (std::strncmp(*e, "ROCPROF", 7) == 0 || std::strncmp(*e, "ROCP_", 5) == 0)
            return true;
    return false;
}

[[noreturn]] void finish(int code)
{
    std::fflush(stdout);
    std::fflush(stderr);
    if (tool_attached()) std::exit(code);
    ::_exit(code);
}

struct Input {
    const char* data = nullptr;   // the text in memory (pipes, or mapped for --host-parse)
    size_t len = 0;
    void* map = nullptr;
    std::string owned;
    int fd = -1;                  // regular file: mapped by the engine (sid_engine_source_file)
};

void map_input(Input& in, bool populate)
{
    if (in.data || in.fd < 0 || !in.len) return;
    in.map = mmap(nullptr, in.len, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), in.fd, 0);
    if (in.map == MAP_FAILED) {
        in.map = nullptr;
        in.owned.resize(in.len);
        size_t off = 0;
        while (off < in.len) {
            ssize_t r = ::pread(in.fd, &in.owned[off], in.len - off, (off_t)off);
            if (r <= 0) break;
            off += (size_t)r;
        }
        in.owned.resize(off);
        in.data = in.owned.data();
        in.len = off;
    } else {
        madvise(in.map, in.len, MADV_SEQUENTIAL);
        in.data = (const char*)in.map;
    }
}

// std::ifstream semantics: open failure -> "Could not open file" (sid.cpp:86-89)
bool open_input(const char* path, Input& in)
{
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
        in.len = (size_t)st.st_size;
        in.fd = fd;   // kept open
        return true;
    }
    if (fstat(fd, &st) == 0 && S_ISDIR(st.st_mode)) {
        // std::ifstream opens a directory, getline then fails: no records
        in.len = 0;
    } else {   // pipe / character device
        char buf[1 << 16];
        ssize_t r;
        while ((r = ::read(fd, buf, sizeof buf)) > 0) in.owned.append(buf, (size_t)r);
        in.data = in.owned.data();
        in.len = in.owned.size();
    }
    ::close(fd);
    return true;
}

struct Shard {
    size_t begin = 0, end = 0;            // global site range
    sid_ctx* ctx = nullptr;
    const uint16_t* d_counts = nullptr;   // the shard's counts
    uint16_t* d_own_counts = nullptr;     // host-parse path: uploaded counts
    uint8_t* d_code = nullptr;
    double* d_hom = nullptr;
    double* d_het = nullptr;
    hipStream_t stream = nullptr;
};

}  // namespace

int main(int argc, char** argv)
{
    const double t_entry = unix_now();
    // host<->device copies on the copy engines (set before the HIP runtime
    // starts; an explicit setting in the environment wins): with the
    // runtime's default, device->host ran at 30 GB/s, with SDMA at ~57 GB/s
    // and concurrently with host->device (tools/debug/pcie_probe.cpp)
    setenv("HSA_ENABLE_SDMA", "1", 0);
    Options opt;
    sid_opts_default(&opt.o);
    static const struct option LONG[] = {{"devices", required_argument, nullptr, 1},
                                         {"threads", required_argument, nullptr, 2},
                                         {"stats", no_argument, nullptr, 3},
                                         {"host-parse", no_argument, nullptr, 4},
                                         {"chunk-bytes", required_argument, nullptr, 5},
                                         {"hold-bytes", required_argument, nullptr, 6},
                                         {"retain-bytes", required_argument, nullptr, 7},
                                         {"host-hold", required_argument, nullptr, 8},
                                         {nullptr, 0, nullptr, 0}};
    int flag;
    while ((flag = getopt_long(argc, argv, "E:Rhm:p:r:", LONG, nullptr)) != -1) {
        switch (flag) {
        case 'E': opt.o.site_error_threshold = std::atof(optarg); break;
        case 'R': opt.o.estimate_prior = 1; break;
        case 'm': opt.method = optarg; break;
        case 'p': opt.o.significance_level = std::atof(optarg); break;
        case 'r': opt.o.snp_prior = std::atof(optarg); break;
        case 'h':
            std::fputs("sid [flags] input_file\n", stdout);
            for (const auto& o : OPTIONS) {
                std::printf("\t-%c", o.flag);
                if (o.has_arg > 0) std::printf(" %s", o.name);
                std::printf("\t%s\n", o.description);
            }
            break;
        case 1: opt.devices = std::max(1, std::atoi(optarg)); break;
        case 2: opt.threads = std::max(1, std::atoi(optarg)); break;
        case 3: opt.stats = true; break;
        case 4: opt.host_parse = true; break;
        case 5: opt.chunk_bytes = std::strtoull(optarg, nullptr, 10); break;
        case 6: opt.hold_bytes = std::strtoull(optarg, nullptr, 10); break;
        case 7: opt.retain_bytes = std::strtoull(optarg, nullptr, 10); break;
        case 8: opt.host_hold = std::strtoull(optarg, nullptr, 10); break;
        default: std::exit(EXIT_FAILURE);
        }
    }
    if (optind >= argc) {
        std::fflush(stdout);
        std::fputs("No file name given!\n", stderr);
        std::exit(EXIT_FAILURE);
    }
    const char* path = argv[optind];
    Input in;
    if (!open_input(path, in)) {
        std::fflush(stdout);
        std::fprintf(stderr, "Could not open file: %s\n", path);
        std::exit(EXIT_FAILURE);
    }
    int method = -1;
    if (opt.method == "local") method = SID_METHOD_LOCAL;
    else if (opt.method == "bayes") method = SID_METHOD_BAYES;
    else if (opt.method == "likelihood_ratio") method = SID_METHOD_LIKELIHOOD_RATIO;
    else if (opt.method == "quality") method = SID_METHOD_QUALITY;   // call.cpp:291-372
    if (method < 0) {   // sid.cpp:92-102: unknown method -> header only
        std::printf("chrom,pos,label,gt,hom_conf,het_conf,conf_type\n");
        return 0;
    }
    opt.o.method = method;
    if (method == SID_METHOD_BAYES) opt.o.estimate_prior = 0;   // callBayes(in) ignores -R/-r/-p
    const int T = opt.threads > 0 ? opt.threads
                                  : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));

    // The engine path over a regular file of up to 8 GiB: the HIP runtime's
    // start-up and the engine's creation (60-240 ms: the runtime's
    // initialisation, the contexts' class tables, the streams' hardware
    // queues) on a second thread while this one maps the file and populates
    // its page tables (~30 ms for 4 GB).
    const bool overlap = !opt.host_parse && in.fd >= 0 && !in.data && in.len && in.len <= (8ull << 30);
    int ndev = 0, D = 0;
    sid_engine* eng = nullptr;
    sid_engine_cfg cfg;
    sid_engine_cfg_default(&cfg);
    auto make_engine = [&]() -> int {
        cfg.devices = D;
        cfg.chunk_bytes = opt.chunk_bytes;
        cfg.hold_bytes = opt.hold_bytes;
        cfg.retain_bytes = opt.retain_bytes;
        cfg.host_hold_bytes = opt.host_hold;
        cfg.host_threads = T;
        cfg.verbose = 1;
        return sid_engine_create(&opt.o, &cfg, &eng);
    };
    int dev_rc = SID_OK, eng_rc = SID_OK;
    double t0 = 0, tc = 0;
    const char* pre_map = nullptr;
    auto start_devices = [&](bool engine) {
        dev_rc = sid_device_count(&ndev);
        if (dev_rc != SID_OK || ndev <= 0) return;
        D = opt.devices > 0 ? opt.devices : ndev;
        if (!engine) return;
        t0 = now();
        eng_rc = make_engine();
        tc = now();
    };
    if (overlap) {
        std::thread th(start_devices, true);
        void* m = mmap(nullptr, in.len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, in.fd, 0);
        if (m != MAP_FAILED) {
            (void)madvise(m, in.len, MADV_SEQUENTIAL);
            pre_map = (const char*)m;
        }
        th.join();
    } else {
        start_devices(false);
    }
    CHECK(dev_rc, "device query");
    if (ndev <= 0) {
        std::fflush(stdout);
        std::fputs("sid: no HIP device available\n", stderr);
        std::exit(EXIT_FAILURE);
    }
    // shard d runs on device d % ndev (more shards than devices: a
    // multi-device run's splitting and merging on fewer GPUs)
    const bool quality = method == SID_METHOD_QUALITY;
    // the Lynch estimate: LR and bayes always, local and quality with -R
    const bool lynch = method == SID_METHOD_LIKELIHOOD_RATIO || method == SID_METHOD_BAYES || opt.o.estimate_prior;
    // per-read qualities live in the text: -m quality always takes the device text path
    if (quality) opt.host_parse = false;
    const char* conf_type = method == SID_METHOD_BAYES ? "probability" : "p_value";
    std::vector<Shard> sh(D);
    auto on_parse_error = [&](int prc) {
        if (prc == SID_EMALFORMED) terminate_like("std::invalid_argument", "Malformed pileup line");
        if (prc == SID_EMISSING_MQ)   // pileup.cpp:10,63
            terminate_like("std::invalid_argument", "Malformed pileup line or missing mapping qualities");
        if (prc == SID_ENULLCHROM || prc == SID_ENOBQ) {
            // pileup.cpp:18 assigns a NULL char* to std::string (or, for
            // -m quality, pileup.cpp:158 reads a NULL field): the reference
            // dies with SIGSEGV, printing nothing
            std::fflush(stdout);
            std::signal(SIGSEGV, SIG_DFL);
            std::raise(SIGSEGV);
        }
        CHECK(prc, "parse");
    };
    auto make_ctx = [&](int d) {
        Shard& s = sh[d];
        CHECK(sid_create(d % ndev, &opt.o, &s.ctx), "context");
        HCHECK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "stream");
    };
    auto alloc_out = [&](Shard& s) {
        const size_t m = std::max<size_t>(s.end - s.begin, 1);
        HCHECK(hipMalloc(&s.d_code, m), "device code");
        HCHECK(hipMalloc(&s.d_hom, m * 8), "device hom_conf");
        HCHECK(hipMalloc(&s.d_het, m * 8), "device het_conf");
    };
    auto parallel = [&](auto fn) {
        std::vector<std::thread> th;
        for (int d = 1; d < D; ++d) th.emplace_back(fn, d);
        fn(0);
        for (auto& x : th) x.join();
    };

    auto write_all = [](void*, const char* p, size_t len) -> int {
        size_t off = 0;
        while (off < len) {
            ssize_t w = ::write(1, p + off, len - off);
            if (w <= 0) return -1;
            off += (size_t)w;
        }
        return 0;
    };
    const char* HEADER = "chrom,pos,label,gt,hom_conf,het_conf,conf_type\n";

    // ------------------------------------------------ streaming engine path --
    if (!opt.host_parse) {
        if (!overlap) {
            t0 = now();
            eng_rc = make_engine();
            tc = now();
        }
        CHECK(eng_rc, "engine");
        if (pre_map) CHECK(sid_engine_source_text(eng, pre_map, in.len), "input");   // (mapped above)
        else if (in.fd >= 0 && !in.data) CHECK(sid_engine_source_file(eng, in.fd, 0, in.len), "input");
        else CHECK(sid_engine_source_text(eng, in.data, in.len), "input");
        sid_run_stats st;
        std::memset(&st, 0, sizeof st);
        int rc = sid_engine_ingest(eng, &st);
        if (rc != SID_OK) on_parse_error(rc);
        const double t1 = now();
        rc = sid_engine_estimate(eng, nullptr, &st.estimate);
        if (rc == SID_EEMPTY) {
            std::fflush(stdout);
            std::fputs("sid: no profile with coverage >= 4 (the reference crashes here)\n", stderr);
            std::exit(139);
        }
        if (rc == SID_EBADFUNC) {
            std::fflush(stdout);
            std::fputs("gsl: nmsimplex2.c: ERROR: non-finite function value encountered\n"
                       "Default GSL error handler invoked.\n", stderr);
            std::abort();
        }
        CHECK(rc, "estimate");
        const double t2 = now();
        std::fflush(stdout);
        rc = sid_engine_emit(eng, HEADER, write_all, nullptr, &st);
        if (rc == SID_EIO) std::exit(EXIT_FAILURE);
        CHECK(rc, "emit");
        const double t3 = now();
        std::string place;   // per pipeline: its GPU, the CPUs its threads ran on, its pinned buffers' NUMA nodes
        if (opt.stats)
            for (int i = 0; i < sid_engine_devices(eng); ++i) {
                sid_placement pl;
                if (sid_engine_placement(eng, i, &pl) != SID_OK) continue;
                char b[256];
                std::snprintf(b, sizeof b,
                              "%s{\"device\": %d, \"pci\": \"%s\", \"gpu_numa_node\": %d, \"cpus\": %d, "
                              "\"first_cpu\": %d, \"arena_numa_node\": %d, \"ring_numa_node\": %d}",
                              place.empty() ? "" : ", ", pl.device, pl.pci, pl.gpu_numa_node, pl.cpus, pl.first_cpu,
                              pl.arena_numa_node, pl.ring_numa_node);
                place += b;
            }
        if (opt.stats)
            std::fprintf(stderr,
                         "{\"sites\": %llu, \"devices\": %d, \"threads\": %d, \"path\": \"stream\", "
                         "\"create_s\": %.6f, \"parse_s\": %.6f, \"device_s\": %.6f, \"emit_s\": %.6f, \"total_s\": %.6f, "
                         "\"sites_per_s\": %.1f, \"chunks\": %llu, \"chunks_held\": %llu, "
                         "\"chunks_retained\": %llu, \"chunks_reloaded\": %llu, \"bytes_in\": %llu, "
                         "\"bytes_out\": %llu, \"ingest_s\": %.6f, \"chunks_registered\": %llu, "
                         "\"register_s\": %.6f, \"h2d_s\": %.6f, \"h2d_bytes\": %llu, \"chunks_tiled\": %llu, "
                         "\"tile_overflows\": %llu, \"tile_overflows_queued\": %llu, \"placement\": [%s], "
                         "\"main_entry_unix\": %.6f, \"main_exit_unix\": %.6f}\n",
                         (unsigned long long)st.sites, D, T, tc - t0, t1 - t0, t2 - t1, t3 - t2, t3 - t0,
                         st.sites / std::max(1e-9, t3 - t0), (unsigned long long)st.chunks,
                         (unsigned long long)st.chunks_held, (unsigned long long)st.chunks_retained,
                         (unsigned long long)st.chunks_reloaded, (unsigned long long)st.bytes_in,
                         (unsigned long long)st.bytes_out, st.ingest_s, (unsigned long long)st.chunks_registered,
                         st.register_s, st.h2d_s, (unsigned long long)st.h2d_bytes,
                         (unsigned long long)st.chunks_tiled, (unsigned long long)st.tile_overflows,
                         (unsigned long long)st.tile_overflows_queued, place.c_str(),
                         t_entry,
                         unix_now());
        // device memory, pinned staging and the mapping go with the process
        finish(0);
    }

    // ------------------------------------------------------ host-parse path --
    t0 = now();
    sid_sites* sites = nullptr;
    size_t n = 0;
    {
        uint64_t bad = 0;
        map_input(in, true);
        int prc = sid_parse_text(in.data, in.len, T, &sites, &bad);
        on_parse_error(prc);
        if (in.map) munmap(in.map, in.len);
        in.map = nullptr;
        n = sid_sites_count(sites);
        const uint16_t* h_counts = sid_sites_counts(sites);
        for (int d = 0; d < D; ++d) {
            sh[d].begin = n * d / D;
            sh[d].end = n * (d + 1) / D;
        }
        parallel([&](int d) {
            make_ctx(d);
            Shard& s = sh[d];
            HCHECK(hipMalloc(&s.d_own_counts, std::max<size_t>(s.end - s.begin, 1) * 8), "device counts");
            s.d_counts = s.d_own_counts;
            if (s.end > s.begin)
                HCHECK(hipMemcpyAsync(s.d_own_counts, h_counts + 4 * s.begin, (s.end - s.begin) * 8,
                                      hipMemcpyHostToDevice, s.stream),
                       "H2D");
            alloc_out(s);
            HCHECK(hipStreamSynchronize(s.stream), "H2D");
        });
    }
    double t1 = now();

    // -------------------------------------------------------------- compute --
    if (lynch) {
        parallel([&](int d) {
            Shard& s = sh[d];
            (void)hipSetDevice(d % ndev);
            CHECK(sid_profile_reset(s.ctx, s.stream), "histogram");
            CHECK(sid_profile_accumulate(s.ctx, s.d_counts, s.end - s.begin, s.stream), "histogram");
        });
        // merge the per-device histograms (the single exchange of the path)
        std::vector<uint64_t> keys, cnts;
        for (int d = 0; d < D; ++d) {
            (void)hipSetDevice(d % ndev);
            size_t u = 0;
            CHECK(sid_profile_table(sh[d].ctx, nullptr, nullptr, 0, &u), "profile table");
            size_t at = keys.size();
            keys.resize(at + u);
            cnts.resize(at + u);
            CHECK(sid_profile_table(sh[d].ctx, keys.data() + at, cnts.data() + at, u, &u), "profile table");
        }
        std::vector<int> rcs(D, SID_OK);
        std::vector<sid_estimate> est(D);
        auto prep = [&](int d) {
            (void)hipSetDevice(d % ndev);
            if (D > 1) {
                int rc = sid_profile_load(sh[d].ctx, keys.data(), cnts.data(), keys.size());
                if (rc) {
                    rcs[d] = rc;
                    return;
                }
            }
            rcs[d] = sid_lynch_prepare(sh[d].ctx, d == 0, &est[d]);
            if (rcs[d] == SID_OK && method == SID_METHOD_LOCAL)
                rcs[d] = sid_set_prior(sh[d].ctx, est[d].heterozygosity);   // call.cpp:233, :305
        };
        // device 0 prints the reference's diagnostics; the others run the same
        // deterministic estimate silently
        prep(0);
        if (rcs[0] == SID_EEMPTY) {
            std::fflush(stdout);
            std::fputs("sid: no profile with coverage >= 4 (the reference crashes here)\n", stderr);
            std::exit(139);
        }
        if (rcs[0] == SID_EBADFUNC) {
            std::fflush(stdout);
            std::fputs("gsl: nmsimplex2.c: ERROR: non-finite function value encountered\n"
                       "Default GSL error handler invoked.\n", stderr);
            std::abort();
        }
        CHECK(rcs[0], "estimate");
        std::vector<std::thread> th;
        for (int d = 1; d < D; ++d) th.emplace_back(prep, d);
        for (auto& x : th) x.join();
        for (int d = 1; d < D; ++d) CHECK(rcs[d], "estimate");
    }
    parallel([&](int d) {
        Shard& s = sh[d];
        (void)hipSetDevice(d % ndev);
        const size_t m = s.end - s.begin;
        if (method == SID_METHOD_LOCAL)
            CHECK(sid_call_local(s.ctx, s.d_counts, m, s.d_code, s.d_hom, s.d_het, s.stream), "local");
        else
            CHECK(sid_lookup_sites(s.ctx, s.d_counts, m, s.d_code, s.d_hom, s.d_het, s.stream), "lookup");
        HCHECK(hipStreamSynchronize(s.stream), "compute");
    });
    double t2 = now();

    // ----------------------------------------------------------------- emit --
    std::fputs(HEADER, stdout);
    std::fflush(stdout);
    {
        uint8_t* h_code = nullptr;
        double *h_hom = nullptr, *h_het = nullptr;
        const size_t nn = std::max<size_t>(n, 1);
        if (hipHostMalloc((void**)&h_code, nn, hipHostMallocDefault) != hipSuccess) h_code = (uint8_t*)std::malloc(nn);
        if (hipHostMalloc((void**)&h_hom, nn * 8, hipHostMallocDefault) != hipSuccess) h_hom = (double*)std::malloc(nn * 8);
        if (hipHostMalloc((void**)&h_het, nn * 8, hipHostMallocDefault) != hipSuccess) h_het = (double*)std::malloc(nn * 8);
        (void)hipGetLastError();   // a failed pinning above falls back to malloc: not an error
        parallel([&](int d) {
            Shard& s = sh[d];
            (void)hipSetDevice(d % ndev);
            const size_t m = s.end - s.begin;
            if (m) {
                HCHECK(hipMemcpyAsync(h_code + s.begin, s.d_code, m, hipMemcpyDeviceToHost, s.stream), "D2H");
                HCHECK(hipMemcpyAsync(h_hom + s.begin, s.d_hom, m * 8, hipMemcpyDeviceToHost, s.stream), "D2H");
                HCHECK(hipMemcpyAsync(h_het + s.begin, s.d_het, m * 8, hipMemcpyDeviceToHost, s.stream), "D2H");
            }
            HCHECK(hipStreamSynchronize(s.stream), "D2H");
        });
        const size_t BLOCK = 1u << 18;
        const size_t nblocks = (n + BLOCK - 1) / BLOCK;
        std::vector<std::vector<char>> bufs(nblocks);
        std::vector<size_t> lens(nblocks, 0);
        std::vector<std::atomic<int>> ready(nblocks);
        for (auto& r : ready) r.store(0);
        std::atomic<size_t> next{0};
        auto worker = [&] {
            for (;;) {
                size_t b = next.fetch_add(1);
                if (b >= nblocks) return;
                size_t lo = b * BLOCK, hi = std::min(n, lo + BLOCK);
                size_t need = 0;
                sid_format_csv(sites, lo, hi, h_code, h_hom, h_het, conf_type, nullptr, 0, &need);
                bufs[b].resize(need);
                size_t len = 0;
                int rc = sid_format_csv(sites, lo, hi, h_code, h_hom, h_het, conf_type, bufs[b].data(), need, &len);
                lens[b] = rc == SID_OK ? len : 0;
                ready[b].store(1, std::memory_order_release);
            }
        };
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back(worker);
        for (size_t b = 0; b < nblocks; ++b) {
            while (!ready[b].load(std::memory_order_acquire)) std::this_thread::yield();
            size_t off = 0;
            while (off < lens[b]) {
                ssize_t w = ::write(1, bufs[b].data() + off, lens[b] - off);
                if (w <= 0) break;
                off += (size_t)w;
            }
            std::vector<char>().swap(bufs[b]);
        }
        for (auto& x : th) x.join();
    }
    double t3 = now();
    if (opt.stats) {
        std::fprintf(stderr,
                     "{\"sites\": %zu, \"devices\": %d, \"threads\": %d, \"path\": \"%s\", \"parse_s\": %.6f, "
                     "\"device_s\": %.6f, \"emit_s\": %.6f, \"total_s\": %.6f, \"sites_per_s\": %.1f, "
                     "\"main_entry_unix\": %.6f, \"main_exit_unix\": %.6f}\n",
                     n, D, T, "host", t1 - t0, t2 - t1, t3 - t2, t3 - t0,
                     n / std::max(1e-9, t3 - t0), t_entry, unix_now());
    }
    // device memory, pinned staging and mappings go with the process: freeing
    // gigabytes of HBM and pinned host memory one by one only delays the exit
    finish(0);
}
