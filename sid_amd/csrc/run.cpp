// run.cpp — the streaming engine: one sid run, pileup text in, CSV out, over
// line-aligned chunks with bounded host memory (include/sid.h "streaming
// engine").
//
// It replaces the reference's whole-input flow -- readFile materialising
// every site (call.cpp:11-20), callX over the vector (call.cpp:62-289), the
// output loop (sid.cpp:102-105) -- by a pipeline per device:
//
//   uploader   source chunk -> device text buffer (ring of `slots`, or a
//              retained buffer); H2D on its own stream
//   compute    line index -> (sync: sites) -> parse -> call -> record lengths
//              -> (sync: bytes) -> records into a device CSV buffer
//   drain      CSV buffer -> pinned ring -> writer (D2H on its own stream)
//   writer     one for all devices: write() in chunk = file order
//
// Two passes keep the reference's all-or-nothing output (a malformed line
// aborts before anything is printed):
//   pass 1  every chunk is indexed and parsed (validation); -m local / quality
//           also call and format it, the records held in HBM (hold budget);
//           the Lynch methods accumulate the profile histogram instead.
//   (first error in file order -> return it, nothing written)
//   (Lynch: merge the device histograms, one estimate, class tables)
//   pass 2  header, then every chunk in file order: held records are copied
//           back as they are; the others are processed again from their text
//           (kept in HBM within the retain budget, else read again).
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "sid_internal.h"
#include "synth.h"

namespace {

constexpr uint64_t PAD = 256;   // readable bytes past every chunk's end (16-B windows, zeroed)

double wall()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// bounded blocking queue; close() wakes every waiter (push fails, pop drains)
template <class T>
class Chan {
public:
    bool push(T v)
    {
        std::unique_lock<std::mutex> l(m_);
        if (closed_) return false;
        q_.push_back(std::move(v));
        cv_.notify_one();
        return true;
    }
    bool pop(T& v)
    {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return !q_.empty() || closed_; });
        if (q_.empty()) return false;
        v = std::move(q_.front());
        q_.pop_front();
        return true;
    }
    // without waiting: false when nothing is queued right now
    bool try_pop(T& v)
    {
        std::lock_guard<std::mutex> l(m_);
        if (q_.empty()) return false;
        v = std::move(q_.front());
        q_.pop_front();
        return true;
    }
    void close()
    {
        std::lock_guard<std::mutex> l(m_);
        closed_ = true;
        cv_.notify_all();
    }
    void reset()
    {
        std::lock_guard<std::mutex> l(m_);
        q_.clear();
        closed_ = false;
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<T> q_;
    bool closed_ = false;
};

// Device buffers reused across chunks and runs (hipMalloc/hipFree are slow and
// hipFree waits for the device).  A buffer returned with an event is reused
// on another stream only after that event.
class DevPool {
public:
    int device = 0;
    ~DevPool() { release(); }
    // A fitting buffer whose last use is done is taken first; while every
    // fitting one is still in use (its event pending), up to two of them, a
    // new one is allocated rather than waited for -- the records' buffer of
    // a chunk is in use until its D2H completes, and the next chunk's writer
    // waiting for that copy serialised writer and D2H chunk after chunk (the
    // PCIe leg's last chunks then drained one D2H at a time after the last
    // upload)
    char* get(uint64_t need, uint64_t* cap, hipStream_t st)
    {
        std::lock_guard<std::mutex> l(m_);
        const uint64_t top = 2 * need + (64u << 20);
        const auto lo = free_.lower_bound(need);
        auto it = free_.end();
        int busy = 0;
        for (auto jt = lo; jt != free_.end() && jt->first <= top; ++jt) {
            if (!jt->second.ev || jt->second.st == st) {   // (returned on this stream: ordered, no wait)
                it = jt;
                break;
            }
            const hipError_t q = hipEventQuery(jt->second.ev);
            if (q == hipSuccess) {
                it = jt;
                break;
            }
            (void)hipGetLastError();   // (hipErrorNotReady: not an error of this thread's work)
            ++busy;
        }
        if (it == free_.end() && busy >= 2) it = lo;   // (growth bounded: wait for the first)
        if (it != free_.end()) {
            Entry en = it->second;
            *cap = it->first;
            free_.erase(it);
            if (en.ev) {
                (void)hipStreamWaitEvent(st, en.ev, 0);
                evs_.push_back(en.ev);
            }
            return en.p;
        }
        const uint64_t c = (need + PAD + (4u << 20) - 1) & ~(uint64_t)((4u << 20) - 1);
        char* p = nullptr;
        if (hipMalloc(&p, c) != hipSuccess) {
            // the caller falls back (ring slot, pass 2, arena): clear the
            // runtime's sticky last error, or the next launch check on this
            // thread (hipGetLastError) reports this failed allocation
            (void)hipGetLastError();
            return nullptr;
        }
        all_.push_back(p);
        bytes_ += c;
        *cap = c;
        return p;
    }
    // `after` (may be null): the buffer is free once the work before it on
    // its stream has run
    void put(char* p, uint64_t cap, hipStream_t after)
    {
        if (!p || !cap) return;   // cap 0: not a pooled buffer (the hold arena)
        std::lock_guard<std::mutex> l(m_);
        Entry en{p, nullptr, after};
        if (after) {
            if (evs_.empty()) {
                hipEvent_t ev;
                if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) evs_.push_back(ev);
            }
            if (!evs_.empty()) {
                en.ev = evs_.back();
                evs_.pop_back();
                (void)hipEventRecord(en.ev, after);
            }
        }
        free_.emplace(cap, en);
    }
    uint64_t bytes() const { return bytes_; }
    void release()
    {
        (void)hipSetDevice(device);
        for (char* p : all_) (void)hipFree(p);
        for (auto& kv : free_)
            if (kv.second.ev) (void)hipEventDestroy(kv.second.ev);
        for (hipEvent_t ev : evs_) (void)hipEventDestroy(ev);
        all_.clear();
        free_.clear();
        evs_.clear();
        bytes_ = 0;
    }

private:
    struct Entry {
        char* p;
        hipEvent_t ev;
        hipStream_t st;   // the stream the event was recorded on
    };
    std::mutex m_;
    std::multimap<uint64_t, Entry> free_;
    std::vector<char*> all_;
    std::vector<hipEvent_t> evs_;
    uint64_t bytes_ = 0;
};

struct ChunkRec {
    uint64_t off = 0, len = 0;       // input bytes (host / file / device text sources)
    uint64_t site0 = 0, nsites = 0;  // synthetic sources: sites [site0, site0 + nsites)
    int dev = 0;
    uint64_t parsed = 0;             // sites found by the index
    char* held = nullptr;            // CSV records formatted in pass 1 (device)
    uint64_t held_cap = 0, held_len = 0;
    char* kept = nullptr;            // text kept for pass 2 (device)
    uint64_t kept_cap = 0, kept_len = 0;
    char* pre = nullptr;             // Lynch paths: the pass-1 parse (line offsets, counts, formatter
    uint64_t pre_cap = 0;            // header pairs: n x 28 B) kept for pass 2, which skips index + parse
    uint64_t err = ~0ull;            // min(offset * 8 + kind) of the chunk's malformed lines
    const char* host = nullptr;      // its records in the host arena (host_hold_bytes), or null
    uint64_t host_len = 0;
    bool host1 = false;              // copied there during pass 1 (the emit only writes them)
    bool sunk = false;               // device sink: formatted in pass 1 and dropped (held_len bytes)
};

enum SrcKind { SRC_NONE, SRC_HOST, SRC_FILE, SRC_DEVICE, SRC_SYNTH_HOST, SRC_SYNTH_DEVICE };

struct Loaded {
    uint64_t j = 0;
    int kind = 0;            // 0 = text in a ring slot / kept buffer / device source, 1 = held records
    int slot = -1;           // ring slot, or -1
    const char* base = nullptr;
    uint64_t c0 = 0, c1 = 0;
    hipEvent_t ev = nullptr; // upload done (slot only)
};

struct OutItem {
    uint64_t j = 0;
    char* buf = nullptr;
    uint64_t cap = 0, len = 0;
    hipEvent_t ev = nullptr;  // records written (null: already complete)
    bool pooled = true;
};

struct Piece {
    uint64_t j = 0;
    int ps = -1;              // pinned slot, -1: no bytes
    uint64_t len = 0;
    bool last = false;
    char* buf = nullptr;      // the chunk's device CSV buffer, returned after the last piece
    uint64_t cap = 0;
    const char* host = nullptr;  // the whole chunk copied into the host arena instead (ps = -1)
    hipEvent_t hev = nullptr;    // that copy done
};

struct Slot {
    char* text = nullptr;
    uint64_t cap = 0;
    hipEvent_t ev_up = nullptr;    // upload done
    hipEvent_t ev_free = nullptr;  // last read of the text done
    bool used = false;
};

struct Dev {
    int index = 0, device = 0;
    // host placement (sid_engine_placement): the CPUs local to the GPU's PCI
    // device within the process's own, and its NUMA node
    cpu_set_t cpus;
    int ncpus = 0, first_cpu = -1, numa_node = -1;
    char pci[16] = {0};
    sid_ctx* ctx = nullptr;
    hipStream_t s_up = nullptr, s_comp = nullptr, s_d2h = nullptr;
    std::vector<Slot> slots;
    Chan<int> free_slots;
    Chan<Loaded> loaded;
    Chan<OutItem> drain_q;
    Chan<Piece> out_q;
    Chan<int> free_pinned;
    std::vector<char*> pinned;
    std::vector<hipEvent_t> pinned_ev;
    uint64_t pinned_cap = 0;
    sid_chunk_ws ws;
    uint64_t* h_small = nullptr;   // pinned, 16 words: [0] sites [4] error key [6..7] generator [8..11] formatter
    DevPool pool;
    // hold arena: the records formatted in pass 1, packed one after another
    // in segments of HBM kept across runs; a chunk reserves its upper bound
    // and commits its exact bytes
    std::vector<std::pair<char*, uint64_t>> arena;
    size_t arena_seg = 0;
    uint64_t arena_off = 0;
    // `left`: what the hold budget still allows (a new segment is not made
    // larger than that, nor than 4 GiB, nor smaller than `need`); null when
    // the HBM is not there (the caller formats the chunk in pass 2 instead)
    char* arena_reserve(uint64_t need, uint64_t left)
    {
        while (arena_seg < arena.size() && arena_off + need > arena[arena_seg].second) ++arena_seg, arena_off = 0;
        if (arena_seg == arena.size()) {
            const uint64_t want = std::min<uint64_t>(4ull << 30, std::max(need, left));
            const uint64_t c = (std::max(need, want) + (2u << 20) - 1) & ~(uint64_t)((2u << 20) - 1);
            char* p = nullptr;
            if (hipMalloc(&p, c) != hipSuccess) {
                (void)hipGetLastError();   // not an error: the chunk is formatted in pass 2 (see DevPool::get)
                return nullptr;
            }
            arena.push_back({p, c});
            arena_off = 0;
        }
        return arena[arena_seg].first + arena_off;
    }
    void arena_commit(uint64_t bytes) { arena_off += (bytes + 255) & ~(uint64_t)255; }
    uint64_t arena_bytes() const
    {
        uint64_t b = 0;
        for (auto& a : arena) b += a.second;
        return b;
    }
    // host arena (sid_engine_cfg.host_hold_bytes): pinned host memory, made
    // once and reused by every run, that receives the records D2H -- in pass
    // 1 while later chunks upload (full duplex), in pass 2 instead of the
    // pinned ring; bump-allocated, reset by every ingest
    char* hh = nullptr;
    uint64_t hh_cap = 0, hh_off = 0;
    bool hh_full = false;
    bool hh_alloc(uint64_t bytes)
    {
        if (hipHostMalloc((void**)&hh, bytes, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            hh = nullptr;
            return false;
        }
        hh_cap = bytes;
        return true;
    }
    void hh_free()
    {
        if (hh) (void)hipHostFree(hh);
        hh = nullptr;
        hh_cap = 0;
    }
    char* hh_take(uint64_t bytes)
    {
        if (!hh || hh_off + bytes > hh_cap) return nullptr;
        char* p = hh + hh_off;
        hh_off += (bytes + 255) & ~(uint64_t)255;
        return p;
    }
    // the tile parse (sid_chunk_tile_local): its slots per tile for the next
    // chunk (tile_next / tile_over), its shape (a quad of lanes per line for
    // lines over 256 B on average), and whether it takes the lines at all (at
    // most SID_TILE_CAP_MAX a tile)
    uint32_t tile_cap = 288;
    bool tile_quad = false;
    bool tile_ok = true;
    // slots per tile for at most `lines` lines a tile: multiples of 16, up to
    // the shape's list (a quad tile of lines too short for its list: the lane
    // shape instead)
    uint64_t tile_hi = 0;   // the lines a tile should have room for (a decaying maximum over chunks)
    void tile_set(uint64_t lines, bool quad)
    {
        if (quad && lines > SID_TILE_CAP_MAX_QUAD) {
            quad = false;
            lines = lines * sid_tile_unit(false) / sid_tile_unit(true) + 1;
        }
        tile_quad = quad;
        tile_hi = lines;
        tile_cap = (uint32_t)std::min<uint64_t>(quad ? SID_TILE_CAP_MAX_QUAD : SID_TILE_CAP_MAX,
                                                std::max<uint64_t>(SID_TILE_CAP_MIN, (lines + 15) & ~15ull));
    }
    // after a tiled chunk of n sites over `bytes` of text whose tiles had at
    // most maxl lines: the next chunk's shape (a quad of lanes per line over
    // 256 B a line) and slots (the same shape: maxl, a thirty-second and 2 on
    // top, or the room recent chunks needed, less a sixty-fourth a chunk --
    // chunks whose fullest tiles alternate would otherwise overflow every
    // other chunk; a new shape: from this chunk's lines per byte, a quarter on
    // top)
    void tile_next(uint64_t maxl, uint64_t n, uint64_t bytes, bool quad)
    {
        const bool q2 = bytes > 256 * n;
        if (q2 == quad)
            tile_set(std::max<uint64_t>(maxl + maxl / 32 + 2, tile_hi - tile_hi / 64), q2);
        else
            tile_set((uint64_t)((double)n * sid_tile_unit(q2) / (double)std::max<uint64_t>(1, bytes) * 1.25) + 1, q2);
    }
    // a tile had more lines than slots (the chunk goes the two-pass way); the
    // tile parse stays off while no shape has room for them: judged in the
    // units of the shape tile_set chose (a quad tile's lines counted in lane
    // tiles when it switched to the lane shape)
    void tile_over(uint64_t maxl, bool quad)
    {
        tile_set(maxl + maxl / 32 + 2, quad);
        const uint64_t need = quad && !tile_quad ? maxl * sid_tile_unit(false) / sid_tile_unit(true) + 1 : maxl;
        tile_ok = need <= (tile_quad ? SID_TILE_CAP_MAX_QUAD : SID_TILE_CAP_MAX);
    }
    // the tile parse off (a run of tiny lines): after a two-pass chunk of n
    // sites over `bytes` whose lines per byte leave a lane tile half its
    // largest list, on again with that chunk's density (a quarter on top);
    // a tile of tiny lines in it overflows and turns it off again
    void tile_retry(uint64_t n, uint64_t bytes)
    {
        const uint64_t per = (uint64_t)((double)n * sid_tile_unit(false) / (double)std::max<uint64_t>(1, bytes) * 1.25) + 1;
        if (tile_ok || 2 * per > SID_TILE_CAP_MAX) return;
        tile_hi = 0;
        tile_set(per, false);
        tile_ok = true;
    }
    // a new run: a device the last run left with the tile parse off starts
    // from the defaults (a run that kept it on keeps its shape and slots, the
    // next run's likely fit)
    void tile_reset()
    {
        if (tile_ok) return;
        tile_cap = 288;
        tile_quad = false;
        tile_hi = 0;
        tile_ok = true;
    }
    uint64_t hold_budget = 0, retain_budget = 0;
    std::atomic<uint64_t> hold_used{0}, retain_used{0};
    std::atomic<bool> hold_full{false};
    // the ingest's host-to-device copies, timed on the upload stream (pairs
    // of timing events, summed after the ingest's sync)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> h2d_pending;
    std::vector<hipEvent_t> h2d_free;
    uint64_t h2d_bytes = 0;
    uint64_t tiled = 0, tile_overflows = 0, tile_over_queued = 0;   // this run's chunks (the device's compute thread)
    hipEvent_t h2d_event()
    {
        hipEvent_t ev = nullptr;
        if (!h2d_free.empty()) {
            ev = h2d_free.back();
            h2d_free.pop_back();
        } else if (hipEventCreate(&ev) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return ev;
    }
    // device time of the uploads timed since the last call (the stream
    // drained): each uploader's span, first copy's start to last copy's end
    double h2d_collect()
    {
        double s = 0;
        for (auto& pr : h2d_pending) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) s += ms * 1e-3;
            h2d_free.push_back(pr.first);
            h2d_free.push_back(pr.second);
        }
        (void)hipGetLastError();
        h2d_pending.clear();
        return s;
    }
    std::mutex ev_m;
    std::vector<hipEvent_t> ev_cache;   // events marking a chunk's records written (compute -> drain)
    // sid_engine_profile: (stage, start, end) per stage and chunk, read after a sync
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> prof_pending;
    std::vector<hipEvent_t> prof_free;
    uint64_t prof_chunks = 0;
    hipEvent_t prof_begin(bool on)
    {
        if (!on) return nullptr;
        hipEvent_t ev = nullptr;
        if (!prof_free.empty()) {
            ev = prof_free.back();
            prof_free.pop_back();
        } else if (hipEventCreate(&ev) != hipSuccess) {
            return nullptr;
        }
        (void)hipEventRecord(ev, s_comp);
        return ev;
    }
    void prof_end(int stage, hipEvent_t start)
    {
        if (!start) return;
        hipEvent_t ev = prof_begin(true);
        if (ev) prof_pending.push_back({stage, {start, ev}});
    }
    hipEvent_t take_event()
    {
        std::lock_guard<std::mutex> l(ev_m);
        hipEvent_t ev = nullptr;
        if (!ev_cache.empty()) {
            ev = ev_cache.back();
            ev_cache.pop_back();
        } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            ev = nullptr;
        }
        return ev;
    }
    void give_event(hipEvent_t ev)
    {
        std::lock_guard<std::mutex> l(ev_m);
        ev_cache.push_back(ev);
    }
};

// The CPUs of a sysfs cpulist ("0-15,128-143") within `allowed`
int parse_cpulist(const char* txt, const cpu_set_t& allowed, cpu_set_t* out, int* first)
{
    CPU_ZERO(out);
    int n = 0;
    *first = -1;
    const char* p = txt;
    while (*p) {
        char* q = nullptr;
        const long lo = std::strtol(p, &q, 10);
        if (q == p) break;
        long hi = lo;
        p = q;
        if (*p == '-') {
            hi = std::strtol(p + 1, &q, 10);
            p = q;
        }
        for (long c = lo; c <= hi && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET(c, &allowed) && !CPU_ISSET(c, out)) {
                CPU_SET(c, out);
                if (*first < 0 || c < *first) *first = (int)c;
                ++n;
            }
        while (*p == ',' || *p == '\n' || *p == ' ') ++p;
    }
    return n;
}

// d's GPU: its PCI bus id, NUMA node and local CPUs (sysfs), kept for
// binding when they are a proper subset of the process's CPUs
void find_placement(Dev& d)
{
    CPU_ZERO(&d.cpus);
    if (hipDeviceGetPCIBusId(d.pci, sizeof d.pci, d.device) != hipSuccess) {
        (void)hipGetLastError();
        d.pci[0] = 0;
        return;
    }
    for (char* c = d.pci; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    char path[128], buf[4096];
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", d.pci);
    if (FILE* f = std::fopen(path, "r")) {
        if (std::fscanf(f, "%d", &d.numa_node) != 1) d.numa_node = -1;
        std::fclose(f);
    }
    std::snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/local_cpulist", d.pci);
    FILE* f = std::fopen(path, "r");
    if (!f) return;
    const size_t m = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[m] = 0;
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return;
    cpu_set_t mine;
    int first = -1;
    const int n = parse_cpulist(buf, allowed, &mine, &first);
    if (n == 0 || n == CPU_COUNT(&allowed)) return;   // nothing to choose
    d.cpus = mine;
    d.ncpus = n;
    d.first_cpu = first;
}

// the calling thread onto d's CPUs (no-op when not bound)
void bind_thread(const Dev& d)
{
    if (d.ncpus > 0) (void)pthread_setaffinity_np(pthread_self(), sizeof d.cpus, &d.cpus);
}

// NUMA node of the page holding p (-1: unknown)
int page_node(const void* p)
{
    if (!p) return -1;
    int node = -1;
    // get_mempolicy(&node, NULL, 0, p, MPOL_F_NODE | MPOL_F_ADDR)
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0ul, p, 1ul | 2ul) != 0) return -1;
    return node;
}

// f() on a thread bound to d's CPUs (pinned host buffers then come from the
// GPU's NUMA node: the pages are allocated by the thread that pins them)
template <class F>
void on_node(const Dev& d, F f)
{
    if (d.ncpus == 0) return f();
    std::thread t([&] {
        bind_thread(d);
        f();
    });
    t.join();
}

// The engine's run threads, kept across runs (spawning a run's uploader and
// compute threads took 0.08-0.15 ms of every run, the device idle behind
// them): run() gives each task of a batch a thread of its own (uploader and
// compute wait on each other through the queues) and returns when all are
// done.  A task starts with the affinity its thread was created with (the
// caller's), as a thread spawned for it would.
class Crew {
  public:
    Crew() = default;
    Crew(const Crew&) = delete;
    Crew& operator=(const Crew&) = delete;
    ~Crew()
    {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // the batch started (one batch at a time); wait() returns when it is done
    void start(std::vector<std::function<void()>>& fs)
    {
        std::lock_guard<std::mutex> l(m_);
        if (tasks_.size() < fs.size()) tasks_.resize(fs.size());
        while (th_.size() < fs.size()) {
            const size_t k = th_.size();
            th_.emplace_back([this, k] { loop(k); });
        }
        for (size_t k = 0; k < fs.size(); ++k) tasks_[k] = std::move(fs[k]);
        pending_ = fs.size();
        cv_.notify_all();
    }
    void wait()
    {
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return pending_ == 0; });
    }
    void run(std::vector<std::function<void()>>& fs)
    {
        start(fs);
        wait();
    }

  private:
    void loop(size_t k)
    {
        cpu_set_t base;
        const bool aff = pthread_getaffinity_np(pthread_self(), sizeof base, &base) == 0;
        std::unique_lock<std::mutex> l(m_);
        for (;;) {
            cv_.wait(l, [&] { return stop_ || tasks_[k] != nullptr; });
            if (stop_) return;
            std::function<void()> f = std::move(tasks_[k]);
            tasks_[k] = nullptr;
            l.unlock();
            if (aff) (void)pthread_setaffinity_np(pthread_self(), sizeof base, &base);
            f();
            l.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    std::vector<std::function<void()>> tasks_;   // (resized under m_ only, before a worker can see its slot)
    size_t pending_ = 0;
    bool stop_ = false;
};

}  // namespace

struct sid_engine {
    sid_opts opts{};
    sid_engine_cfg cfg{};
    std::vector<std::unique_ptr<Dev>> devs;
    // source
    int src = SRC_NONE;
    const char* text = nullptr;     // SRC_HOST / SRC_FILE (mapping) / SRC_DEVICE
    uint64_t text_len = 0;
    bool reg_upload = false;        // SRC_HOST / SRC_FILE pageable: chunks registered for DMA (upload_register)
    void* map = nullptr;
    uint64_t map_len = 0, map_skew = 0;
    uint64_t synth_seed = 0, synth_first = 0, synth_n = 0, synth_spc = 0, synth_per = 0;
    double synth_depth = 30.0;
    std::vector<uint64_t> synth_cdf;
    uint64_t* d_cdf = nullptr;       // on the first device (SRC_SYNTH_DEVICE)
    std::vector<uint64_t*> d_cdf_dev;
    std::vector<sid_synth_gen_ws> gen_ws;
    std::vector<ChunkRec> recs;
    // run state
    bool lynch = false, quality = false, ingested = false, estimated = false;
    bool hist_merged = false;        // the pipelines' Lynch histograms hold the merged table
    const char* conf_type = "p_value";
    std::atomic<int> rc{SID_OK};
    std::atomic<uint64_t> first_err{UINT64_MAX};
    std::atomic<uint64_t> reloaded{0};
    std::atomic<uint64_t> sink_bytes{0};   // device sink: CSV bytes formatted and dropped
    // SID_ENGINE_TIMING: host time (ns) spent in compute-stream syncs and in
    // the writer's waits for D2H pieces, printed per phase
    std::atomic<uint64_t> t_comp_sync{0}, t_write_wait{0};
    std::atomic<uint64_t> reg_chunks{0};   // chunks uploaded from registered pages (upload_register)
    std::atomic<uint64_t> t_register{0};   // ns in hipHostRegister / hipHostUnregister (the uploaders)
    // host-generated input: pinned buffers
    std::vector<char*> gen_buf;
    std::vector<uint64_t> gen_cap;
    std::vector<hipEvent_t> gen_ev;   // H2D of the buffer done (recorded by the uploader)
    std::vector<int> gen_dev;         // device whose stream recorded gen_ev
    uint64_t per_chunk_cap = 0;
    sid_estimate est{};
    bool prof = false;
    double prof_ms[6] = {0, 0, 0, 0, 0, 0};   // sid_engine_prof order: index parse call hist fmt_len fmt_write
    uint64_t prof_chunks = 0;
    Crew crew;   // (last: its threads joined first when the engine is deleted)
};

namespace {

void close_all(sid_engine* e)
{
    for (auto& d : e->devs) {
        d->free_slots.close();
        d->loaded.close();
        d->drain_q.close();
        d->out_q.close();
        d->free_pinned.close();
    }
}

// the first failure wins; every queue closes so no thread waits on a peer
// that has stopped
void fail(sid_engine* e, int rc)
{
    int ok = SID_OK;
    e->rc.compare_exchange_strong(ok, rc);
    close_all(e);
}

int hipfail(sid_engine* e, hipError_t x)
{
    if (x == hipSuccess) return SID_OK;
    const int rc = sid_set_hip_error(x);
    fail(e, rc);
    return rc;
}

// default chunk sizes: input that crosses PCIe in 128 MiB pieces (the pipeline
// fills and drains in a few ms); text already in HBM, or generated there, in
// larger ones (every chunk costs a few fixed launches and two host round
// trips; the workspace is a few hundred MB per GiB of text)
const uint64_t CHUNK_HOST = 128ull << 20;
const uint64_t CHUNK_DEVICE = 4000ull << 20;   // C2 2.95-2.97 vs 2.97-2.99 ms with 2 GiB, C5 13.7 vs 14.2 ms (round 5)
const uint64_t CHUNK_SYNTH = 512ull << 20;

uint64_t chunk_bytes(const sid_engine* e)
{
    // (32-bit line offsets: a chunk spans less than 4 GiB, sid_off_t)
    if (e->cfg.chunk_bytes) return std::min<uint64_t>(e->cfg.chunk_bytes, SID_CHUNK_MAX - (64ull << 20));
    return e->src == SRC_DEVICE ? CHUNK_DEVICE : e->src == SRC_SYNTH_DEVICE ? CHUNK_SYNTH : CHUNK_HOST;
}

// first line start at or after c (one past the next '\n')
uint64_t next_line_start(const char* t, uint64_t len, uint64_t c)
{
    if (c == 0 || c >= len) return std::min(c, len);
    const char* nl = (const char*)std::memchr(t + c - 1, '\n', len - c + 1);
    return nl ? (uint64_t)(nl - t) + 1 : len;
}

void split_host_text(sid_engine* e, const char* t, uint64_t len)
{
    const uint64_t C = chunk_bytes(e);
    e->recs.clear();
    uint64_t at = 0;
    while (at < len) {
        // the last chunks' work (compute, then their records' copies back)
        // runs after the last upload: the last two chunks' worth of text is
        // cut in halves down to 8-16 MiB, so each chunk's D2H (~0.6 of its
        // upload's time) runs under the uploads still to come, and what is
        // left after the last upload is one small chunk's
        const uint64_t rem = len - at;
        const uint64_t want = rem <= 2 * C && rem > (16ull << 20) ? std::min(C, rem / 2) : C;
        uint64_t end = next_line_start(t, len, std::max(at + 1, std::min(len, at + want)));
        if (end <= at) end = len;
        ChunkRec r;
        r.off = at;
        r.len = end - at;
        e->recs.push_back(r);
        at = end;
    }
}

// ------------------------------------------------------------- generator --
// the synthetic text of sites [first, first + n) into dst (cap bytes); the
// same bytes as sid_synth_text (capi.cpp), without intermediate strings.
// Returns the length, or UINT64_MAX when it does not fit.
uint64_t synth_host(const std::vector<uint64_t>& cdf, uint64_t seed, uint64_t first, uint64_t n, uint64_t spc,
                    char* dst, uint64_t cap)
{
    static const char UP[] = "ACGT", LO[] = "acgt";
    const uint32_t k = (uint32_t)cdf.size();
    char* o = dst;
    char* const end = dst + cap;
    auto put_u = [&](uint64_t v) {
        char tmp[24];
        int m = 0;
        do {
            tmp[m++] = (char)('0' + v % 10);
            v /= 10;
        } while (v);
        while (m) *o++ = tmp[--m];
    };
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t site = first + i;
        const uint64_t chrom = spc ? site / spc + 1 : 1;
        const uint64_t pos = spc ? site % spc + 1 : site + 1;
        sid_synth_site s = sid_synth_site_header(seed, site, cdf.data(), k);
        // worst case of this line: names and numbers (64) + 4 bytes per read
        if ((uint64_t)(end - o) < 64 + 5ull * s.depth) return UINT64_MAX;
        *o++ = 'c';
        *o++ = 'h';
        *o++ = 'r';
        put_u(chrom);
        *o++ = '\t';
        put_u(pos);
        *o++ = '\t';
        *o++ = UP[s.ref];
        *o++ = '\t';
        put_u(s.depth);
        *o++ = '\t';
        if (s.depth == 0) {
            *o++ = '*';
            *o++ = '\t';
            *o++ = '*';
            *o++ = '\n';
            continue;
        }
        char* q = o + 4 * s.depth;   // qualities after the bases: written in one walk
        char* qs = q;
        for (uint32_t r = 0; r < s.depth; ++r) {
            uint32_t strand;
            const uint32_t b = sid_synth_read_base(&s, r, &strand);
            int st, en;
            uint32_t ql;
            sid_synth_read_marks(&s, r, &st, &en, &ql);
            if (st) {
                *o++ = '^';
                *o++ = ']';
            }
            *o++ = b == s.ref ? (strand ? '.' : ',') : (strand ? UP[b] : LO[b]);
            if (en) *o++ = '$';
            *q++ = (char)('!' + ql);
        }
        *o++ = '\t';
        std::memmove(o, qs, s.depth);
        o += s.depth;
        *o++ = '\n';
    }
    return (uint64_t)(o - dst);
}

}  // namespace

// ================================================================= C ABI ==
extern "C" void sid_engine_cfg_default(sid_engine_cfg* c)
{
    if (!c) return;
    std::memset(c, 0, sizeof *c);
}

extern "C" int sid_engine_create(const sid_opts* opts, const sid_engine_cfg* cfg, sid_engine** out)
{
    if (!out) return SID_EINVAL;
    *out = nullptr;
    int nvis = 0;
    if (hipGetDeviceCount(&nvis) != hipSuccess || nvis <= 0) return SID_EHIP;
    sid_engine* e = new sid_engine();
    if (opts) e->opts = *opts; else sid_opts_default(&e->opts);
    if (cfg) e->cfg = *cfg; else sid_engine_cfg_default(&e->cfg);
    const int G = e->cfg.devices > 0 ? e->cfg.devices : nvis;
    const int lanes = std::max(1, e->cfg.lanes);
    const int D = G * lanes;   // pipelines
    const int R = e->cfg.slots > 0 ? e->cfg.slots : 3;
    for (int i = 0; i < D; ++i) {
        auto d = std::make_unique<Dev>();
        d->index = i;
        d->device = (e->cfg.first_device + i / lanes) % nvis;
        d->pool.device = d->device;
        e->devs.push_back(std::move(d));
    }
    // every pipeline's context (class tables, the first kernel launches on
    // its GPU), streams and events: one thread per GPU, its pipelines in
    // order -- the GPUs' start-up costs (tens of ms each) overlap instead of
    // adding up on a whole node
    std::vector<int> rcs(D, SID_OK);
    // (the streams -- a hardware queue each, ~8 ms apiece -- are created on a
    // second thread while sid_create builds the class tables)
    auto make = [&](int i) {
        Dev* d = e->devs[i].get();
        find_placement(*d);
        bind_thread(*d);   // (this GPU's start-up thread: its host allocations local to it)
        hipError_t x = hipSuccess;
        std::thread qs([&] {
            bind_thread(*d);
            x = hipSetDevice(d->device);
            if (x == hipSuccess) x = hipStreamCreateWithFlags(&d->s_up, hipStreamNonBlocking);
            if (x == hipSuccess) x = hipStreamCreateWithFlags(&d->s_comp, hipStreamNonBlocking);
            if (x == hipSuccess) x = hipStreamCreateWithFlags(&d->s_d2h, hipStreamNonBlocking);
            if (x == hipSuccess) x = hipHostMalloc((void**)&d->h_small, 128, hipHostMallocDefault);
            d->slots.resize(R);
            for (auto& s : d->slots) {
                if (x == hipSuccess) x = hipEventCreateWithFlags(&s.ev_up, hipEventDisableTiming);
                if (x == hipSuccess) x = hipEventCreateWithFlags(&s.ev_free, hipEventDisableTiming);
            }
        });
        int rc = sid_create(d->device, &e->opts, &d->ctx);
        qs.join();
        if (rc == SID_OK && x != hipSuccess) rc = sid_set_hip_error(x);
        rcs[i] = rc;
    };
    auto per_gpu = [&](int g) {
        for (int i = g * lanes; i < std::min(D, (g + 1) * lanes); ++i) make(i);
    };
    {   // (each on a thread of its own: make() binds its thread to the GPU's CPUs)
        std::vector<std::thread> th;
        for (int g = 0; g < G; ++g) th.emplace_back(per_gpu, g);
        for (auto& t : th) t.join();
    }
    (void)hipSetDevice(e->devs[0]->device);
    for (int rc : rcs)
        if (rc != SID_OK) {
            sid_engine_destroy(e);
            return rc;
        }
    *out = e;
    return SID_OK;
}

static void drop_source(sid_engine* e)
{
    if (e->map) munmap(e->map, e->map_len);
    e->map = nullptr;
    for (auto& r : e->recs) {
        Dev& d = *e->devs[r.dev];
        if (r.held) d.pool.put(r.held, r.held_cap, nullptr);
        if (r.kept) d.pool.put(r.kept, r.kept_cap, nullptr);
        if (r.pre) d.pool.put(r.pre, r.pre_cap, nullptr);
        r.held = r.kept = r.pre = nullptr;
    }
    e->recs.clear();
    e->src = SRC_NONE;
    e->text = nullptr;
    e->text_len = 0;
    e->ingested = e->estimated = false;
}

extern "C" int sid_engine_destroy(sid_engine* e)
{
    if (!e) return SID_OK;
    for (auto& d : e->devs) (void)hipSetDevice(d->device), (void)hipDeviceSynchronize();
    drop_source(e);
    for (auto& d : e->devs) {
        (void)hipSetDevice(d->device);
        for (auto& s : d->slots) {
            if (s.text) (void)hipFree(s.text);
            if (s.ev_up) (void)hipEventDestroy(s.ev_up);
            if (s.ev_free) (void)hipEventDestroy(s.ev_free);
        }
        for (char* p : d->pinned) (void)hipHostFree(p);
        d->hh_free();
        for (hipEvent_t ev : d->pinned_ev) (void)hipEventDestroy(ev);
        for (hipEvent_t ev : d->ev_cache) (void)hipEventDestroy(ev);
        for (auto& pr : d->prof_pending) (void)hipEventDestroy(pr.second.first), (void)hipEventDestroy(pr.second.second);
        for (hipEvent_t ev : d->prof_free) (void)hipEventDestroy(ev);
        for (auto& pr : d->h2d_pending) (void)hipEventDestroy(pr.first), (void)hipEventDestroy(pr.second);
        for (hipEvent_t ev : d->h2d_free) (void)hipEventDestroy(ev);
        sid_chunk_release(&d->ws);
        if (d->h_small) (void)hipHostFree(d->h_small);
        for (hipStream_t s : {d->s_up, d->s_comp, d->s_d2h})
            if (s) (void)hipStreamDestroy(s);
        d->pool.release();
        for (auto& a : d->arena) (void)hipFree(a.first);
        sid_destroy(d->ctx);
    }
    for (size_t i = 0; i < e->d_cdf_dev.size(); ++i)
        if (e->d_cdf_dev[i]) (void)hipSetDevice(e->devs[i]->device), (void)hipFree(e->d_cdf_dev[i]);
    for (size_t i = 0; i < e->gen_ws.size(); ++i) {
        (void)hipSetDevice(e->devs[i]->device);
        sid_synth_gen_release(&e->gen_ws[i]);
    }
    for (char* p : e->gen_buf) (void)hipHostFree(p);
    for (hipEvent_t ev : e->gen_ev)
        if (ev) (void)hipEventDestroy(ev);
    delete e;
    return SID_OK;
}

extern "C" int sid_engine_devices(const sid_engine* e) { return e ? (int)e->devs.size() : 0; }

extern "C" sid_ctx* sid_engine_context(sid_engine* e, int i)
{
    if (!e || i < 0 || i >= (int)e->devs.size()) return nullptr;
    return e->devs[i]->ctx;
}

extern "C" int sid_engine_placement(const sid_engine* e, int i, sid_placement* out)
{
    if (!e || !out || i < 0 || i >= (int)e->devs.size()) return SID_EINVAL;
    const Dev& d = *e->devs[i];
    std::memset(out, 0, sizeof *out);
    out->device = d.device;
    out->gpu_numa_node = d.numa_node;
    out->cpus = d.ncpus;
    out->first_cpu = d.first_cpu;
    out->arena_numa_node = page_node(d.hh);
    out->ring_numa_node = d.pinned.empty() ? -1 : page_node(d.pinned[0]);
    std::memcpy(out->pci, d.pci, sizeof out->pci);
    out->pci[sizeof out->pci - 1] = 0;
    return SID_OK;
}

static void assign_devices(sid_engine* e)
{
    const int D = (int)e->devs.size();
    for (size_t j = 0; j < e->recs.size(); ++j) e->recs[j].dev = (int)(j % D);
}

// Pageable host text (a file's mapping, or host memory the caller did not
// pin) is uploaded chunk by chunk from registered pages: each chunk's page-
// aligned body is pinned (hipHostRegister, read-only) by the uploader while
// the previous chunk's DMA runs, copied straight from the page cache, and
// released once its copy is done; the partial pages at its ends (shared with
// the neighbouring chunks) take the runtime's pageable path.  Without it the
// runtime copies every byte through its own pinned staging buffers first
// (a CPU copy per byte: at a whole node's N uploads, host memory traffic).
// SID_UPLOAD_REGISTER=0: the pageable path for everything (A/B).
static bool upload_register()
{
    static const bool on = [] {
        const char* v = std::getenv("SID_UPLOAD_REGISTER");
        return !v || std::atoi(v) != 0;
    }();
    return on;
}

// host memory the runtime already maps for the device (pinned or registered)
static bool host_pinned(const char* p)
{
    hipPointerAttribute_t a;
    const bool pinned = hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost;
    (void)hipGetLastError();   // (pageable memory: an error to clear, not to report)
    return pinned;
}

extern "C" int sid_engine_source_text(sid_engine* e, const char* text, uint64_t len)
{
    if (!e || (!text && len)) return SID_EINVAL;
    drop_source(e);
    e->src = SRC_HOST;
    e->text = text;
    e->text_len = len;
    e->reg_upload = upload_register() && len && !host_pinned(text);
    split_host_text(e, text, len);
    assign_devices(e);
    return SID_OK;
}

extern "C" int sid_engine_source_file(sid_engine* e, int fd, uint64_t offset, uint64_t len)
{
    if (!e || fd < 0) return SID_EINVAL;
    struct stat sb;
    // a range past the end of the file would fault (SIGBUS) on the first read
    if (fstat(fd, &sb) != 0) return SID_EIO;
    if (S_ISREG(sb.st_mode) && (offset > (uint64_t)sb.st_size || len > (uint64_t)sb.st_size - offset))
        return SID_EINVAL;
    drop_source(e);
    if (len == 0) {
        e->src = SRC_HOST;
        return SID_OK;
    }
    const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
    const uint64_t a = offset & ~(pg - 1);
    e->map_skew = offset - a;
    e->map_len = len + e->map_skew;
    // populated up front below 8 GiB (one kernel pass over the page tables was
    // measured fastest); larger inputs are populated chunk by chunk
    // ahead of the uploads and released behind them
    const bool populate = len <= (8ull << 30);
    void* m = mmap(nullptr, e->map_len, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, (off_t)a);
    if (m == MAP_FAILED) return SID_EIO;
    (void)madvise(m, e->map_len, MADV_SEQUENTIAL);
    e->map = m;
    e->src = SRC_FILE;
    e->text = (const char*)m + e->map_skew;
    e->text_len = len;
    e->reg_upload = upload_register();
    split_host_text(e, e->text, len);
    assign_devices(e);
    return SID_OK;
}

extern "C" int sid_engine_source_device_text(sid_engine* e, const char* d_text, uint64_t len)
{
    if (!e || (!d_text && len)) return SID_EINVAL;
    drop_source(e);
    e->src = SRC_DEVICE;
    e->text = d_text;
    e->text_len = len;
    // line-aligned cuts: a window around each nominal cut is read back
    Dev& d0 = *e->devs[0];
    if (hipSetDevice(d0.device) != hipSuccess) return SID_EHIP;
    const uint64_t C = chunk_bytes(e);
    std::vector<char> w(1 << 16);
    uint64_t at = 0;
    while (at < len) {
        uint64_t c = std::min(len, at + C);
        while (c < len) {   // the next '\n' at or after c - 1
            const uint64_t m = std::min<uint64_t>(w.size(), len - (c - 1));
            if (hipMemcpy(w.data(), d_text + c - 1, m, hipMemcpyDeviceToHost) != hipSuccess) return SID_EHIP;
            const char* nl = (const char*)std::memchr(w.data(), '\n', m);
            if (nl) {
                c = c - 1 + (uint64_t)(nl - w.data()) + 1;
                break;
            }
            c += m;
        }
        c = std::min(c, len);
        ChunkRec r;
        r.off = at;
        r.len = c - at;
        e->recs.push_back(r);
        at = c;
    }
    // the text lives on the first GPU: its pipelines take the chunks in turn
    const int lanes = std::max(1, e->cfg.lanes);
    for (size_t j = 0; j < e->recs.size(); ++j) e->recs[j].dev = (int)(j % std::min<size_t>(lanes, e->devs.size()));
    return SID_OK;
}

extern "C" int sid_engine_source_synth(sid_engine* e, uint64_t seed, double mean_depth, uint64_t first_site,
                                       uint64_t n, uint64_t sites_per_chrom, uint64_t sites_per_chunk, int on_device)
{
    if (!e || !(mean_depth >= 0) || mean_depth > 600) return SID_EINVAL;
    drop_source(e);
    e->src = on_device ? SRC_SYNTH_DEVICE : SRC_SYNTH_HOST;
    e->synth_seed = seed;
    e->synth_depth = mean_depth;
    e->synth_first = first_site;
    e->synth_n = n;
    e->synth_spc = sites_per_chrom;
    sid_poisson_cdf(mean_depth, e->synth_cdf);
    // about 2.7 B per read (base, quality, marks) + 20 B of fields per site
    const double per_site = 20.0 + 2.75 * mean_depth;
    uint64_t per = sites_per_chunk ? sites_per_chunk : (uint64_t)(chunk_bytes(e) / per_site);
    per = std::max<uint64_t>(per, 1);
    e->synth_per = per;
    // capacity: the mean plus a wide margin (the generator reports overflow)
    e->per_chunk_cap = (uint64_t)(per * per_site * 1.25) + (64ull + 5ull * e->synth_cdf.size()) + (1u << 20);
    for (uint64_t s = 0; s < n; s += per) {
        ChunkRec r;
        r.site0 = first_site + s;
        r.nsites = std::min(per, n - s);
        e->recs.push_back(r);
    }
    assign_devices(e);
    if (on_device) {
        const size_t D = e->devs.size();
        e->d_cdf_dev.resize(D, nullptr);
        e->gen_ws.resize(D);
        for (size_t i = 0; i < D; ++i) {
            if (hipSetDevice(e->devs[i]->device) != hipSuccess) return SID_EHIP;
            if (e->d_cdf_dev[i]) (void)hipFree(e->d_cdf_dev[i]);
            e->d_cdf_dev[i] = nullptr;
            if (hipMalloc(&e->d_cdf_dev[i], e->synth_cdf.size() * 8) != hipSuccess ||
                hipMemcpy(e->d_cdf_dev[i], e->synth_cdf.data(), e->synth_cdf.size() * 8, hipMemcpyHostToDevice) !=
                    hipSuccess)
                return SID_EHIP;
        }
    }
    return SID_OK;
}

// --------------------------------------------------------------- threads --
namespace {

bool needs_format_pass1(const sid_engine* e) { return !e->lynch; }

// The device sink (cfg.device_sink 1: records formatted into HBM and dropped)
// formats every -m local / quality chunk in pass 1 into a pooled scratch
// buffer whose bytes are counted and dropped at once (no hold arena, whose
// HBM a 2 GiB chunk's record bound then lacked beside C4's 244 GB of
// resident text: SID_ENOMEM, profiles/bench_c4_2gib_chunks_r04.err).  Nothing is written
// anywhere, so the all-or-nothing output that makes the other sinks hold
// records until every chunk is validated does not apply, and no chunk is
// indexed and parsed a second time in pass 2 (C4 on one GPU: 131 GB of
// records against a hold budget of ~16 GB).
bool sink_all_pass1(const sid_engine* e) { return e->cfg.device_sink == 1 && needs_format_pass1(e); }

// An uploader's registered chunk bodies (upload_register): at most the one
// being copied and the next, each released once its copy's event is done.
struct UploadReg {
    struct Reg {
        uint64_t j = UINT64_MAX;
        char* p = nullptr;          // page-aligned body, registered
        uint64_t n = 0;
        hipEvent_t ev = nullptr;    // its copy done
        bool copied = false;
    };
    sid_engine* e;
    bool on;
    std::deque<Reg> regs;
    std::vector<hipEvent_t> evs;
    UploadReg(sid_engine* e_, int pass) : e(e_), on(e_->reg_upload && (pass == 1 || e_->src == SRC_FILE)) {}
    ~UploadReg()
    {
        for (auto& r : regs) {
            if (r.ev) (void)hipEventSynchronize(r.ev);
            unregister(r.p);
        }
        for (auto& r : regs)
            if (r.ev) (void)hipEventDestroy(r.ev);
        for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
    }
    Reg* find(uint64_t j)
    {
        for (auto& r : regs)
            if (r.j == j) return &r;
        return nullptr;
    }
    // pin chunk j's whole pages (bodies of at least 1 MiB; smaller chunks
    // take the pageable path, and so does every chunk after a registration
    // fails)
    void pin(uint64_t j)
    {
        if (!on || j == UINT64_MAX || find(j)) return;
        const ChunkRec& r = e->recs[j];
        const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
        const uintptr_t s = (uintptr_t)(e->text + r.off), t = s + r.len;
        const uintptr_t a = (s + pg - 1) & ~(uintptr_t)(pg - 1), b = t & ~(uintptr_t)(pg - 1);
        if (b <= a || b - a < (1u << 20)) return;
        const double t0 = wall();
        const bool ok = hipHostRegister((void*)a, b - a, hipHostRegisterReadOnly) == hipSuccess ||
                        ((void)hipGetLastError(), hipHostRegister((void*)a, b - a, hipHostRegisterDefault) == hipSuccess);
        e->t_register += (uint64_t)((wall() - t0) * 1e9);
        if (!ok) {
            (void)hipGetLastError();   // not an error: the pageable path from now on
            on = false;
            return;
        }
        Reg g;
        g.j = j;
        g.p = (char*)a;
        g.n = b - a;
        regs.push_back(g);
    }
    void ahead(uint64_t j)
    {
        release_done();
        pin(j);
    }
    // chunk j (pinned now if it is not yet) into dst on stream st
    hipError_t copy(char* dst, uint64_t j, hipStream_t st)
    {
        const ChunkRec& r = e->recs[j];
        const char* src = e->text + r.off;
        pin(j);
        Reg* g = find(j);
        if (!g) return hipMemcpyAsync(dst, src, r.len, hipMemcpyHostToDevice, st);
        const uint64_t head = (uint64_t)(g->p - src), body = g->n, tail = r.len - head - body;
        hipError_t x = hipSuccess;
        if (head) x = hipMemcpyAsync(dst, src, head, hipMemcpyHostToDevice, st);
        if (x == hipSuccess) x = hipMemcpyAsync(dst + head, g->p, body, hipMemcpyHostToDevice, st);
        if (x == hipSuccess) e->reg_chunks++;
        if (x == hipSuccess && tail) x = hipMemcpyAsync(dst + head + body, g->p + body, tail, hipMemcpyHostToDevice, st);
        if (x == hipSuccess) {
            if (evs.empty()) {
                hipEvent_t ev = nullptr;
                x = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
                if (x == hipSuccess) evs.push_back(ev);
            }
            if (x == hipSuccess) {
                g->ev = evs.back();
                evs.pop_back();
                x = hipEventRecord(g->ev, st);
                g->copied = true;
            }
        }
        return x;
    }
    void unregister(char* p)
    {
        const double t0 = wall();
        (void)hipHostUnregister(p);
        e->t_register += (uint64_t)((wall() - t0) * 1e9);
    }
    // unregister the bodies whose copies are done (in copy order)
    void release_done()
    {
        while (!regs.empty() && regs.front().copied && hipEventQuery(regs.front().ev) == hipSuccess) {
            unregister(regs.front().p);
            evs.push_back(regs.front().ev);
            regs.pop_front();
        }
        (void)hipGetLastError();   // (hipEventQuery's "not ready")
    }
};

// the uploader of device d: the chunks of `list` into device buffers, in order
void uploader(sid_engine* e, Dev& d, const std::vector<uint64_t>& list, int pass)
{
    bind_thread(d);
    if (hipSetDevice(d.device) != hipSuccess) return (void)fail(e, SID_EHIP);
    UploadReg reg(e, pass);
    // the ingest's uploads timed as one span on the upload stream, from the
    // first copy's start to the last one's end (the copies run back to back;
    // a pair of events around every copy cost the step ~0.3 ms)
    struct Span {
        Dev& d;
        hipEvent_t t0 = nullptr;
        uint64_t bytes = 0;
        ~Span()
        {
            if (!t0) return;
            hipEvent_t t1 = d.h2d_event();
            if (t1 && hipEventRecord(t1, d.s_up) == hipSuccess) {
                d.h2d_pending.push_back({t0, t1});
                d.h2d_bytes += bytes;
            } else {
                d.h2d_free.push_back(t0);
                if (t1) d.h2d_free.push_back(t1);
            }
        }
    } span{d};
    // the chunk this uploader copies after j from the host (UINT64_MAX: none)
    size_t at = 0;
    auto next_of = [&](uint64_t j) -> uint64_t {
        while (at < list.size() && list[at] != j) ++at;
        for (size_t k = at + 1; k < list.size(); ++k) {
            const ChunkRec& q = e->recs[list[k]];
            if (pass == 2 && (q.host1 || q.sunk || q.held || q.kept)) continue;
            return list[k];
        }
        return UINT64_MAX;
    };
    for (uint64_t j : list) {
        if (e->rc.load() != SID_OK) break;
        if (pass == 1 && j > e->first_err.load()) break;
        ChunkRec& r = e->recs[j];
        Loaded L;
        L.j = j;
        if (pass == 2 && (r.host1 || r.sunk)) continue;   // in host memory already (the writer takes it), or sunk
        if (pass == 2 && r.held) {
            L.kind = 1;
            if (!d.loaded.push(L)) break;
            continue;
        }
        if (e->src == SRC_DEVICE) {   // resident text: a view, 16-B aligned base
            const uint64_t a = (uint64_t)(uintptr_t)(e->text + r.off);
            L.base = (const char*)(uintptr_t)(a & ~(uint64_t)15);
            L.c0 = a & 15;
            L.c1 = L.c0 + r.len;
            if (!d.loaded.push(L)) break;
            continue;
        }
        if (pass == 2 && r.kept) {
            L.base = r.kept;
            L.c0 = 0;
            L.c1 = r.kept_len;
            if (!d.loaded.push(L)) break;
            continue;
        }
        // text length (synthetic sources: a bound until generated)
        uint64_t need = e->src == SRC_SYNTH_HOST || e->src == SRC_SYNTH_DEVICE ? e->per_chunk_cap : r.len;
        // keep it for pass 2?  Lynch always needs a second pass; local and
        // quality only once the hold budget ran out
        // (the device sink formats every -m local / quality chunk in pass 1:
        // nothing to keep for a second pass)
        bool want_keep = pass == 1 && (e->lynch || (d.hold_full.load() && !sink_all_pass1(e))) &&
                         d.retain_used.load() + need + PAD <= d.retain_budget;
        char* dst = nullptr;
        uint64_t dcap = 0;
        int slot = -1;
        hipError_t x = hipSuccess;
        if (want_keep) {
            dst = d.pool.get(need + PAD, &dcap, d.s_up);
            if (dst) d.retain_used += dcap;
            else want_keep = false;   // no HBM for it: a ring slot, read again in pass 2
        }
        if (!want_keep) {
            if (!d.free_slots.pop(slot)) break;
            Slot& s = d.slots[slot];
            if (s.cap < need) {   // grow: wait for the slot's last reader first
                if (s.used) x = hipEventSynchronize(s.ev_free);
                if (s.text) (void)hipFree(s.text);
                s.text = nullptr;
                s.cap = 0;
                const uint64_t c = std::max<uint64_t>(need, chunk_bytes(e) + (chunk_bytes(e) >> 3));
                if (x == hipSuccess) x = hipMalloc(&s.text, c + PAD);
                if (x == hipSuccess) s.cap = c;
                s.used = false;
            } else if (s.used) {
                // the slot's last reader (compute stream) is long done by now:
                // waited for here, not by the copy engine's queue (a cross-
                // queue wait in front of every copy)
                x = hipEventSynchronize(s.ev_free);
            }
            if (x != hipSuccess) return (void)hipfail(e, x);
            dst = s.text;
            dcap = s.cap + PAD;
            s.used = true;
        }
        uint64_t len = r.len;
        if (e->src == SRC_HOST || e->src == SRC_FILE) {
            if (pass == 1 && len && !span.t0 && (span.t0 = d.h2d_event())) x = hipEventRecord(span.t0, d.s_up);
            if (len && x == hipSuccess) x = reg.copy(dst, j, d.s_up);
            if (pass == 1 && span.t0 && x == hipSuccess) span.bytes += len;
            // the next chunk's pages pinned while this copy runs; the ones
            // whose copies are done released
            if (x == hipSuccess) reg.ahead(next_of(j));
            if (e->src == SRC_FILE && x == hipSuccess && e->text_len > (8ull << 30)) {
                // large mapped inputs: drop the chunk's page-table entries once
                // copied (the page cache keeps the data; RSS stays bounded)
                x = hipStreamSynchronize(d.s_up);
                reg.release_done();
                const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
                const uint64_t a = (e->map_skew + r.off + pg - 1) & ~(pg - 1);
                const uint64_t b = (e->map_skew + r.off + len) & ~(pg - 1);
                if (b > a) (void)madvise((char*)e->map + a, b - a, MADV_DONTNEED);
            }
        } else if (e->src == SRC_SYNTH_HOST) {
            // generated by host threads into this device's pinned staging,
            // one region per thread, each region DMA'd to its place
            const size_t gi = (size_t)d.index;
            const int T = std::max(1, e->cfg.host_threads > 0 ? e->cfg.host_threads : 8);
            const uint64_t region = e->per_chunk_cap / T + e->per_chunk_cap / (4 * T) + 64 + 5 * e->synth_cdf.size();
            x = hipEventSynchronize(e->gen_ev[gi]);   // the previous chunk's copies are done
            if (x == hipSuccess && e->gen_cap[gi] < region * T) {
                if (e->gen_buf[gi]) (void)hipHostFree(e->gen_buf[gi]);
                e->gen_buf[gi] = nullptr;
                e->gen_cap[gi] = 0;
                x = hipHostMalloc((void**)&e->gen_buf[gi], region * T, hipHostMallocDefault);
                if (x == hipSuccess) e->gen_cap[gi] = region * T;
            }
            std::vector<uint64_t> plen(T, 0);
            if (x == hipSuccess) {
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const uint64_t a = r.nsites * t / T, b = r.nsites * (t + 1) / T;
                        plen[t] = synth_host(e->synth_cdf, e->synth_seed, r.site0 + a, b - a, e->synth_spc,
                                             e->gen_buf[gi] + region * t, region);
                    });
                for (auto& t : th) t.join();
            }
            len = 0;
            for (int t = 0; t < T && x == hipSuccess; ++t) {
                if (plen[t] == UINT64_MAX || len + plen[t] > dcap - PAD) return (void)fail(e, SID_ENOMEM);
                if (plen[t])
                    x = hipMemcpyAsync(dst + len, e->gen_buf[gi] + region * t, plen[t], hipMemcpyHostToDevice,
                                       d.s_up);
                len += plen[t];
            }
            if (x == hipSuccess) x = hipEventRecord(e->gen_ev[gi], d.s_up);
        } else if (e->src == SRC_SYNTH_DEVICE) {
            sid_synth_gen_ws& G = e->gen_ws[d.index];
            x = sid_launch_synth_text(e->synth_seed, e->d_cdf_dev[d.index], (uint32_t)e->synth_cdf.size(), r.site0,
                                      r.nsites, e->synth_spc, &G, dst, dcap - PAD, d.s_up, e->synth_depth);
            if (x == hipSuccess) x = hipMemcpyAsync(d.h_small + 6, G.res, 16, hipMemcpyDeviceToHost, d.s_up);
            if (x == hipSuccess) x = hipStreamSynchronize(d.s_up);
            if (x == hipSuccess) {
                if (d.h_small[7]) return (void)fail(e, SID_ENOMEM);   // beyond the generator's margin
                len = d.h_small[6];
            }
        }
        // the bytes past the chunk only need to be readable (every kernel
        // bounds its reads by the chunk's end), which the buffers' PAD
        // guarantees; zeroing them per chunk put a fill kernel between every
        // two copies of the upload stream (copy engine -> shader -> copy
        // engine), so it is done only where a kernel already wrote the text
        if (x == hipSuccess && e->src == SRC_SYNTH_DEVICE) x = hipMemsetAsync(dst + len, 0, PAD, d.s_up);
        hipEvent_t ev = nullptr;
        if (slot >= 0) {
            ev = d.slots[slot].ev_up;
            if (x == hipSuccess) x = hipEventRecord(ev, d.s_up);
        } else if (x == hipSuccess) {
            x = hipStreamSynchronize(d.s_up);   // kept buffers: no per-buffer event
        }
        if (x != hipSuccess) return (void)hipfail(e, x);
        if (want_keep) {
            r.kept = dst;
            r.kept_cap = dcap;
            r.kept_len = len;
        }
        L.slot = slot;
        L.base = dst;
        L.c0 = 0;
        L.c1 = len;
        L.ev = ev;
        if (pass == 2) e->reloaded++;
        if (!d.loaded.push(L)) break;
    }
    d.loaded.close();
}

int call_sites(sid_engine* e, Dev& d, const Loaded& L, uint64_t n)
{
    sid_chunk_ws& W = d.ws;
    if (n == 0) return SID_OK;
    const int m = e->opts.method;
    if (m == SID_METHOD_QUALITY) return sid_chunk_quality(d.ctx, &W, L.base, L.c1, n, d.s_comp);
    if (m == SID_METHOD_LOCAL)
        return sid_call_local(d.ctx, (const uint16_t*)W.counts, n, W.code, W.hom, W.het, d.s_comp);
    return sid_lookup_sites(d.ctx, (const uint16_t*)W.counts, n, W.code, W.hom, W.het, d.s_comp);
}

// the compute thread of device d, for one pass
void compute(sid_engine* e, Dev& d, int pass)
{
    bind_thread(d);
    if (hipSetDevice(d.device) != hipSuccess) return (void)fail(e, SID_EHIP);
    sid_chunk_ws& W = d.ws;
    uint64_t* hs = d.h_small;
    const int qmode = e->quality ? 1 : 0;
    auto sync = [&]() {
        const double a = wall();
        const hipError_t r = hipStreamSynchronize(d.s_comp);
        e->t_comp_sync += (uint64_t)((wall() - a) * 1e9);
        return r;
    };
    // (an event instead of the stream: the work queued behind it is not waited for)
    auto sync_ev = [&](hipEvent_t ev) {
        const double a = wall();
        const hipError_t r = hipEventSynchronize(ev);
        e->t_comp_sync += (uint64_t)((wall() - a) * 1e9);
        return r;
    };
    // the next chunk, taken early so that its line index runs behind this
    // chunk's formatter (the GPU then does not idle over the host round trip
    // that reads the formatter's byte count); indexed: its site count is in hs[0]
    Loaded nextL;
    bool have_next = false, next_indexed = false;
    // ... or its tile parse behind this chunk's writer (tiled: with next_lg
    // slots a tile, the next_quad shape)
    bool next_tiled = false, next_quad = false;
    uint32_t next_lg = 0;
    auto take = [&](Loaded& out) {
        if (have_next) {
            out = nextL;
            have_next = false;
            return true;
        }
        return d.loaded.pop(out);
    };
    Loaded L;
    while (take(L)) {
        const bool pre_indexed = next_indexed;
        next_indexed = false;
        bool pre_tiled = next_tiled;
        next_tiled = false;
        if (e->rc.load() != SID_OK) break;
        ChunkRec& r = e->recs[L.j];
        auto release_slot = [&]() {
            if (L.slot < 0) return;
            (void)hipEventRecord(d.slots[L.slot].ev_free, d.s_comp);
            d.free_slots.push(L.slot);
        };
        if (L.kind == 1) {   // pass 2: records held since pass 1
            OutItem it;
            it.j = L.j;
            it.buf = r.held;
            it.cap = r.held_cap;
            it.len = r.held_len;
            r.held = nullptr;
            if (e->cfg.device_sink == 1) e->sink_bytes += it.len, d.pool.put(it.buf, it.cap, nullptr);
            else if (!d.drain_q.push(it)) break;
            continue;
        }
        if (pass == 1 && L.j > e->first_err.load()) {
            if (pre_tiled) W.slot_cap = 0;
            release_slot();
            continue;
        }
        int rc = SID_OK;
        hipError_t x = hipSuccess;
        if (L.ev && !pre_indexed && !pre_tiled) x = hipStreamWaitEvent(d.s_comp, L.ev, 0);
        const bool P = e->prof;
        if (P && pass == 1) d.prof_chunks++;   // chunks, not passes: a Lynch run formats each chunk again in pass 2
        if (!pre_tiled) {
            W.lens_ready = false;   // (set by this chunk's parse when it computes the -m local record lengths)
            W.cls_ready = false;    // (... and the class words)
        }
        const uint64_t tbytes = L.c1 - (L.c0 & ~(uint64_t)15);
        if (x == hipSuccess && !pre_indexed && !pre_tiled) rc = sid_chunk_reserve(&W, tbytes, 0);
        const bool lynch_hist = pass == 1 && e->lynch;
        const bool format = pass == 2 || (needs_format_pass1(e) && (!d.hold_full.load() || sink_all_pass1(e)));
        // -m local / quality (and pass 2 of the Lynch paths): call, then the
        // one-pass formatter into a buffer of the records' upper bound -- the
        // device's hold arena in pass 1 (committed to the exact bytes after),
        // else a pooled scratch buffer
        char* out = nullptr;
        uint64_t cap = 0;   // 0: arena memory (never returned to the pool)
        bool via_host = false;   // pass 1: records go on to the host arena (a pooled device buffer meanwhile)
        bool sunk = false;       // pass 1, device sink: a scratch buffer, dropped
        hipEvent_t pe = nullptr;
        uint64_t n = 0;
        // the tile path: this chunk's records and byte count done (recorded
        // before the next chunk's tile parse is queued behind the writer: the
        // host and the records' D2H wait for this, not for that parse, which
        // waits for the next chunk's upload -- each chunk's D2H then runs
        // behind its own writer instead of a chunk later)
        struct Done {
            Dev& d;
            hipEvent_t ev = nullptr;
            void drop()
            {
                if (ev) d.give_event(ev);
                ev = nullptr;
            }
            ~Done() { drop(); }
        } done{d};
        // -m local formatting in this pass, lines of up to 256 B on average (as
        // the device's last chunk had): the tile parse -- the text read once,
        // no host round trip before the writer (sid_chunk_tile_local).  A tile
        // with more lines than its slots sends the chunk again through the
        // two-pass path below (its records dropped), the next chunks with
        // more slots
        // (pre_tiled: this chunk's tile parse already ran behind the previous
        // chunk's writer, with the slots and shape of that time)
        bool tiled = false;
        const bool tile_was_off = !d.tile_ok;   // (this chunk then goes the two-pass way, and may turn it on)
        const bool tile_path =x == hipSuccess && rc == SID_OK && format && !lynch_hist && !qmode &&
                               (d.tile_ok || pre_tiled) && e->opts.method == SID_METHOD_LOCAL &&
                               sid_chunk_local_ok(d.ctx) && !(pass == 2 && r.pre);
        if (pre_tiled && !tile_path) {
            W.slot_cap = 0;   // (its slots unused: the dense layout again)
            pre_tiled = false;
        }
        if (tile_path) {
            const uint32_t lg = pre_tiled ? next_lg : d.tile_cap;
            const bool quad = pre_tiled ? next_quad : d.tile_quad;
            if (!pre_tiled) rc = sid_chunk_reserve(&W, tbytes, sid_chunk_tile_slots(L.c0, L.c1, lg, quad));
            if (rc != SID_OK) return (void)fail(e, rc);
            const uint64_t bound = sid_chunk_tile_bound(L.c0, L.c1, lg, quad);
            // the records' buffer, taken as the two-pass path below takes it
            // (near the hold budget that path decides, with its exact bound)
            if (pass == 1 && d.hh && !d.hh_full) {
                out = d.pool.get(bound, &cap, d.s_comp);
                via_host = out != nullptr;
                if (!out) cap = 0;
            }
            if (via_host) {
            } else if (pass == 1 && sink_all_pass1(e)) {
                out = d.pool.get(bound, &cap, d.s_comp);
                sunk = out != nullptr;
                if (!out) cap = 0;
            } else if (pass == 1 && d.hold_used.load() + bound > d.hold_budget) {
            } else if (pass == 1) {
                out = d.arena_reserve(bound, d.hold_budget - d.hold_used.load());
            } else {
                out = d.pool.get(bound, &cap, d.s_comp);
                if (!out) cap = 0;
            }
            if (!out && pre_tiled) {
                W.slot_cap = 0;
                pre_tiled = false;
            }
            if (out) {
                if (!pre_tiled) {
                    pe = d.prof_begin(P);
                    rc = sid_chunk_tile_local(d.ctx, &W, L.base, L.c0, L.c1, lg, quad, e->conf_type, d.s_comp);
                    d.prof_end(1, pe);
                }
                if (rc == SID_OK) {
                    pe = d.prof_begin(P);
                    rc = sid_chunk_local_put(d.ctx, &W, L.base, L.c1, 0, e->conf_type, out, d.s_comp);
                    d.prof_end(5, pe);
                }
                W.slot_cap = 0;   // (the workspace's dense layout again for the two-pass path)
                if (rc != SID_OK) return (void)fail(e, rc);
                // bytes, range flag, sites, parse error key, the most lines in a tile
                x = hipMemcpyAsync(hs + 8, W.lb + 1, 5 * 8, hipMemcpyDeviceToHost, d.s_comp);
                if (x == hipSuccess && (done.ev = d.take_event())) x = hipEventRecord(done.ev, d.s_comp);
                // the next chunk's tile parse behind this writer (stream order:
                // it rewrites the slots and W.lb after the writer and the copy
                // have read them), so the GPU does not idle over the host round
                // trip; with this chunk's slots and shape (a change takes effect
                // a chunk later), dropped if this chunk overflows
                if (x == hipSuccess && !have_next && d.loaded.try_pop(nextL)) {
                    have_next = true;
                    const ChunkRec& r2 = e->recs[nextL.j];
                    if (nextL.kind == 0 && !(pass == 2 && r2.pre) && !(pass == 1 && nextL.j > e->first_err.load())) {
                        const uint32_t lg2 = d.tile_cap;
                        const bool q2 = d.tile_quad;
                        if (nextL.ev) x = hipStreamWaitEvent(d.s_comp, nextL.ev, 0);
                        int rc2 = SID_OK;
                        // growth frees buffers: hipFree waits for the queued work first
                        if (x == hipSuccess)
                            rc2 = sid_chunk_reserve(&W, nextL.c1 - (nextL.c0 & ~(uint64_t)15),
                                                    sid_chunk_tile_slots(nextL.c0, nextL.c1, lg2, q2));
                        hipEvent_t pe2 = d.prof_begin(P);
                        if (rc2 == SID_OK && x == hipSuccess)
                            rc2 = sid_chunk_tile_local(d.ctx, &W, nextL.base, nextL.c0, nextL.c1, lg2, q2,
                                                       e->conf_type, d.s_comp);
                        d.prof_end(1, pe2);
                        if (rc2 != SID_OK) return (void)fail(e, rc2);
                        next_tiled = x == hipSuccess;
                        next_lg = lg2;
                        next_quad = q2;
                    }
                }
                if (x == hipSuccess) x = done.ev ? sync_ev(done.ev) : sync();
                if (x != hipSuccess) return (void)hipfail(e, x);
                const uint64_t maxl = hs[12];
                if (maxl <= lg) {
                    tiled = true;
                    ++d.tiled;
                    n = hs[10];
                    r.parsed = n;
                    hs[4] = hs[11];
                    // the next chunk's shape and slots (a new shape: from this
                    // chunk's lines per byte, a quarter on top)
                    d.tile_next(maxl, n, L.c1 - L.c0, quad);
                } else {
                    if (cap) d.pool.put(out, cap, d.s_comp);
                    out = nullptr;
                    cap = 0;
                    via_host = sunk = false;
                    done.drop();
                    ++d.tile_overflows;
                    d.tile_over_queued += have_next;
                    d.tile_over(maxl, quad);
                    // this chunk goes the two-pass way through the workspace:
                    // the next chunk's tile parse is dropped (it runs again)
                    W.slot_cap = 0;
                    next_tiled = false;
                }
            }
        }
        // The Lynch paths' first pass likewise: the tile parse into every
        // site's counts and header pair, compacted into the buffer kept for
        // pass 2 (the two-pass parse's layout), then the histogram.  Without
        // room for that buffer (the retain budget), the two-pass path below
        // (pass 2 then indexes and parses the text again).
        if (!tiled && x == hipSuccess && rc == SID_OK && lynch_hist && !qmode && d.tile_ok) {
            const uint32_t cp = d.tile_cap;
            const bool quad = d.tile_quad;
            rc = sid_chunk_reserve(&W, tbytes, sid_chunk_tile_slots(L.c0, L.c1, cp, quad));
            if (rc != SID_OK) return (void)fail(e, rc);
            pe = d.prof_begin(P);
            rc = sid_chunk_tile_counts(&W, L.base, L.c0, L.c1, cp, quad, d.s_comp);
            if (rc != SID_OK) return (void)fail(e, rc);
            x = hipMemcpyAsync(hs, W.state, 8, hipMemcpyDeviceToHost, d.s_comp);   // sites
            if (x == hipSuccess) x = hipMemcpyAsync(hs + 4, W.state + 4, 8, hipMemcpyDeviceToHost, d.s_comp);
            if (x == hipSuccess) x = hipMemcpyAsync(hs + 12, W.lb + 5, 8, hipMemcpyDeviceToHost, d.s_comp);
            if (x == hipSuccess) x = sync();
            if (x != hipSuccess) return (void)hipfail(e, x);
            const uint64_t maxl = hs[12], m = hs[0];
            if (maxl > cp) {   // a tile with more lines than slots: the two-pass path
                W.slot_cap = 0;
                d.prof_end(1, pe);
                ++d.tile_overflows;
                d.tile_over(maxl, quad);
            } else {
                const uint64_t m2 = (m + 1) & ~(uint64_t)1, m4 = (m + 3) & ~(uint64_t)3;
                const uint64_t pre_bytes = 4 * m4 + 24 * m2;
                uint64_t pc = 0;
                char* pre = m && d.retain_used.load() + pre_bytes <= d.retain_budget
                                ? d.pool.get(pre_bytes, &pc, d.s_comp) : nullptr;
                if (m == 0 || pre) {
                    uint64_t* counts = nullptr;
                    if (pre) {
                        r.pre = pre;
                        r.pre_cap = pc;
                        d.retain_used += pc;
                        counts = (uint64_t*)(pre + 4 * m4);
                        rc = sid_chunk_tile_compact(&W, (sid_off_t*)pre, counts, counts + m2, d.s_comp);
                        if (rc != SID_OK) return (void)fail(e, rc);
                    }
                    W.slot_cap = 0;
                    d.prof_end(1, pe);
                    n = m;
                    r.parsed = n;
                    pe = d.prof_begin(P);
                    rc = sid_profile_accumulate(d.ctx, (const uint16_t*)counts, n, d.s_comp);   // synchronises
                    d.prof_end(3, pe);
                    if (rc == SID_OK && n == 0) x = sync();
                    if (rc != SID_OK) return (void)fail(e, rc);
                    if (x != hipSuccess) return (void)hipfail(e, x);
                    tiled = true;
                    ++d.tiled;
                    d.tile_next(maxl, n, L.c1 - L.c0, quad);
                } else {
                    W.slot_cap = 0;   // no room to keep the parse: the two-pass path
                    d.prof_end(1, pe);
                }
            }
        }
        if (!tiled) {
        // pass 2 of a Lynch path: the parse kept since pass 1 stands in for the
        // workspace's line offsets, counts and header pairs (restored below)
        struct View {
            sid_chunk_ws& W;
            sid_off_t* starts;
            uint64_t *counts, *hdr;
            bool on = false;
            ~View()
            {
                if (on) W.starts = starts, W.counts = counts, W.hdr = hdr;
            }
        } view{W, W.starts, W.counts, W.hdr};
        // the kept parse's layout: starts (4 B), counts (8 B), header pairs
        // (16 B), each at a 16-B aligned offset (the lookup reads counts as
        // 16-B site pairs)
        auto use_pre = [&](char* pre, uint64_t m) {
            view.starts = W.starts, view.counts = W.counts, view.hdr = W.hdr, view.on = true;
            const uint64_t m2 = (m + 1) & ~(uint64_t)1, m4 = (m + 3) & ~(uint64_t)3;
            W.starts = (sid_off_t*)pre;
            W.counts = (uint64_t*)(pre + 4 * m4);
            W.hdr = W.counts + m2;
        };
        if (pass == 2 && r.pre) {
            n = r.parsed;
            rc = sid_chunk_reserve(&W, 0, n);
            if (rc != SID_OK) return (void)fail(e, rc);
            use_pre(r.pre, n);
            if (x == hipSuccess) x = hipMemsetAsync(W.state + 4, 0xFF, sizeof(uint64_t), d.s_comp);   // no parse error
            if (x != hipSuccess) return (void)hipfail(e, x);
        } else {
            if (!pre_indexed) {
                pe = d.prof_begin(P);
                if (rc == SID_OK && x == hipSuccess) rc = sid_chunk_index(&W, L.base, L.c0, L.c1, d.s_comp);
                d.prof_end(0, pe);
                if (rc == SID_OK && x == hipSuccess) x = hipMemcpyAsync(hs, W.state, 8, hipMemcpyDeviceToHost, d.s_comp);
                if (rc == SID_OK && x == hipSuccess) x = sync();
            }
            if (x != hipSuccess) return (void)hipfail(e, x);
            if (rc != SID_OK) return (void)fail(e, rc);
            n = hs[0];
            rc = sid_chunk_reserve(&W, 0, n);
            if (rc != SID_OK) return (void)fail(e, rc);
            r.parsed = n;
            if (tile_was_off && !qmode) d.tile_retry(n, L.c1 - L.c0);
            // Lynch paths: the parse goes straight into a buffer kept for
            // pass 2 (which then skips index and parse) while the retain
            // budget allows: 28 B a site, cheaper than indexing and parsing
            // the text again
            const uint64_t pre_bytes = 4 * ((n + 3) & ~(uint64_t)3) + 24 * ((n + 1) & ~(uint64_t)1);
            if (pass == 1 && e->lynch && n && !qmode && d.retain_used.load() + pre_bytes <= d.retain_budget) {
                uint64_t pc = 0;
                char* pre = d.pool.get(pre_bytes, &pc, d.s_comp);
                if (pre) {
                    r.pre = pre;
                    r.pre_cap = pc;
                    d.retain_used += pc;
                    use_pre(pre, n);
                }
            }
            pe = d.prof_begin(P);
            // -m local: the records' lengths come out of the parse when this
            // pass formats (sid_parse_len_kernel; the length kernel is skipped)
            const bool lens = e->opts.method == SID_METHOD_LOCAL && sid_chunk_local_ok(d.ctx) && !qmode &&
                              !(pass == 1 && e->lynch) && (pass == 2 || needs_format_pass1(e));
            if (rc == SID_OK) rc = sid_chunk_parse(&W, L.base, L.c0, L.c1, n, qmode, d.s_comp, lens ? d.ctx : nullptr);
            d.prof_end(1, pe);
            if (rc != SID_OK) return (void)fail(e, rc);
        }
        if (lynch_hist) {
            x = hipMemcpyAsync(hs + 4, W.state + 4, 8, hipMemcpyDeviceToHost, d.s_comp);
            if (x != hipSuccess) return (void)hipfail(e, x);
            pe = d.prof_begin(P);
            rc = sid_profile_accumulate(d.ctx, (const uint16_t*)W.counts, n, d.s_comp);   // synchronises
            d.prof_end(3, pe);
            if (rc == SID_OK && n == 0) x = sync();
            if (rc != SID_OK) return (void)fail(e, rc);
            if (x != hipSuccess) return (void)hipfail(e, x);
        }
        // -m local: the call fused into the formatter (sid_chunk_local_*)
        const bool fused = e->opts.method == SID_METHOD_LOCAL && sid_chunk_local_ok(d.ctx);
        // likelihood_ratio / bayes pass 2: the class lookup fused into the
        // formatter (sid_chunk_lynch_*; the records' tails prebuilt per class)
        sid_lynch_fmt lv;
        const bool lfused = pass == 2 && !fused && sid_lynch_fmt_view(d.ctx, &lv) == SID_OK;
        if (format && !lynch_hist) {
            if (!fused && !lfused) {
                pe = d.prof_begin(P);
                rc = call_sites(e, d, L, n);
                d.prof_end(2, pe);
                if (rc != SID_OK) return (void)fail(e, rc);
            }
            const uint64_t bound = sid_chunk_fmt_bound(n, L.c1 - L.c0);
            if (n && pass == 1 && d.hh && !d.hh_full) {
                out = d.pool.get(bound, &cap, d.s_comp);
                via_host = out != nullptr;
                if (!out) cap = 0;
            }
            if (n == 0 || via_host) {
            } else if (pass == 1 && sink_all_pass1(e)) {
                // (no hold arena: nothing is emitted, so no record need wait
                // in HBM; the pooled buffer is reused chunk after chunk)
                out = d.pool.get(bound, &cap, d.s_comp);
                sunk = out != nullptr;   // (no HBM for it: formatted in pass 2 instead)
                if (!out) cap = 0, d.hold_full = true;
            } else if (pass == 1 && d.hold_used.load() + bound > d.hold_budget) {
                d.hold_full = true;   // this chunk and the rest: formatted in pass 2
            } else if (pass == 1) {
                // no HBM for the arena: formatted in pass 2 instead
                if (!(out = d.arena_reserve(bound, d.hold_budget - d.hold_used.load()))) d.hold_full = true;
            } else {
                if (!(out = d.pool.get(bound, &cap, d.s_comp))) return (void)fail(e, SID_ENOMEM);
            }
            if (out) {
                pe = d.prof_begin(P);
                rc = fused    ? sid_chunk_local_len(d.ctx, &W, L.base, L.c1, n, e->conf_type, d.s_comp)
                     : lfused ? sid_chunk_lynch_len(d.ctx, &W, L.base, L.c1, n, d.s_comp)
                              : sid_chunk_fmt_len(&W, L.base, L.c1, n, e->conf_type, d.s_comp);
                d.prof_end(4, pe);
                if (rc != SID_OK) return (void)fail(e, rc);
                pe = d.prof_begin(P);
                rc = fused    ? sid_chunk_local_put(d.ctx, &W, L.base, L.c1, n, e->conf_type, out, d.s_comp)
                     : lfused ? sid_chunk_lynch_put(d.ctx, &W, L.base, L.c1, n, out, d.s_comp)
                              : sid_chunk_fmt_put(&W, L.base, L.c1, n, e->conf_type, out, d.s_comp);
                d.prof_end(5, pe);
                if (rc != SID_OK) return (void)fail(e, rc);
                x = hipMemcpyAsync(hs + 8, W.lb + 1, 32, hipMemcpyDeviceToHost, d.s_comp);   // bytes, flags, error
                // the next chunk's line index behind the formatter (stream
                // order: it rewrites W.state only after the formatter has read it)
                // (not when the tile path already took the next chunk: this
                // chunk overflowed its slots and came here)
                if (x == hipSuccess && !have_next && d.loaded.try_pop(nextL)) {
                    have_next = true;
                    const ChunkRec& r2 = e->recs[nextL.j];
                    if (nextL.kind == 0 && !(pass == 2 && r2.pre) && !(pass == 1 && nextL.j > e->first_err.load())) {
                        if (nextL.ev) x = hipStreamWaitEvent(d.s_comp, nextL.ev, 0);
                        int rc2 = SID_OK;
                        // growth frees buffers: hipFree waits for the queued work first
                        if (x == hipSuccess) rc2 = sid_chunk_reserve(&W, nextL.c1 - (nextL.c0 & ~(uint64_t)15), 0);
                        hipEvent_t pe2 = d.prof_begin(P);
                        if (rc2 == SID_OK && x == hipSuccess)
                            rc2 = sid_chunk_index(&W, nextL.base, nextL.c0, nextL.c1, d.s_comp);
                        d.prof_end(0, pe2);
                        if (rc2 == SID_OK && x == hipSuccess)
                            x = hipMemcpyAsync(hs, W.state, 8, hipMemcpyDeviceToHost, d.s_comp);
                        if (rc2 != SID_OK) return (void)fail(e, rc2);
                        next_indexed = x == hipSuccess;
                    }
                }
                if (x == hipSuccess) x = sync();
                if (x != hipSuccess) return (void)hipfail(e, x);
                hs[4] = hs[11];
            }
        }
        }   // (the two-pass path)
        if (!lynch_hist && !out) {
            x = hipMemcpyAsync(hs + 4, W.state + 4, 8, hipMemcpyDeviceToHost, d.s_comp);
            if (x == hipSuccess) x = sync();
            if (x != hipSuccess) return (void)hipfail(e, x);
            hs[8] = 0;
        }
        const uint64_t err = hs[4];
        if (err != ~0ull) {   // a malformed line: the rest of the input is moot
            r.err = err - 8 * L.c0;
            if (out && cap) d.pool.put(out, cap, d.s_comp);
            uint64_t cur = e->first_err.load();
            while (L.j < cur && !e->first_err.compare_exchange_weak(cur, L.j)) {
            }
            release_slot();
            if (pass == 2) return (void)fail(e, SID_EMALFORMED);   // cannot happen: pass 1 validated
            continue;
        }
        if (pass == 1 && n == 0 && format && !lynch_hist) {
            // a chunk without sites has no records: done in pass 1 for the
            // sinks that take records then (else the emit would start its
            // threads and a second pass for it)
            if (sink_all_pass1(e)) {
                r.sunk = true;
                r.held_len = 0;
            } else if (d.hh) {
                r.host = d.hh;
                r.host_len = 0;
                r.host1 = true;
            }
        }
        if (!format || lynch_hist || (pass == 1 && !out)) {
            release_slot();
            continue;
        }
        if (out && hs[9]) return (void)fail(e, SID_ERANGE);
        const uint64_t bytes = hs[8];
        release_slot();
        if (pass == 2 && r.kept) {   // kept text done with: back to the pool after this stream's work
            d.pool.put(r.kept, r.kept_cap, d.s_comp);
            r.kept = nullptr;
        }
        if (pass == 2 && r.pre) {
            d.pool.put(r.pre, r.pre_cap, d.s_comp);
            r.pre = nullptr;
        }
        if (pass == 1 && sunk) {
            r.sunk = true;
            r.held_len = bytes;
            d.pool.put(out, cap, d.s_comp);   // reused on this stream only: ordered
            continue;
        }
        if (pass == 1 && via_host) {
            char* hp = d.hh_take(bytes);
            if (hp) {   // D2H behind this chunk's formatter, while the next chunks upload
                hipEvent_t ev = done.ev ? nullptr : d.take_event();
                if (!done.ev && !ev) return (void)fail(e, SID_EHIP);
                if (ev) x = hipEventRecord(ev, d.s_comp);
                if (x == hipSuccess) x = hipStreamWaitEvent(d.s_d2h, ev ? ev : done.ev, 0);
                if (ev) d.give_event(ev);
                if (x == hipSuccess && bytes) x = hipMemcpyAsync(hp, out, bytes, hipMemcpyDeviceToHost, d.s_d2h);
                if (x != hipSuccess) return (void)hipfail(e, x);
                d.pool.put(out, cap, d.s_d2h);   // reusable once the copy is done
                r.host = hp;
                r.host_len = bytes;
                r.host1 = true;
                continue;
            }
            // the host arena is full: keep the records on the device while
            // the hold budget allows, else format the chunk again in pass 2
            d.hh_full = true;
            if (d.hold_used.load() + cap <= d.hold_budget) {
                r.held = out;
                r.held_cap = cap;
                r.held_len = bytes;
                d.hold_used += cap;
            } else {
                d.hold_full = true;
                d.pool.put(out, cap, d.s_comp);
            }
            continue;
        }
        if (pass == 1) {
            d.arena_commit(bytes);
            r.held = out;
            r.held_cap = 0;
            r.held_len = bytes;
            d.hold_used += (bytes + 255) & ~(uint64_t)255;
            continue;
        }
        if (e->cfg.device_sink == 1) {
            e->sink_bytes += bytes;
            d.pool.put(out, cap, nullptr);   // reused on this stream only: ordered
            continue;
        }
        OutItem it;
        it.j = L.j;
        it.buf = out;
        it.cap = cap;
        it.len = bytes;
        hipEvent_t ev = done.ev;
        done.ev = nullptr;
        if (!ev) {
            if (!(ev = d.take_event())) return (void)fail(e, SID_EHIP);
            (void)hipEventRecord(ev, d.s_comp);
        }
        it.ev = ev;
        if (!d.drain_q.push(it)) break;
    }
    W.slot_cap = 0;   // (a tile parse run ahead for a chunk this pass then skipped)
    if (pass == 2) d.drain_q.close();
}

// the drain of device d: CSV buffers through the pinned ring to the writer
void drain(sid_engine* e, Dev& d)
{
    bind_thread(d);
    if (hipSetDevice(d.device) != hipSuccess) return (void)fail(e, SID_EHIP);
    OutItem it;
    while (d.drain_q.pop(it)) {
        if (e->rc.load() != SID_OK) break;
        hipError_t x = hipSuccess;
        if (it.ev) {
            x = hipStreamWaitEvent(d.s_d2h, it.ev, 0);
            // free again once the wait is enqueued: the wait is on the record
            // made before it, a later record does not affect it
            d.give_event(it.ev);
        }
        if (x != hipSuccess) return (void)hipfail(e, x);
        if (it.len == 0) {
            if (d.hh) e->recs[it.j].host = d.hh, e->recs[it.j].host_len = 0;
            Piece p;
            p.j = it.j;
            p.last = true;
            p.buf = it.buf;
            p.cap = it.cap;
            if (!d.out_q.push(p)) break;
            continue;
        }
        if (char* hp = d.hh_take(it.len)) {   // the whole chunk into the host arena, one copy
            hipEvent_t ev = d.take_event();
            if (!ev) return (void)fail(e, SID_EHIP);
            x = hipMemcpyAsync(hp, it.buf, it.len, hipMemcpyDeviceToHost, d.s_d2h);
            if (x == hipSuccess) x = hipEventRecord(ev, d.s_d2h);
            if (x != hipSuccess) return (void)hipfail(e, x);
            e->recs[it.j].host = hp;
            e->recs[it.j].host_len = it.len;
            Piece p;
            p.j = it.j;
            p.len = it.len;
            p.last = true;
            p.buf = it.buf;
            p.cap = it.cap;
            p.host = hp;
            p.hev = ev;
            if (!d.out_q.push(p)) return;
            continue;
        }
        for (uint64_t o = 0; o < it.len;) {
            int ps;
            if (!d.free_pinned.pop(ps)) return;
            const uint64_t m = std::min<uint64_t>(d.pinned_cap, it.len - o);
            x = hipMemcpyAsync(d.pinned[ps], it.buf + o, m, hipMemcpyDeviceToHost, d.s_d2h);
            if (x == hipSuccess) x = hipEventRecord(d.pinned_ev[ps], d.s_d2h);
            if (x != hipSuccess) return (void)hipfail(e, x);
            o += m;
            Piece p;
            p.j = it.j;
            p.ps = ps;
            p.len = m;
            p.last = o == it.len;
            if (p.last) {
                p.buf = it.buf;
                p.cap = it.cap;
            }
            if (!d.out_q.push(p)) return;
        }
    }
    d.out_q.close();
}

}  // namespace

// ------------------------------------------------------------------ phases --
static void timing_report(sid_engine* e, const char* phase, double s)
{
    static const bool on = std::getenv("SID_ENGINE_TIMING") != nullptr;
    if (on)
        std::fprintf(stderr,
                     "{\"engine_phase\": \"%s\", \"s\": %.6f, \"compute_sync_s\": %.6f, \"writer_wait_s\": %.6f, "
                     "\"chunks_registered\": %llu}\n",
                     phase, s, e->t_comp_sync.load() * 1e-9, e->t_write_wait.load() * 1e-9,
                     (unsigned long long)e->reg_chunks.load());
    e->t_comp_sync = e->t_write_wait = 0;
    e->reg_chunks = 0;
    e->t_register = 0;
}

static void reset_run(sid_engine* e)
{
    e->rc = SID_OK;
    e->first_err = UINT64_MAX;
    const int m = e->opts.method;
    e->quality = m == SID_METHOD_QUALITY;
    e->lynch = m == SID_METHOD_LIKELIHOOD_RATIO || m == SID_METHOD_BAYES || e->opts.estimate_prior;
    e->conf_type = m == SID_METHOD_BAYES ? "probability" : "p_value";
    for (auto& r : e->recs) {
        Dev& d = *e->devs[r.dev];
        if (r.held) d.pool.put(r.held, r.held_cap, nullptr);
        if (r.kept) d.pool.put(r.kept, r.kept_cap, nullptr);
        if (r.pre) d.pool.put(r.pre, r.pre_cap, nullptr);
        r.held = r.kept = r.pre = nullptr;
        r.held_len = r.kept_len = 0;
        r.host = nullptr;
        r.host_len = 0;
        r.host1 = false;
        r.sunk = false;
        r.err = ~0ull;
        r.parsed = 0;
    }
    for (auto& dp : e->devs) {
        Dev& d = *dp;
        d.hold_used = 0;
        d.retain_used = 0;
        d.hold_full = false;
        d.arena_seg = 0;
        d.arena_off = 0;
        d.hh_off = 0;
        d.hh_full = false;
        (void)d.h2d_collect();   // (a failed run's copies: its devices were synchronised)
        d.h2d_bytes = 0;
        d.tiled = d.tile_overflows = d.tile_over_queued = 0;
        d.tile_reset();
        d.ws.slot_cap = 0;   // (a failed run may leave the slot layout set)
    }
    e->hist_merged = false;
}

static void start_queues(sid_engine* e)
{
    for (auto& dp : e->devs) {
        Dev& d = *dp;
        d.free_slots.reset();
        d.loaded.reset();
        d.drain_q.reset();
        d.out_q.reset();
        d.free_pinned.reset();
        for (int s = 0; s < (int)d.slots.size(); ++s) d.free_slots.push(s);
    }
}

static int setup_budgets(sid_engine* e)
{
    for (auto& dp : e->devs) {
        Dev& d = *dp;
        if (hipSetDevice(d.device) != hipSuccess) return SID_EHIP;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) return SID_EHIP;
        const uint64_t avail = fr + d.pool.bytes() + d.arena_bytes();   // pooled buffers and the arena are reusable
        // the GPU's pipelines share its memory (avail: what this one sees free)
        const double share = 0.40 / std::max(1, e->cfg.lanes);
        d.hold_budget = e->cfg.hold_bytes ? e->cfg.hold_bytes : (uint64_t)(avail * share);
        d.retain_budget = e->cfg.retain_bytes ? e->cfg.retain_bytes : (uint64_t)(avail * share);
        // the host arena: pinned (and so populated) once, reused by every run
        const uint64_t hb = e->cfg.device_sink == 1 ? 0 : e->cfg.host_hold_bytes;
        if (hb && d.hh_cap < hb) {
            d.hh_free();
            bool ok = false;
            on_node(d, [&] { ok = hipSetDevice(d.device) == hipSuccess && d.hh_alloc(hb); });
            if (!ok) return SID_ENOMEM;
        }
    }
    return SID_OK;
}

static int setup_generator(sid_engine* e)
{
    const size_t D = e->devs.size();
    if (e->src == SRC_SYNTH_HOST && e->gen_buf.size() != D) {
        e->gen_buf.assign(D, nullptr);
        e->gen_cap.assign(D, 0);
        e->gen_ev.assign(D, nullptr);
        for (size_t i = 0; i < D; ++i) {
            if (hipSetDevice(e->devs[i]->device) != hipSuccess) return SID_EHIP;
            if (hipEventCreateWithFlags(&e->gen_ev[i], hipEventDisableTiming) != hipSuccess) return SID_EHIP;
            if (hipEventRecord(e->gen_ev[i], e->devs[i]->s_up) != hipSuccess) return SID_EHIP;
        }
    }
    return SID_OK;
}

// The emit's pinned ring per device: 4 x 16 MiB (pinned once, reused by
// every run; 8 x 16, 4 x 64, 4 x 128 and 16 x 8 MiB measured slower: the
// pinning slows the ingest beside it and the exit tail grows with it)
constexpr int EMIT_RING_N = 4;
constexpr uint64_t EMIT_RING_BYTES = 16ull << 20;
static int alloc_ring_here(Dev& d);
// (on a thread bound to the GPU's CPUs: the ring's pages from its NUMA node)
static int alloc_ring(Dev& d)
{
    int rc = SID_OK;
    on_node(d, [&] { rc = alloc_ring_here(d); });
    return rc;
}
static int alloc_ring_here(Dev& d)
{
    if (hipSetDevice(d.device) != hipSuccess) return SID_EHIP;
    const uint64_t bytes = EMIT_RING_BYTES;
    while ((int)d.pinned.size() < EMIT_RING_N) {
        char* p = nullptr;
        hipEvent_t ev;
        if (hipHostMalloc((void**)&p, bytes, hipHostMallocDefault) != hipSuccess) return SID_ENOMEM;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipHostFree(p);
            return SID_EHIP;
        }
        d.pinned.push_back(p);
        d.pinned_ev.push_back(ev);
    }
    d.pinned_cap = bytes;
    return SID_OK;
}

extern "C" int sid_engine_ingest(sid_engine* e, sid_run_stats* st)
{
    if (!e || e->src == SRC_NONE) return SID_EINVAL;
    const double t0 = wall();
    reset_run(e);
    int rc = setup_budgets(e);
    const double t_budget = wall();
    if (rc == SID_OK) rc = setup_generator(e);
    if (rc != SID_OK) return rc;
    start_queues(e);
    const double t_setup = wall();
    const int D = (int)e->devs.size();
    // SID_ENGINE_TIMING: the first device's GPU timeline of the run -- its
    // start, and after the join the ends of its compute and D2H streams,
    // against its upload span (the head before the first copy, the tail
    // after the last)
    const bool timing = std::getenv("SID_ENGINE_TIMING") != nullptr;
    hipEvent_t tz[3] = {nullptr, nullptr, nullptr};
    if (timing) {
        Dev& d0 = *e->devs[0];
        for (auto& ev : tz) ev = d0.h2d_event();
        if (tz[0]) (void)hipEventRecord(tz[0], d0.s_up);
    }
    if (e->lynch)
        for (auto& dp : e->devs)
            if ((rc = sid_profile_reset(dp->ctx, dp->s_comp)) != SID_OK) return rc;
    std::vector<std::vector<uint64_t>> lists(D);
    for (uint64_t j = 0; j < e->recs.size(); ++j) lists[e->recs[j].dev].push_back(j);
    std::vector<std::function<void()>> th;
    for (int i = 0; i < D; ++i) {
        Dev& d = *e->devs[i];
        const std::vector<uint64_t>& li = lists[i];
        th.emplace_back([e, &d, &li] { uploader(e, d, li, 1); });
        th.emplace_back([e, &d] { compute(e, d, 1); });
    }
    // the emit's pinned ring, pinned on a thread of its own during the ingest
    // of a run that writes its records through it (no host arena, no device
    // sink); a failure here leaves the ring to the emit, which reports it
    if (e->cfg.device_sink == 0 && e->cfg.host_hold_bytes == 0)
        th.emplace_back([e] {
            for (auto& dp : e->devs) (void)alloc_ring(*dp);
        });
    const double t_spawn = wall();
    e->crew.run(th);
    const double t_join = wall();
    if (e->rc.load() != SID_OK) {
        close_all(e);
        for (auto& dp : e->devs) (void)hipSetDevice(dp->device), (void)hipDeviceSynchronize();
        return e->rc.load();
    }
    if (timing) {
        Dev& d0 = *e->devs[0];
        if (tz[1]) (void)hipEventRecord(tz[1], d0.s_comp);
        if (tz[2]) (void)hipEventRecord(tz[2], d0.s_d2h);
        (void)hipSetDevice(d0.device);
        float head = -1.f, tc = -1.f, td = -1.f;
        if (hipStreamSynchronize(d0.s_comp) == hipSuccess && hipStreamSynchronize(d0.s_d2h) == hipSuccess &&
            hipStreamSynchronize(d0.s_up) == hipSuccess && !d0.h2d_pending.empty() && tz[0] && tz[1] && tz[2]) {
            (void)hipEventElapsedTime(&head, tz[0], d0.h2d_pending.front().first);
            (void)hipEventElapsedTime(&tc, d0.h2d_pending.back().second, tz[1]);
            (void)hipEventElapsedTime(&td, d0.h2d_pending.back().second, tz[2]);
        }
        (void)hipGetLastError();
        for (auto ev : tz)
            if (ev) d0.h2d_free.push_back(ev);
        std::fprintf(stderr,
                     "{\"ingest_setup_s\": %.6f, \"budgets_s\": %.6f, \"spawn_s\": %.6f, \"join_s\": %.6f, "
                     "\"gpu_head_ms\": %.3f, \"gpu_tail_comp_ms\": %.3f, \"gpu_tail_d2h_ms\": %.3f, \"join_after_ms\": %.3f}\n",
                     t_setup - t0, t_budget - t0, t_spawn - t_setup, t_join - t_spawn, head, tc, td,
                     (wall() - t_join) * 1e3);
    }
    double h2d_s = 0;
    uint64_t h2d_bytes = 0, tiled = 0, tile_over = 0, tile_oq = 0;
    for (auto& dp : e->devs) {
        (void)hipSetDevice(dp->device);
        if (hipStreamSynchronize(dp->s_comp) != hipSuccess || hipStreamSynchronize(dp->s_up) != hipSuccess ||
            hipStreamSynchronize(dp->s_d2h) != hipSuccess)
            return SID_EHIP;
        h2d_s += dp->h2d_collect();
        h2d_bytes += dp->h2d_bytes;
        dp->h2d_bytes = 0;
        tiled += dp->tiled;
        tile_over += dp->tile_overflows;
        tile_oq += dp->tile_over_queued;
        dp->tiled = dp->tile_overflows = dp->tile_over_queued = 0;
    }
    uint64_t sites = 0, bytes = 0, held = 0, kept = 0;
    for (auto& r : e->recs) {
        sites += r.parsed;
        bytes += r.len;
        held += r.held != nullptr || r.host1 || r.sunk;
        kept += r.kept != nullptr;
    }
    if (st) {
        st->sites = sites;
        st->chunks = e->recs.size();
        st->bytes_in = e->src == SRC_SYNTH_HOST || e->src == SRC_SYNTH_DEVICE ? 0 : bytes;
        st->chunks_held = held;
        st->chunks_retained = kept;
        st->devices = D;
        st->status_kind = 0;
        st->err_offset = 0;
        st->ingest_s = wall() - t0;
        st->chunks_registered = e->reg_chunks.load();
        st->register_s = e->t_register.load() * 1e-9;
        st->h2d_s = h2d_s;
        st->h2d_bytes = h2d_bytes;
        st->chunks_tiled = tiled;
        st->tile_overflows = tile_over;
        st->tile_overflows_queued = tile_oq;
    }
    timing_report(e, "ingest", wall() - t0);
    const uint64_t fe = e->first_err.load();
    if (fe != UINT64_MAX) {
        const ChunkRec& r = e->recs[fe];
        const unsigned kind = (unsigned)(r.err & 7);
        const int prc = kind == 1 ? SID_EMALFORMED : kind == 2 ? SID_ENULLCHROM : kind == 3 ? SID_EMISSING_MQ
                                                                                             : SID_ENOBQ;
        if (st) {
            st->status_kind = prc;
            st->err_offset = r.off + (r.err >> 3);
        }
        return prc;
    }
    e->ingested = true;
    e->estimated = !e->lynch;
    return SID_OK;
}

// the pipelines' Lynch histograms merged (KB-sized tables) and loaded into
// every context, once per ingest (a second estimate, or a table loaded with
// sid_engine_profile_load, must not be merged again)
static int merge_histograms(sid_engine* e)
{
    const int D = (int)e->devs.size();
    if (D == 1 || e->hist_merged) {
        e->hist_merged = true;
        return SID_OK;
    }
    std::vector<std::vector<uint64_t>> k(D), v(D);
    std::vector<int> rcs(D, SID_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < D; ++i)
        th.emplace_back([&, i] {
            size_t u = 0;
            sid_ctx* c = e->devs[i]->ctx;
            rcs[i] = sid_profile_table(c, nullptr, nullptr, 0, &u);
            if (rcs[i]) return;
            k[i].resize(u);
            v[i].resize(u);
            rcs[i] = sid_profile_table(c, k[i].data(), v[i].data(), u, &u);
        });
    for (auto& t : th) t.join();
    for (int r : rcs)
        if (r) return r;
    std::vector<uint64_t> K, V;
    for (int i = 0; i < D; ++i) {
        K.insert(K.end(), k[i].begin(), k[i].end());
        V.insert(V.end(), v[i].begin(), v[i].end());
    }
    for (int i = 0; i < D; ++i) {
        const int rc = sid_profile_load(e->devs[i]->ctx, K.data(), V.data(), K.size());
        if (rc != SID_OK) return rc;
    }
    e->hist_merged = true;
    return SID_OK;
}

extern "C" int sid_engine_profile_table(sid_engine* e, uint64_t* keys, uint64_t* counts64, size_t cap, size_t* u)
{
    if (!e || !u) return SID_EINVAL;
    if (!e->ingested || !e->lynch) return SID_ESTATE;
    const int rc = merge_histograms(e);
    if (rc != SID_OK) return rc;
    return sid_profile_table(e->devs[0]->ctx, keys, counts64, cap, u);
}

extern "C" int sid_engine_profile_load(sid_engine* e, const uint64_t* keys, const uint64_t* counts64, size_t u)
{
    if (!e || (!keys && u) || (!counts64 && u)) return SID_EINVAL;
    if (!e->ingested || !e->lynch) return SID_ESTATE;
    for (auto& dp : e->devs) {
        const int rc = sid_profile_load(dp->ctx, keys, counts64, u);
        if (rc != SID_OK) return rc;
    }
    e->hist_merged = true;
    return SID_OK;
}

extern "C" int sid_engine_records(sid_engine* e, uint64_t chunk, const char** bytes, uint64_t* len)
{
    if (!e || !bytes || !len || chunk >= e->recs.size()) return SID_EINVAL;
    const ChunkRec& r = e->recs[chunk];
    if (!r.host) return SID_ESTATE;
    *bytes = r.host;
    *len = r.host_len;
    return SID_OK;
}

extern "C" int sid_engine_estimate(sid_engine* e, const sid_estimate* given, sid_estimate* out)
{
    if (!e || !e->ingested) return SID_ESTATE;
    if (!e->lynch) {
        e->estimated = true;
        return SID_OK;
    }
    const int D = (int)e->devs.size();
    const int verbose = e->cfg.verbose;
    int rc = merge_histograms(e);
    if (rc != SID_OK) return rc;
    // one estimate (device 0, prints the reference's lines), the others
    // classify with its (pi, eps)
    sid_estimate est{};
    rc = sid_lynch_prepare_given(e->devs[0]->ctx, verbose, given, &est);
    if (rc != SID_OK) return rc;
    if (D > 1) {
        std::vector<int> rcs(D, SID_OK);
        std::vector<std::thread> th;
        for (int i = 1; i < D; ++i)
            th.emplace_back([&, i] { rcs[i] = sid_lynch_prepare_given(e->devs[i]->ctx, 0, &est, nullptr); });
        for (auto& t : th) t.join();
        for (int r : rcs)
            if (r) return r;
    }
    const int m = e->opts.method;
    if (m == SID_METHOD_LOCAL || m == SID_METHOD_QUALITY)   // -R: call.cpp:223-234, :305
        for (auto& dp : e->devs)
            if ((rc = sid_set_prior(dp->ctx, est.heterozygosity)) != SID_OK) return rc;
    e->est = est;
    if (out) *out = est;
    e->estimated = true;
    return SID_OK;
}

extern "C" int sid_engine_emit(sid_engine* e, const char* header, sid_write_fn write, void* user,
                               sid_run_stats* st)
{
    if (!e || !e->ingested || !e->estimated) return SID_ESTATE;
    const int sink = e->cfg.device_sink;   // 0 write, 1 HBM only, 2 D2H only
    if (sink == 0 && !write) return SID_EINVAL;
    const double t0 = wall();
    e->rc = SID_OK;
    e->reloaded = 0;
    e->sink_bytes = 0;
    for (const auto& r : e->recs)
        if (r.sunk) e->sink_bytes += r.held_len;   // formatted and dropped in pass 1
    // every chunk's records already in the host arena (-m local / quality
    // with host_hold_bytes): nothing left for the devices, only the writes
    bool all_host = sink != 1;
    for (const auto& r : e->recs) all_host = all_host && r.host1;
    if (all_host) {
        uint64_t out = 0;
        bool ok = !(sink == 0 && header && write(user, header, std::strlen(header)) != 0);
        for (const auto& r : e->recs) {
            if (ok && sink == 0 && r.host_len && write(user, r.host, r.host_len) != 0) ok = false;
            out += r.host_len;
        }
        if (st) {
            st->chunks_reloaded = 0;
            st->bytes_out = out;
            st->emit_s = wall() - t0;
        }
        timing_report(e, "emit", wall() - t0);
        e->ingested = false;
        return ok ? SID_OK : SID_EIO;
    }
    // the device sink with every chunk's records held in HBM since pass 1: no
    // pass 2 for the devices (the ingest synchronised their streams), only the
    // byte count -- no threads to start for a run that has nothing left to do
    bool all_held = sink == 1 && !e->recs.empty();
    for (const auto& r : e->recs) all_held = all_held && (r.held || r.sunk);
    if (all_held) {
        uint64_t out = 0;
        for (auto& r : e->recs) {
            Dev& d = *e->devs[r.dev];
            out += r.held_len;
            if (r.held) d.pool.put(r.held, r.held_cap, nullptr);
            if (r.kept) d.pool.put(r.kept, r.kept_cap, nullptr);
            if (r.pre) d.pool.put(r.pre, r.pre_cap, nullptr);
            r.held = r.kept = r.pre = nullptr;
        }
        e->sink_bytes = out;
        if (st) {
            st->chunks_reloaded = 0;
            st->bytes_out = out;
            st->emit_s = wall() - t0;
        }
        timing_report(e, "emit", wall() - t0);
        e->ingested = false;
        return SID_OK;
    }
    start_queues(e);
    const int D = (int)e->devs.size();
    if (sink != 1)
        for (auto& dp : e->devs) {
            Dev& d = *dp;
            const int rc = alloc_ring(d);
            if (rc != SID_OK) return rc;
            for (int i = 0; i < EMIT_RING_N; ++i) d.free_pinned.push(i);
        }
    std::vector<std::vector<uint64_t>> lists(D);
    for (uint64_t j = 0; j < e->recs.size(); ++j) lists[e->recs[j].dev].push_back(j);
    std::atomic<uint64_t> out_bytes{0};
    std::vector<std::function<void()>> th;
    for (int i = 0; i < D; ++i) {
        Dev& d = *e->devs[i];
        const std::vector<uint64_t>& li = lists[i];
        th.emplace_back([e, &d, &li] { uploader(e, d, li, 2); });
        th.emplace_back([e, &d] { compute(e, d, 2); });
        if (sink != 1) th.emplace_back([e, &d] { drain(e, d); });
    }
    e->crew.start(th);
    // the writer: header, then every chunk's pieces in file order
    if (sink != 1) {
        bool ok = true;
        if (sink == 0 && header && write(user, header, std::strlen(header)) != 0) ok = false;
        for (uint64_t j = 0; j < e->recs.size() && e->rc.load() == SID_OK; ++j) {
            Dev& d = *e->devs[e->recs[j].dev];
            const ChunkRec& rj = e->recs[j];
            if (rj.host1) {   // copied back during the ingest (which waited for the copies)
                if (ok && sink == 0 && rj.host_len && write(user, rj.host, rj.host_len) != 0) ok = false;
                out_bytes += rj.host_len;
                if (!ok) break;
                continue;
            }
            Piece p;
            bool got_last = false;
            while (d.out_q.pop(p)) {
                if (p.host) {
                    const double w0 = wall();
                    const hipError_t ws = hipEventSynchronize(p.hev);
                    e->t_write_wait += (uint64_t)((wall() - w0) * 1e9);
                    d.give_event(p.hev);
                    if (ws != hipSuccess) {
                        fail(e, SID_EHIP);
                        break;
                    }
                    if (ok && sink == 0 && write(user, p.host, p.len) != 0) ok = false;
                    out_bytes += p.len;
                } else if (p.ps >= 0) {
                    const double w0 = wall();
                    const hipError_t ws = hipEventSynchronize(d.pinned_ev[p.ps]);
                    e->t_write_wait += (uint64_t)((wall() - w0) * 1e9);
                    if (ws != hipSuccess) {
                        fail(e, SID_EHIP);
                        break;
                    }
                    if (ok && sink == 0 && write(user, d.pinned[p.ps], p.len) != 0) ok = false;
                    out_bytes += p.len;
                    d.free_pinned.push(p.ps);
                }
                if (p.last) {
                    d.pool.put(p.buf, p.cap, nullptr);   // its D2H completed (event above)
                    got_last = true;
                    break;
                }
            }
            if (!ok) fail(e, SID_EIO);
            if (!got_last) break;
        }
        if (!ok) fail(e, SID_EIO);
        if (e->rc.load() != SID_OK) close_all(e);
    }
    e->crew.wait();
    for (auto& dp : e->devs) {
        (void)hipSetDevice(dp->device);
        if (hipDeviceSynchronize() != hipSuccess) fail(e, SID_EHIP);
    }
    if (st) {
        st->chunks_reloaded = e->reloaded.load();
        st->bytes_out = sink == 1 ? e->sink_bytes.load() : out_bytes.load();
        st->emit_s = wall() - t0;
    }
    timing_report(e, "emit", wall() - t0);
    // every held / kept buffer went back to the pools
    for (auto& r : e->recs) {
        Dev& d = *e->devs[r.dev];
        if (r.held) d.pool.put(r.held, r.held_cap, nullptr);
        if (r.kept) d.pool.put(r.kept, r.kept_cap, nullptr);
        if (r.pre) d.pool.put(r.pre, r.pre_cap, nullptr);
        r.held = r.kept = r.pre = nullptr;
    }
    e->ingested = false;
    return e->rc.load();
}

extern "C" int sid_engine_run(sid_engine* e, const char* header, sid_write_fn write, void* user,
                              sid_run_stats* st)
{
    if (!e) return SID_EINVAL;
    sid_run_stats local{};
    sid_run_stats* s = st ? st : &local;
    std::memset(s, 0, sizeof *s);
    int rc = sid_engine_ingest(e, s);
    if (rc != SID_OK) return rc;
    const double t0 = wall();
    rc = sid_engine_estimate(e, nullptr, &s->estimate);
    s->estimate_s = wall() - t0;
    if (rc != SID_OK) return rc;
    return sid_engine_emit(e, header, write, user, s);
}

extern "C" int sid_engine_profile(sid_engine* e, int enable)
{
    if (!e) return SID_EINVAL;
    e->prof = enable != 0;
    return SID_OK;
}

// sums the pending event pairs of every device (after their streams drained)
extern "C" int sid_engine_profile_read(sid_engine* e, sid_engine_prof* out)
{
    if (!e || !out) return SID_EINVAL;
    for (auto& dp : e->devs) {
        Dev& d = *dp;
        if (hipSetDevice(d.device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SID_EHIP;
        for (auto& pr : d.prof_pending) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, pr.second.first, pr.second.second) == hipSuccess) e->prof_ms[pr.first] += ms;
            d.prof_free.push_back(pr.second.first);
            d.prof_free.push_back(pr.second.second);
        }
        d.prof_pending.clear();
        e->prof_chunks += d.prof_chunks;
        d.prof_chunks = 0;
    }
    std::memset(out, 0, sizeof *out);
    out->chunks = e->prof_chunks;
    out->index_ms = e->prof_ms[0];
    out->parse_ms = e->prof_ms[1];
    out->call_ms = e->prof_ms[2];
    out->hist_ms = e->prof_ms[3];
    out->fmt_len_ms = e->prof_ms[4];
    out->fmt_write_ms = e->prof_ms[5];
    for (double& v : e->prof_ms) v = 0;
    e->prof_chunks = 0;
    return SID_OK;
}
