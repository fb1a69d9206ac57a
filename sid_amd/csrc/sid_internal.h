// sid_internal.h — libsid.so internals shared by the C-ABI translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/sid.h"
#include "sid_math.h"

// Second-level class table of -m local (L2-resident, 4 MiB): (nf, ns, r2)
// with nf < 512, ns < 128, r2 < 8 covers the 30x and 200x het sites (ns >= 8) and the
// 200x sites with r2 >= 4 that the LDS table (nf < 256, ns < 8, r2 < 4) leaves out.
#define SID_TAB2_NF 512
#define SID_TAB2_NS 128
#define SID_TAB2_NR 8
#define SID_TAB2_N (SID_TAB2_NF * SID_TAB2_NS * SID_TAB2_NR)

// -m local workspace (class table + miss list), one per context
struct sid_local_ws {
    double* table = nullptr;     // SID_TAB_N entries (local.hip), copied to LDS
    double* table2 = nullptr;    // SID_TAB2_N entries, the fix-up's L2-resident table
    uint32_t* miss = nullptr;    // miss list
    uint32_t cap = 0;            // miss list capacity
    uint32_t* ctr = nullptr;     // [2] miss counters, alternating per call
    int parity = 0;
    int table_grid = 4096;       // blocks of the table kernel (2 resident per CU; 8 rounds)
    int tail = 1;                // SID_TABLE_TAIL=0: no inline second-level lookup, every miss to the fix-up
    hipEvent_t ev_mid = nullptr; // set only while timing: recorded between main and fix-up
    // the record tails per class entry (the engine's -m local formatter):
    // SID_STR_BYTES per entry of table / table2 (local.hip), and their lengths
    char* str1 = nullptr;
    uint8_t* len1 = nullptr;
    char* str2 = nullptr;
    uint8_t* len2 = nullptr;
};
#define SID_STR_BYTES 32   // entry: [0] tail length, [1] het, [8..32) the tail, zero-padded
#define SID_STR_TEXT 8

struct sid_timing_ev {
    hipEvent_t start, mid, end;
};

// kernels (local.hip, synth.hip, lynch.hip)
extern "C" hipError_t sid_launch_local(const uint16_t* counts, size_t n, uint8_t* code,
                                       double* hom, double* het, const sid_local_k* K,
                                       const double* d_lnt, const sid_local_ws* ws, int grid_cap,
                                       hipStream_t stream);
extern "C" hipError_t sid_launch_local_table_build(const sid_local_k* K, const double* d_lnt,
                                                   double* d_table, double* d_table2, hipStream_t stream);
extern "C" hipError_t sid_launch_local_str_build(const sid_local_k* K, const double* d_table, const double* d_table2,
                                                 const sid_local_ws* ws, hipStream_t stream);
extern "C" hipError_t sid_launch_synth(uint64_t seed, uint64_t first, size_t n,
                                       const uint64_t* d_cdf, uint32_t kmax, uint16_t* counts,
                                       hipStream_t stream);

// Lynch-path device state (lynch.hip)
struct sid_lynch_dev;
sid_lynch_dev* sid_lynch_dev_create(int* err);
void sid_lynch_dev_destroy(sid_lynch_dev* L);

// The Lynch classes as the engine's fused formatter reads them (after
// sid_lynch_prepare for likelihood_ratio / bayes): a site's class is
// dense_cidx[dense code] or, for the other profiles, the class hash
// (ckeys / cidx / cmask / special_idx); none = the profile was filtered (no
// record).  Per class SID_LSTR_BYTES of record tail: [0] its length, from
// [8] "label,gt,conf1,conf2,conf_type\n"; dlen[d] = the tail length of
// dense code d's class (0: none).
#define SID_LSTR_BYTES 64
struct sid_lynch_fmt {
    const uint32_t* dense_cidx;
    const unsigned long long* ckeys;
    const uint32_t* cidx;
    uint64_t cmask;
    uint32_t special_idx;
    const char* lstr;
    const uint8_t* dlen;
    int empty;   // no class at all: every site dropped
};
int sid_lynch_fmt_view(const sid_ctx* c, sid_lynch_fmt* v);
// textpath.hip: the tails of the U classes and the dense codes' lengths
hipError_t sid_launch_lynch_str_build(const uint8_t* pcode, const double* cc, uint32_t U, const char* conf_type,
                                      const uint32_t* dense_cidx, char* lstr, uint8_t* dlen, uint32_t* bad,
                                      hipStream_t st);

#define SID_STAGE_N 8                   // reader threads / pinned input buffers
#define SID_STAGE_BYTES (16u << 20)     // bytes per input buffer

struct sid_ctx {
    int device = 0;
    sid_opts opts{};
    sid_local_k K{};
    double* d_lnt = nullptr;     // ln(k), k < SID_LUTN
    int grid_cap = 2048;
    // synthetic generator: Poisson CDF thresholds for the last mean depth
    uint64_t* d_cdf = nullptr;
    uint32_t cdf_k = 0;
    double cdf_mean = -1.0;
    sid_local_ws ws;
    // measurement (sid_timing_enable / sid_timing_read)
    int timing = 0;
    std::vector<sid_timing_ev> ev_pool, ev_pending;
    // Lynch path
    sid_lynch_dev* lynch = nullptr;
    // device CSV formatter (textpath.hip): staging kept for the context's
    // lifetime (pinning host memory costs ~5 GB/s, too slow per call)
    char* fmt_d[2] = {nullptr, nullptr};
    char* fmt_h[2] = {nullptr, nullptr};
    size_t fmt_cap[2] = {0, 0};
    // sid_dtext_parse_fd: pinned read staging, one buffer per reader thread
    char* in_h[SID_STAGE_N] = {};
    // -m quality (textpath.hip): per-quality terms and log_gamma, host-computed
    double* d_qtab = nullptr;   // 4 x 256
    double* d_lg = nullptr;     // log_gamma(x), x < lg_n
    size_t lg_n = 0;
    uint32_t* d_scratch = nullptr;
    double* d_qlo = nullptr;    // -m quality phase 1 -> 2: lo parts of the two sums, 16 B per site
    size_t qlo_n = 0;
};

// ----------------------------------------------------- chunk pipeline ----
// textpath.hip: one line-aligned chunk of text resident on the device,
// processed in place by the streaming engine (run.cpp).  Grow-only device
// workspace; every function is asynchronous on `st`.
//
// Invariant: the chunk is the bytes [c0, c1) of `base`, and every kernel
// bounds what it USES by c1.  The bytes past c1 (at least 256 readable, for
// whole 16-B windows) are NOT zero: a ring slot keeps a previous, longer
// chunk's text there, and resident text has the next chunk there.  A kernel
// may load them but must mask them (as the index's line-start masks, the
// parse's token scans and the formatters do); a kernel that needs NUL
// padding must write it itself (tests/test_engine_gpu.py
// test_stale_ring_slot_behind_a_last_line_without_newline).
//
// Line offsets of a chunk, relative to its 16-B aligned base: 32 bits (a
// chunk spans less than 4 GiB; sid_chunk_index refuses a longer one), 4 B a
// site written by the index and read by the parse (the whole-text sid_dtext_*
// path keeps 64-bit offsets)
typedef uint32_t sid_off_t;
constexpr uint64_t SID_CHUNK_MAX = (4ull << 30) - (1ull << 20);   // bytes a chunk may span

struct sid_chunk_ws {
    uint64_t site_cap = 0, tile_cap = 0;
    sid_off_t* starts = nullptr;  // line start offsets (relative to the chunk's base)
    uint64_t* counts = nullptr;   // profile_t per site
    uint64_t* hdr = nullptr;      // per site for the formatter: (chrom / position word, chrom's first 8 bytes)
    uint32_t* fb = nullptr;       // three site lists of site_cap entries: the lines the first parse pass
                                  // leaves (count in state[6]); the second pass's leftovers, or the lines the
                                  // general routine parsed for the fused -m local lengths ([7]); the
                                  // -m local fix-up's sites (lb[0])
    bool lens_ready = false;      // the parse computed the -m local record lengths (sid_chunk_parse lctx)
    uint32_t* cls = nullptr;      // with lens_ready: per site its -m local class word (the table entry and the
                                  // major / minor bases, or SID_CLS_MISS); the counts are then written only for
                                  // the fix-up's sites
    bool cls_ready = false;       // cls holds this chunk's words (set by the parse, read by sid_chunk_local_put)
    ulonglong2* twv = nullptr;    // the tile parse's wave entries (-m local, lane shape: chrom and position
                                  // of the compact class words; site_cap / 32 + 1)
    uint8_t* code = nullptr;
    double* hom = nullptr;
    double* het = nullptr;
    uint32_t* tcnt = nullptr;     // per 16 KiB tile line counts (+ scan workspace)
    uint64_t* toff = nullptr;
    uint32_t* bsum = nullptr;     // per 256-site block record bytes (+ scan workspace)
    uint64_t* boff = nullptr;
    uint16_t* masks = nullptr;    // line-start masks of the index, a u16 per lane per 4 KiB tile
    unsigned long long* lb = nullptr;   // formatter flags and totals (sid_chunk_fmt_len)
    uint64_t* state = nullptr;    // [0] sites [1..2] parse range [3] CSV bytes [4] first error key [5] range flag
                                  // [6] [7] fallback lines
    uint32_t slot_cap = 0;        // 0: sites in file order (index + parse); else the tile parse's layout: slots
    uint64_t slots = 0;           // of slot_cap per tile, `slots` of them (sid_chunk_tile_local)
    bool tile_quad = false;       // the tile parse's shape (the compaction; the -m local writer: wave entries or not)
    uint64_t tile_ntp = 0;
};
int sid_chunk_reserve(sid_chunk_ws* W, uint64_t bytes, uint64_t sites);
void sid_chunk_release(sid_chunk_ws* W);
int sid_chunk_index(sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, hipStream_t st);
// lctx (optional, -m local with class tables, sid_chunk_local_ok): the
// records' lengths computed by the parse, for sid_chunk_local_len next
int sid_chunk_parse(sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, uint64_t n, int qmode,
                    hipStream_t st, const sid_ctx* lctx = nullptr);
// the formatter: records of the n sites into out, which must hold
// sid_chunk_fmt_bound(n, text bytes).  _len: record bytes per 512-site block
// and their offsets; _put: the records.  Afterwards lb[1], lb[2], lb[4] =
// {bytes, range flag, the chunk's parse error key (state[4])}.  The fmt_
// pair formats code / hom / het (any method's call kernel); the local_ pair
// is -m local fused with the call (counts in; sid_chunk_local_ok: options
// the class tables cover)
uint64_t sid_chunk_fmt_bound(uint64_t n, uint64_t text_bytes);
int sid_chunk_fmt_len(sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, const char* conf_type,
                      hipStream_t st);
int sid_chunk_fmt_put(sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, const char* conf_type, char* out,
                      hipStream_t st);
bool sid_chunk_local_ok(const sid_ctx* ctx);
int sid_chunk_local_len(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n,
                        const char* conf_type, hipStream_t st);
int sid_chunk_local_put(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n,
                        const char* conf_type, char* out, hipStream_t st);
// -m local (sid_chunk_local_ok) in one pass over the text: the tile parse of
// [c0, c1) with cap slots per tile (a multiple of 16, SID_TILE_CAP_MIN .. _MAX), the
// record lengths, the fix-up and the writer's offsets; sid_chunk_local_put
// then writes the records into a buffer of sid_chunk_tile_bound.  No host
// round trip inside.  Afterwards lb[1] bytes, lb[2] range flag, lb[3] sites,
// lb[4] the parse error key (after the put), lb[5] the most lines in one tile:
// above the cap the chunk's results are void (run it again with a larger cap,
// or through sid_chunk_index + sid_chunk_parse).  quad: 24 KiB tiles and a
// quad of lanes per line (lines over 256 B on average), else 20 KiB tiles and
// a lane per line.
constexpr uint32_t SID_TILE_CAP_MIN = 64, SID_TILE_CAP_MAX = 1024;   // slots per tile (multiples of 16)
constexpr uint32_t SID_TILE_CAP_MAX_QUAD = 256;                       // ... of the quad shape
uint64_t sid_chunk_tile_slots(uint64_t c0, uint64_t c1, uint32_t cap, bool quad);
uint32_t sid_tile_unit(bool quad);   // text bytes per tile (the slot layout's unit)
uint64_t sid_chunk_tile_bound(uint64_t c0, uint64_t c1, uint32_t cap, bool quad);
int sid_chunk_tile_local(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, uint32_t cap,
                         bool quad, const char* conf_type, hipStream_t st);
// The Lynch paths' first pass in one pass over the text: the tile parse of
// [c0, c1) into every site's counts and header pair (slots as above), the
// general routine's lines, and the tiles' prefix; afterwards state[0] = the
// chunk's sites, state[4] the parse error key, lb[5] the most lines in one
// tile (above the cap: void, as sid_chunk_tile_local).  Then
// sid_chunk_tile_compact writes the sites in file order into the caller's
// arrays (line offsets, counts, header pairs: the two-pass parse's layout).
int sid_chunk_tile_counts(sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, uint32_t cap, bool quad,
                          hipStream_t st);
int sid_chunk_tile_compact(sid_chunk_ws* W, sid_off_t* starts, uint64_t* counts, uint64_t* hdr, hipStream_t st);
// likelihood_ratio / bayes fused with the class lookup (sid_lynch_fmt_view)
int sid_chunk_lynch_len(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, hipStream_t st);
int sid_chunk_lynch_put(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, char* out,
                        hipStream_t st);
int sid_chunk_quality(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, hipStream_t st);
// synth.hip: the synthetic text of sites [first, first + n) (the bytes of
// sid_synth_text) generated on the device into out (cap bytes): res[0] =
// bytes, res[1] != 0 when they did not fit (nothing usable written then)
struct sid_synth_gen_ws {
    uint32_t* len = nullptr;      // per site line length (+ scan workspace)
    uint64_t* off = nullptr;      // per site line offset
    uint64_t* res = nullptr;      // [0] bytes, [1] overflow
    uint64_t cap = 0;             // sites
};
hipError_t sid_launch_synth_text(uint64_t seed, const uint64_t* d_cdf, uint32_t kmax, uint64_t first, uint64_t n,
                                 uint64_t sites_per_chrom, sid_synth_gen_ws* ws, char* out, uint64_t cap,
                                 hipStream_t st, double mean_depth);
void sid_synth_gen_release(sid_synth_gen_ws* ws);
// textpath.hip: exclusive u32 -> u64 scan (three kernels) from *base
size_t sid_scan_ws_bytes(uint64_t m);
hipError_t sid_scan_u32(const uint32_t* in, uint64_t m, uint64_t* out, uint64_t* base, uint64_t* ws, hipStream_t st);

// host helpers (capi.cpp)
int sid_set_hip_error(hipError_t e);
double sid_gsl_lngamma(double x);   // GSL 2.7.1 gsl_sf_lngamma restated (x >= 0.5)
void sid_build_local_k(const sid_opts& o, sid_local_k* K);
// Poisson(mean) CDF as 64-bit thresholds (synth.h); returns kmax
uint32_t sid_poisson_cdf(double mean, std::vector<uint64_t>& cdf);
