/*
 * sid.h — C ABI of libsid.so, the MI355X-native per-site genotype caller.
 *
 * Drop-in boundary.  EvolBioInf/sid has no plugin/FFI API; its internal seam
 * is the four method functions declared at call.hpp:40-43,
 *     std::vector<OutputRecord> callX(std::istream&, ...)
 * called only from sid.cpp:92-100.  This header replaces that seam with plain
 * pointers and sizes (no C++ or torch types), split where the data crosses the
 * host/device boundary:
 *
 *   host text --(sid_parse_*: pileup.cpp:13-153)--> SoA counts (u16 x 4 per site)
 *   counts --(sid_call_local / sid_profile_* + sid_lynch_* + sid_lookup_sites:
 *             call.cpp:62-289, lynch.hpp/.cpp, stats.cpp)--> code + 2 x f64 per site
 *   code + confs --(sid_format_csv: call.hpp:29-38, sid.cpp:102-105)--> CSV text
 *
 * Conventions
 *   - Caller owns every buffer.  "device" pointers are HIP device memory
 *     (hipMalloc / torch); "host" pointers are ordinary or pinned host memory.
 *   - No exception crosses the ABI: every function returns SID_OK (0) or a
 *     SID_E* status; sid_strerror() names it.
 *   - Device work is asynchronous on the caller's stream (hipStream_t passed as
 *     void*, NULL = default stream) unless the function says it synchronises.
 *   - One sid_ctx per device and host thread (thread-compatible, not
 *     thread-safe).
 *   - Per-site result code: bits 0-1 = gt[0] base (0..3 = A,C,G,T), bits 2-3 =
 *     gt[1] base, bit 7 = het label, bit 6 = site dropped (its profile was
 *     filtered, coverage < 4, and the reference prints no record for it:
 *     call.cpp:131-140).
 *   - Counts layout: profile_t (pileup.hpp:7) = 4 x uint16 {A,C,G,T} per site,
 *     array of structures, 8 bytes per site.
 */
#ifndef SID_H
#define SID_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- status -- */
enum {
    SID_OK = 0,
    SID_EINVAL = 1,      /* bad argument (null pointer, misuse)                     */
    SID_EHIP = 2,        /* HIP runtime error (sid_last_hip_error() has the code)   */
    SID_ENOMEM = 3,      /* host or device allocation failed                        */
    SID_EMALFORMED = 4,  /* "Malformed pileup line"                pileup.cpp:9       */
    SID_EMISSING_MQ = 5, /* "Malformed pileup line or missing mapping qualities" :10 */
    SID_ENULLCHROM = 6,  /* no first token: the reference assigns a NULL char* to a
                            std::string (pileup.cpp:18) and dies with SIGSEGV       */
    SID_ESTATE = 7,      /* call order violated (e.g. lookup before lynch_prepare)  */
    SID_EBADFUNC = 8,    /* non-finite objective at the simplex start: GSL would
                            abort (nmsimplex2 set; optimization.hpp:55)            */
    SID_EEMPTY = 9,      /* no profile with coverage >= 4: the reference indexes an
                            empty vector in adjustBenjaminiHochberg (stats.cpp:73) */
    SID_EIO = 10,        /* the output callback reported a write failure            */
    SID_ERANGE = 11,     /* a confidence outside the device formatter's range
                            (|v| >= 2^63; p-values and posteriors never are)        */
    SID_ENOBQ = 12,      /* -m quality, no base-quality field: parseQualities(NULL)
                            dereferences NULL (pileup.cpp:54,158): SIGSEGV          */
    SID_ELINE = 13,      /* a line that makes a chunk span 4 GiB or more (line
                            offsets on the device are 32-bit)                      */
};
const char* sid_strerror(int status);
int sid_last_hip_error(void);
/* Library version string, e.g. "sid-mi355x 0.1.0 (gfx950)". */
const char* sid_version(void);

/* --------------------------------------------------------------- options -- */
/* per-site result code bits (see Conventions) */
#define SID_CODE_HET 0x80
#define SID_CODE_DROPPED 0x40

enum { SID_METHOD_LOCAL = 0, SID_METHOD_LIKELIHOOD_RATIO = 1, SID_METHOD_BAYES = 2, SID_METHOD_QUALITY = 3 };

/* GlobalOptions, sid.cpp:11-17 */
typedef struct {
    int method;                  /* -m   (default SID_METHOD_LOCAL)                */
    int estimate_prior;          /* -R   (default 0)                               */
    double snp_prior;            /* -r   (default -1 = no prior)                   */
    double significance_level;   /* -p   (default 0.05)                            */
    double site_error_threshold; /* -E   (default 0.1)                             */
} sid_opts;
void sid_opts_default(sid_opts* o);

/* ------------------------------------------------------------- contexts -- */
typedef struct sid_ctx sid_ctx;
int sid_device_count(int* n);
/* Binds `device` (hipSetDevice) for the calling thread and builds the
 * per-context constant tables (log table, chi-square constants). */
int sid_create(int device, const sid_opts* opts, sid_ctx** out);
int sid_destroy(sid_ctx* ctx);
/* Replaces snp_prior after the -R estimate (call.cpp:223-234). */
int sid_set_prior(sid_ctx* ctx, double snp_prior);

/* ------------------------------------------------------- -m local (a5-a8) --
 * Per-site replacement of callSiteMLError's per-profile loop + per-site gather
 * (call.cpp:213-289; likelihoods lynch.hpp:48-55,76-80,92-96; LRT
 * stats.cpp:29-37).  counts/code/hom_conf/het_conf are device pointers. */
int sid_call_local(sid_ctx* ctx, const uint16_t* counts, size_t n, uint8_t* code,
                   double* hom_conf, double* het_conf, void* stream);

/* Measurement (bench.py): while enabled, sid_call_local records HIP events on
 * its stream around its main (class-table) kernel and its fix-up kernel.
 * sid_timing_read synchronises on them, returns the per-call averages of
 * the calls since the previous read, and resets. */
int sid_timing_enable(sid_ctx* ctx, int enable);
int sid_timing_read(sid_ctx* ctx, uint64_t* calls, double* main_ms, double* fixup_ms);

/* ---------------------------------------------- Lynch path (a11-a17) -------
 * 1. sid_profile_reset + sid_profile_accumulate (any number of batches):
 *    device hash histogram of the site profiles (countUniqueProfiles,
 *    pileup.cpp:169-196).
 * 2. optional multi-device / multi-rank merge: sid_profile_table exports the
 *    sorted unique profiles (cached until the histogram changes),
 *    sid_profile_load replaces the context's table by a merged one: the
 *    concatenated per-device tables may repeat keys, it sorts them and sums
 *    the counts of equal keys itself.
 * 3. sid_lynch_prepare: coverage >= 4 filter (call.cpp:66-70), nucleotide
 *    distribution (pileup.cpp:198-217), Nelder-Mead estimate of (pi, eps)
 *    with the objective evaluated on the GPU (lynch.cpp:17-61,
 *    optimization.hpp:50-89), per-profile 10-genotype likelihoods at eps-hat
 *    (lynch.hpp:57-74,82-90), then the per-method class table:
 *    likelihood_ratio: LRT + Benjamini-Hochberg (call.cpp:85-127,
 *    stats.cpp:58-80); bayes: posteriors (call.cpp:170-194); local -R: only
 *    the prior (use sid_set_prior + sid_call_local afterwards).
 * 4. sid_lookup_sites: per-site gather of the class table (call.cpp:129-140). */
typedef struct {
    double heterozygosity;   /* pi-hat   ("# heterozygosity: %e", call.cpp:79)   */
    double error_rate;       /* eps-hat  ("# error: %e", call.cpp:80)            */
    double fval;             /* objective at the returned vertex                */
    double dist[4];          /* nucleotide distribution                         */
    int iterations;          /* NM iterations (optimization.hpp:70)             */
    int converged;           /* 0: "did not converge in 1000 iterations"        */
    uint64_t evaluations;    /* objective evaluations                           */
    uint64_t n_unique;       /* profiles after the coverage filter ("# unique profiles") */
} sid_estimate;

int sid_profile_reset(sid_ctx* ctx, void* stream);
int sid_profile_accumulate(sid_ctx* ctx, const uint16_t* counts, size_t n, void* stream);
/* Synchronises.  keys[i] = A<<48 | C<<32 | G<<16 | T (numeric order ==
 * lexicographic profile_t order); counts64[i] = sites with that profile.
 * With keys == NULL only *u is returned. */
int sid_profile_table(sid_ctx* ctx, uint64_t* keys, uint64_t* counts64, size_t cap, size_t* u);
int sid_profile_load(sid_ctx* ctx, const uint64_t* keys, const uint64_t* counts64, size_t u);
/* Objective -sum count*log((1-pi)Lhom+pi*Lhet) over the filtered table at
 * (pi, eps), lynch.cpp:37-61.  Valid after sid_lynch_prepare (or
 * sid_lynch_setup).  Synchronises. */
int sid_lynch_setup(sid_ctx* ctx, sid_estimate* est /* dist, n_unique filled */);
int sid_lynch_objective(sid_ctx* ctx, double pi, double eps, double* out);
/* verbose != 0 prints the reference's "# ..." stderr lines. Synchronises.
 * -m bayes with no profile of coverage >= 4 succeeds and drops every site
 * (callBayes prints the header only); likelihood_ratio returns SID_EEMPTY. */
int sid_lynch_prepare(sid_ctx* ctx, int verbose, sid_estimate* est);
/* The same with (pi-hat, eps-hat) taken from `given` (an estimate another
 * device or rank computed on the same merged table, SURVEY.md §8(e) steps
 * 3-4): no Nelder-Mead here, only the per-profile classification.  Prints
 * only the "# unique profiles" line when verbose. */
int sid_lynch_prepare_given(sid_ctx* ctx, int verbose, const sid_estimate* given, sid_estimate* est);
int sid_lookup_sites(sid_ctx* ctx, const uint16_t* counts, size_t n, uint8_t* code,
                     double* hom_conf, double* het_conf, void* stream);

/* ----------------------------------------------------- synthetic input -----
 * Counter-based generator (BASELINE.md "Synthetic generator"): site i of a
 * run is a pure function of (seed, first_site + i), identical on host and
 * device.  sites_per_chrom splits the run into chromosomes chr1, chr2, ...
 * (positions restart at 1; keeps positions < 2^31). */
int sid_synth_counts(sid_ctx* ctx, uint64_t seed, double mean_depth, uint64_t first_site,
                     size_t n, uint16_t* counts /* device */, void* stream);
/* The same text generated on the device into out (cap bytes, device memory),
 * stream-ordered, then synchronised: *len = its bytes; SID_ERANGE when they
 * exceed cap (then out holds no usable text). */
int sid_synth_text_device(sid_ctx* ctx, uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                          uint64_t sites_per_chrom, char* out /* device */, size_t cap, size_t* len, void* stream);
/* Host text of sites [first_site, first_site+n).  Returns the bytes needed in
 * *len; writes at most cap bytes (call with buf == NULL to size). */
int sid_synth_text(uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                   uint64_t sites_per_chrom, char* buf, size_t cap, size_t* len);
/* The same text with a 7th column of mapping qualities (samtools mpileup -s,
 * uniform 0..60 per read), as the quality method requires. */
int sid_synth_text_mq(uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                      uint64_t sites_per_chrom, char* buf, size_t cap, size_t* len);
/* Host counts of the same sites (for tests; no GPU needed). */
int sid_synth_counts_host(uint64_t seed, double mean_depth, uint64_t first_site, size_t n,
                          uint16_t* counts);

/* ------------------------------------------------------ host parser --------
 * parsePileupLine / parseReadBases semantics (pileup.cpp:13-153) over a text
 * buffer, multi-threaded.  Empty lines are skipped (call.cpp:14).  On a
 * malformed line the status is SID_EMALFORMED / SID_ENULLCHROM and
 * *err_line is the 0-based line number of the first bad line. */
typedef struct sid_sites sid_sites;
int sid_parse_text(const char* text, size_t len, int nthreads, sid_sites** out,
                   uint64_t* err_line);
void sid_sites_free(sid_sites* s);
size_t sid_sites_count(const sid_sites* s);
const uint16_t* sid_sites_counts(const sid_sites* s);   /* host, n x 4          */
const int32_t* sid_sites_positions(const sid_sites* s); /* host, n              */
/* Chromosome runs: segment k covers sites [start_k, start_{k+1}). */
size_t sid_sites_chrom_segments(const sid_sites* s);
const char* sid_sites_chrom_name(const sid_sites* s, size_t k, uint64_t* start);

/* ------------------------------------------------------ CSV emitter --------
 * Formats records [begin, end) exactly like operator<<(OutputRecord)
 * (call.hpp:29-38: chrom,pos,label,gt,%g,%g,conf_type) into buf; sites with
 * code bit 6 set are skipped.  conf_type: "p_value" or "probability".
 * Returns bytes written in *len, or SID_ENOMEM if cap is too small (then *len
 * is a sufficient size). */
int sid_format_csv(const sid_sites* s, size_t begin, size_t end, const uint8_t* code,
                   const double* hom_conf, const double* het_conf, const char* conf_type,
                   char* buf, size_t cap, size_t* len);
/* %g formatting of one double exactly as std::ostream does (precision 6). */
int sid_format_double(double v, char* buf, size_t cap);

/* ------------------------------------ device text path
 * The same parse and the same CSV, on the device: the text of one shard is
 * copied to HBM, indexed (line starts) and parsed there, and stays resident
 * (the formatter re-reads chrom and pos from it).
 *
 * sid_dtext_parse: host text -> device counts (sid_dtext_counts, 4 x u16 per
 *   non-empty line, as sid_parse_text).  Synchronises.  `chunk` (0 = 256 MiB)
 *   is the size of the individual host-to-device copies.  On a malformed line
 *   returns SID_EMALFORMED or SID_ENULLCHROM for the first one in file order
 *   and its byte offset in *err_offset; *out stays NULL.
 * sid_dtext_format: the records of sites [begin, end) with the given device
 *   code/confs, formatted on the device and handed to write() in order, in
 *   pieces valid only during the call (write returns 0, else SID_EIO).
 *   Synchronises. */
typedef struct sid_dtext sid_dtext;
typedef int (*sid_write_fn)(void* user, const char* bytes, size_t len);
int sid_dtext_parse(sid_ctx* ctx, const char* text, size_t len, size_t chunk, sid_dtext** out,
                    uint64_t* err_offset, void* stream);
/* The same for bytes [offset, offset+len) of an open file (offset at a line
 * start): `threads` host threads (0 = 8) pread() into pinned staging owned by
 * the context, each buffer DMA'd to HBM as it fills -- no file mapping. */
int sid_dtext_parse_fd(sid_ctx* ctx, int fd, uint64_t offset, uint64_t len, int threads, sid_dtext** out,
                       uint64_t* err_offset, void* stream);
size_t sid_dtext_count(const sid_dtext* t);
const uint16_t* sid_dtext_counts(const sid_dtext* t);   /* device */
int sid_dtext_format(sid_ctx* ctx, const sid_dtext* t, size_t begin, size_t end, const uint8_t* code,
                     const double* hom_conf, const double* het_conf, const char* conf_type,
                     sid_write_fn write, void* user, void* stream);
int sid_dtext_free(sid_dtext* t);
/* -m quality (call.cpp:291-372) over a shard parsed by a context whose method
 * is SID_METHOD_QUALITY (7 fields per line): the read bases and both quality
 * fields are read from the resident text.  snp_prior / significance_level
 * from the context's options (sid_set_prior after a -R estimate). */
int sid_call_quality(sid_ctx* ctx, const sid_dtext* t, uint8_t* code, double* hom_conf, double* het_conf,
                     void* stream);
/* The device formatter's %g, host build (tests) and device batch: out gets
 * 16 bytes per value, NUL-padded. */
int sid_format_g6(double v, char* buf, size_t cap);
int sid_format_g6_device(sid_ctx* ctx, const double* values, size_t n, char* out, void* stream);


/* ------------------------------------------------ streaming engine -------
 * The whole path of one sid run -- pileup text in, CSV records out, in file
 * order -- replacing readFile + callX + the output loop (call.cpp:11-20,
 * call.cpp:62-289, sid.cpp:92-105) with a bounded-memory pipeline over
 * line-aligned chunks of the input:
 *
 *   host text --H2D (ring of device buffers)--> line index + parse
 *     [-m local / quality: call + CSV format, held in HBM]
 *     [Lynch (likelihood_ratio, bayes, -R): profile histogram]
 *   (the whole input validated; Lynch: merge + one estimate + class tables)
 *   [second pass over the chunks not formatted yet: parse, call / lookup,
 *    format] --D2H (pinned ring)--> write() in file order
 *
 * Chunk j runs on pipeline j % (devices x lanes) (pipeline i on GPU i / lanes);
 * every pipeline formats and copies back
 * concurrently and one writer keeps file order.  As in the reference, no
 * record is written before the whole input has parsed: the first malformed
 * line in file order is reported (its input byte offset in err_offset) and
 * nothing is written.  Host memory stays bounded (pinned rings); device
 * memory holds the formatted records of the chunks processed before the input
 * was validated, up to hold_bytes per device, beyond which chunks are
 * formatted in the second pass (their text kept in HBM up to retain_bytes,
 * else read again from the source).
 *
 * Usage: sid_engine_create, one sid_engine_source_*, then sid_engine_run --
 * or the three phases separately (multi-rank runs exchange the Lynch
 * histogram between ingest and estimate: sid_engine_context + the
 * sid_profile_* calls).  An engine is reusable: set a new source and run
 * again.  Not thread-safe. */
typedef struct sid_engine sid_engine;
typedef struct {
    int devices;            /* GPUs used (0 = every visible one); chunk j runs on
                               device (first_device + j % devices) % visible       */
    int first_device;
    uint64_t chunk_bytes;   /* input text per chunk (0 = 128 MiB)                  */
    int slots;              /* device text buffers per device (0 = 3)              */
    uint64_t hold_bytes;    /* per device, HBM for records held until the input is
                               validated (0 = 40% of free HBM)                     */
    uint64_t retain_bytes;  /* per device, HBM for text kept for the second pass
                               (0 = 40% of free HBM)                               */
    int host_threads;       /* host threads generating / prefetching input (0 = 8) */
    int verbose;            /* the reference's "# ..." lines on stderr             */
    int device_sink;        /* 0: write() in file order; 1: records stay in HBM,
                               nothing is copied back (measurement); 2: records
                               copied back to pinned host memory, no write
                               (measurement of the PCIe path; with
                               host_hold_bytes they stay there for
                               sid_engine_records)                               */
    int lanes;              /* pipelines per GPU (0 = 1): each its own streams,
                               context and workspace, chunks dealt over all of
                               them, so one chunk's kernels run while another
                               waits on its host sync                            */
    uint64_t host_hold_bytes; /* per pipeline, pinned host memory (made once,
                               reused by every run) for the records: -m local /
                               quality copy each chunk's records into it during
                               the ingest, while later chunks upload (PCIe both
                               ways at once), and the emit only write()s them;
                               the second pass copies into it instead of the
                               pinned ring.  Chunks beyond it take the HBM hold.
                               0 = off.  Ignored with device_sink 1             */
} sid_engine_cfg;
typedef struct {
    uint64_t sites;              /* non-empty lines parsed                           */
    uint64_t chunks;
    uint64_t bytes_in;           /* input text bytes                                 */
    uint64_t bytes_out;          /* CSV bytes (header excluded)                      */
    uint64_t chunks_held;        /* formatted in the first pass                      */
    uint64_t chunks_retained;    /* text kept in HBM for the second pass             */
    uint64_t chunks_reloaded;    /* text read from the source a second time          */
    int devices;
    int status_kind;             /* parse error status of the first bad line, or 0   */
    uint64_t err_offset;         /* its input byte offset                            */
    double ingest_s, estimate_s, emit_s;
    sid_estimate estimate;       /* Lynch paths                                      */
    /* the ingest's uploads of host text (host memory or a file's mapping):     */
    uint64_t chunks_registered;  /* copied from pages registered for DMA (the
                                    others: the runtime's pageable path, or the
                                    source was pinned already)                     */
    double register_s;           /* host time in hipHostRegister / Unregister,
                                    summed over the uploaders                      */
    double h2d_s;                /* device time of the host-to-device copies: the
                                    span from each upload stream's first copy to
                                    its last (HIP events), summed over the
                                    devices                                        */
    uint64_t h2d_bytes;          /* bytes those copies moved                       */
    uint64_t chunks_tiled;       /* parsed by the tile parse (text read once)       */
    uint64_t tile_overflows;     /* chunks with a tile of more lines than its slots
                                    (parsed again by the two-pass path; the next
                                    chunks get more slots)                         */
    uint64_t tile_overflows_queued; /* of those, overflows with the device's next
                                    chunk already popped behind it (its run-ahead
                                    tile parse dropped, the chunk kept)            */
} sid_run_stats;
void sid_engine_cfg_default(sid_engine_cfg* cfg);
int sid_engine_create(const sid_opts* opts, const sid_engine_cfg* cfg, sid_engine** out);
int sid_engine_destroy(sid_engine* e);
int sid_engine_devices(const sid_engine* e);
sid_ctx* sid_engine_context(sid_engine* e, int i);
/* Host placement of pipeline i (a multi-GPU node: each GPU's uploader,
 * compute and drain threads run on the CPUs local to its PCI device, and its
 * pinned host buffers are allocated from them, so their pages sit on the
 * GPU's NUMA node and its DMA does not cross sockets). */
typedef struct {
    int device;             /* HIP device                                          */
    int gpu_numa_node;      /* NUMA node of the GPU's PCI device (-1: unknown)     */
    int cpus;               /* CPUs its threads are bound to (0: not bound)        */
    int first_cpu;          /* the lowest of them (-1: not bound)                  */
    int arena_numa_node;    /* NUMA node of the host arena's first page (-1: none) */
    int ring_numa_node;     /* ... of the emit ring's first page (-1: none)        */
    char pci[16];           /* PCI bus id, e.g. "0000:05:00.0"                     */
} sid_placement;
int sid_engine_placement(const sid_engine* e, int i, sid_placement* out);
/* Sources.  The engine keeps the pointer / descriptor until the next source. */
int sid_engine_source_text(sid_engine* e, const char* text, uint64_t len);          /* host memory */
int sid_engine_source_file(sid_engine* e, int fd, uint64_t offset, uint64_t len);   /* regular file */
/* Text already in HBM on the engine's first device (measurement): d_text must
 * be readable for 256 bytes past len. */
int sid_engine_source_device_text(sid_engine* e, const char* d_text, uint64_t len);
/* The synthetic generator (sid_synth_text) streamed, never stored: sites
 * [first_site, first_site + n), sites_per_chunk per chunk (0 = about
 * chunk_bytes of text), generated by host threads into pinned buffers
 * (on_device = 0) or by a kernel straight into the device buffer (1). */
int sid_engine_source_synth(sid_engine* e, uint64_t seed, double mean_depth, uint64_t first_site, uint64_t n,
                            uint64_t sites_per_chrom, uint64_t sites_per_chunk, int on_device);
/* Phases.  ingest returns the parse status of the first malformed line
 * (stats->err_offset); estimate runs the Lynch estimate when the method needs
 * it (given != NULL: skip the Nelder-Mead, use given's pi/eps) and returns its
 * status (SID_EEMPTY, SID_EBADFUNC); emit writes `header` (unless NULL) and
 * the records through write(). */
int sid_engine_ingest(sid_engine* e, sid_run_stats* stats);
int sid_engine_estimate(sid_engine* e, const sid_estimate* given, sid_estimate* out);
int sid_engine_emit(sid_engine* e, const char* header, sid_write_fn write, void* user, sid_run_stats* stats);
int sid_engine_run(sid_engine* e, const char* header, sid_write_fn write, void* user, sid_run_stats* stats);
/* Multi-rank Lynch runs: after ingest, the merged unique-
 * profile table of all the engine's pipelines (sid_profile_table layout;
 * keys == NULL: only *u), and the load of a table merged across ranks into
 * every pipeline (it is not merged again by sid_engine_estimate). */
int sid_engine_profile_table(sid_engine* e, uint64_t* keys, uint64_t* counts64, size_t cap, size_t* u);
int sid_engine_profile_load(sid_engine* e, const uint64_t* keys, const uint64_t* counts64, size_t u);
/* With host_hold_bytes: the CSV records of chunk `chunk` (0 .. stats.chunks-1,
 * file order) in the host arena, after the emit (device_sink 2: the records
 * are not written anywhere else), valid until the next ingest or source;
 * SID_ESTATE when that chunk's records did not go through the host arena. */
int sid_engine_records(sid_engine* e, uint64_t chunk, const char** bytes, uint64_t* len);
/* Measurement: with profiling on, every stage of every chunk is bracketed by
 * a pair of HIP events on its device's compute stream; _read sums the stages'
 * device time over the chunks and devices since the last read (synchronises). */
typedef struct {
    uint64_t chunks;        /* chunks processed (either pass)                      */
    double index_ms;        /* line index: line starts per tile + scan             */
    double parse_ms;        /* line offsets + parse to counts                      */
    double call_ms;         /* sid_call_local / sid_lookup_sites / quality kernels */
    double hist_ms;         /* Lynch profile histogram                             */
    double fmt_len_ms;      /* record lengths + scan                               */
    double fmt_write_ms;    /* records written                                     */
} sid_engine_prof;
int sid_engine_profile(sid_engine* e, int enable);
int sid_engine_profile_read(sid_engine* e, sid_engine_prof* out);

#ifdef __cplusplus
}
#endif
#endif /* SID_H */
