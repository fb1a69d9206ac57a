// textpath.hip — pileup text -> counts and records -> CSV on the device
// (SURVEY.md §8(f) #1 GPU-side tokenisation, #4 GPU-side CSV formatting).
//
// The host hands over the raw text (e.g. a file mapping); it is copied to HBM
// in line-aligned chunks and, chunk by chunk while the next one is in flight:
//
//   sid_lines_count_kernel   line starts per 4 KiB tile (16-B loads, lanes
//                            contiguous)
//   sid_scan_*_kernel        exclusive scan of the tile counts (block sums,
//                            one block over those, block scans), continuing
//                            the running site count of the shard
//   sid_lines_emit_kernel    the byte offset of every non-empty line
//                            (call.cpp:14 skips empty lines)
//   sid_parse_kernel         one lane per line: parsePileupLine +
//                            parseReadBases (pileup.cpp:13-153) into
//                            profile_t counts; the first malformed line in
//                            file order is kept as min(offset*8 + kind)
//
// and for output, per piece of sites:
//
//   sid_fmt_len_kernel       record length per site (call.hpp:29-38), block sums
//   sid_scan_*_kernel        block offsets
//   sid_fmt_write_kernel     records assembled in LDS, written with 16-B stores
//
// chrom and pos are re-tokenised from the resident text when formatting, so
// parsing stores only the 8-B counts (and 8-B line offsets) per site.
// Semantics are those of parse.cpp (the host parser, tested against the
// reference's own pileup.cpp) and emit.cpp; the %g digits come from fmt.h.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <climits>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/sid.h"
#include "fmt.h"
#include "local_site.h"

namespace {

constexpr int TB = 256;                 // threads per block (4 waves)
constexpr int TILE = TB * 16;           // bytes per line-index tile
constexpr int SCAN_TB = 1024;

// ------------------------------------------------------------ block scan --
// inclusive scans over the wave by DPP (no LDS round trip): row_shr 1/2/4/8
// within each row of 16 lanes, then row_bcast 15 / 31 carry the rows' sums
// up.  The 64-bit form moves both halves and adds with the carry.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
// the wave's maximum of unsigned values, wave-uniform (0 fills the lanes a
// shift leaves empty: the identity)
__device__ __forceinline__ uint32_t wave_max(uint32_t x)
{
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
template <int CTRL, int ROWS, bool BOUND>
__device__ __forceinline__ uint64_t dpp64(uint64_t x)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, ROWS, 0xF, BOUND);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, ROWS, 0xF, BOUND);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_scan_incl64(uint64_t x)
{
    x += dpp64<0x111, 0xF, true>(x);
    x += dpp64<0x112, 0xF, true>(x);
    x += dpp64<0x114, 0xF, true>(x);
    x += dpp64<0x118, 0xF, true>(x);
    x += dpp64<0x142, 0xA, false>(x);
    x += dpp64<0x143, 0xC, false>(x);
    return x;
}

// exclusive scan of one u32 per thread over a 256-thread block; returns the
// prefix, *total = block sum
template <int NT = TB>
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* total)
{
    __shared__ uint32_t wsum[NT / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t x = wave_scan_incl(v);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int w = 0; w < NT / 64; ++w) {
        if (w < wid) base += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();   // wsum reused by the next call
    *total = tot;
    return base + x - v;
}

// Exclusive scan of m u32 values into u64 offsets, continuing from *base;
// *base advances by the sum (stream-ordered running total); range (if set)
// receives {*base before, *base after}.  Three kernels: block sums over
// 4096-element blocks, one block scanning those sums, the blocks' own scans.
// (A single block walking the whole array took 0.6 ms for 400k tile counts.)
constexpr int SCAN_PER = 16;                  // elements per thread
constexpr uint64_t SCAN_BLK = TB * SCAN_PER;  // elements per block

__device__ __forceinline__ uint64_t block_exscan64(uint64_t v, uint64_t* total)
{
    __shared__ uint64_t wsum[TB / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t x = wave_scan_incl64(v);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint64_t base = 0, tot = 0;
    for (int w = 0; w < TB / 64; ++w) {
        if (w < wid) base += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// the wave's sum, wave-uniform (a scalar)
__device__ __forceinline__ uint32_t wave_sum(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_incl(x), 63);
}
// a lane's value from a lane of its quad by DPP quad_perm (no LDS round trip
// as __shfl's ds_bpermute takes; the quad's four lanes active together):
// QP = the source lane for lanes 0-3, two bits each
template <uint32_t QP>
__device__ __forceinline__ uint32_t quad_get(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, (int)QP, 0xF, 0xF, false);
}
constexpr uint32_t QP_LEFT = 0x93;    // lane j <- j-1 mod 4 (3, 0, 1, 2)
constexpr uint32_t QP_LANE3 = 0xFF;   // every lane <- 3
constexpr uint32_t QP_XOR1 = 0xB1;    // (1, 0, 3, 2)
constexpr uint32_t QP_XOR2 = 0x4E;    // (2, 3, 0, 1)

// exclusive scan of one u32 per thread over an NT-thread block, once per
// kernel (its LDS slots are not reused): the waves by DPP (wave_scan_incl),
// their sums as scalars after one barrier; returns the prefix, *total = the
// block's sum.  (The writers' scan: 0.93 us of a 6.3 us writer block with
// the shuffle scan and its two barriers, profiles/tile_stamps_r05.log.)
template <int NT>
__device__ __forceinline__ uint32_t block_exscan_once(uint32_t v, uint32_t* total)
{
    __shared__ uint32_t wsum[NT / 64];
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t x = wave_scan_incl(v);
    if ((threadIdx.x & 63u) == 63u) wsum[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) {
        const uint32_t t = __builtin_amdgcn_readfirstlane(wsum[w]);
        base += w < wid ? t : 0u;
        tot += t;
    }
    *total = tot;
    return base + x - v;
}

// this thread's SCAN_PER inputs (16-B loads when the run is whole)
__device__ __forceinline__ void scan_load(const uint32_t* __restrict__ in, uint64_t m, uint64_t b0, uint32_t* v)
{
    if (b0 + SCAN_PER <= m) {
        const uint4* p = (const uint4*)(in + b0);   // b0 is a multiple of 16 elements
#pragma unroll
        for (int k = 0; k < SCAN_PER / 4; ++k) {
            const uint4 q = p[k];
            v[4 * k] = q.x;
            v[4 * k + 1] = q.y;
            v[4 * k + 2] = q.z;
            v[4 * k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_PER; ++k) v[k] = b0 + k < m ? in[b0 + k] : 0u;
    }
}

__global__ __launch_bounds__(TB) void sid_scan_reduce_kernel(const uint32_t* __restrict__ in, uint64_t m,
                                                             uint64_t* __restrict__ bsum)
{
    uint32_t v[SCAN_PER];
    scan_load(in, m, (uint64_t)blockIdx.x * SCAN_BLK + threadIdx.x * SCAN_PER, v);
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) s += v[k];
    uint64_t tot;
    block_exscan64(s, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// one block: exclusive scan of the nb block sums from *base (in place)
__global__ __launch_bounds__(SCAN_TB) void sid_scan_top_kernel(uint64_t* __restrict__ bsum, uint64_t nb,
                                                              uint64_t* base, uint64_t* __restrict__ range)
{
    __shared__ uint64_t wsum[SCAN_TB / 64];
    const uint64_t per = (nb + SCAN_TB - 1) / SCAN_TB;
    const uint64_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += bsum[i];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t x = wave_scan_incl64(s);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    const uint64_t b = *base;
    uint64_t before = b, tot = b;
    for (int w = 0; w < SCAN_TB / 64; ++w) {
        if (w < wid) before += wsum[w];
        tot += wsum[w];
    }
    uint64_t acc = before + x - s;
    for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t v = bsum[i];
        bsum[i] = acc;
        acc += v;
    }
    __syncthreads();   // every thread has read *base
    if (threadIdx.x == 0) {
        *base = tot;
        if (range) {
            range[0] = b;
            range[1] = tot;
        }
    }
}

__global__ __launch_bounds__(TB) void sid_scan_down_kernel(const uint32_t* __restrict__ in, uint64_t m,
                                                           const uint64_t* __restrict__ boff,
                                                           uint64_t* __restrict__ out)
{
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_BLK + threadIdx.x * SCAN_PER;
    uint32_t v[SCAN_PER];
    scan_load(in, m, b0, v);
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) s += v[k];
    uint64_t tot;
    uint64_t acc = boff[blockIdx.x] + block_exscan64(s, &tot);
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        if (b0 + k < m) out[b0 + k] = acc;
        acc += v[k];
    }
}

// workspace: one u64 per 4096 inputs
static size_t scan_ws_bytes(uint64_t m) { return ((m + SCAN_BLK - 1) / SCAN_BLK + 1) * 8; }

static void launch_scan(const uint32_t* in, uint64_t m, uint64_t* out, uint64_t* base, uint64_t* range,
                        uint64_t* ws, hipStream_t st)
{
    const uint64_t nb = (m + SCAN_BLK - 1) / SCAN_BLK;
    if (nb) sid_scan_reduce_kernel<<<(unsigned)nb, TB, 0, st>>>(in, m, ws);
    sid_scan_top_kernel<<<1, SCAN_TB, 0, st>>>(ws, nb, base, range);
    if (nb) sid_scan_down_kernel<<<(unsigned)nb, TB, 0, st>>>(in, m, ws, out);
}

// ---- SWAR helpers: bit 7 of each byte of the result flags a byte of w
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x)
{
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t k4) { return zero_bytes(w ^ k4); }
// bytes < 0x21: the separators, '\n', NUL (and other control bytes)
__device__ __forceinline__ uint32_t low_bytes(uint32_t w)
{
    return ~(((w & 0x7F7F7F7Fu) + 0x5F5F5F5Fu) | w) & 0x80808080u;
}

// bit 7 of each byte of four words -> 16 bits (word w's byte k at bit 4w+k):
// the bytes (0x00 or 0x80) weighted by v_dot4 (1, 2, 4, 8 and 16 .. 128) and
// summed, two words a dot product pair: 6 instructions where a shift-or
// ladder over nibble-interleaved flags took 16 (round 6, profiles/ab_tile_r06.log)
__device__ __forceinline__ uint32_t compress16(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    const uint32_t lo = __builtin_amdgcn_udot4(b, 0x80402010u, __builtin_amdgcn_udot4(a, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(d, 0x80402010u, __builtin_amdgcn_udot4(c, 0x08040201u, 0u, false), false);
    return (lo >> 7) | (hi << 1);   // (hi: 128 x the high byte's bits)
}
// a 16-B load marked non-temporal (streamed data read once: kept out of the
// caches the data read again needs)
// the intermediate arrays (line-start masks, line offsets, counts, header
// pairs: hundreds of MB a chunk, read back once by the next kernel, from HBM
// in any case) stored non-temporal, out of the way of the text the kernels
// read (index 0.896 -> 0.877, parse 2.015 -> 2.003 ms per C2 step, A/B)
#define ST_MID(ptr, val) __builtin_nontemporal_store((val), (ptr))
__device__ __forceinline__ uint4 ld_nt(const void* p)
{
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 t = __builtin_nontemporal_load((const u32x4*)p);
    return make_uint4(t.x, t.y, t.z, t.w);
}

// ------------------------------------------------------------ line index --
// 16 bytes per lane; bit j of the result = byte j starts a non-empty line.
// Bytes outside [c0, c1) never start a line; c0 is a line start.  SWAR: the
// '\n' bytes of the four words as a 16-bit mask, the previous byte's from the
// neighbouring lane (a load at a wave's first lane).
__device__ __forceinline__ uint32_t line_start_mask(const char* __restrict__ text, uint64_t tile0, uint64_t c0,
                                                    uint64_t c1)
{
    const uint64_t at = tile0 + (uint64_t)threadIdx.x * 16;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (at < c1 && at + 16 > c0) v = *(const uint4*)(text + at);
    uint32_t nl = compress16(eq_bytes(v.x, 0x0A0A0A0Au), eq_bytes(v.y, 0x0A0A0A0Au), eq_bytes(v.z, 0x0A0A0A0Au),
                             eq_bytes(v.w, 0x0A0A0A0Au));
    // is the byte before `at` a '\n': the neighbour lane's bit 15, or a load at a wave start
    uint32_t prev = (uint32_t)__shfl_up((int)(nl >> 15), 1, 64);
    if ((threadIdx.x & 63) == 0) prev = (at > c0 && at - 1 < c1) ? (text[at - 1] == '\n') : 1u;
    uint32_t m = ((nl << 1) | prev) & ~nl & 0xFFFFu;
    if (at + 16 > c0 && at <= c0) {   // c0 in this lane: it starts a line (unless a '\n'), nothing before it does
        const uint32_t j = (uint32_t)(c0 - at);
        m = (m | ((1u << j) & ~nl)) & ~((1u << j) - 1u);
    }
    if (at + 16 > c1) m &= c1 > at ? (1u << (uint32_t)(c1 - at)) - 1u : 0u;
    if (at + 16 <= c0) m = 0;
    return m;
}

__global__ __launch_bounds__(TB) void sid_lines_count_kernel(const char* __restrict__ text, uint64_t tile_base,
                                                             uint64_t c0, uint64_t c1, uint32_t* __restrict__ cnt)
{
    const uint64_t tile0 = tile_base + (uint64_t)blockIdx.x * TILE;
    const uint32_t m = __popc(line_start_mask(text, tile0, c0, c1));
    uint32_t tot;
    block_exscan(m, &tot);
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(TB) void sid_lines_emit_kernel(const char* __restrict__ text, uint64_t tile_base,
                                                            uint64_t c0, uint64_t c1,
                                                            const uint64_t* __restrict__ toff,
                                                            uint64_t* __restrict__ starts)
{
    const uint64_t tile0 = tile_base + (uint64_t)blockIdx.x * TILE;
    uint32_t mask = line_start_mask(text, tile0, c0, c1);
    uint32_t tot;
    uint64_t o = toff[blockIdx.x] + block_exscan(__popc(mask), &tot);
    const uint64_t at = tile0 + (uint64_t)threadIdx.x * 16;
    while (mask) {
        const int j = __ffs(mask) - 1;
        starts[o++] = at + j;
        mask &= mask - 1;
    }
}

// Line index of a chunk (the engine's path), two passes over 16 KiB tiles:
//   sid_index_count_kernel  4 lane-contiguous 4 KiB sub-tiles per tile, one
//                           16-B load per lane each (4 loads in flight per
//                           lane, the next tile's 4 issued before this one is
//                           counted; 8 measured slower): line-start masks (u16
//                           per lane and sub-tile, a lane's four in one 8-B
//                           word; 1/8 of the text) and the
//                           tile's count
//   (scan of the tile counts -> tile offsets, state[0] = sites)
//   sid_index_emit_kernel   the offsets of every line start, from the masks
// (A single pass with a decoupled look-back was measured 25x slower: the
// prefix chain crosses XCDs, whose L2s only meet in memory, ~0.4 us a link.)
constexpr int IX_SUB = 4;   // (a lane's IX_SUB 16-bit masks share one 8-B word)
static_assert(IX_SUB == 4, "masks are packed four to a u64");
constexpr uint64_t IX_TILE = (uint64_t)TILE * IX_SUB;   // 16 KiB

// the 16 bytes of a lane's window and, for a wave's first lane, the byte
// before it (1 when there is none: the window starts the range)
struct IxWin {
    uint4 v;
    uint32_t prev;
};
__device__ __forceinline__ IxWin ix_load(const char* __restrict__ text, uint64_t at, uint64_t c0, uint64_t c1)
{
    IxWin w{make_uint4(0, 0, 0, 0), 1u};
    // non-temporal: each byte is read once here (index 0.93 -> 0.90 ms per C2 step, A/B)
    if (at < c1 && at + 16 > c0) w.v = ld_nt(text + at);
    if ((threadIdx.x & 63) == 0 && at > c0 && at - 1 < c1) w.prev = text[at - 1] == '\n';
    return w;
}
// line_start_mask's arithmetic on a loaded window
__device__ __forceinline__ uint32_t ix_mask(const IxWin& w, uint64_t at, uint64_t c0, uint64_t c1)
{
    const uint4 v = w.v;
    uint32_t nl = compress16(eq_bytes(v.x, 0x0A0A0A0Au), eq_bytes(v.y, 0x0A0A0A0Au), eq_bytes(v.z, 0x0A0A0A0Au),
                             eq_bytes(v.w, 0x0A0A0A0Au));
    uint32_t prev = (uint32_t)__shfl_up((int)(nl >> 15), 1, 64);
    if ((threadIdx.x & 63) == 0) prev = w.prev;
    uint32_t m = ((nl << 1) | prev) & ~nl & 0xFFFFu;
    if (at + 16 > c0 && at <= c0) {
        const uint32_t j = (uint32_t)(c0 - at);
        m = (m | ((1u << j) & ~nl)) & ~((1u << j) - 1u);
    }
    if (at + 16 > c1) m &= c1 > at ? (1u << (uint32_t)(c1 - at)) - 1u : 0u;
    if (at + 16 <= c0) m = 0;
    return m;
}

// Blocks stride over the tiles (a fixed grid of a few per CU), the next
// tile's four windows per lane in flight while this one is counted; the tile
// count is a block reduction (two LDS slots alternate: one barrier a tile).
__global__ __launch_bounds__(TB) void sid_index_count_kernel(const char* __restrict__ text, uint64_t tile_base,
                                                             uint64_t c0, uint64_t c1, uint64_t ntiles,
                                                             uint16_t* __restrict__ masks,
                                                             uint32_t* __restrict__ cnt, uint64_t* __restrict__ state)
{
    __shared__ uint32_t red[2][TB / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // the scan's running base, and no parse error yet
        state[0] = 0;
        state[4] = ~0ull;
    }
    uint64_t t = blockIdx.x;
    IxWin w[IX_SUB];
    if (t < ntiles) {
#pragma unroll
        for (int k = 0; k < IX_SUB; ++k)
            w[k] = ix_load(text, tile_base + t * IX_TILE + (uint64_t)k * TILE + threadIdx.x * 16, c0, c1);
    }
    for (int par = 0; t < ntiles; t += gridDim.x, par ^= 1) {
        const uint64_t t0 = tile_base + t * IX_TILE;
        IxWin cur[IX_SUB];
#pragma unroll
        for (int k = 0; k < IX_SUB; ++k) cur[k] = w[k];
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles) {
#pragma unroll
            for (int k = 0; k < IX_SUB; ++k)
                w[k] = ix_load(text, tile_base + tn * IX_TILE + (uint64_t)k * TILE + threadIdx.x * 16, c0, c1);
        }
        uint32_t c = 0;
        uint64_t mw = 0;   // the lane's four sub-tile masks in one 8-B word
#pragma unroll
        for (int k = 0; k < IX_SUB; ++k) {
            const uint64_t at = t0 + (uint64_t)k * TILE + threadIdx.x * 16;
            const uint32_t m = ix_mask(cur[k], at, c0, c1);
            c += __popc(m);
            mw |= (uint64_t)m << (16 * k);
        }
        ST_MID((uint64_t*)masks + t * TB + threadIdx.x, mw);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
        if (lane == 0) red[par][wid] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
#pragma unroll
            for (int k = 0; k < TB / 64; ++k) tot += red[par][k];
            cnt[t] = tot;
        }
    }
}

// Zeroes on the way (for the kernels behind it, instead of memset launches):
// z32[0, n32), z64a[0, 8), z64b[0, 2) when set.
__global__ __launch_bounds__(TB) void sid_index_emit_kernel(const uint16_t* __restrict__ masks, uint64_t tile_base,
                                                            uint64_t ntiles, const uint64_t* __restrict__ toff,
                                                            sid_off_t* __restrict__ starts,
                                                            uint32_t* __restrict__ z32 = nullptr, uint64_t n32 = 0,
                                                            unsigned long long* __restrict__ z64a = nullptr,
                                                            unsigned long long* __restrict__ z64b = nullptr)
{
    for (uint64_t k = (uint64_t)blockIdx.x * TB + threadIdx.x; k < n32; k += (uint64_t)gridDim.x * TB) z32[k] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 8 && z64a) z64a[threadIdx.x] = 0;
    if (blockIdx.x == 0 && threadIdx.x < 2 && z64b) z64b[threadIdx.x] = 0;
    // blocks stride over the tiles as in the count kernel, the next tile's
    // masks loaded ahead (measured the same as a block per tile: 137 vs 140 us
    // per 2 GiB chunk; the scattered 8-B offset stores set its pace)
    uint64_t t = blockIdx.x;
    uint64_t mw_next = t < ntiles ? ((const uint64_t*)masks)[t * TB + threadIdx.x] : 0;
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t mw = mw_next;
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles) mw_next = ((const uint64_t*)masks)[tn * TB + threadIdx.x];
        uint32_t m[IX_SUB];
#pragma unroll
        for (int k = 0; k < IX_SUB; ++k) m[k] = (uint32_t)(mw >> (16 * k)) & 0xFFFFu;
        uint64_t o = toff[t];
        const uint64_t t0 = tile_base + t * IX_TILE;
        uint64_t packed = 0;
#pragma unroll
        for (int k = 0; k < IX_SUB; ++k) packed |= (uint64_t)__popc(m[k]) << (16 * k);
        uint64_t tot;
        const uint64_t pre = block_exscan64(packed, &tot);   // four sub-tiles: 16-bit fields stay < 2^16
#pragma unroll
        for (int k = 0; k < IX_SUB; ++k) {
            uint64_t q = o + ((pre >> (16 * k)) & 0xFFFF);
            const uint64_t at = t0 + (uint64_t)k * TILE + (uint64_t)threadIdx.x * 16;
            uint32_t mk = m[k];
            while (mk) {
                const int j = __ffs(mk) - 1;
                ST_MID(starts + q, (sid_off_t)(at + j));
                ++q;
                mk &= mk - 1;
            }
            o += (tot >> (16 * k)) & 0xFFFF;
        }
    }
}

// ----------------------------------------------------------------- parse --
// Byte reader over the resident text with a 16-B window.
struct Reader {
    const char* text;
    uint64_t limit;    // first byte not to read (end of text)
    uint64_t wpos = ~0ull;
    uint4 win;
    __device__ __forceinline__ uint32_t at(uint64_t i)
    {
        const uint64_t w = i & ~15ull;
        if (w != wpos) {
            wpos = w;
            win = *(const uint4*)(text + w);   // text is padded to a 16-B multiple
        }
        // byte k of the window by a select of the 8-byte half and a 64-bit
        // shift: a word select on k was turned into a dynamically indexed
        // stack array (scratch store + load per byte) in the quality kernel
        const uint32_t k = (uint32_t)(i & 15);
        const uint64_t half = (k & 8) ? (((uint64_t)win.w << 32) | win.z) : (((uint64_t)win.y << 32) | win.x);
        return (uint32_t)(half >> (8 * (k & 7))) & 0xffu;
    }
};

__device__ __forceinline__ bool is_sep(uint32_t c) { return c == ' ' || c == '\t'; }
__device__ __forceinline__ bool is_c_space(uint32_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
__device__ __forceinline__ bool is_digit(uint32_t c) { return c >= '0' && c <= '9'; }

// parse.cpp ClassTable: 1..4 = A C G T (either case), 5 = '^', 6 = '+'/'-', 0 = other
__host__ __device__ constexpr uint32_t base_class(uint32_t c)
{
    switch (c) {
    case 'A': case 'a': return 1;
    case 'C': case 'c': return 2;
    case 'G': case 'g': return 3;
    case 'T': case 't': return 4;
    case '^': return 5;
    case '+': case '-': return 6;
    default: return 0;
    }
}

// end of the line starting at s: the '\n' or the end of the text; and the
// end of its C string (first NUL), as parsePileupLine sees it
struct Line {
    uint64_t s, le, end;
};

// tokens on ' '/'\t' runs within [s, end): up to `want` tokens
__device__ __forceinline__ int tokenize(Reader& R, uint64_t s, uint64_t end, int want, uint64_t* tb, uint64_t* te)
{
    uint64_t q = s;
    int nt = 0;
    while (nt < want) {
        while (q < end && is_sep(R.at(q))) ++q;
        if (q >= end) break;
        tb[nt] = q;
        while (q < end && !is_sep(R.at(q))) ++q;
        te[nt] = q;
        ++nt;
    }
    return nt;
}

__device__ __forceinline__ Line find_line(Reader& R, uint64_t s)
{
    Line L;
    L.s = s;
    uint64_t q = s, z = ~0ull;
    while (q < R.limit) {
        const uint32_t c = R.at(q);
        if (c == '\n') break;
        if (c == 0 && z == ~0ull) z = q;
        ++q;
    }
    L.le = q;
    L.end = z < q ? z : q;
    return L;
}

// (int)strtol over [b, e) (parse.cpp atoi_like)
__device__ int atoi_like(Reader& R, uint64_t b, uint64_t e)
{
    while (b < e && is_c_space(R.at(b))) ++b;
    bool neg = false;
    if (b < e && (R.at(b) == '+' || R.at(b) == '-')) {
        neg = R.at(b) == '-';
        ++b;
    }
    unsigned long long v = 0;
    bool ovf = false;
    while (b < e && is_digit(R.at(b))) {
        const unsigned d = R.at(b) - '0';
        if (v > (ULLONG_MAX - d) / 10) ovf = true;
        else v = v * 10 + d;
        ++b;
    }
    long r;
    if (!neg) r = (ovf || v > (unsigned long long)LONG_MAX) ? LONG_MAX : (long)v;
    else r = (ovf || v > (unsigned long long)LONG_MAX + 1ull) ? LONG_MIN : (long)(0ull - v);
    return (int)(unsigned)(unsigned long)r;
}

// One pass over each line, stopping at the end of the fifth token (the
// quality and mapping-quality fields are never read): tokenisation on ' '/'\t'
// runs up to a NUL or '\n' (parsePileupLine sees a C string), and the read
// bases of token 4 counted on the fly with the reference's skip rules
// (pileup.cpp:70-153, parse.cpp read_bases):
//   '^' skips the next byte; '+'/'-' followed by a digit skips the digits and
//   then strtol(digits) more bytes; '.'/',' count as toupper/tolower(ref);
//   the skips end with the token.
// Byte classes come from a 256-entry LDS table; the counts are updated without
// branches on the class.
enum : uint32_t { K_IGN = 0, K_A = 1, K_C = 2, K_G = 3, K_T = 4, K_CARET = 5, K_INDEL = 6 };

// The per-byte walk: the general routine, for every line the fast path below
// does not take (indels, '^' runs, a '\n'/NUL or an over-long header before
// token 4, a ref whose '.'/',' class is '^'/'+'/'-', malformed lines) and for
// the quality-mode validation of tokens 5 and 6.
__device__ __noinline__ void parse_line_serial(const char* __restrict__ text, uint64_t len, uint64_t s0,
                                               const uint8_t* cls, uint64_t* out,
                                               unsigned long long* __restrict__ err, int qmode)
{
    Reader R{text, len};
    int nt = 0;              // tokens started
    bool in_tok = false;
    uint64_t tb2 = 0, te2 = 0;
    uint32_t cdot = 0, ccomma = 0;
    uint32_t nA = 0, nC = 0, nG = 0, nT = 0;
    uint64_t skip = 0;       // bytes of token 4 still to skip
    int ind = 0;             // 1: after '+'/'-'; 2: in its number
    uint64_t num = 0;
    bool ovf = false;
    for (uint64_t q = s0; q < len; ++q) {
        const uint32_t c = R.at(q);
        if (c == '\n' || c == 0) break;   // end of the line / of the C string
        const bool sep = c == ' ' || c == '\t';
        if (!in_tok) {
            if (sep) continue;
            in_tok = true;
            ++nt;
            if (nt == 7) break;                // quality mode: both quality fields exist
            if (nt == 3) tb2 = q;
            if (nt == 5) {   // token 2 is complete: the '.'/',' classes
                const uint32_t ref = R.at(tb2);
                const uint32_t up = (ref >= 'a' && ref <= 'z') ? ref - 32 : ref;
                const uint32_t lw = (ref >= 'A' && ref <= 'Z') ? ref + 32 : ref;
                cdot = cls[up];
                ccomma = cls[lw];
            }
        } else if (sep) {
            in_tok = false;
            if (nt == 3) te2 = q;
            if (nt == 5 && !qmode) break;  // token 4 done: the rest is never read
            continue;
        }
        if (nt != 5) continue;
        // ---- a byte of the read-bases token
        if (ind == 1) {   // byte after '+'/'-'
            ind = 0;
            if (c >= '0' && c <= '9') {
                ind = 2;
                num = c - '0';
                ovf = false;
                continue;
            }
        } else if (ind == 2) {
            if (c >= '0' && c <= '9') {
                const unsigned d = c - '0';
                if (!ovf) {
                    if (num > ((unsigned long long)LONG_MAX - d) / 10) ovf = true;
                    else num = num * 10 + d;
                }
                continue;
            }
            ind = 0;
            skip = ovf ? (uint64_t)LONG_MAX : num;   // this byte is the first skipped
        }
        if (skip) {
            --skip;
            continue;
        }
        const uint32_t k = c == '.' ? cdot : (c == ',' ? ccomma : cls[c]);
        nA += k == K_A;
        nC += k == K_C;
        nG += k == K_G;
        nT += k == K_T;
        if (k == K_CARET) skip = 1;
        else if (k == K_INDEL) ind = 1;
    }
    if (in_tok && nt == 3) te2 = ~0ull;   // token 2 ran to the end: length checked below
    int code = SID_OK;
    if (nt < 1) code = SID_ENULLCHROM;
    else if (nt < 3) code = SID_EMALFORMED;
    else {
        // token 2 length: its end is te2, or (if the line ended inside it) the
        // first '\n'/NUL/end after tb2
        uint64_t e2 = te2;
        if (e2 == 0 || e2 == ~0ull) {
            e2 = tb2;
            while (e2 < len) {
                const uint32_t c = R.at(e2);
                if (c == '\n' || c == 0 || c == ' ' || c == '\t') break;
                ++e2;
            }
        }
        if (e2 - tb2 != 1 || nt < 5) code = SID_EMALFORMED;
        // readFile(in, true, true) (call.cpp:292): parseQualities(NULL) on a
        // missing 6th field (SIGSEGV), then the mapping-quality check
        else if (qmode && nt == 5) code = SID_ENOBQ;
        else if (qmode && nt == 6) code = SID_EMISSING_MQ;
    }
    if (code != SID_OK) {   // first in file order: min(offset * 8 + kind)
        const uint32_t kind = code == SID_EMALFORMED ? 1u : code == SID_ENULLCHROM ? 2u
                            : code == SID_EMISSING_MQ ? 3u : 4u;
        atomicMin(err, (unsigned long long)(s0 * 8 + kind));
        *out = 0;
        return;
    }
    *out = (uint64_t)(uint16_t)nA | ((uint64_t)(uint16_t)nC << 16) | ((uint64_t)(uint16_t)nG << 32) |
                ((uint64_t)(uint16_t)nT << 48);
}

__device__ __forceinline__ int ctz64(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }

constexpr int HDR_BYTES = 48;   // bytes staged per lane for the header (3 aligned windows)

// 8 bytes from a lane's staged header at any offset < HDR_BYTES + 16: two
// aligned 8-B LDS reads and a funnel shift (past the lane's 48 bytes: the next
// lane's, or the block's padding -- garbage, masked by the caller)
__device__ __forceinline__ uint64_t stage_u64(const char* stage, uint32_t off)
{
    const uint32_t a = off & ~7u, sh = 8u * (off & 7u);
    const uint64_t lo = *(const uint64_t*)(stage + a), hi = *(const uint64_t*)(stage + a + 8);
    return (lo >> sh) | ((hi << 1) << (63u - sh));   // (no lane branch around the second read)
}
// bit 7 of each byte of x that is not an ASCII digit
__device__ __forceinline__ uint32_t not_digit(uint32_t x)
{
    const uint32_t lt30 = ~(((x & 0x7F7F7F7Fu) + 0x50505050u) | x) & 0x80808080u;   // b < '0'
    const uint32_t lt3a = ~(((x & 0x7F7F7F7Fu) + 0x46464646u) | x) & 0x80808080u;   // b < ':'
    return lt30 | (~lt3a & 0x80808080u);
}

// The LDS table of the read-bases counts (pileup.cpp:76-150): a byte's
// increments in 5-bit fields -- a 16-byte window adds at most 16 to a field:
// bits 0-4 A/a, 5-9 C/c, 10-14 G/g, 15-19 T/t, 20-24 '.'/',' (the ref's,
// added to its base at the end), 25-29 '+'/'-' (an indel: the line takes the
// general routine), bit 30 a control byte other than '\t' / '\n' ending the
// token (only the token's end byte is looked up among the low bytes: the
// general routine then has strtok_r's view of it); every other byte 0.
// Bytes not to count are zeroed before the lookup (NUL's entry is 0).
constexpr uint32_t RB_M_SHIFT = 20, RB_BAD_SHIFT = 25;
__host__ __device__ constexpr uint32_t rb_entry(uint32_t c)
{
    switch (c) {
    case 'A': case 'a': return 1u;
    case 'C': case 'c': return 1u << 5;
    case 'G': case 'g': return 1u << 10;
    case 'T': case 't': return 1u << 15;
    case '.': case ',': return 1u << RB_M_SHIFT;
    case '+': case '-': return 1u << RB_BAD_SHIFT;
    case ' ': case '\t': case '\n': case 0: return 0;
    default: return c < 0x21 ? 1u << 30 : 0;
    }
}

// The parse kernels' two LDS tables, built at compile time: each block copies
// them in (a load a lane) instead of evaluating both switches per lane (the
// branches of every case, serial in a wave, in every block: 13 % of the tile
// parse's time, C2 parse 1.712 -> 1.51 ms, C5 10.13 -> 8.76 ms per step,
// profiles/ab_tile_r06.log)
// rb[256 + m]: the 4-bit mask m as the bytes 0x00 / 0xFF of a word (the
// read bases' kept bytes: one LDS read a word; round 6 first spread the bits
// by a 24-bit multiply and multiplied by 0xFF -- v_perm's constant selectors,
// or (b << 8) - b, were no faster)
constexpr uint32_t RB_LUT_N = 256 + 16;
struct TpTables {
    uint32_t rb[RB_LUT_N];
    uint8_t cls[256];
};
constexpr TpTables make_tp_tables()
{
    TpTables t{};
    for (uint32_t c = 0; c < 256; ++c) {
        t.rb[c] = rb_entry(c);
        t.cls[c] = (uint8_t)base_class(c);
    }
    for (uint32_t m = 0; m < 16; ++m)
        t.rb[256 + m] = (m & 1 ? 0xFFu : 0u) | (m & 2 ? 0xFF00u : 0u) | (m & 4 ? 0xFF0000u : 0u) | (m & 8 ? 0xFF000000u : 0u);
    return t;
}
__device__ constexpr TpTables k_tp_tables = make_tp_tables();

// the four bytes of x through the table (byte b at LDS word b)
__device__ __forceinline__ uint32_t rb_word(const uint32_t* lut, uint32_t x)
{
    return lut[x & 0xFFu] + lut[(x >> 8) & 0xFFu] + lut[(x >> 16) & 0xFFu] + lut[x >> 24];
}

// One 16-B window of token 4 over its 16-bit masks: the token-end (the
// first byte < 0x21; `done` from then on) and '^' bytes of the four words
// compressed to 16 bits once; the '^' skip (carried into the next window), a
// '^' run (bad), the bytes before the end kept and the skipped ones dropped;
// then the kept bytes expanded back per word for four table lookups each (the
// token's end byte is looked up too: its entry flags a control byte).
// MASKED: only the bytes `valid` (the window's bytes at or after the token's
// start and before the text's end, room = bytes before the end) count; else
// the whole window lies inside the text.  (A per-word form of the same logic
// measured 1-2 % slower at 30x, 4 % at 200x.)
// (Lpre: the window's low-byte mask when the caller has it -- the header
// parse's mask of the line's first 48 bytes holds the first window's; ~0u:
// computed here)
template <bool MASKED>
__device__ __forceinline__ uint32_t rb_window16(const uint4 v, uint32_t valid, int room, const uint32_t* lut,
                                                bool& done, uint32_t& carry, bool& bad, uint32_t Lpre = ~0u)
{
    const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
    const uint32_t L = Lpre != ~0u ? Lpre
                                   : compress16(low_bytes(ws[0]), low_bytes(ws[1]), low_bytes(ws[2]), low_bytes(ws[3]));
    const uint32_t C = compress16(eq_bytes(ws[0], 0x5E5E5E5Eu), eq_bytes(ws[1], 0x5E5E5E5Eu),
                                  eq_bytes(ws[2], 0x5E5E5E5Eu), eq_bytes(ws[3], 0x5E5E5E5Eu));
    uint32_t vm = done ? 0u : (MASKED ? valid : 0xFFFFu);
    const uint32_t lo = L & vm;
    const uint32_t first = lo & (0u - lo);      // the token's end, if in this window
    vm &= first - 1u;                           // bytes before it (all if none)
    done = done || first != 0 || (MASKED && room < 16);
    const uint32_t caret = C & vm;
    const uint32_t skip = ((caret << 1) | carry) & vm;
    bad = bad || (caret & skip) != 0;           // '^' run
    carry = (caret >> 15) & 1u;
    const uint32_t cm = (vm | first) & ~skip;   // the bytes looked up
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += rb_word(lut, ws[k] & lut[256 + ((cm >> (4 * k)) & 15u)]);
    return acc;
}

// The read-bases count by the table: the first window (the token's start
// inside it) masked, then whole windows while they lie inside the text.
// first: the first window's 16 bytes, in LDS with the header (no second load
// of bytes the header already read).  ld(a): the 16-B window at text offset a
// (global memory, or the tile parse's LDS copy).  (The next windows from the
// per-line parse's stage too, where its 48 staged bytes hold them, measured
// slower: the loads hit the caches already)  Off: the
// offsets' type (32-bit for the tile parse's offsets from its tile).
template <class Ld, class Off = uint64_t>
__device__ __forceinline__ bool read_bases_lut(Ld ld, Off len, Off q, uint32_t kd, const uint32_t* lut,
                                               const uint4* first, uint64_t* out, uint32_t Lfirst = ~0u)
{
    uint32_t nA = 0, nC = 0, nG = 0, nT = 0, nM = 0;
    Off a = q & ~(Off)15;
    uint32_t carry = 0;   // 1: byte 0 of the next window is skipped
    bool done = false, bad = false;
    uint4 vn = ld(a + 16);   // the next window in flight while the first is counted
    uint32_t acc = 0;
    auto masked = [&](const uint4& v, uint32_t lead, uint32_t Lpre) {
        const int room = len > a ? (int)min(len - a, (Off)16) : 0;
        const uint32_t valid = ((room >= 16 ? 0xFFFFu : ((1u << room) - 1u)) >> lead) << lead;
        return rb_window16<true>(v, valid, room, lut, done, carry, bad, Lpre);
    };
    // the windows' 5-bit fields summed in two words with 10 bits a field (A,
    // G, '.' in one, C, T in the other: 4 instructions a window instead of
    // 10), into the counters every 63 windows (a field gains at most 16 a
    // window) and at the end (C2 parse 1.331-1.336 -> 1.320-1.323 ms)
    uint32_t ev = 0, od = 0, nw = 0;
    auto flush = [&]() {
        nA += ev & 1023u;
        nG += (ev >> 10) & 1023u;
        nM += ev >> 20;
        nC += (od >> 5) & 1023u;
        nT += od >> 15;
        ev = od = nw = 0;
    };
    auto add = [&](uint32_t w) {
        ev += w & 0x01F07C1Fu;
        od += w & 0x000F83E0u;
        acc |= w;
        if (++nw == 63) flush();
    };
    add(masked(*first, (uint32_t)(q & 15), Lfirst));
    a += 16;
    while (!done) {
        const uint4 v = vn;
        vn = ld(a + 16);
        add(a + 16 <= len ? rb_window16<false>(v, 0u, 16, lut, done, carry, bad) : masked(v, 0u, ~0u));
        a += 16;
    }
    if (bad || (acc >> RB_BAD_SHIFT) != 0) return false;
    flush();
    nA += kd == K_A ? nM : 0;
    nC += kd == K_C ? nM : 0;
    nG += kd == K_G ? nM : 0;
    nT += kd == K_T ? nM : 0;
    *out = (uint64_t)(uint16_t)nA | ((uint64_t)(uint16_t)nC << 16) | ((uint64_t)(uint16_t)nG << 32) |
           ((uint64_t)(uint16_t)nT << 48);
    return true;
}

// read_bases_lut for a line worked by a quad of 4 lanes (long lines, the
// quad parse below): window k of token 4 (16-B aligned, from q's window) goes
// to lane k mod 4, so a quad reads 64 consecutive bytes a step and a line
// needs a quarter of the steps.  A window's '^' carry-in is whether the byte
// before it is a '^' (the previous window's lane; a '^' that is itself
// skipped is a '^' run, which fails in that lane); the token ends in the
// quad's first window holding its end, and the windows after it are dropped.
// Every lane of the quad returns the same result.
template <class Ld, class Off = uint64_t>
__device__ __forceinline__ bool read_bases_quad(Ld ld, Off len, Off q, uint32_t kd, const uint32_t* lut,
                                                const uint4* first, uint64_t* out)
{
    const uint32_t j = threadIdx.x & 3u;
    const Off a0 = q & ~(Off)15;
    uint32_t nA = 0, nC = 0, nG = 0, nT = 0, nM = 0, acc = 0;
    bool bad = false;
    uint32_t prev3 = 0;   // lane 3's last byte was a '^' (the previous step's window 4(it-1)+3)
    for (uint32_t it = 0;; ++it) {   // uniform across the quad
        const uint32_t k = 4u * it + j;
        const Off a = a0 + (Off)16 * k;
        const uint4 v = k == 0 ? *first : ld(a);   // (past the line's end: the readable padding)
        const int room = len > a ? (int)min(len - a, (Off)16) : 0;
        const uint32_t lead = k == 0 ? (uint32_t)(q & 15) : 0u;
        const uint32_t valid = ((room >= 16 ? 0xFFFFu : ((1u << room) - 1u)) >> lead) << lead;
        const uint32_t last_caret = (v.w >> 24) == 0x5Eu ? 1u : 0u;
        const uint32_t from_left = quad_get<QP_LEFT>(last_caret);
        const uint32_t cin = k == 0 ? 0u : (j ? from_left : prev3);
        prev3 = quad_get<QP_LANE3>(last_caret);
        bool done = false, wbad = false;
        uint32_t carry = cin;
        const uint32_t w = rb_window16<true>(v, valid, room, lut, done, carry, wbad);
        // the quad's first window that ends the token (or the text)
        const uint64_t bal = __ballot(done);
        const uint32_t qb = (uint32_t)(bal >> (threadIdx.x & 60u)) & 15u;
        const bool keep = qb == 0 || j <= (uint32_t)__builtin_ctz(qb);
        if (keep) {
            nA += w & 31u;
            nC += (w >> 5) & 31u;
            nG += (w >> 10) & 31u;
            nT += (w >> 15) & 31u;
            nM += (w >> RB_M_SHIFT) & 31u;
            acc |= w;
            bad = bad || wbad;
        }
        if (qb) break;
    }
    auto quad_sum = [](uint32_t& x) {
        x += quad_get<QP_XOR1>(x);
        x += quad_get<QP_XOR2>(x);
    };
    auto quad_or = [](uint32_t& x) {
        x |= quad_get<QP_XOR1>(x);
        x |= quad_get<QP_XOR2>(x);
    };
    quad_sum(nA);
    quad_sum(nC);
    quad_sum(nG);
    quad_sum(nT);
    quad_sum(nM);
    uint32_t bf = acc | (bad ? 1u << 31 : 0u);   // (bit 31 of the entries' sum never set: bits 0-30)
    quad_or(bf);
    acc = bf & 0x7FFFFFFFu;
    bad = (bf >> 31) != 0;
    if (bad || (acc >> RB_BAD_SHIFT) != 0) return false;
    nA += kd == K_A ? nM : 0;
    nC += kd == K_C ? nM : 0;
    nG += kd == K_G ? nM : 0;
    nT += kd == K_T ? nM : 0;
    *out = (uint64_t)(uint16_t)nA | ((uint64_t)(uint16_t)nC << 16) | ((uint64_t)(uint16_t)nG << 32) |
           ((uint64_t)(uint16_t)nT << 48);
    return true;
}

// The fast path's header (pileup.cpp:13-46), branch-free over SWAR byte
// masks: the 48 bytes from the line's 16-B window (v0..v2, also at `stage`
// in LDS for byte reads) -> low-byte (< 0x21) mask -> token starts 1-4 by bit
// tricks; token 0 at the line start, exactly one ' '/'\t' before each of
// tokens 1-4 and a one-byte token 2 (else the general routine, which has
// strtok_r's semantics); ref and the position digits from the LDS copy.
// sh: the line's offset in v0; avail: the chunk's bytes from the line start.
// hdr: the formatter's header pair; returns the offset of token 4 from the
// line start (< 48), or -1 for the general routine; *kd: the class '.'/','
// stand for.
__device__ __forceinline__ int parse_header(const uint4 v0, const uint4 v1, const uint4 v2, const char* stage,
                                            uint32_t sh, uint64_t avail, const uint8_t* cls, uint64_t* hdr,
                                            uint32_t* kdp, uint64_t* low48 = nullptr)
{
    // low bytes (< 0x21: the separators, '\n', NUL, every other control byte)
    // of the 48 staged bytes as a 48-bit mask: 3 instructions a word
    const uint32_t w[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
    uint32_t lowb[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) lowb[k] = low_bytes(w[k]);
    const uint32_t l_lo = compress16(lowb[0], lowb[1], lowb[2], lowb[3]) |
                          (compress16(lowb[4], lowb[5], lowb[6], lowb[7]) << 16);
    const uint32_t l_hi = compress16(lowb[8], lowb[9], lowb[10], lowb[11]);
    if (low48) *low48 = ((uint64_t)l_hi << 32) | l_lo;   // (the staged windows' low-byte masks, for the read bases)
    // bit j = byte s0 + j, for the bytes inside the text and the 48 staged
    const uint32_t nb = (uint32_t)min((uint64_t)(HDR_BYTES - sh), avail);
    const uint64_t valid = (1ull << nb) - 1;   // (nb <= 48)
    const uint64_t L = ((((uint64_t)l_hi << 32) | l_lo) >> sh) & valid;
    const uint64_t N = ~L & valid;
    uint64_t T = N & ~(N << 1) & ~1ull;   // starts of tokens 1, 2, ...
    const int t1 = ctz64(T);
    T &= T - 1;
    const int t2 = ctz64(T);
    T &= T - 1;
    const int t3 = ctz64(T);
    T &= T - 1;
    const int t4 = ctz64(T);
    // the low bytes before token 4 are then the four gaps, which must be ' '
    // or '\t' (a '\n', NUL or other control byte there ends or splits a
    // token differently)
    // (no early exits: every check folded into ok, the byte reads clamped to
    // the 48 staged bytes -- each exit was an exec-masked branch and its
    // own copy of the outputs' defaults)
    bool ok = ((N & 1) != 0) & (t4 < (int)nb) & (t3 == t2 + 2);
    ok &= __popcll(L & ((1ull << (t4 & 63)) - 1)) == 4;
    auto at = [&](int t) { return (uint32_t)(uint8_t)stage[sh + (uint32_t)min(max(t, 0), 47)]; };
    const uint32_t gaps = at(t1 - 1) | (at(t2 - 1) << 8) | (at(t2 + 1) << 16) | (at(t4 - 1) << 24);
    ok &= (eq_bytes(gaps, 0x20202020u) | eq_bytes(gaps, 0x09090909u)) == 0x80808080u;
    const int t0 = 0;
    const int l0 = t1 - 1;
    const int lp = t2 - 1 - t1;
    const uint32_t ref = at(t2);
    // the position: its first 8 bytes by two aligned 8-B LDS reads and a
    // funnel shift, digit-checked in SWAR, left-padded with zero digits and
    // summed by v_dot4 pairs (10, 1) and two 24-bit multiply-adds; a 9th digit
    // on top (at most 9: < 2^31, as the per-digit loop this replaces)
    const uint32_t L8 = min((uint32_t)lp, 8u);
    const uint64_t p8 = stage_u64(stage, sh + (uint32_t)min(max(t1, 0), 47));
    const uint32_t plo = (uint32_t)p8, phi = (uint32_t)(p8 >> 32);
    const uint64_t nd = (uint64_t)not_digit(plo) | ((uint64_t)not_digit(phi) << 32);
    const uint64_t inl = L8 >= 8 ? ~0ull : ((1ull << (8 * L8)) - 1);
    const uint32_t d9 = at(t1 + 8) - '0';   // (read within the staged bytes whenever lp == 9)
    // (a leading zero: the position's digits then differ from its printed
    // ones -- the formatter's tokeniser takes it, so a valid pair's digit
    // count is the printed position's, sid_i32_len)
    const bool lz = lp > 1 && (plo & 0xFFu) == '0';
    const bool pos_ok = !lz && lp >= 1 && lp <= 9 && (nd & inl) == 0 && (lp < 9 || d9 < 10u);
    // digit values (garbage above the digits only borrows upward, then shifts out)
    const uint64_t dv = ((uint64_t)(phi - 0x30303030u) << 32) | (plo - 0x30303030u);
    const uint64_t dz = L8 == 0 ? 0 : dv << ((8 * (8 - L8)) & 63);
    const uint32_t q0 = (uint32_t)dz, q1 = (uint32_t)(dz >> 32);
    const uint32_t h4 = __umul24(__builtin_amdgcn_udot4(q0, 0x0000010Au, 0u, false), 100u) +
                        __builtin_amdgcn_udot4(q0, 0x010A0000u, 0u, false);
    const uint32_t l4 = __umul24(__builtin_amdgcn_udot4(q1, 0x0000010Au, 0u, false), 100u) +
                        __builtin_amdgcn_udot4(q1, 0x010A0000u, 0u, false);
    uint32_t pos = __umul24(h4, 10000u) + l4;
    if (lp == 9) pos = pos * 10u + d9;
    // chrom (offset: bits 44-58, length: 32-43), position (0-31) and its
    // digits (59-62) for the formatter (bit 63: valid)
    hdr[0] = pos_ok ? (1ull << 63) | ((uint64_t)lp << 59) | ((uint64_t)t0 << 44) | ((uint64_t)l0 << 32) | pos : 0ull;
    // the chrom's first 8 bytes: the formatter then never reads the text for
    // names up to 8 bytes (reading them back fetched every line's cache lines)
    const uint64_t c8 = stage_u64(stage, sh + t0) & (l0 >= 8 ? ~0ull : ((1ull << (8 * l0)) - 1));
    hdr[1] = c8;
    const uint32_t up = (ref >= 'a' && ref <= 'z') ? ref - 32 : ref;
    const uint32_t lw = (ref >= 'A' && ref <= 'Z') ? ref + 32 : ref;
    const uint32_t kd = cls[up], kc = cls[lw];
    ok &= (kd < K_CARET) & (kc < K_CARET) & (kd == kc);
    *kdp = kd;
    return ok ? t4 : -1;
}

// The fast path of one line (pileup.cpp:13-46 + :70-153 for the lines that
// need none of the general routine's cases): the header (parse_header), then
// the read bases (token 4) 16 bytes per step, per 4-byte word:
//   A/C/G/T either case     -> their counters
//   '.' / ','               -> one "matches ref" counter, added to the ref's
//                              class at the end
//   '^'                     -> the next byte is skipped; a '^' that is itself
//                              skipped (a '^' run) fails
//   '+'/'-'                 -> fail (indel: the general routine)
//   first byte < 0x21       -> end of the token, which must be ' ', '\t',
//                              '\n' or NUL, else fail
// Returns false when the line needs the general routine.  The 48 header bytes
// are staged in the lane's LDS slot for byte reads.
// QUAD: the read bases counted by the line's quad of lanes (read_bases_quad;
// every lane of the quad parses the same line, so its header is the same in
// all four)
template <bool QUAD = false>
__device__ __forceinline__ bool parse_line_fast(const char* __restrict__ text, uint64_t len, uint64_t s0,
                                                const uint8_t* cls, char* stage, uint64_t* out, uint64_t* hdr,
                                                const uint32_t* rbl)
{
    const uint64_t a0 = s0 & ~(uint64_t)15;
    const uint32_t sh = (uint32_t)(s0 & 15);
    const uint4 v0 = *(const uint4*)(text + a0);
    const uint4 v1 = *(const uint4*)(text + a0 + 16);
    const uint4 v2 = *(const uint4*)(text + a0 + 32);
    *(uint4*)(stage) = v0;
    *(uint4*)(stage + 16) = v1;
    *(uint4*)(stage + 32) = v2;
    uint32_t kd = 0;
    const int t4 = parse_header(v0, v1, v2, stage, sh, len > s0 ? len - s0 : 0, cls, hdr, &kd);
    if (t4 < 0) return false;
    auto ld = [text](uint64_t a) { return *(const uint4*)(text + a); };
    const uint4* first = (const uint4*)(stage + ((sh + t4) & 0x30));
    if (QUAD) return read_bases_quad(ld, len, s0 + (uint64_t)t4, kd, rbl, first, out);
    return read_bases_lut(ld, len, s0 + (uint64_t)t4, kd, rbl, first, out);
}

// Pass 1: the fast path over every line; a line it cannot take is appended to
// the fallback list fb (count in *fbn).  Pass 2 (sid_parse_serial_kernel):
// the general routine over that list -- or over every line, for -m quality.
template <class Off>
__global__ __launch_bounds__(TB) void sid_parse_kernel(const char* __restrict__ text, uint64_t len,
                                                       const Off* __restrict__ starts,
                                                       const uint64_t* __restrict__ range,   // [lo, hi)
                                                       uint64_t* __restrict__ counts, uint64_t* __restrict__ hdr,
                                                       uint32_t* __restrict__ fb, unsigned long long* fbn)
{
    __shared__ uint8_t cls[256];
    __shared__ uint32_t rbl[RB_LUT_N];
    __shared__ __attribute__((aligned(16))) char stage[TB * HDR_BYTES + 64];
    if (threadIdx.x < 256) {
        cls[threadIdx.x] = k_tp_tables.cls[threadIdx.x];
        rbl[threadIdx.x] = k_tp_tables.rb[threadIdx.x];
        if (threadIdx.x < RB_LUT_N - 256) rbl[256 + threadIdx.x] = k_tp_tables.rb[256 + threadIdx.x];
    }
    __syncthreads();
    const uint64_t lo = range[0], hi = range[1];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t s_next = i < hi ? starts[i] : 0;
    for (; i < hi; i += stride) {
        const uint64_t s0 = s_next;
        if (i + stride < hi) s_next = starts[i + stride];   // the next line's offset in flight
        uint64_t c = 0, h[2] = {0, 0};
        if (parse_line_fast(text, len, s0, cls, stage + threadIdx.x * HDR_BYTES, &c, h, rbl)) {
            counts[i] = c;
            *(ulonglong2*)(hdr + 2 * i) = make_ulonglong2(h[0], h[1]);
        } else {
            fb[atomicAdd(fbn, 1ull)] = (uint32_t)(i - lo);
        }
    }
}

// sid_parse_kernel for long lines (> 256 B on average: 200x) with a quad of
// lanes per line (parse_line_fast<true>): 16 lines a wave, each quad reading
// 64 consecutive bytes of its line a step, instead of 64 lanes walking 64
// lines 16 bytes at a time (whose in-flight lines are a cache working set
// the 200x lines overflow, line_walk_grid).
template <class Off>
__global__ __launch_bounds__(TB) void sid_parse_quad_kernel(const char* __restrict__ text, uint64_t len,
                                                            const Off* __restrict__ starts,
                                                            const uint64_t* __restrict__ range,   // [lo, hi)
                                                            uint64_t* __restrict__ counts, uint64_t* __restrict__ hdr,
                                                            uint32_t* __restrict__ fb, unsigned long long* fbn)
{
    __shared__ uint8_t cls[256];
    __shared__ uint32_t rbl[RB_LUT_N];
    __shared__ __attribute__((aligned(16))) char stage[TB * HDR_BYTES + 64];
    if (threadIdx.x < 256) {
        cls[threadIdx.x] = k_tp_tables.cls[threadIdx.x];
        rbl[threadIdx.x] = k_tp_tables.rb[threadIdx.x];
        if (threadIdx.x < RB_LUT_N - 256) rbl[256 + threadIdx.x] = k_tp_tables.rb[256 + threadIdx.x];
    }
    __syncthreads();
    constexpr uint32_t LPB = TB / 4;   // lines per block step
    const uint64_t lo = range[0], hi = range[1];
    const uint64_t stride = (uint64_t)gridDim.x * LPB;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * LPB + (threadIdx.x >> 2); i < hi; i += stride) {
        uint64_t c = 0, h[2] = {0, 0};
        const bool ok = parse_line_fast<true>(text, len, starts[i], cls, stage + threadIdx.x * HDR_BYTES, &c, h, rbl);
        if ((threadIdx.x & 3u) == 0) {
            if (ok) {
                ST_MID(counts + i, c);
                ST_MID(hdr + 2 * i, h[0]);
                ST_MID(hdr + 2 * i + 1, h[1]);
            } else {
                fb[atomicAdd(fbn, 1ull)] = (uint32_t)(i - lo);
            }
        }
    }
}

// late (optional): the lines it parsed, for the -m local record lengths the
// fused parse computes for its own lines (sid_local_len_list_kernel)
template <class Off>
__global__ __launch_bounds__(TB) void sid_parse_serial_kernel(const char* __restrict__ text, uint64_t len,
                                                              const Off* __restrict__ starts,
                                                              const uint64_t* __restrict__ range,
                                                              uint64_t* __restrict__ counts,
                                                              uint64_t* __restrict__ hdr,
                                                              const uint32_t* __restrict__ fb,
                                                              const unsigned long long* fbn,
                                                              unsigned long long* __restrict__ err, int qmode,
                                                              uint32_t* __restrict__ late = nullptr,
                                                              unsigned long long* nlate = nullptr)
{
    __shared__ uint8_t cls[256];
    if (threadIdx.x < 256) cls[threadIdx.x] = k_tp_tables.cls[threadIdx.x];
    __syncthreads();
    const uint64_t lo = range[0];
    const uint64_t m = fb ? *fbn : range[1] - lo;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = lo + (fb ? fb[k] : k);
        uint64_t c = 0;
        parse_line_serial(text, len, starts[i], cls, &c, err, qmode);
        counts[i] = c;
        hdr[2 * i] = 0;   // the formatter tokenises these lines itself
        if (late) late[atomicAdd(nlate, 1ull)] = (uint32_t)(i - lo);
    }
}

// Grid of a kernel in which every lane walks its own line: the lines a CU
// has in flight are its cache working set.  At 30x (~81 B a line) a full CU
// fits; at 200x (~430 B) 32 waves of lines thrash L1/L2 and the text is
// fetched again.  Blocks per CU ~ 1000 B / bytes per line, at most 8 (the
// full grid, `cap`).  Parse on a C5 shard (200x): 8 blocks a CU 14.1 ms, 4:
// 10.9, 2: 10.5, 1: 13.8; C2 best at the full grid.
static unsigned line_walk_grid(uint64_t n, uint64_t len, unsigned cap)
{
    if (!n) return cap;
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const long bpc = std::lround(1000.0 * (double)n / (double)std::max<uint64_t>(len, 1));
    if (bpc >= 8) return cap;
    return (unsigned)std::min<uint64_t>(cap, (uint64_t)std::max(1L, bpc) * (uint64_t)ncu);
}

// the two passes over sites [range[0], range[1]) (the range lives on the device)
template <class Off>
static void launch_parse(const char* text, uint64_t len, const Off* starts, const uint64_t* range, uint64_t n,
                         uint64_t* counts, uint64_t* hdr, uint32_t* fb, unsigned long long* fbn,
                         unsigned long long* err, int qmode, hipStream_t st)
{
    constexpr uint64_t PG = 16384;   // blocks of the grid-stride parse
    const unsigned pg = (unsigned)std::min<uint64_t>(std::max<uint64_t>((n + TB - 1) / TB, 1), PG);
    if (qmode) {   // (the byte-wise walks of -m quality measured slower on the smaller grid: 925 vs 626 us at 200x)
        sid_parse_serial_kernel<<<pg, TB, 0, st>>>(text, len, starts, range, counts, hdr, nullptr, nullptr, err, 1);
        return;
    }
    (void)hipMemsetAsync(fbn, 0, sizeof *fbn, st);
    if (n && len > 256 * n) {   // long lines (over 256 B on average): a quad of lanes per line, the full grid
        const unsigned pq = (unsigned)std::min<uint64_t>(std::max<uint64_t>((n + TB / 4 - 1) / (TB / 4), 1), PG);
        sid_parse_quad_kernel<Off><<<pq, TB, 0, st>>>(text, len, starts, range, counts, hdr, fb, fbn);
    } else {
        sid_parse_kernel<Off><<<line_walk_grid(n, len, pg), TB, 0, st>>>(text, len, starts, range, counts, hdr, fb,
                                                                         fbn);
    }
    sid_parse_serial_kernel<<<256, TB, 0, st>>>(text, len, starts, range, counts, hdr, fb, fbn, err, 0);
}

// ---------------------------------------------------------------- format --
struct CType {
    char s[16];
    int len;
};

// chrom token [cb, cb + clen) and position of the site whose line starts at
// `start`: from the parse's header word when it is valid, else tokenised here
// (a parsed line has >= 5 tokens before any NUL or newline, so its first two
// tokens are plain separator-delimited runs; the scan also stops at a newline
// or NUL: the streaming engine formats a chunk before it knows whether one of
// its lines is malformed -- it then discards the records -- and such a line
// must not send the scan past its end)
struct Head {
    uint64_t cb;
    uint32_t clen;
    int32_t pos;
    uint64_t c8;   // the chrom's bytes when clen <= 8 and the header word is valid (else 0)
};

// hdr: the parse's (header word, chrom's first 8 bytes) of the site, or null;
// the line's offset (*startp) is read only when the text is (a chrom longer
// than 8 bytes, or no valid header word)
// (hw: the header pair, loaded by the caller)
template <class Off>
__device__ __forceinline__ Head site_head_hw(Reader& R, const Off* startp, const ulonglong2 hw)
{
    Head h;
    h.c8 = 0;
    if (hw.x >> 63) {
        h.clen = (uint32_t)(hw.x >> 32) & 0xFFFu;
        h.pos = (int32_t)(uint32_t)hw.x;
        h.c8 = h.clen <= 8 ? hw.y : 0;
        h.cb = (h.c8 || h.clen == 0) ? 0 : *startp + ((hw.x >> 44) & 0x7FFFull);
        return h;
    }
    uint64_t q = *startp;
    while (is_sep(R.at(q))) ++q;
    h.cb = q;
    for (uint32_t ch = R.at(q); !is_sep(ch) && ch != '\n' && ch != 0; ch = R.at(++q)) {
    }
    h.clen = (uint32_t)(q - h.cb);
    while (is_sep(R.at(q))) ++q;
    const uint64_t pb = q;
    for (uint32_t ch = R.at(q); !is_sep(ch) && ch != '\n' && ch != 0; ch = R.at(++q)) {
    }
    h.pos = atoi_like(R, pb, q);
    return h;
}

template <class Off>
__device__ __forceinline__ Head site_head(Reader& R, const Off* startp, const uint64_t* hdr)
{
    return site_head_hw(R, startp, hdr ? *(const ulonglong2*)hdr : make_ulonglong2(0, 0));
}

// record length of a site (call.hpp:29-38): 0 for a filtered profile (no
// record, call.cpp:131-140), -1 for a confidence outside the formatter's range
__device__ __forceinline__ int record_len(const Head& h, uint8_t c, const sid_g6& gh, const sid_g6& gt, int tlen)
{
    if (c & 0x40) return 0;
    const int a = sid_g6_len(gh), b = sid_g6_len(gt);
    if (a < 0 || b < 0) return -1;
    // chrom , pos , hom|het , XY , hom_conf , het_conf , conf_type \n
    return (int)h.clen + 1 + sid_i32_len(h.pos) + 1 + 3 + 1 + 2 + 1 + a + 1 + b + 1 + tlen + 1;
}

__device__ __forceinline__ void record_put(Reader& R, const Head& h, uint8_t c, const sid_g6& gh, const sid_g6& gt,
                                           const CType& ct, char* out)
{
    if (h.c8 || h.clen == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (k < (int)h.clen) out[k] = (char)(h.c8 >> (8 * k));
    } else {
        for (uint32_t k = 0; k < h.clen; ++k) out[k] = (char)R.at(h.cb + k);
    }
    int n = (int)h.clen;
    out[n++] = ',';
    n += sid_fmt_i32(h.pos, out + n);
    out[n++] = ',';
    const bool het = c & 0x80;
    out[n++] = 'h';
    out[n++] = het ? 'e' : 'o';
    out[n++] = het ? 't' : 'm';
    out[n++] = ',';
    out[n++] = "ACGT"[c & 3];
    out[n++] = "ACGT"[(c >> 2) & 3];
    out[n++] = ',';
    n += sid_g6_put(gh, out + n);
    out[n++] = ',';
    n += sid_g6_put(gt, out + n);
    out[n++] = ',';
#pragma unroll
    for (int k = 0; k < 16; ++k)
        if (k < ct.len) out[n + k] = ct.s[k];
    out[n + ct.len] = '\n';
}

// the block's LDS copy of the 10^k table of the %g fast path (a dependent
// global load per confidence otherwise); synchronises the block
__device__ __forceinline__ void load_p10(double* p10)
{
    for (int k = threadIdx.x; k < SID_P10_N; k += blockDim.x) p10[k] = sid_p10_d[k];
    __syncthreads();
}

__global__ __launch_bounds__(TB) void sid_fmt_len_kernel(const char* __restrict__ text, uint64_t len,
                                                         const uint64_t* __restrict__ starts,
                                                         const uint64_t* __restrict__ hdr, uint64_t s0,
                                                         uint64_t s1, const uint8_t* __restrict__ code,
                                                         const double* __restrict__ hom,
                                                         const double* __restrict__ het, CType ct,
                                                         uint32_t* __restrict__ bsum, int* __restrict__ bad)
{
    __shared__ double p10[SID_P10_N];
    load_p10(p10);
    const uint64_t i = s0 + (uint64_t)blockIdx.x * TB + threadIdx.x;
    int l = 0;
    if (i < s1) {
        const uint8_t c = code[i];
        if (!(c & 0x40)) {
            Reader R{text, len};
            const Head h = site_head(R, starts + i, hdr ? hdr + 2 * i : nullptr);
            l = record_len(h, c, sid_g6_prep(hom[i], p10), sid_g6_prep(het[i], p10), ct.len);
            if (l < 0) {
                atomicExch(bad, 1);
                l = 0;
            }
        }
    }
    uint32_t tot;
    block_exscan((uint32_t)l, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

constexpr int FMT_LDS = 16 * 1024;   // 64 B per record: 8 blocks (32 waves) per CU

__global__ __launch_bounds__(TB) void sid_fmt_write_kernel(const char* __restrict__ text, uint64_t len,
                                                           const uint64_t* __restrict__ starts,
                                                           const uint64_t* __restrict__ hdr, uint64_t s0,
                                                           uint64_t s1, const uint8_t* __restrict__ code,
                                                           const double* __restrict__ hom,
                                                           const double* __restrict__ het, CType ct,
                                                           const uint64_t* __restrict__ boff, uint64_t out0,
                                                           char* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) char buf[FMT_LDS + 32];
    __shared__ double p10[SID_P10_N];
    load_p10(p10);
    const uint64_t i = s0 + (uint64_t)blockIdx.x * TB + threadIdx.x;
    Reader R{text, len};
    int l = 0;
    uint8_t c = 0x40;
    Head h{0, 0, 0, 0};
    sid_g6 gh{}, gt{};
    if (i < s1) {
        c = code[i];
        if (!(c & 0x40)) {
            h = site_head(R, starts + i, hdr ? hdr + 2 * i : nullptr);
            gh = sid_g6_prep(hom[i], p10);
            gt = sid_g6_prep(het[i], p10);
            l = record_len(h, c, gh, gt, ct.len);
            if (l < 0) l = 0;
        }
    }
    uint32_t tot;
    const uint32_t my = block_exscan((uint32_t)l, &tot);
    const uint64_t base = boff[blockIdx.x] - out0;   // offset of this block in `out`
    if (tot > FMT_LDS) {   // long records (long chromosome names): straight to global
        if (l) record_put(R, h, c, gh, gt, ct, out + base + my);
        return;
    }
    // assemble in LDS at the same 16-B phase as the destination, then 16-B stores
    const uint32_t phase = (uint32_t)((uintptr_t)(out + base) & 15u);
    if (l) record_put(R, h, c, gh, gt, ct, buf + phase + my);
    __syncthreads();
    char* dst = out + base - phase;   // 16-B aligned
    const uint32_t span = phase + tot;
    for (uint32_t k = threadIdx.x * 16; k < span; k += TB * 16) {
        if (k >= phase && k + 16 <= span) {
            *(uint4*)(dst + k) = *(const uint4*)(buf + k);
        } else {
            for (uint32_t j = k; j < k + 16 && j < span; ++j)
                if (j >= phase) dst[j] = buf[j];
        }
    }
}

// The engine's formatter: the records of a chunk's sites, in file order,
// with no block ever waiting on another (a decoupled look-back across blocks
// stalls when another process's kernels share the GPU and its waves are
// swapped out): (1) every FTB-site block's record bytes, (2) a scan of the
// block sums into block offsets, (3) every block assembles its records in LDS
// and stores them at its offset with 16-B stores.
//
// lb (zeroed before (1)): [1] the records' bytes (the scan's running total),
// [2] != 0: a confidence outside the formatter's range, [4] a copy of
// state[4] (the chunk's parse error key), written by (3)
constexpr int FTB = 512;                  // threads (= sites) per formatter block
constexpr int FMT_LDS2 = 32 * 1024;       // its record buffer: 4 blocks (32 waves) per CU
constexpr int LPB = 8;                    // formatter blocks per workgroup of the -m local length kernel
constexpr int SID_PUT_WAVES = 8;          // the -m local writer's min waves per SIMD (its LDS allows 8)

// sum of one u32 per thread over an NT-thread block (every thread gets it)
template <int NT>
__device__ __forceinline__ uint32_t block_sum(uint32_t v)
{
    __shared__ uint32_t wsum[NT / 64];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += wsum[w];
    __syncthreads();   // wsum reused by the next call
    return t;
}

// the block's records, assembled at buf[0, tot), to dst (any alignment):
// destination window k covers dst - phase + 16k; the inner windows read two
// aligned LDS quads and shift them by the block-uniform (-phase) & 15 bytes
// (QW words and R bytes): one copy of the loop per QW, so no lane selects
// the words (15 v_cndmask a window when QW was a variable)
template <bool SWZ, uint32_t QW>
__device__ __forceinline__ void block_store_q(const char* buf, uint32_t phase, uint32_t span, uint32_t r,
                                              char* __restrict__ dst)
{
    // SWZ: buf's quads are swizzled as swz_quad (the -m local writer's buffer)
    auto quad = [](uint32_t Q) { return SWZ ? (Q ^ ((Q >> 3) & 7u)) : Q; };
    const uint4* B = (const uint4*)buf;
    for (uint32_t k = threadIdx.x * 16; k < span; k += FTB * 16) {
        if (k >= phase && k + 16 <= span) {
            const uint32_t a16 = (k - phase) >> 4;   // quad holding byte k - phase
            const uint4 lo = B[quad(a16)], hi = B[quad(a16 + 1)];
            const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            // streaming (non-temporal) stores: the records are not read again on
            // the device, and kept out of the caches they leave room for the next
            // chunk's text (writer 0.965 -> 0.934 ms and the index behind it
            // 0.975 -> 0.93 ms per C2 step, A/B of builds on one box)
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 nv = {__builtin_amdgcn_alignbyte(w[QW + 1], w[QW], r),
                              __builtin_amdgcn_alignbyte(w[QW + 2], w[QW + 1], r),
                              __builtin_amdgcn_alignbyte(w[QW + 3], w[QW + 2], r),
                              __builtin_amdgcn_alignbyte(w[QW + 4], w[QW + 3], r)};
            __builtin_nontemporal_store(nv, (u32x4*)(dst + k));
        } else {
            for (uint32_t j = k; j < k + 16 && j < span; ++j)
                if (j >= phase) dst[j] = buf[quad((j - phase) >> 4) * 16 + ((j - phase) & 15u)];
        }
    }
}
template <bool SWZ = false>
__device__ __forceinline__ void block_store(const char* buf, uint32_t tot, char* __restrict__ dst0)
{
    const uint32_t phase = (uint32_t)((uintptr_t)dst0 & 15u);
    char* dst = dst0 - phase;   // 16-B aligned
    const uint32_t span = phase + tot;
    const uint32_t sh = (16u - phase) & 15u, r = sh & 3u;
    switch (sh >> 2) {   // (block-uniform)
    case 0: block_store_q<SWZ, 0>(buf, phase, span, r, dst); break;
    case 1: block_store_q<SWZ, 1>(buf, phase, span, r, dst); break;
    case 2: block_store_q<SWZ, 2>(buf, phase, span, r, dst); break;
    default: block_store_q<SWZ, 3>(buf, phase, span, r, dst); break;
    }
}

// ---- any method: code / hom_conf / het_conf per site (call kernels) ----
__global__ __launch_bounds__(FTB) void sid_fmt_blen_kernel(const char* __restrict__ text, uint64_t len,
                                                          const sid_off_t* __restrict__ starts,
                                                          const uint64_t* __restrict__ hdr, uint64_t n,
                                                          const uint8_t* __restrict__ code,
                                                          const double* __restrict__ hom,
                                                          const double* __restrict__ het, CType ct,
                                                          uint32_t* __restrict__ bsum, unsigned long long* lb)
{
    __shared__ double p10[SID_P10_N];
    load_p10(p10);
    const uint64_t i = (uint64_t)blockIdx.x * FTB + threadIdx.x;
    int l = 0;
    if (i < n) {
        const uint8_t c = code[i];
        if (!(c & 0x40)) {
            Reader R{text, len};
            const Head h = site_head(R, starts + i, hdr + 2 * i);
            l = record_len(h, c, sid_g6_prep(hom[i], p10), sid_g6_prep(het[i], p10), ct.len);
            if (l < 0) {
                atomicExch(lb + 2, 1ull);
                l = 0;
            }
        }
    }
    const uint32_t tot = block_sum<FTB>((uint32_t)l);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(FTB) void sid_fmt_put_kernel(const char* __restrict__ text, uint64_t len,
                                                         const sid_off_t* __restrict__ starts,
                                                         const uint64_t* __restrict__ hdr, uint64_t n,
                                                         const uint8_t* __restrict__ code,
                                                         const double* __restrict__ hom,
                                                         const double* __restrict__ het, CType ct,
                                                         const uint64_t* __restrict__ boff, const uint64_t* state,
                                                         unsigned long long* lb, char* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) char buf[FMT_LDS2 + 32];
    __shared__ double p10[SID_P10_N];
    load_p10(p10);
    const uint64_t i = (uint64_t)blockIdx.x * FTB + threadIdx.x;
    Reader R{text, len};
    int l = 0;
    uint8_t c = 0x40;
    Head h{0, 0, 0, 0};
    sid_g6 gh{}, gt{};
    if (i < n) {
        c = code[i];
        if (!(c & 0x40)) {
            h = site_head(R, starts + i, hdr + 2 * i);
            gh = sid_g6_prep(hom[i], p10);
            gt = sid_g6_prep(het[i], p10);
            l = record_len(h, c, gh, gt, ct.len);
            if (l < 0) l = 0;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) lb[4] = state[4];
    uint32_t tot;
    const uint32_t my = block_exscan<FTB>((uint32_t)l, &tot);
    char* const dst = out + boff[blockIdx.x];
    if (tot > FMT_LDS2) {   // long records (long chromosome names): straight to global
        if (l) record_put(R, h, c, gh, gt, ct, dst + my);
        return;
    }
    if (l) record_put(R, h, c, gh, gt, ct, buf + my);
    __syncthreads();
    block_store(buf, tot, dst);
}

// ---- -m local, fused with the call: the class of a site (local_site.h)
// gives its code and the text of its two confidences (the class tables'
// string tables, built with them per option set), so the call kernel's
// code / hom_conf / het_conf never round-trip HBM and no %g is computed
// per site.  Sites neither class table covers go through the fix-up (the
// fast / emulated evaluation of call.cpp:238-273), which adds their record
// bytes to the block sums and leaves code / confs for the writer.

// the class-table entry of a profile: 0 .. SID_TAB_N-1 (LDS table), then
// SID_TAB_N + the second-level index, or UINT32_MAX (neither)
__device__ __forceinline__ uint32_t local_entry(uint32_t nf, uint32_t ns, uint32_t r2)
{
    if (nf < SID_TAB_NF && ns < SID_TAB_NS && r2 < SID_TAB_NR) return sid_tab_slot(nf, ns, r2);
    if (nf < SID_TAB2_NF && ns < SID_TAB2_NS && r2 < SID_TAB2_NR)
        return SID_TAB_N + (nf * SID_TAB2_NS + ns) * SID_TAB2_NR + r2;
    return UINT32_MAX;
}

// chrom , pos , "hom,XY," / "het,XY," then the class's tail (the entry's
// "hom_conf,het_conf,p_value\n")
__device__ __forceinline__ int local_rec_len(const Head& h, uint32_t tail)
{
    return (int)h.clen + 1 + sid_i32_len(h.pos) + 1 + 7 + (int)tail;
}

// a site's -m local record length from its counts and header (the call's
// class-table entry -> the tail length); 0 and the site listed for the
// fix-up when neither table covers it
struct LocalLen {
    const uint8_t* len1;            // tail lengths of the LDS table's entries
    const uint8_t* len2;            // ... of the second-level table's
    uint32_t* bsum;                 // per FTB-site block: record bytes (zeroed before)
    uint32_t* miss;                 // sites for sid_local_fixlen_kernel
    unsigned long long* nmiss;
    uint32_t* cls;                  // per site its class word (sid_local_word)
};

// The -m local class word of a tabulated site, for the writer: the class-
// table entry (< 2^20) in bits 0-19, the major base in bits 28-29, the minor
// in 30-31.  SID_CLS_MISS (bits 20-27 set: no entry has them): the fix-up's
// site, whose record comes from its code and confidences.  The writer then
// reads 4 B a site instead of the 8 B counts, and skips getMajorAlleleIndices.
constexpr uint32_t SID_CLS_MISS = 0xFFFFFFFFu;
static_assert(SID_TAB_N + SID_TAB2_N <= (1u << 20), "class entries fit the word's 20 bits");
__device__ __forceinline__ uint32_t local_word(uint32_t k, uint32_t f, uint32_t s)
{
    return k | (f << 28) | (s << 30);
}
// The tile parse's compact word (lane shape): SID_CLS_COMPACT set and the
// position's offset (0..127) from its wave's reference line in bits 20-26;
// the chrom (at most 8 bytes) and the reference position are the wave's
// entry (tile_wave_store), so the site needs no header pair (the slot's 4 B
// instead of 20 B, each way).  No compact word is SID_CLS_MISS: k < 0xFFFFF.
constexpr uint32_t SID_CLS_COMPACT = 1u << 27;
constexpr uint32_t SID_CLS_DPOS = 128;   // offsets 0 .. 127
static_assert(SID_TAB_N + SID_TAB2_N < 0xFFFFFu, "a compact word never equals SID_CLS_MISS");
__device__ __forceinline__ bool cls_compact(uint32_t w) { return (w & SID_CLS_COMPACT) && w != SID_CLS_MISS; }

// The site's record length (0: a fix-up site, listed in LL.miss; a record
// is never empty) and its class word into LL.cls[i]
// local_site_tail: the tail's length of the record (its bytes after "chrom,
// pos,label,"; local_rec_len), -1 for a fix-up site.  (The tail lengths of
// the ~200x profiles copied into LDS by every quad-shape block, 4 KiB, took
// C5's parse 11.41 -> 11.28 ms per step, but cost more than it saved beside
// quad_head: 11.19 with it, 11.03 without; for the lane shape, 2 KiB of the
// ~30x profiles: C2 parse 1.79 -> 1.92 ms.)
// the class word and tail length alone (-1 and SID_CLS_MISS: a fix-up site)
__device__ __forceinline__ int local_site_word(uint64_t c, const uint8_t* L1, const LocalLen& LL, uint32_t* w)
{
    uint32_t f, s, nf, ns, cov;
    sid_major(c, f, s, nf, ns, cov);
    const uint32_t k = local_entry(nf, ns, cov - nf - ns);
    const uint32_t L = k < SID_TAB_N ? L1[k] : k != UINT32_MAX ? LL.len2[k - SID_TAB_N] : 0xFFu;
    *w = L == 0xFFu ? SID_CLS_MISS : local_word(k, f, s);
    return L == 0xFFu ? -1 : (int)L;
}
template <bool LIST = true>   // LIST: a fix-up site listed in LL.miss (else the caller fixes it up)
__device__ __forceinline__ int local_site_tail(uint64_t c, uint64_t i, const uint8_t* L1, const LocalLen& LL)
{
    uint32_t w;
    const int L = local_site_word(c, L1, LL, &w);
    const bool miss = L < 0;
    LL.cls[i] = w;   // (read back by the writer soon: through the caches)
    if (miss) {
        if (LIST) LL.miss[atomicAdd(LL.nmiss, 1ull)] = (uint32_t)i;   // its bytes: the fix-up's
        return -1;
    }
    return (int)L;
}
__device__ __forceinline__ int local_site_len(const Head& h, uint64_t c, uint64_t i, const uint8_t* L1,
                                              const LocalLen& LL)
{
    const int L = local_site_tail(c, i, L1, LL);
    return L < 0 ? 0 : local_rec_len(h, (uint32_t)L);
}

// (out of line: its tokeniser would set the parse's register count)
__device__ __noinline__ int local_site_len_text(const char* text, uint64_t len, uint64_t s0, uint64_t c, uint64_t i,
                                                LocalLen LL)
{
    Reader R{text, len};
    return local_site_len(site_head(R, &s0, nullptr), c, i, LL.len1, LL);
}

// The parse with the -m local call's record lengths fused in (the length
// kernel then only has the fix-up left): the per-line fast path as
// sid_parse_kernel, then each parsed line's class entry and record length,
// summed per wave (a wave's 64 lines lie in one FTB-site block) into the
// block's byte count.  Lines the fast path leaves get theirs after the
// general routine (sid_local_len_list_kernel).  The tail-length table is read
// through the caches (an LDS copy would cost the parse a block per CU).
// (the two-pass fallback's parse since the tile parse: 7 waves a SIMD)
__global__ __launch_bounds__(TB) void sid_parse_len_kernel(const char* __restrict__ text, uint64_t len,
                                                           const sid_off_t* __restrict__ starts,
                                                           const uint64_t* __restrict__ range,
                                                           uint64_t* __restrict__ counts,
                                                           uint64_t* __restrict__ hdr, uint32_t* __restrict__ fb,
                                                           unsigned long long* fbn, LocalLen LL)
{
    static_assert(FTB % 64 == 0 && TB % 64 == 0, "a wave's lines lie in one formatter block");
    __shared__ uint8_t cls[256];
    __shared__ uint32_t rbl[RB_LUT_N];
    __shared__ __attribute__((aligned(16))) char stage[TB * HDR_BYTES + 64];
    if (threadIdx.x < 256) {
        cls[threadIdx.x] = k_tp_tables.cls[threadIdx.x];
        rbl[threadIdx.x] = k_tp_tables.rb[threadIdx.x];
        if (threadIdx.x < RB_LUT_N - 256) rbl[256 + threadIdx.x] = k_tp_tables.rb[256 + threadIdx.x];
    }
    __syncthreads();
    const uint64_t lo = range[0], hi = range[1];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t w0 = lo + (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);   // the wave's first line
    uint64_t i = w0 + (threadIdx.x & 63u);
    uint64_t s_next = i < hi ? starts[i] : 0;
    for (uint64_t wb = w0; wb < hi; wb += stride, i += stride) {   // wave-uniform trip count
        const uint64_t s0 = s_next;
        if (i + stride < hi) s_next = starts[i + stride];
        int l = 0;
        if (i < hi) {
            uint64_t c = 0, h[2] = {0, 0};
            if (parse_line_fast(text, len, s0, cls, stage + threadIdx.x * HDR_BYTES, &c, h, rbl)) {
                ST_MID(hdr + 2 * i, h[0]);
                ST_MID(hdr + 2 * i + 1, h[1]);
                if (h[0] >> 63) {
                    Head hd;
                    hd.clen = (uint32_t)(h[0] >> 32) & 0xFFFu;
                    hd.pos = (int32_t)(uint32_t)h[0];
                    l = local_site_len(hd, c, i - lo, LL.len1, LL);
                } else {   // position not a plain 1-9 digit run: the formatter's tokeniser
                    l = local_site_len_text(text, len, s0, c, i - lo, LL);
                }
                if (l == 0) counts[i] = c;   // a fix-up site: the fix-up reads its counts (the writer, the class word)
            } else {
                fb[atomicAdd(fbn, 1ull)] = (uint32_t)(i - lo);
            }
        }
        const uint32_t sl = wave_sum((uint32_t)l);
        if ((threadIdx.x & 63u) == 0 && sl) atomicAdd(LL.bsum + (wb - lo) / FTB, sl);
    }
}

// the record lengths of listed sites (the lines the general routine parsed)
__global__ __launch_bounds__(TB) void sid_local_len_list_kernel(const char* __restrict__ text, uint64_t len,
                                                               const sid_off_t* __restrict__ starts,
                                                               const uint64_t* __restrict__ hdr,
                                                               const uint64_t* __restrict__ counts,
                                                               const uint32_t* __restrict__ list,
                                                               const unsigned long long* nlist, LocalLen LL)
{
    const uint64_t m = *nlist;
    for (uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x; j < m; j += (uint64_t)gridDim.x * TB) {
        const uint32_t i = list[j];
        Reader R{text, len};
        const int l = local_site_len(site_head(R, starts + i, hdr + 2 * i), counts[i], i, LL.len1, LL);
        if (l) atomicAdd(LL.bsum + i / FTB, (uint32_t)l);
    }
}

// ------------------------------------------------------------ tile parse --
// The engine's -m local path for lines of up to 256 B on average (30x): the
// line index fused into the parse, so the text is fetched from HBM once and
// no host round trip separates index and parse (pileup.cpp:13-153 +
// call.cpp:213-289 up to the record lengths).  One 256-thread block per tile
// of TP_TILE bytes, copied to LDS with a halo (tp_halo) after it (a
// line that starts in the tile is read from LDS to its end in nearly every
// case; one that runs past the halo reads the rest from HBM):
//   load    the tile's 16-B windows, lanes contiguous, non-temporal (each
//           byte is read once), into LDS
//   index   line starts per window (the index kernel's masks), one block scan
//           in file order -> the offsets of the tile's lines in LDS
//   parse   one lane per line: the fast path (parse_header + read_bases_lut)
//           from LDS; the call's class entry and record length
//           (local_site_len), summed per wave into the writer block's bytes
//   write   per line its slot g = tile * cap + j (j: the line's rank in the
//           tile): class word and header pair; per tile its site count
// Outputs are laid out per tile, cap slots each (slots past a tile's count
// are never written or read), so no prefix over the tiles is needed before
// the parse.  A tile with more lines than cap leaves the rest unparsed and
// reports its count (lb[5]): the host runs the chunk again with a larger cap
// (the chunk's records are dropped), or through the two-pass path.
// The header pair's second word holds the chrom's first 8 bytes when the
// pair is valid and the chrom at most 8 bytes long, else the line's offset
// (slot_head): the writer never needs a line offset array.
// Two shapes: 20 KiB tiles with a lane per line (30x: ~253 lines of ~81 B
// per tile: one round of the block's 256 lanes, a few lines of a second now
// and then; 16 KiB tiles, ~202 lines, left a fifth of the lanes idle), and
// 24 KiB tiles with a quad of lanes per line (200x: ~58 lines of ~426 B, 232
// lanes; read_bases_quad, each quad reading 64 consecutive bytes a step).
constexpr uint32_t TP_ROWS = 5;                 // (the lane-per-line shape: ~253 lines a tile, one round of 256 lanes)
constexpr uint32_t TP_ROWS_QUAD = 6;
// the halo and the line list per shape: the quad shape's tiles hold few
// lines (the host picks it for lines over 256 B on average), so 256 slots.
// (A 512-B halo, LDS for six blocks a CU instead of five, measured slower:
// 12.93 vs 12.78 ms per C5 step; again with the loads issued together and
// no tail-length window, 11.46 vs 11.28 ms; with the window, still five
// blocks, 11.24 vs 11.28 ms: noise.  The LDS limit is byte-exact:
// tools/debug/lds_occ_probe.hip, 27306 B six blocks, 27307 B five.)
__host__ __device__ constexpr uint32_t tp_halo(bool) { return 1024; }
__host__ __device__ constexpr uint32_t tp_cap_max(bool quad) { return quad ? SID_TILE_CAP_MAX_QUAD : SID_TILE_CAP_MAX; }
__host__ __device__ constexpr uint32_t tp_tile(bool quad) { return (quad ? TP_ROWS_QUAD : TP_ROWS) * TILE; }

struct TileOut {
    uint32_t cap;               // slots per tile (a multiple of 16, powers of 2 included, SID_TILE_CAP_MIN .. _MAX)
    uint32_t* tcnt;             // per tile: its lines (above the cap: overflow; the writer takes the first cap)
    uint64_t* hdr;              // per slot: the header pair
    uint64_t* counts;           // per slot: counts of the fix-up's and the general routine's sites
    uint32_t* fb;               // the general routine's lines: slots,
    uint32_t* fbo;              // ... and line offsets
    unsigned long long* lb;     // [6] fallback count (zeroed before); [3] sites and [5] the most lines in a
                                //   tile from tcnt (sid_tile_serial_kernel)
    uint64_t* state;            // [4] the chunk's parse error key: none yet
    ulonglong2* twv;            // -m local, lane shape: per tile nwv wave entries (tile_wave_store), entry
    uint32_t nwv;               //   j / 64 for the tile's slot j
};

// a slot's chrom and position from its header pair (the tile parse's layout)
__device__ __forceinline__ Head slot_head(Reader& R, const ulonglong2 hw)
{
    if (hw.x >> 63) {
        Head h;
        h.clen = (uint32_t)(hw.x >> 32) & 0xFFFu;
        h.pos = (int32_t)(uint32_t)hw.x;
        h.c8 = h.clen <= 8 ? hw.y : 0;
        h.cb = h.clen <= 8 ? 0 : (uint64_t)(uint32_t)hw.y + ((hw.x >> 44) & 0x7FFFull);
        return h;
    }
    const uint64_t s0 = (uint32_t)hw.y;
    return site_head_hw(R, &s0, make_ulonglong2(0, 0));
}

// One line of a lane-shape tile from its LDS copy (tl: the copy of the text
// from global offset g0 on, ld: a 16-B window at an offset from g0, from LDS
// or past its end from HBM): the fast path (parse_header, then
// read_bases_lut), then the line's outputs into slot g (header pair; -m
// local's class word and record length, returned; the Lynch paths' counts),
// or its slot and offset listed for the general routine.  (The quad shape:
// quad_head, then quad_line.)
// -m local's lines with a valid header pair, a chrom of at most 8 bytes and a
// tabulated class leave their slot words to the wave (tile_wave_store): ws.
struct LaneSlot {
    uint64_t h0 = 0, h1 = 0;   // the header pair
    uint32_t w = 0;            // the class word
    uint32_t pl = 0;           // the position's digits
    bool elig = false;         // the words are the wave's to store
};
template <bool LOCAL, class Ld>
__device__ __forceinline__ int tile_line(const char* __restrict__ text, const char* tl, Ld ld, uint64_t g0, uint32_t r0,
                                         uint64_t g, uint32_t len_t, uint64_t c1, const uint8_t* cls,
                                         const uint32_t* rbl, const TileOut& O, const LocalLen& LL, LaneSlot& ws)
{
    int l = 0;
    const uint64_t s0 = g0 + r0;
    const char* stage = tl + (r0 & ~15u);
    const uint32_t sh = r0 & 15u;
    const uint4 v0 = *(const uint4*)stage, v1 = *(const uint4*)(stage + 16), v2 = *(const uint4*)(stage + 32);
    uint64_t c = 0, h[2] = {0, 0}, low48 = 0;
    uint32_t kd = 0;
    const int t4 = parse_header(v0, v1, v2, stage, sh, len_t - r0, cls, h, &kd, &low48);
    bool ok = t4 >= 0;
    if (ok) {
        const uint32_t fw = (sh + (uint32_t)t4) & 0x30u;   // the read bases' first window (0, 16 or 32)
        ok = read_bases_lut<Ld, uint32_t>(ld, len_t, r0 + (uint32_t)t4, kd, rbl, (const uint4*)(stage + fw), &c,
                                          (uint32_t)(low48 >> fw) & 0xFFFFu);
    }
    if (ok) {
        const bool hv = (h[0] >> 63) != 0;
        const uint32_t clen = (uint32_t)(h[0] >> 32) & 0xFFFu;
        if (!hv || clen > 8) h[1] = (uint32_t)s0;   // the writer reads the chrom, or tokenises, from the line
        Head hd;
        hd.clen = clen;
        hd.pos = (int32_t)(uint32_t)h[0];
        if (LOCAL && hv && clen <= 8) {
            uint32_t w;
            const int L = local_site_word(c, LL.len1, LL, &w);
            if (L >= 0) {   // (a fix-up site: stored here, below)
                ws.h0 = h[0];
                ws.h1 = h[1];
                ws.w = w;
                ws.pl = (uint32_t)(h[0] >> 59) & 15u;   // (parse_header: the printed digits)
                ws.elig = true;
                return (int)(clen + ws.pl + 9 + (uint32_t)L);   // (local_rec_len)
            }
        }
        ST_MID(O.hdr + 2 * g, h[0]);
        ST_MID(O.hdr + 2 * g + 1, h[1]);
        if (!LOCAL) {
            ST_MID(O.counts + g, c);
        } else if (hv) {
            l = local_site_len(hd, c, g, LL.len1, LL);
        } else {   // position not a plain 1-9 digit run: the formatter's tokeniser
            l = local_site_len_text(text, c1, s0, c, g, LL);
        }
        if (LOCAL && l == 0) O.counts[g] = c;   // a fix-up site: the fix-up reads its counts
    } else {
        const unsigned long long k = atomicAdd(O.lb + 6, 1ull);
        O.fb[k] = (uint32_t)g;
        O.fbo[k] = (uint32_t)s0;
    }
    return l;
}

// The wave's deferred slot words (converged lanes, slot g): the lowest lane
// with words is the wave's reference, its chrom and position the wave's entry
// (*e); a lane of the same chrom within SID_CLS_DPOS positions after it
// stores only its compact class word, the others the class word and the
// header pair.  The entry: the chrom's 8 bytes; the position p0, the chrom's
// length (bits 32-43), p0's digits n (44-47) and the offsets from p0 where
// the digits grow, 10^n - p0 and 10^(n+1) - p0 (48-55, 56-63; 255: not below
// SID_CLS_DPOS), so the writer counts a compact site's digits in 4
// instructions (wave_pos_digits)
__device__ constexpr uint64_t k_pow10[16] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
                                              10000000ull, 100000000ull, 1000000000ull, 10000000000ull,
                                              100000000000ull, 0, 0, 0, 0};
__device__ __forceinline__ void tile_wave_store(const LaneSlot& ws, uint64_t g, ulonglong2* e, const TileOut& O,
                                                const LocalLen& LL)
{
    const uint64_t em = __ballot(ws.elig);
    if (em == 0) return;   // (wave-uniform)
    const int r = __builtin_ctzll(em);
    const uint32_t c8lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ws.h1, r);
    const uint32_t c8hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ws.h1 >> 32), r);
    const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ws.h0, r);
    const uint32_t cl0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ws.h0 >> 32), r) & 0xFFFu;
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)ws.pl, r);
    const uint64_t c8 = c8lo | ((uint64_t)c8hi << 32);
    const uint32_t dp = (uint32_t)ws.h0 - p0;
    const bool cmp = ws.elig && ws.h1 == c8 && (((uint32_t)(ws.h0 >> 32) & 0xFFFu) == cl0) && dp < SID_CLS_DPOS;
    if ((int)(threadIdx.x & 63u) == r) {
        const uint64_t p10 = k_pow10[n0 & 15u];   // (n0 <= 9: a valid pair's position has at most 9 digits)
        const uint64_t d1 = p10 - p0, d2 = 10u * p10 - p0;
        const uint64_t y = (uint64_t)p0 | ((uint64_t)cl0 << 32) | ((uint64_t)n0 << 44) |
                           ((d1 < SID_CLS_DPOS ? d1 : 255ull) << 48) | ((d2 < SID_CLS_DPOS ? d2 : 255ull) << 56);
        *e = make_ulonglong2(c8, y);
    }
    if (cmp) {
        LL.cls[g] = ws.w | SID_CLS_COMPACT | (dp << 20);
    } else if (ws.elig) {
        LL.cls[g] = ws.w;
        ST_MID(O.hdr + 2 * g, ws.h0);
        ST_MID(O.hdr + 2 * g + 1, ws.h1);
    }
}

// The quad shape in two steps.  A line's header is the same work in each of
// its quad's four lanes, so it is parsed a lane per line first (the tile's
// ~58 lines of 200x: one wave instead of four), its outputs stored, and what
// the quad needs passed on in LDS: bit 0 the header parsed, bits 1-6 the
// offset of token 4, 7-9 the class '.'/',' stand for, 10 the header pair
// valid, 11-23 the record's length but its tail ("chrom,pos,label,":
// local_rec_len with no tail).  A line whose header takes the general
// routine is listed for it here.
template <bool LOCAL>
__device__ __forceinline__ uint32_t quad_head(const char* tl, uint64_t g0, uint32_t r0, uint64_t g, uint32_t len_t,
                                              const uint8_t* cls, const TileOut& O)
{
    const uint64_t s0 = g0 + r0;
    const char* stage = tl + (r0 & ~15u);
    const uint32_t sh = r0 & 15u;
    const uint4 v0 = *(const uint4*)stage, v1 = *(const uint4*)(stage + 16), v2 = *(const uint4*)(stage + 32);
    uint64_t h[2] = {0, 0};
    uint32_t kd = 0;
    const int t4 = parse_header(v0, v1, v2, stage, sh, len_t - r0, cls, h, &kd);
    if (t4 < 0) {
        const unsigned long long k = atomicAdd(O.lb + 6, 1ull);
        O.fb[k] = (uint32_t)g;
        O.fbo[k] = (uint32_t)s0;
        return 0;
    }
    const bool hv = (h[0] >> 63) != 0;
    const uint32_t clen = (uint32_t)(h[0] >> 32) & 0xFFFu;
    if (!hv || clen > 8) h[1] = (uint32_t)s0;   // the writer reads the chrom, or tokenises, from the line
    // (stored before the read bases are counted: a line the general routine
    // then takes gets both words again from sid_tile_serial_kernel)
    ST_MID(O.hdr + 2 * g, h[0]);
    ST_MID(O.hdr + 2 * g + 1, h[1]);
    Head hd;
    hd.clen = clen;
    hd.pos = (int32_t)(uint32_t)h[0];
    const uint32_t base = hv ? (uint32_t)local_rec_len(hd, 0) : 0u;   // (< 2^13: the chrom below 4096 B)
    return 1u | ((uint32_t)t4 << 1) | (kd << 7) | ((uint32_t)hv << 10) | (base << 11);
}

// the quad's part of a line (its header from quad_head): the read bases
// counted by the quad; the lead lane lists the line for the general routine
// when they need it, else stores its counts (the Lynch paths'), or, for
// -m local, keeps them in LDS for quad_tail (bit 31 of the line's word: counted)
template <bool LOCAL, class Ld>
__device__ __forceinline__ void quad_bases(const char* tl, Ld ld, uint64_t g0, uint32_t r0, uint32_t* meta,
                                           uint64_t* cnt_l, uint64_t g, uint32_t len_t, bool lead,
                                           const uint32_t* rbl, const TileOut& O)
{
    const uint32_t mt = *meta;
    if (!(mt & 1u)) return;   // (the whole quad: the general routine's line)
    const uint32_t q = r0 + ((mt >> 1) & 63u), kd = (mt >> 7) & 7u;
    uint64_t c = 0;
    const bool ok = read_bases_quad<Ld, uint32_t>(ld, len_t, q, kd, rbl, (const uint4*)(tl + (q & ~15u)), &c);
    if (!lead) return;
    if (!ok) {
        const unsigned long long k = atomicAdd(O.lb + 6, 1ull);
        O.fb[k] = (uint32_t)g;
        O.fbo[k] = (uint32_t)(g0 + r0);
    } else if (!LOCAL) {
        ST_MID(O.counts + g, c);
    } else {
        *cnt_l = c;
        *meta = mt | (1u << 31);
    }
}

// -m local's call of a counted quad-shape line, a lane per line as the
// header: the class word, the record's length (returned; 0 for a fix-up site
// or a line not counted here)
__device__ __forceinline__ int quad_tail(const char* __restrict__ text, uint64_t s0, uint32_t mt, uint64_t c, uint64_t g,
                                         uint64_t c1, const TileOut& O, const LocalLen& LL)
{
    if (!(mt >> 31)) return 0;
    int l;
    if ((mt >> 10) & 1u) {
        const int L = local_site_tail(c, g, LL.len1, LL);
        l = L < 0 ? 0 : (int)((mt >> 11) & 0x1FFFu) + L;
    } else {   // position not a plain 1-9 digit run: the formatter's tokeniser
        l = local_site_len_text(text, c1, s0, c, g, LL);
    }
    if (l == 0) O.counts[g] = c;   // a fix-up site: the fix-up reads its counts
    return l;
}

// LOCAL: -m local's class words and record lengths (sid_chunk_tile_local);
// else every site's counts (the Lynch paths' first pass, sid_chunk_tile_counts).
// One block per tile.  (Round 5 kept a later tile's lines in flight into L2
// while a block parsed, one 4-B load per 128-B line: with the tile loaded by
// LDS-DMA that prefetch fetched 101 B a site for 86 without it, and the
// parse took 1.714-1.722 ms per C2 step for 1.698-1.702: profiles/ab_tile_r06.log.)
#ifdef SID_TP_STAMP
// (diagnostic builds: per-phase wall-clock stamps of the tile parse's and the
// -m local writer's blocks, thread 0 of each)
constexpr uint32_t TP_STAMP_N = 1u << 20;
__device__ uint32_t tp_stamp[TP_STAMP_N][4];
__device__ uint32_t put_stamp[TP_STAMP_N][4];
#define TP_STAMP_AT(v) const uint64_t v = tid == 0 ? wall_clock64() : 0
#define PUT_STAMP_AT(v) const uint64_t v = threadIdx.x == 0 ? wall_clock64() : 0
#else
#define TP_STAMP_AT(v)
#define PUT_STAMP_AT(v)
#endif
template <bool QUAD, bool LOCAL>
__global__ __launch_bounds__(TB) void sid_tile_parse_kernel(const char* __restrict__ text, uint64_t tile_base,
                                                            uint64_t c0, uint64_t c1, TileOut O, LocalLen LL)
{
    constexpr uint32_t ROWS = QUAD ? TP_ROWS_QUAD : TP_ROWS, TP_TILE = ROWS * TILE;
    constexpr uint32_t LPR = QUAD ? TB / 4 : TB;   // lines per round of the block
    // a window has at most 8 line starts, a wave's row at most 512: 10-bit
    // fields, three rows a word
    constexpr uint32_t NW = (ROWS + 2) / 3;
    static_assert(TB == 256 && ROWS <= 9, "a lane's windows: three u32s of line-start counts");
    static_assert(FTB % 64 == 0, "a wave's slots lie in one writer block");
    constexpr uint32_t TP_HALO = tp_halo(QUAD);
    static_assert(TP_HALO % 1024 == 0 && TP_HALO / 16 <= TB, "the halo loaded by whole waves, a window a lane");
    __shared__ __attribute__((aligned(16))) char tl[TP_TILE + TP_HALO + 64];
    __shared__ uint16_t ls[tp_cap_max(QUAD) + TB];   // (+ a dummy slot per thread: the index's absent starts)
    __shared__ uint8_t cls[256];
    __shared__ uint32_t rbl[RB_LUT_N];
    __shared__ uint32_t wtot[TB / 64][NW];
    __shared__ uint32_t qmeta[QUAD ? tp_cap_max(true) : 1];   // the quad shape's headers (quad_head)
    __shared__ uint64_t qcnt[QUAD && LOCAL ? tp_cap_max(true) : 1];   // ... and counts (quad_bases)
    const uint32_t tid = threadIdx.x;
    if (blockIdx.x == 0 && tid == 0) O.state[4] = ~0ull;   // no parse error yet
    const uint32_t cap = O.cap;
    {
        const uint64_t t = blockIdx.x;
        TP_STAMP_AT(st0);
        // the load and the index (block-wide barriers: a block waits for its
        // slowest wave) at raised priority over other blocks' per-line parse:
        // C2 parse 1.777 -> 1.747 ms; the quad shape at 2 once its loads are
        // out (C5 10.91 -> 10.85; at 3 throughout: 10.92)
        __builtin_amdgcn_s_setprio(3);
        const uint64_t g0 = tile_base + t * TP_TILE;           // the tile's first byte (16-B aligned)
        // a tile inside the chunk (all but its first and last): no window needs
        // the chunk's bounds (block-uniform)
        const bool inner = g0 > c0 && g0 + TP_TILE <= c1;
        // ---- load: the tile and its halo straight into LDS by LDS-DMA
        // (global_load_lds_dwordx4: one wave-instruction fills 1 KiB at the
        // wave's base, lane-linear; no VGPR holds the tile), then each lane's
        // windows read back for the index.  A window at or past the chunk's
        // end loads the tile's first window instead (g0 < c1, readable as
        // every window before c1 is) and is zeroed once it has landed.
        // (Against register loads stored to LDS: C2 parse 1.701-1.707 vs
        // 1.714-1.726 ms per step, C5 10.19 vs 10.19-10.22: profiles/ab_tile_r06.log.)
        const uint64_t hat = g0 + TP_TILE + tid * 16;
        const bool hok = hat < c1;
        // the byte before the tile (one address for the block)
        const bool pok = g0 > c0 && g0 - 1 < c1;
        const uint32_t pbyte = (uint8_t)text[pok ? g0 - 1 : g0];
        {
            typedef __attribute__((address_space(3))) void lds_void;
            // (the wave's LDS base and the tile's text as scalars; an inner
            // tile's rows at a 32-bit lane offset from it: no per-lane 64-bit
            // bounds select a row)
            const uint32_t wb = __builtin_amdgcn_readfirstlane((tid & ~63u) * 16u);
            const char* const gt = text + g0;
            if (inner) {
#pragma unroll
                for (uint32_t k = 0; k < ROWS; ++k)
                    __builtin_amdgcn_global_load_lds((const void*)(gt + (k * TILE + tid * 16)),
                                                     (lds_void*)(tl + k * TILE + wb), 16, 0, 2 /* nt */);
            } else {
#pragma unroll
                for (uint32_t k = 0; k < ROWS; ++k) {
                    const uint64_t at = g0 + k * TILE + tid * 16;
                    __builtin_amdgcn_global_load_lds((const void*)(text + (at < c1 ? at : g0)),
                                                     (lds_void*)(tl + k * TILE + wb), 16, 0, 2 /* nt */);
                }
            }
            if (tid < TP_HALO / 16)   // (whole waves)
                __builtin_amdgcn_global_load_lds((const void*)(text + (hok ? hat : g0)), (lds_void*)(tl + TP_TILE + wb),
                                                 16, 0, 0);
            // the LDS tables, loaded while the tile's pieces are in flight
            // (copied in before them, their load's wait came before the
            // tile's loads were issued)
            // (all three loads issued before any LDS store: a store waits for
            // every load ahead of it, the DMA's included)
            const uint8_t cv = k_tp_tables.cls[tid];
            const uint32_t rv = k_tp_tables.rb[tid], nv = k_tp_tables.rb[256 + (tid & (RB_LUT_N - 257))];
            cls[tid] = cv;
            rbl[tid] = rv;
            rbl[256 + (tid & (RB_LUT_N - 257))] = nv;   // (every lane: the same values, no branch to sink the load into)
            __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): this wave's pieces have landed
            if (!inner) {
#pragma unroll
                for (uint32_t k = 0; k < ROWS; ++k)
                    if (g0 + k * TILE + tid * 16 >= c1) *(uint4*)(tl + k * TILE + tid * 16) = make_uint4(0, 0, 0, 0);
            }
            if (tid < TP_HALO / 16 && !hok) *(uint4*)(tl + TP_TILE + tid * 16) = make_uint4(0, 0, 0, 0);
            // (the padding after the halo zeroed once the wave's pieces have
            // landed: an LDS store issued before the wait made the compiler
            // wait for the wave's DMA first, ahead of the tables' loads)
            if (tid < 4) *(uint32_t*)(tl + TP_TILE + TP_HALO + 4 * tid) = 0u;
        }
        if constexpr (QUAD) __builtin_amdgcn_s_setprio(2);
        // is the byte before the tile a '\n' (1 when there is none: the tile starts the chunk)
        const uint32_t prev0 = tid ? 0u : pok ? (pbyte == '\n') : 1u;
        __syncthreads();
        uint4 v[ROWS];
#pragma unroll
        for (uint32_t k = 0; k < ROWS; ++k) v[k] = *(const uint4*)(tl + k * TILE + tid * 16);
        TP_STAMP_AT(st1);
        // ---- line starts (bit j: byte j of the window starts a non-empty line in [c0, c1))
        // (the windows' newline masks computed before the barrier, while the
        // block's other loads land, measured 1 % slower: parse 1.912 vs 1.889
        // ms per C2 step)
        uint32_t m[ROWS];
        uint32_t packed[NW];
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) packed[w] = 0;
        // the byte before each window (one LDS round trip for all rows)
        uint32_t pb[ROWS];
#pragma unroll
        for (uint32_t k = 0; k < ROWS; ++k) pb[k] = (uint8_t)tl[max(k * TILE + tid * 16, 1u) - 1];
#pragma unroll
        for (uint32_t k = 0; k < ROWS; ++k) {
            const uint64_t at = g0 + k * TILE + tid * 16;
            const uint4 w = v[k];
            const uint32_t nl = compress16(eq_bytes(w.x, 0x0A0A0A0Au), eq_bytes(w.y, 0x0A0A0A0Au),
                                           eq_bytes(w.z, 0x0A0A0A0Au), eq_bytes(w.w, 0x0A0A0A0Au));
            const uint32_t prev = (k == 0 && tid == 0) ? prev0 : (uint32_t)(pb[k] == '\n');
            uint32_t mk = ((nl << 1) | prev) & ~nl & 0xFFFFu;
            if (!inner) {
                if (at + 16 > c0 && at <= c0) {   // c0 in this window: it starts a line (unless a '\n'), nothing before it does
                    const uint32_t j = (uint32_t)(c0 - at);
                    mk = (mk | ((1u << j) & ~nl)) & ~((1u << j) - 1u);
                }
                if (at + 16 > c1) mk &= c1 > at ? (1u << (uint32_t)(c1 - at)) - 1u : 0u;
                if (at + 16 <= c0) mk = 0;
            }
            m[k] = mk;
            packed[k / 3] |= (uint32_t)__popc(mk) << (10 * (k % 3));
        }
        // their ranks in file order: a scan over the wave's lanes (DPP, no
        // LDS round trip), the waves before this one from LDS
        uint32_t incl[NW];
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) incl[w] = wave_scan_incl(packed[w]);
        const uint32_t wid = __builtin_amdgcn_readfirstlane(tid >> 6);
        if ((tid & 63u) == 63u) {
#pragma unroll
            for (uint32_t w = 0; w < NW; ++w) wtot[wid][w] = incl[w];
        }
        __syncthreads();
        // the waves' sums, wave-uniform (scalar): a word's fields 0 and 2,
        // and field 1, summed apart (up to 2048 a row: 12 bits, room to grow)
        uint32_t bA[NW], bB[NW], tA[NW], tB[NW];
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w) {
            bA[w] = bB[w] = tA[w] = tB[w] = 0;
#pragma unroll
            for (uint32_t w2 = 0; w2 < TB / 64; ++w2) {
                const uint32_t x = __builtin_amdgcn_readfirstlane(wtot[w2][w]);
                const uint32_t xa = x & 0x3FF003FFu, xb = x & 0x000FFC00u;
                tA[w] += xa;
                tB[w] += xb;
                bA[w] += w2 < wid ? xa : 0u;
                bB[w] += w2 < wid ? xb : 0u;
            }
        }
        uint32_t nlines = 0;
#pragma unroll
        for (uint32_t k = 0; k < ROWS; ++k) {
            const uint32_t sh = 10 * (k % 3), w = k / 3;
            const uint32_t before = (((k % 3) == 1 ? bB[w] : bA[w]) >> sh) & 4095u;
            const uint32_t total = (((k % 3) == 1 ? tB[w] : tA[w]) >> sh) & 4095u;
            const uint32_t q = nlines + before + (((incl[w] - packed[w]) >> sh) & 1023u);
            // the window's first start written unconditionally (to the
            // thread's dummy slot when absent or past the cap), the rest --
            // lines under 16 B -- one by one: no exec-masked loop per window
            const uint32_t mk = m[k], off = k * TILE + tid * 16, dummy = tp_cap_max(QUAD) + tid;
            ls[mk && q < cap ? q : dummy] = (uint16_t)(off + (uint32_t)__builtin_ctz(mk | 0x10000u));
            uint32_t q2 = q + 1;
            for (uint32_t r = mk & (mk - 1); r; r &= r - 1, ++q2)
                if (q2 < cap) ls[q2] = (uint16_t)(off + (uint32_t)(__ffs(r) - 1));
            nlines += total;
        }
        const uint32_t cnt = min(nlines, cap);
        if (tid == 0) O.tcnt[t] = nlines;   // (no atomics on one address from every block: summed by the next kernel)
        __syncthreads();
        TP_STAMP_AT(st2);
        __builtin_amdgcn_s_setprio(0);
        // ---- parse, one lane (a quad of lanes) per line, from LDS; offsets
        // from the tile's first byte (32 bits: a chunk spans less than 4 GiB)
        const char* gtile = text + g0;
        // (the global load non-temporal: two loads of a kind would be merged into
        // one generic-address (flat) load of a selected pointer, the LDS reads too)
        auto ld = [&](uint32_t r) -> uint4 {
            if (r <= TP_TILE + TP_HALO - 16) return *(const uint4*)(tl + r);
            return ld_nt(gtile + r);   // (a line running past the halo)
        };
        const uint32_t len_t = (uint32_t)(c1 - g0);   // the chunk's end
        const uint64_t g_tile = t * (uint64_t)cap;
        // the record bytes of a round's lines (slot g_tile + j0 + lane's line)
        // into the writer blocks' sums: a wave's slots (64, or 16 with quads,
        // from a multiple of 16) lie in one block or two
        auto bsum_add = [&](uint32_t wslot0, uint32_t j, int l) {
            wslot0 = __builtin_amdgcn_readfirstlane(wslot0);
            const uint64_t gw = (g_tile + wslot0) / FTB;
            if ((g_tile + wslot0 + 63) / FTB == gw) {   // (most waves: their slots in one block, one sum)
                const uint32_t s = wave_sum((uint32_t)l);
                if ((tid & 63u) == 0 && s) atomicAdd(LL.bsum + gw, s);
                return;
            }
            const uint32_t lo = (g_tile + j) / FTB == gw ? (uint32_t)l : 0u;
            const uint32_t slo = wave_sum(lo), shi = wave_sum((uint32_t)l - lo);
            if ((tid & 63u) == 0 && slo) atomicAdd(LL.bsum + gw, slo);
            if ((tid & 63u) == 0 && shi) atomicAdd(LL.bsum + gw + 1, shi);
        };
        if constexpr (QUAD) {
            // the headers a lane per line, the read bases a quad per line,
            // -m local's call a lane per line again (cnt <= cap <= TB)
            static_assert(tp_cap_max(true) <= TB, "a lane per line of the quad shape's tile");
            // (the header and the call steps, one wave's work while the block
            // waits at a barrier, at priority 2 over other blocks' quads: C5
            // parse 10.84 -> 10.50 ms)
            __builtin_amdgcn_s_setprio(2);
            if (tid < cnt) qmeta[tid] = quad_head<LOCAL>(tl, g0, ls[tid], g_tile + tid, len_t, cls, O);
            __builtin_amdgcn_s_setprio(0);
            __syncthreads();
            for (uint32_t j0 = 0; j0 < cnt; j0 += LPR) {   // block-uniform trip count
                const uint32_t j = j0 + (tid >> 2);
                if (j < cnt)
                    quad_bases<LOCAL>(tl, ld, g0, ls[j], qmeta + j, qcnt + (LOCAL ? j : 0), g_tile + j, len_t,
                                      (tid & 3u) == 0, rbl, O);
            }
            if constexpr (LOCAL) {
                __syncthreads();
                __builtin_amdgcn_s_setprio(2);
                int l = 0;
                if (tid < cnt) l = quad_tail(text, g0 + ls[tid], qmeta[tid], qcnt[tid], g_tile + tid, c1, O, LL);
                bsum_add(tid & ~63u, tid, l);
            }
        } else {
            for (uint32_t j0 = 0; j0 < cnt; j0 += LPR) {   // block-uniform trip count
                const uint32_t j = j0 + tid;
                int l = 0;
                LaneSlot ws;
                if (j < cnt) l = tile_line<LOCAL>(text, tl, ld, g0, ls[j], g_tile + j, len_t, c1, cls, rbl, O, LL, ws);
                if constexpr (LOCAL) {
                    tile_wave_store(ws, g_tile + j, O.twv + t * O.nwv + ((j0 + (tid & ~63u)) >> 6), O, LL);
                    bsum_add(j0 + (tid & ~63u), j, l);
                }
            }
        }
#ifdef SID_TP_STAMP
        __syncthreads();
        if (tid == 0 && t < TP_STAMP_N) {
            const uint64_t st3 = wall_clock64();
            tp_stamp[t][0] = (uint32_t)(st1 - st0);
            tp_stamp[t][1] = (uint32_t)(st2 - st1);
            tp_stamp[t][2] = (uint32_t)(st3 - st2);
            tp_stamp[t][3] = (uint32_t)(st0 >> 4);   // start (160 ns units)
        }
#endif
    }
}

// (64 blocks: the tiles' sum and maximum are one atomic per block on one
// address each, which serialise; 256 blocks took 20 us a launch)
constexpr unsigned TILE_SERIAL_GRID = 64;

// -m local's fix-up (the sites no class table covers: local.hip's
// fixup_site) and its record length into the writer block's bytes
struct LocalFix {
    LocalLen LL;
    sid_local_k K;
    const double* lnt;
    CType ct;
    uint8_t* code;
    double* hom;
    double* het;
};
__device__ __forceinline__ void fix_site(uint64_t i, const Head& hd, uint64_t c, const LocalFix& F,
                                         unsigned long long* lb)
{
    double h, t;
    const uint32_t code = fixup_site(c, nullptr, F.K, F.lnt, h, t);
    F.code[i] = (uint8_t)code;
    F.hom[i] = h;
    F.het[i] = t;
    int l = record_len(hd, (uint8_t)code, sid_g6_prep(h), sid_g6_prep(t), F.ct.len);
    if (l < 0) {
        atomicExch(lb + 2, 1ull);
        l = 0;
    }
    atomicAdd(F.LL.bsum + i / FTB, (uint32_t)l);
}

// the general routine over the tile parse's leftovers (slot, line offset):
// counts and a header pair with no chrom (the formatter tokenises the line),
// the slot listed for its record length; and the tiles' line counts summed
// (lb[3]: sites, the counts capped at the slots) and maxed (lb[5]).
// LOCAL (-m local, sid_chunk_tile_local): also each leftover line's call and
// record length, a fix-up where no class table covers it, and the fix-ups
// the tile parse listed (LL.miss) -- the work of two more launches a chunk
// (a record-length kernel over the leftovers, then the fix-up kernel)
template <bool LOCAL>
__global__ __launch_bounds__(TB) void sid_tile_serial_kernel(const char* __restrict__ text, uint64_t len,
                                                             const uint32_t* __restrict__ fb,
                                                             const uint32_t* __restrict__ fbo,
                                                             unsigned long long* lb, const uint32_t* __restrict__ tcnt,
                                                             uint64_t ntiles, uint32_t cap,
                                                             uint64_t* __restrict__ counts, uint64_t* __restrict__ hdr,
                                                             unsigned long long* __restrict__ err, LocalFix F)
{
    __shared__ uint8_t cls[256];
    __shared__ uint32_t red[2][TB / 64];
    if (threadIdx.x < 256) cls[threadIdx.x] = k_tp_tables.cls[threadIdx.x];
    {
        // four tiles a 16-B load, four loads in flight a lane (one pass over
        // ~200k tiles at this grid; a load a tile, each waited for before the
        // next, took ~12 us a chunk)
        uint32_t sum = 0, mx = 0;
        auto add = [&](uint32_t c) {
            sum += min(c, cap);
            mx = max(mx, c);
        };
        const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x, nq = ntiles / 4;
        const uint4* tq = (const uint4*)tcnt;   // (hipMalloc'd: 16-B aligned)
        for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += 4 * nthr) {
            uint4 c4[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t qu = q + u * nthr;
                c4[u] = qu < nq ? tq[qu] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                add(c4[u].x);
                add(c4[u].y);
                add(c4[u].z);
                add(c4[u].w);
            }
        }
        if (blockIdx.x == 0 && threadIdx.x < ntiles - 4 * nq) add(tcnt[4 * nq + threadIdx.x]);
        sum = wave_sum(sum);
        mx = wave_max(mx);
        if ((threadIdx.x & 63u) == 0) red[0][threadIdx.x >> 6] = sum, red[1][threadIdx.x >> 6] = mx;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int w = 1; w < TB / 64; ++w) sum += red[0][w], mx = max(mx, red[1][w]);
            if (sum) atomicAdd(lb + 3, (unsigned long long)sum);
            if (mx) atomicMax(lb + 5, (unsigned long long)mx);
        }
    }
    const uint64_t m = lb[6];
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t g = fb[k];
        const uint64_t s0 = fbo[k];
        uint64_t c = 0;
        parse_line_serial(text, len, s0, cls, &c, err, 0);
        counts[g] = c;
        hdr[2 * g] = 0;
        hdr[2 * g + 1] = s0;
        if constexpr (LOCAL) {
            Reader R{text, len};
            const Head hd = slot_head(R, make_ulonglong2(0, s0));
            const int L = local_site_tail<false>(c, g, F.LL.len1, F.LL);
            if (L >= 0) atomicAdd(F.LL.bsum + g / FTB, (uint32_t)local_rec_len(hd, (uint32_t)L));
            else fix_site(g, hd, c, F, lb);
        }
    }
    if constexpr (LOCAL) {   // the tile parse's fix-up sites
        const uint64_t nm = *F.LL.nmiss;
        for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nm; j += (uint64_t)gridDim.x * blockDim.x) {
            const uint64_t i = F.LL.miss[j];
            Reader R{text, len};
            fix_site(i, slot_head(R, *(const ulonglong2*)(hdr + 2 * i)), counts[i], F, lb);
        }
    }
}

// slot -> its tile (slot / cap) by one 32-bit multiply-high: t = mulhi(g, m)
// >> s with s = floor(log2(cap - 1)), m = ceil(2^(32+s) / cap) < 2^32; the
// error m cap - 2^(32+s) < cap <= 2^(s+1) keeps it exact for g < 2^28 (a
// chunk of at most 4 GiB has fewer slots).  (A 64-bit multiply-high by
// ceil(2^64 / cap) took a chain of quarter-rate multiplies a slot.)
struct SlotDiv {
    uint32_t m, s;
};
static SlotDiv slot_div(uint32_t cap)
{
    const uint32_t s = 31u - (uint32_t)__builtin_clz(cap - 1u);
    return SlotDiv{(uint32_t)(((1ull << (32 + s)) + cap - 1) / cap), s};
}
__device__ __forceinline__ uint32_t slot_tile(uint32_t g, SlotDiv d) { return __umulhi(g, d.m) >> d.s; }
// the wave entries of a tile of cap slots (tile_wave_store): at most slots / 32
// of them a chunk, as cap >= SID_TILE_CAP_MIN = 64 (sid_chunk_reserve)
static uint32_t tile_nwv(uint32_t cap) { return (cap + 63) / 64; }
static_assert(SID_TILE_CAP_MIN >= 64, "a tile's wave entries: at most two per 64 slots");
constexpr uint64_t SID_SLOTS_MAX = 1ull << 28;

// The tile parse's sites into file order (the Lynch paths' kept parse,
// run.cpp use_pre: line offsets, counts, header pairs): slot g = tile * cap +
// j goes to toff[tile] + j (toff: the tiles' exclusive prefix of their
// counts); the line offset where the header pair keeps it (a chrom over 8
// bytes, no valid pair), else 0 (unread)
__global__ __launch_bounds__(TB) void sid_tile_compact_kernel(const uint32_t* __restrict__ tcnt,
                                                              const uint64_t* __restrict__ toff, uint64_t slots,
                                                              uint32_t cap, SlotDiv cdiv,
                                                              const uint64_t* __restrict__ counts,
                                                              const uint64_t* __restrict__ hdr,
                                                              sid_off_t* __restrict__ d_starts,
                                                              uint64_t* __restrict__ d_counts,
                                                              uint64_t* __restrict__ d_hdr)
{
    for (uint64_t g = (uint64_t)blockIdx.x * TB + threadIdx.x; g < slots; g += (uint64_t)gridDim.x * TB) {
        const uint32_t t = slot_tile((uint32_t)g, cdiv);
        const uint32_t j = (uint32_t)g - t * cap;
        if (j >= tcnt[t]) continue;
        const uint64_t i = toff[t] + j;
        const ulonglong2 hw = *(const ulonglong2*)(hdr + 2 * g);
        const bool keep = (hw.x >> 63) && ((hw.x >> 32) & 0xFFFu) <= 8;   // the pair holds the chrom's bytes
        d_counts[i] = counts[g];
        *(ulonglong2*)(d_hdr + 2 * i) = hw;
        d_starts[i] = keep ? 0u : (sid_off_t)hw.y;
    }
}

__global__ __launch_bounds__(FTB) void sid_local_len_kernel(const char* __restrict__ text, uint64_t len,
                                                           const sid_off_t* __restrict__ starts,
                                                           const uint64_t* __restrict__ hdr, uint64_t n,
                                                           const uint64_t* __restrict__ counts,
                                                           const uint8_t* __restrict__ len1,
                                                           const uint8_t* __restrict__ len2,
                                                           uint32_t* __restrict__ bsum, uint32_t* __restrict__ miss,
                                                           unsigned long long* nmiss)
{
    static_assert(SID_TAB_N == FTB * 16, "one 16-B load per thread fills the LDS length table");
    __shared__ __attribute__((aligned(16))) uint8_t L1[SID_TAB_N];
    ((uint4*)L1)[threadIdx.x] = ((const uint4*)len1)[threadIdx.x];
    __syncthreads();
    const uint64_t nb = (n + FTB - 1) / FTB;
    for (int it = 0; it < LPB; ++it) {
        const uint64_t b = (uint64_t)blockIdx.x * LPB + it;
        if (b >= nb) break;
        const uint64_t i = b * FTB + threadIdx.x;
        int l = 0;
        if (i < n) {
            uint32_t f, s, nf, ns, cov;
            const uint64_t w = counts[i];
            const ulonglong2 hw = *(const ulonglong2*)(hdr + 2 * i);   // in flight beside the class lookup
            sid_major(w, f, s, nf, ns, cov);
            const uint32_t k = local_entry(nf, ns, cov - nf - ns);
            const uint32_t L = k < SID_TAB_N ? L1[k] : k != UINT32_MAX ? len2[k - SID_TAB_N] : 0xFFu;
            if (L == 0xFFu) {
                miss[atomicAdd(nmiss, 1ull)] = (uint32_t)i;   // its bytes: the fix-up's
            } else {
                Reader R{text, len};
                l = local_rec_len(site_head_hw(R, starts + i, hw), L);
            }
        }
        const uint32_t tot = block_sum<FTB>((uint32_t)l);
        if (threadIdx.x == 0) bsum[b] = tot;
    }
}

// SLOT: the tile parse's layout (site = slot, chrom and position by slot_head)
template <bool SLOT>
__global__ __launch_bounds__(TB) void sid_local_fixlen_kernel(const char* __restrict__ text, uint64_t len,
                                                             const sid_off_t* __restrict__ starts,
                                                             const uint64_t* __restrict__ hdr,
                                                             const uint64_t* __restrict__ counts,
                                                             const uint32_t* __restrict__ miss,
                                                             const unsigned long long* nmiss, sid_local_k K,
                                                             const double* __restrict__ lnt, CType ct,
                                                             uint8_t* __restrict__ code, double* __restrict__ hom,
                                                             double* __restrict__ het, uint32_t* bsum,
                                                             unsigned long long* lb)
{
    const uint64_t m = *nmiss;
    for (uint64_t j = (uint64_t)blockIdx.x * TB + threadIdx.x; j < m; j += (uint64_t)gridDim.x * TB) {
        const uint32_t i = miss[j];
        double h, t;
        const uint32_t c = fixup_site(counts[i], nullptr, K, lnt, h, t);
        code[i] = (uint8_t)c;
        hom[i] = h;
        het[i] = t;
        Reader R{text, len};
        const Head hd = SLOT ? slot_head(R, *(const ulonglong2*)(hdr + 2 * (uint64_t)i))
                             : site_head(R, starts + i, hdr + 2 * i);
        int l = record_len(hd, (uint8_t)c, sid_g6_prep(h), sid_g6_prep(t), ct.len);
        if (l < 0) {
            atomicExch(lb + 2, 1ull);
            l = 0;
        }
        atomicAdd(bsum + i / FTB, (uint32_t)l);
    }
}

// The -m local writer assembles its records in a zeroed LDS buffer by OR-ing
// 8-byte pieces that are zero beyond their fields: a record's neighbours are
// untouched whatever the alignment, and no lane branches per byte (through
// predicated byte stores the writer was branch- and SALU-bound).
// v[0..CNT) = the bytes from buffer offset q on: CNT + 1 ds_or_b64
// The buffer's 16-B quads are swizzled within each 128-B row (quad Q at
// Q ^ (row & 7)): records ~43 B apart put lanes three apart on the same LDS
// bank (3 x 43 = 129), 10-way conflicts on every piece, and the XOR spreads
// them (quads stay whole, so the 16-B copy-out reads are unchanged).
__device__ __forceinline__ uint32_t swz_quad(uint32_t Q) { return Q ^ ((Q >> 3) & 7u); }
__device__ __forceinline__ uint32_t swz_qword(uint32_t w) { return (swz_quad(w >> 1) << 1) | (w & 1u); }

template <int CNT>
__device__ __forceinline__ void lds_or_run(unsigned long long* B, uint32_t q, const uint64_t (&v)[CNT])
{
    const uint32_t w = q >> 3, sh = (q & 7u) * 8u;
    uint64_t prev = 0;
#pragma unroll
    for (int m = 0; m <= CNT; ++m) {
        const uint64_t cur = m < CNT ? v[m] : 0ull;
        const uint64_t x = (cur << sh) | (sh ? prev >> (64u - sh) : 0ull);
        atomicOr(B + swz_qword(w + m), x);
        prev = cur;
    }
}

__device__ __forceinline__ void lds_or_byte(unsigned long long* B, uint32_t q, uint32_t ch)
{
    atomicOr((unsigned*)B + ((swz_qword(q >> 3) << 1) | ((q >> 2) & 1u)), (ch & 0xFFu) << (8u * (q & 3u)));
}

// "," + the decimal of 0 <= v < 10^10 + ",", left-aligned in 16 bytes (lo,
// hi), zero after; nd = its digits
// g < 10^4 as four ASCII digits, most significant first (byte 0): g / 100
// and g % 100 in the two 16-bit halves of a word, both halves divided by 10
// at once ((x 103) >> 10 is x / 10 below 179), full-rate 24-bit multiplies only
__device__ __forceinline__ uint32_t four_digits(uint32_t g)
{
    const uint32_t hi2 = __umul24(g, 5243u) >> 19;   // g / 100 (exact below 43690)
    const uint32_t p = hi2 | ((g - __umul24(hi2, 100u)) << 16);
    const uint32_t t = (__umul24(p, 103u) >> 10) & 0x000F000Fu;
    const uint32_t u = p - __umul24(t, 10u);
    return 0x30303030u + (t | (u << 8));
}
// v < 2^31 with nd digits -> ",digits," in lo (bytes 0-7) and hi: three
// groups of four digits (two 32-bit divisions by 10^4), the twelve digits
// with their leading zeros at bytes 1-12 and a ',' at 13, the zero digit at
// byte 12 - nd made the leading ',', then shifted down by 12 - nd bytes.
// (Eleven divisions by 10, each a quarter-rate multiply-high, before.)
__device__ __forceinline__ void comma_num_comma(uint32_t v, int nd, uint64_t& lo, uint64_t& hi)
{
    const uint32_t q1 = v / 10000u, g0 = v - q1 * 10000u;
    const uint32_t g2 = q1 / 10000u, g1 = q1 - g2 * 10000u;
    const uint32_t w0 = four_digits(g0), w1 = four_digits(g1), w2 = four_digits(g2);
    uint64_t L = ((uint64_t)w2 << 8) | ((uint64_t)w1 << 40);
    uint64_t H = ((uint64_t)w1 >> 24) | ((uint64_t)w0 << 8) | ((uint64_t)',' << 40);
    const uint32_t p = 12u - (uint32_t)nd;   // 2 .. 11
    if (p < 8) L ^= 0x1Cull << (8 * p);      // '0' ^ ',' = 0x1C
    else H ^= 0x1Cull << (8 * (p - 8));
    const uint32_t sh = 8 * p;
    if (sh >= 64) {
        lo = H >> (sh - 64);
        hi = 0;
    } else {
        lo = (L >> sh) | (H << (64 - sh));
        hi = H >> sh;
    }
}

// any record (the fix-up's sites, chroms the parse did not keep, positions
// from the text) byte by byte into the OR buffer
__device__ __forceinline__ void record_or(Reader& R, const Head& h, uint8_t c, const sid_g6& gh, const sid_g6& gt,
                                          const CType& ct, unsigned long long* B, uint32_t q)
{
    uint32_t n = 0;
    if (h.c8 || h.clen == 0) {
        for (uint32_t k = 0; k < h.clen; ++k) lds_or_byte(B, q + n++, (uint32_t)(h.c8 >> (8 * k)));
    } else {
        for (uint32_t k = 0; k < h.clen; ++k) lds_or_byte(B, q + n++, R.at(h.cb + k));
    }
    lds_or_byte(B, q + n++, ',');
    const int pl = sid_i32_len(h.pos);
    uint32_t u = h.pos < 0 ? 0u - (uint32_t)h.pos : (uint32_t)h.pos;
    if (h.pos < 0) lds_or_byte(B, q + n, '-');
    for (int k = pl - 1; k >= (h.pos < 0 ? 1 : 0); --k) {
        lds_or_byte(B, q + n + k, '0' + u % 10u);
        u /= 10u;
    }
    n += pl;
    lds_or_byte(B, q + n++, ',');
    const bool het = c & 0x80;
    lds_or_byte(B, q + n++, 'h');
    lds_or_byte(B, q + n++, het ? 'e' : 'o');
    lds_or_byte(B, q + n++, het ? 't' : 'm');
    lds_or_byte(B, q + n++, ',');
    lds_or_byte(B, q + n++, "ACGT"[c & 3]);
    lds_or_byte(B, q + n++, "ACGT"[(c >> 2) & 3]);
    lds_or_byte(B, q + n++, ',');
    char tmp[SID_FMT_MAX];
    int k = sid_g6_put(gh, tmp);
    for (int j = 0; j < k; ++j) lds_or_byte(B, q + n++, (uint8_t)tmp[j]);
    lds_or_byte(B, q + n++, ',');
    k = sid_g6_put(gt, tmp);
    for (int j = 0; j < k; ++j) lds_or_byte(B, q + n++, (uint8_t)tmp[j]);
    lds_or_byte(B, q + n++, ',');
    for (int j = 0; j < ct.len; ++j) lds_or_byte(B, q + n++, (uint8_t)ct.s[j]);
    lds_or_byte(B, q + n, '\n');
}

// a tabulated site's record byte by byte through put(k, byte): chrom, pos,
// label, gt, then the entry's tail (rare: chroms the parse did not keep,
// positions from the text, blocks of records past the LDS buffer)
template <class Put>
__device__ void record_tail_bytes(Reader& R, const Head& h, uint8_t c, uint4 ea, uint4 eb, Put put)
{
    uint32_t n = 0;
    if (h.c8 || h.clen == 0) {
        for (uint32_t k = 0; k < h.clen; ++k) put(n++, (uint32_t)(h.c8 >> (8 * k)) & 0xFFu);
    } else {
        for (uint32_t k = 0; k < h.clen; ++k) put(n++, R.at(h.cb + k));
    }
    put(n++, ',');
    const int pl = sid_i32_len(h.pos);
    uint32_t u = h.pos < 0 ? 0u - (uint32_t)h.pos : (uint32_t)h.pos;
    if (h.pos < 0) put(n, '-');
    for (int k = pl - 1; k >= (h.pos < 0 ? 1 : 0); --k) {
        put(n + k, '0' + u % 10u);
        u /= 10u;
    }
    n += pl;
    put(n++, ',');
    const bool het = c & 0x80;
    put(n++, 'h');
    put(n++, het ? 'e' : 'o');
    put(n++, het ? 't' : 'm');
    put(n++, ',');
    put(n++, "ACGT"[c & 3]);
    put(n++, "ACGT"[(c >> 2) & 3]);
    put(n++, ',');
    const uint32_t L = ea.x & 0xFFu;
    const uint32_t w[6] = {ea.z, ea.w, eb.x, eb.y, eb.z, eb.w};
#pragma unroll
    for (int j = 0; j < 24; ++j)
        if ((uint32_t)j < L) put(n + j, (w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
}

__device__ __noinline__ void record_put_tail(const char* text, uint64_t len, Head h, uint8_t c, uint4 ea, uint4 eb,
                                             char* out)
{
    Reader R{text, len};
    record_tail_bytes(R, h, c, ea, eb, [&](uint32_t k, uint32_t ch) { out[k] = (char)ch; });
}

__device__ __noinline__ void record_or_tail(const char* text, uint64_t len, Head h, uint8_t c, uint4 ea, uint4 eb,
                                            unsigned long long* B, uint32_t q)
{
    Reader R{text, len};
    record_tail_bytes(R, h, c, ea, eb, [&](uint32_t k, uint32_t ch) { lds_or_byte(B, q + k, ch); });
}

// the fix-up's sites (rare), out of line so that their %g code does not set
// the writer's register count: the record length, and the record
__device__ __noinline__ int miss_len(Head h, uint8_t c, double hm, double ht, CType ct)
{
    const int l = record_len(h, c, sid_g6_prep(hm), sid_g6_prep(ht), ct.len);
    return l < 0 ? 0 : l;
}

__device__ __noinline__ void miss_or(const char* text, uint64_t len, Head h, uint8_t c, double hm, double ht,
                                     CType ct, unsigned long long* B, uint32_t q)
{
    Reader R{text, len};
    record_or(R, h, c, sid_g6_prep(hm), sid_g6_prep(ht), ct, B, q);
}

__device__ __noinline__ void miss_put(const char* text, uint64_t len, Head h, uint8_t c, double hm, double ht,
                                      CType ct, char* out)
{
    Reader R{text, len};
    record_put(R, h, c, sid_g6_prep(hm), sid_g6_prep(ht), ct, out);
}

// CLS: the sites' class words from the fused parse (W->cls) stand in for
// their counts (the entry and the bases come with the word).  tcnt (the tile
// parse's layout): n slots, slot i a site when i mod 2^cap_log2 is below its
// tile's count, chrom and position by slot_head
// WV: the slots' compact words and wave entries (the lane-shape tile parse,
// tile_wave_store); else every slot's header pair
template <bool CLS, bool WV = false>
__global__ __launch_bounds__(FTB, SID_PUT_WAVES) void sid_local_put_kernel(const char* __restrict__ text, uint64_t len,
                                                           const sid_off_t* __restrict__ starts,
                                                           const uint64_t* __restrict__ hdr, uint64_t n,
                                                           const uint32_t* __restrict__ tcnt, uint32_t cap,
                                                           SlotDiv cdiv, const ulonglong2* __restrict__ twv,
                                                           uint32_t nwv, const uint64_t* __restrict__ counts,
                                                           const uint32_t* __restrict__ cwords,
                                                           const char* __restrict__ str1,
                                                           const char* __restrict__ str2,
                                                           const uint8_t* __restrict__ code,
                                                           const double* __restrict__ hom,
                                                           const double* __restrict__ het, CType ct,
                                                           const uint64_t* __restrict__ boff, const uint64_t* state,
                                                           unsigned long long* lb, char* __restrict__ out)
{
    constexpr int NQ = (FMT_LDS2 + 64) / 16;   // records, slack
    PUT_STAMP_AT(ps0);
    // the slot words' and the class entry's loads (a dependent chain) at
    // raised priority over other blocks' LDS assembly and copy-out: writer
    // 0.925 -> 0.898 ms per C2 step, C5 1.216 -> 1.184 (the whole block at
    // 3 up to the copy-out: 0.933)
    __builtin_amdgcn_s_setprio(3);
    __shared__ uint4 buf4[NQ];
    for (int k = threadIdx.x; k < NQ; k += FTB) buf4[k] = make_uint4(0, 0, 0, 0);
    unsigned long long* const B = (unsigned long long*)buf4;
    const uint64_t i = (uint64_t)blockIdx.x * FTB + threadIdx.x;
    int l = 0;
    Head h{0, 0, 0, 0};
    uint32_t f = 0, s = 0;
    uint4 ea = make_uint4(0, 0, 0, 0), eb = ea;
    bool tab = false;
    uint8_t c = 0;
    bool site = i < n;
    // the slot's class word and header pair loaded beside its tile's count
    // (a slot that holds no site: allocated, its words never used)
    // (a compact word: no header pair, the chrom and the position from its
    // wave's entry, loaded beside the word -- one address for most of a wave)
    uint32_t w0 = 0;
    ulonglong2 hw0 = make_ulonglong2(0, 0), te = hw0;
    bool cw = false;
    int pl = 0;   // the position's digits (sid_i32_len)
    if (tcnt && site) {   // slot i = tile * cap + j: a site when j is below the tile's count
        // (without wave entries (the quad shape) every slot's header pair,
        // loaded beside the word -- loaded after it, C5's writer took 1.16
        // ms for 1.08)
        if (CLS) w0 = cwords[i];
        if (!WV) hw0 = *(const ulonglong2*)(hdr + 2 * i);
        const uint32_t t = slot_tile((uint32_t)i, cdiv);   // (i < SID_SLOTS_MAX: t < 2^22, 24-bit products)
        const uint32_t j = (uint32_t)i - __umul24(t, cap);
        if (WV) te = twv[__umul24(t, nwv) + (j >> 6)];
        site = j < tcnt[t];
        cw = WV && cls_compact(w0);
        if (WV && site && !cw) hw0 = *(const ulonglong2*)(hdr + 2 * i);
    }
    if (site) {
        uint32_t k;
        if (CLS) {
            const uint32_t w = tcnt ? w0 : cwords[i];
            k = w == SID_CLS_MISS ? UINT32_MAX : w & 0xFFFFFu;
            f = (w >> 28) & 3u;
            s = w >> 30;
        } else {
            uint32_t nf, ns, cov;
            sid_major(counts[i], f, s, nf, ns, cov);
            k = local_entry(nf, ns, cov - nf - ns);
        }
        // (the record tail's load issued before the header pair's was
        // measured slower here: 0.88-0.89 vs 0.86-0.87 ms per C2 step; in
        // the Lynch writer, which looks the class up first, it pays)
        if (cw) {   // (the entry: tile_wave_store)
            const uint32_t dp = (w0 >> 20) & (SID_CLS_DPOS - 1), m = (uint32_t)(te.y >> 32);
            h.clen = m & 0xFFFu;
            h.pos = (int32_t)((uint32_t)te.y + dp);
            h.c8 = te.x;
            h.cb = 0;
            pl = (int)(((m >> 12) & 15u) + (dp >= ((m >> 16) & 255u)) + (dp >= (m >> 24)));
        } else {
            Reader R{text, len};
            h = tcnt ? slot_head(R, hw0) : site_head(R, starts + i, hdr + 2 * i);
            pl = tcnt && (hw0.x >> 63) ? (int)((hw0.x >> 59) & 15u) : sid_i32_len(h.pos);   // (parse_header's digits)
        }
        if (k != UINT32_MAX) {
            const uint4* e = (const uint4*)(k < SID_TAB_N ? str1 + (size_t)k * SID_STR_BYTES
                                                          : str2 + (size_t)(k - SID_TAB_N) * SID_STR_BYTES);
            ea = e[0];
            eb = e[1];
            tab = (ea.x & 0xFFu) != 0xFFu;
        }
        if (tab) {
            const bool het_l = (ea.x >> 8) & 1u;
            c = (uint8_t)(f | ((het_l ? s : f) << 2) | (het_l ? 0x80u : 0u));
            l = (int)h.clen + pl + 9 + (int)(ea.x & 0xFFu);   // (local_rec_len)
        } else {   // the fix-up's site
            c = code[i];
            l = miss_len(h, c, hom[i], het[i], ct);
        }
    }
    PUT_STAMP_AT(ps1);
    __builtin_amdgcn_s_setprio(0);
    if (blockIdx.x == 0 && threadIdx.x == 0) lb[4] = state[4];
    uint32_t tot;
    const uint32_t my = block_exscan_once<FTB>((uint32_t)l, &tot);   // (its barrier also orders the zeroing)
    PUT_STAMP_AT(ps2);
    char* const dst = out + boff[blockIdx.x];
    if (tot > FMT_LDS2) {   // long records (long chromosome names): straight to global, byte by byte
        if (l && tab) record_put_tail(text, len, h, c, ea, eb, dst + my);
        else if (l) miss_put(text, len, h, c, hom[i], het[i], ct, dst + my);
        return;
    }
    if (l && tab && (h.c8 || h.clen == 0) && h.pos >= 0) {
        // (two runs, chrom + ",pos," and label + tail: 9 LDS ORs a record
        // instead of 11, measured slower: writer 0.947 vs 0.930 ms per C2 step)
        const uint64_t c8[1] = {h.c8};
        lds_or_run<1>(B, my, c8);
        uint64_t pv[2];
        comma_num_comma((uint32_t)h.pos, pl, pv[0], pv[1]);
        const uint32_t q1 = my + h.clen;
        lds_or_run<2>(B, q1, pv);
        const uint64_t ACGT = 0x54474341ull;
        const bool het_l = c & 0x80u;
        const uint64_t lab[1] = {(uint64_t)'h' | ((uint64_t)(het_l ? 'e' : 'o') << 8) |
                                 ((uint64_t)(het_l ? 't' : 'm') << 16) | ((uint64_t)',' << 24) |
                                 (((ACGT >> (8 * (c & 3u))) & 0xFF) << 32) |
                                 (((ACGT >> (8 * ((c >> 2) & 3u))) & 0xFF) << 40) | ((uint64_t)',' << 48)};
        const uint32_t q2 = q1 + (uint32_t)pl + 2;
        lds_or_run<1>(B, q2, lab);
        const uint64_t tv[3] = {((uint64_t)ea.w << 32) | ea.z, ((uint64_t)eb.y << 32) | eb.x,
                                ((uint64_t)eb.w << 32) | eb.z};
        lds_or_run<3>(B, q2 + 7, tv);
    } else if (l && tab) {
        record_or_tail(text, len, h, c, ea, eb, B, my);
    } else if (l) {
        miss_or(text, len, h, c, hom[i], het[i], ct, B, my);
    }
    __syncthreads();
    PUT_STAMP_AT(ps3);
    block_store<true>((const char*)buf4, tot, dst);
#ifdef SID_TP_STAMP
    if (CLS && tcnt && threadIdx.x == 0 && blockIdx.x < TP_STAMP_N) {
        const uint64_t ps4 = wall_clock64();
        put_stamp[blockIdx.x][0] = (uint32_t)(ps1 - ps0);
        put_stamp[blockIdx.x][1] = (uint32_t)(ps2 - ps1);
        put_stamp[blockIdx.x][2] = (uint32_t)(ps3 - ps2);
        put_stamp[blockIdx.x][3] = (uint32_t)(ps4 - ps3);
    }
#endif
}

// ---- likelihood_ratio / bayes, fused with the class lookup: a site's
// class (the Lynch classes of the merged histogram, sid_lynch_fmt) gives its
// whole record tail "label,gt,conf1,conf2,conf_type\n" (built once per class
// by sid_lynch_str_build), so the lookup kernel's code / confs never
// round-trip HBM and no %g is computed per site; a filtered profile
// (coverage < 4, call.cpp:131-140) has no record.
__device__ __forceinline__ uint32_t lynch_class(uint64_t w, const sid_lynch_fmt& V)
{
    const uint32_t d = sid_dense_code(w);
    if (d != SID_DENSE_NONE) return V.dense_cidx[d];   // SID_DENSE_NONE: filtered
    const uint64_t key = sid_profile_key(w);
    if (key == SID_EMPTY_KEY) return V.special_idx;
    uint64_t h = sid_hash64(key) & V.cmask;
    for (uint64_t probe = 0; probe <= V.cmask; ++probe) {
        const unsigned long long k = V.ckeys[h];
        if (k == key) return V.cidx[h];
        if (k == SID_EMPTY_KEY) break;
        h = (h + 1) & V.cmask;
    }
    return 0xFFFFFFFFu;
}

// chrom , pos , then the class's tail
__device__ __forceinline__ int lynch_rec_len(const Head& h, uint32_t tail)
{
    return (int)h.clen + 1 + sid_i32_len(h.pos) + 1 + (int)tail;
}

__global__ __launch_bounds__(FTB) void sid_lynch_len_kernel(const char* __restrict__ text, uint64_t len,
                                                           const sid_off_t* __restrict__ starts,
                                                           const uint64_t* __restrict__ hdr, uint64_t n,
                                                           const uint64_t* __restrict__ counts, sid_lynch_fmt V,
                                                           uint32_t* __restrict__ bsum)
{
    static_assert(SID_DENSE_N == FTB * 32, "two 16-B loads per thread fill the LDS length table");
    __shared__ __attribute__((aligned(16))) uint8_t DL[SID_DENSE_N];
    ((uint4*)DL)[2 * threadIdx.x] = ((const uint4*)V.dlen)[2 * threadIdx.x];
    ((uint4*)DL)[2 * threadIdx.x + 1] = ((const uint4*)V.dlen)[2 * threadIdx.x + 1];
    __syncthreads();
    const uint64_t nb = (n + FTB - 1) / FTB;
    for (int it = 0; it < LPB; ++it) {
        const uint64_t b = (uint64_t)blockIdx.x * LPB + it;
        if (b >= nb) break;
        const uint64_t i = b * FTB + threadIdx.x;
        int l = 0;
        if (i < n && !V.empty) {
            const uint64_t w = counts[i];
            const ulonglong2 hw = *(const ulonglong2*)(hdr + 2 * i);   // in flight beside the class lookup
            const uint32_t d = sid_dense_code(w);
            uint32_t L = 0;
            if (d != SID_DENSE_NONE) {
                L = DL[d];
            } else {
                const uint32_t idx = lynch_class(w, V);
                L = idx == 0xFFFFFFFFu ? 0u : (uint8_t)V.lstr[(size_t)idx * SID_LSTR_BYTES];
            }
            if (L) {
                Reader R{text, len};
                l = lynch_rec_len(site_head_hw(R, starts + i, hw), L);
            }
        }
        const uint32_t tot = block_sum<FTB>((uint32_t)l);
        if (threadIdx.x == 0) bsum[b] = tot;
    }
}

// a record byte by byte through put(k, byte): chrom, pos, the tail (rare:
// chroms the parse did not keep, positions from the text, blocks past the
// LDS buffer)
template <class Put>
__device__ void lynch_record_bytes(Reader& R, const Head& h, const uint4 (&e)[4], Put put)
{
    uint32_t n = 0;
    if (h.c8 || h.clen == 0) {
        for (uint32_t k = 0; k < h.clen; ++k) put(n++, (uint32_t)(h.c8 >> (8 * k)) & 0xFFu);
    } else {
        for (uint32_t k = 0; k < h.clen; ++k) put(n++, R.at(h.cb + k));
    }
    put(n++, ',');
    const int pl = sid_i32_len(h.pos);
    uint32_t u = h.pos < 0 ? 0u - (uint32_t)h.pos : (uint32_t)h.pos;
    if (h.pos < 0) put(n, '-');
    for (int k = pl - 1; k >= (h.pos < 0 ? 1 : 0); --k) {
        put(n + k, '0' + u % 10u);
        u /= 10u;
    }
    n += pl;
    put(n++, ',');
    const uint32_t L = e[0].x & 0xFFu;
    const uint32_t w[14] = {e[0].z, e[0].w, e[1].x, e[1].y, e[1].z, e[1].w, e[2].x,
                            e[2].y, e[2].z, e[2].w, e[3].x, e[3].y, e[3].z, e[3].w};
#pragma unroll
    for (int j = 0; j < SID_LSTR_BYTES - 8; ++j)
        if ((uint32_t)j < L) put(n + j, (w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
}

__device__ __noinline__ void lynch_put_global(const char* text, uint64_t len, Head h, uint4 e0, uint4 e1, uint4 e2,
                                              uint4 e3, char* out)
{
    Reader R{text, len};
    const uint4 e[4] = {e0, e1, e2, e3};
    lynch_record_bytes(R, h, e, [&](uint32_t k, uint32_t ch) { out[k] = (char)ch; });
}

__device__ __noinline__ void lynch_put_or(const char* text, uint64_t len, Head h, uint4 e0, uint4 e1, uint4 e2,
                                          uint4 e3, unsigned long long* B, uint32_t q)
{
    Reader R{text, len};
    const uint4 e[4] = {e0, e1, e2, e3};
    lynch_record_bytes(R, h, e, [&](uint32_t k, uint32_t ch) { lds_or_byte(B, q + k, ch); });
}

__global__ __launch_bounds__(FTB, SID_PUT_WAVES) void sid_lynch_put_kernel(const char* __restrict__ text, uint64_t len,
                                                                          const sid_off_t* __restrict__ starts,
                                                                          const uint64_t* __restrict__ hdr, uint64_t n,
                                                                          const uint64_t* __restrict__ counts,
                                                                          sid_lynch_fmt V,
                                                                          const uint64_t* __restrict__ boff,
                                                                          const uint64_t* state, unsigned long long* lb,
                                                                          char* __restrict__ out)
{
    __builtin_amdgcn_s_setprio(3);   // (the loads and the class lookup: as sid_local_put_kernel)
    constexpr int NQ = (FMT_LDS2 + 64) / 16;   // records, slack
    __shared__ uint4 buf4[NQ];
    for (int k = threadIdx.x; k < NQ; k += FTB) buf4[k] = make_uint4(0, 0, 0, 0);
    unsigned long long* const B = (unsigned long long*)buf4;
    const uint64_t i = (uint64_t)blockIdx.x * FTB + threadIdx.x;
    int l = 0;
    Head h{0, 0, 0, 0};
    uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0, e2 = e0, e3 = e0;
    if (i < n && !V.empty) {
        const uint64_t w = counts[i];
        const ulonglong2 hw = *(const ulonglong2*)(hdr + 2 * i);   // in flight beside the class lookup
        const uint32_t idx = lynch_class(w, V);
        if (idx != 0xFFFFFFFFu) {
            const uint4* e = (const uint4*)(V.lstr + (size_t)idx * SID_LSTR_BYTES);
            e0 = e[0];
            e1 = e[1];
            e2 = e[2];
            e3 = e[3];
            Reader R{text, len};
            h = site_head_hw(R, starts + i, hw);
            l = lynch_rec_len(h, e0.x & 0xFFu);
        }
    }
    __builtin_amdgcn_s_setprio(0);
    if (blockIdx.x == 0 && threadIdx.x == 0) lb[4] = state[4];
    uint32_t tot;
    const uint32_t my = block_exscan_once<FTB>((uint32_t)l, &tot);   // (its barrier also orders the zeroing)
    char* const dst = out + boff[blockIdx.x];
    if (tot > FMT_LDS2) {   // long records (long chromosome names): straight to global, byte by byte
        if (l) lynch_put_global(text, len, h, e0, e1, e2, e3, dst + my);
        return;
    }
    if (l && (h.c8 || h.clen == 0) && h.pos >= 0) {
        const uint64_t c8[1] = {h.c8};
        lds_or_run<1>(B, my, c8);
        const int pl = sid_i32_len(h.pos);
        uint64_t pv[2];
        comma_num_comma((uint32_t)h.pos, pl, pv[0], pv[1]);
        const uint32_t q1 = my + h.clen;
        lds_or_run<2>(B, q1, pv);
        const uint64_t tv[7] = {((uint64_t)e0.w << 32) | e0.z, ((uint64_t)e1.y << 32) | e1.x,
                                ((uint64_t)e1.w << 32) | e1.z, ((uint64_t)e2.y << 32) | e2.x,
                                ((uint64_t)e2.w << 32) | e2.z, ((uint64_t)e3.y << 32) | e3.x,
                                ((uint64_t)e3.w << 32) | e3.z};
        lds_or_run<7>(B, q1 + (uint32_t)pl + 2, tv);
    } else if (l) {
        lynch_put_or(text, len, h, e0, e1, e2, e3, B, my);
    }
    __syncthreads();
    block_store<true>((const char*)buf4, tot, dst);
}

// tails of the U classes (one thread each), then the dense codes' lengths
__global__ __launch_bounds__(256) void sid_lynch_str_kernel(const uint8_t* __restrict__ pcode,
                                                           const double* __restrict__ cc, uint32_t U, CType ct,
                                                           char* __restrict__ lstr, uint32_t* bad)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= U) return;
    char t[SID_LSTR_BYTES];
    const uint8_t c = pcode[i];
    const bool het = c & 0x80;
    int n = 0;
    t[n++] = 'h';
    t[n++] = het ? 'e' : 'o';
    t[n++] = het ? 't' : 'm';
    t[n++] = ',';
    t[n++] = "ACGT"[c & 3];
    t[n++] = "ACGT"[(c >> 2) & 3];
    t[n++] = ',';
    const int a = sid_g6_put(sid_g6_prep(cc[2 * i]), t + n);
    if (a < 0) atomicExch(bad, 1u);
    n += a < 0 ? 0 : a;
    t[n++] = ',';
    const int b = sid_g6_put(sid_g6_prep(cc[2 * i + 1]), t + n);
    if (b < 0) atomicExch(bad, 1u);
    n += b < 0 ? 0 : b;
    t[n++] = ',';
    for (int k = 0; k < ct.len; ++k) t[n++] = ct.s[k];
    t[n++] = '\n';
    if (n > SID_LSTR_BYTES - 8) atomicExch(bad, 1u);   // (45 at most: never)
    char* e = lstr + (size_t)i * SID_LSTR_BYTES;
    for (int k = 0; k < SID_LSTR_BYTES; ++k) e[k] = 0;
    e[0] = (char)n;
    for (int k = 0; k < n && k < SID_LSTR_BYTES - 8; ++k) e[8 + k] = t[k];
}

__global__ __launch_bounds__(256) void sid_lynch_dlen_kernel(const uint32_t* __restrict__ dense_cidx,
                                                            const char* __restrict__ lstr, uint8_t* __restrict__ dlen)
{
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= SID_DENSE_N) return;
    const uint32_t idx = dense_cidx[d];
    dlen[d] = idx == SID_DENSE_NONE ? 0 : (uint8_t)lstr[(size_t)idx * SID_LSTR_BYTES];
}

// ------------------------------------------------------------ -m quality --
// call.cpp:311-369 callQualityBasedSimple, one lane per site, reading the
// read bases and both quality fields straight from the resident text.  The
// j-th counted base pairs with the j-th characters of the base- and
// mapping-quality fields (the reference's index alignment; past their end the
// reference reads outside its vectors -- undefined -- and quality 1 is used).
// Every per-read term is a function of q = min(bq, mq) only, so the four of
// them come from a host table built with the same glibc pow/log the reference
// calls (bit-identical doubles); the long-double sums are double-double here.
struct QParams {
    double sig;
    double prior;
    int prior_on;
    int prior_ld;      // prior >= 1: emulated long-double path
    sid_dd lp1, lp2;   // ln(1 - prior), ln(prior) to ~1e-19
    double lg15;
};

__device__ __forceinline__ void dd_acc(sid_dd& a, double t)
{
    const double s = a.hi + t;
    const double bb = s - a.hi;
    const double e = (a.hi - (s - bb)) + (t - bb);
    a.hi = s;
    a.lo += e;
}

// Two kernels: the walk over the text (phase 1) and the per-site tail
// (phase 2).  In one kernel the tail's double-double, erfc and emulated
// long-double code set the register count for the walk too (203 VGPRs, 2
// waves per SIMD) and the latency-bound walk ran at that occupancy.
// Phase 1 stores the two per-read sums as double-double: the hi parts in
// hom/het (phase 2 overwrites them), the lo parts in lo2.
template <class Off>
__global__ __launch_bounds__(TB) void sid_quality_sum_kernel(const char* __restrict__ text, uint64_t len,
                                                             const Off* __restrict__ starts,
                                                             const uint64_t* __restrict__ counts, uint64_t n,
                                                             const double* __restrict__ g_qtab,
                                                             double* __restrict__ hom, double* __restrict__ het,
                                                             double2* __restrict__ lo2)
{
    __shared__ double T[4 * 256];
    __shared__ uint8_t cls[256];
    for (uint32_t i = threadIdx.x; i < 4 * 256; i += blockDim.x) T[i] = g_qtab[i];
    if (threadIdx.x < 256) cls[threadIdx.x] = k_tp_tables.cls[threadIdx.x];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = counts[i];
        uint32_t f, s2, nf, ns, cov;
        sid_major(w, f, s2, nf, ns, cov);   // getMajorAlleleIndices (same std::sort)
        Reader R{text, len};
        // tokens 2 (ref), 4, 5, 6 of the line (parsed with 7 fields)
        uint64_t b2 = 0, b4 = 0, e4 = 0, b5 = 0, e5 = 0, b6 = 0, e6 = 0;
        {
            uint64_t q = starts[i];
            for (int t = 0; t < 7; ++t) {
                while (is_sep(R.at(q))) ++q;
                const uint64_t tb = q;
                uint32_t c;
                while ((c = R.at(q)) != ' ' && c != '\t' && c != '\n' && c != 0 && q < len) ++q;
                if (t == 2) b2 = tb;
                else if (t == 4) b4 = tb, e4 = q;
                else if (t == 5) b5 = tb, e5 = q;
                else if (t == 6) b6 = tb, e6 = q;
            }
        }
        const uint32_t ref = R.at(b2);
        const uint32_t up = (ref >= 'a' && ref <= 'z') ? ref - 32 : ref;
        const uint32_t lw = (ref >= 'A' && ref <= 'Z') ? ref + 32 : ref;
        const uint32_t cdot = cls[up], ccomma = cls[lw];
        Reader RB{text, len}, RM{text, len};
        const uint64_t nbq = e5 - b5, nmq = e6 - b6;
        sid_dd lph = {0.0, 0.0}, lpt = {0.0, 0.0};
        uint64_t j = 0, skip = 0, num = 0;
        int ind = 0;
        bool ovf = false;
        for (uint64_t q = b4; q < e4; ++q) {
            const uint32_t c = R.at(q);
            if (ind == 1) {
                ind = 0;
                if (c >= '0' && c <= '9') {
                    ind = 2;
                    num = c - '0';
                    ovf = false;
                    continue;
                }
            } else if (ind == 2) {
                if (c >= '0' && c <= '9') {
                    const unsigned d = c - '0';
                    if (!ovf) {
                        if (num > ((unsigned long long)LONG_MAX - d) / 10) ovf = true;
                        else num = num * 10 + d;
                    }
                    continue;
                }
                ind = 0;
                skip = ovf ? (uint64_t)LONG_MAX : num;
            }
            if (skip) {
                --skip;
                continue;
            }
            const uint32_t k = c == '.' ? cdot : (c == ',' ? ccomma : cls[c]);
            if (k >= K_A && k <= K_T) {
                // parseQualities: uint8_t(c - 33), at least 1
                uint32_t bq = 1, mq = 1;
                if (j < nbq) {
                    bq = (RB.at(b5 + j) - 33u) & 0xffu;
                    bq = bq < 1 ? 1 : bq;
                }
                if (j < nmq) {
                    mq = (RM.at(b6 + j) - 33u) & 0xffu;
                    mq = mq < 1 ? 1 : mq;
                }
                const uint32_t qv = bq < mq ? bq : mq;
                const uint32_t b = k - 1;
                dd_acc(lph, T[(b == f ? 0 : 256) + qv]);
                dd_acc(lpt, T[(b == f || b == s2 ? 512 : 768) + qv]);
                ++j;
            } else if (k == K_CARET) {
                skip = 1;
            } else if (k == K_INDEL) {
                ind = 1;
            }
        }
        lph = dd_norm(lph.hi, lph.lo);
        hom[i] = lph.hi;
        het[i] = lpt.hi;
        lo2[i] = make_double2(lph.lo, lpt.lo);
    }
}

__global__ __launch_bounds__(TB) void sid_quality_finish_kernel(const uint64_t* __restrict__ counts, uint64_t n,
                                                                const double* __restrict__ lg, QParams P,
                                                                uint8_t* __restrict__ code, double* __restrict__ hom,
                                                                double* __restrict__ het,
                                                                const double2* __restrict__ lo2)
{
    const sid_dd LN2_LD = {0.6931471805599453, 2.3201926491189795e-17};   // x87 logl(2), exactly
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t f, s2, nf, ns, cov;
        sid_major(counts[i], f, s2, nf, ns, cov);
        const double2 lo = lo2[i];
        sid_dd lph = {hom[i], lo.x}, lpt = {het[i], lo.y};
        // log_probability_heterozygous += logbinom(n, k) - n * logl(2)
        const uint32_t nn = nf + ns, kk = ns;
        const double lb = lg[nn + 1] - lg[nn - kk + 1] - lg[kk + 1];
        sid_dd t = dd_add(sid_dd{lb, 0.0}, dd_neg(dd_mul_d(LN2_LD, (double)nn)));
        lpt = dd_add(dd_norm(lpt.hi, lpt.lo), t);
        double p1, p2;
        if (!P.prior_ld && lph.hi >= SID_FAST_FLOOR && lpt.hi >= SID_FAST_FLOOR) {
            // pp = expl(lp) (* prior) are normal long doubles: the LRTs from
            // the log difference, in double-double
            sid_dd a = lph, b = lpt;
            if (P.prior_on) {
                a = dd_add(a, P.lp1);
                b = dd_add(b, P.lp2);
            }
            const sid_dd dd = dd_add(a, dd_neg(b));
            const double d = dd.hi + dd.lo;
            p1 = sid_chisq_Q(d > 0.0 ? 2.0 * d : 0.0, P.lg15);    // LRT(pp2, pp1)
            p2 = sid_chisq_Q(d < 0.0 ? -2.0 * d : 0.0, P.lg15);   // LRT(pp1, pp2)
        } else {
            sid_ld l1 = ld_round(sid_ld{lph.hi, 0}), l2 = ld_round(sid_ld{lpt.hi, 0});
            if (P.prior_on) {
                l1 = ld_mul(l1, ld_from_double(1 - P.prior));
                l2 = ld_mul(l2, ld_from_double(P.prior));
            }
            p1 = ld_lrt(l2, l1, P.lg15);
            p2 = ld_lrt(l1, l2, P.lg15);
        }
        const bool hz = p2 < P.sig;   // call.cpp:362
        code[i] = (uint8_t)(f | ((hz ? s2 : f) << 2) | (hz ? 0x80u : 0u));
        hom[i] = p1;
        het[i] = p2;
    }
}

__global__ __launch_bounds__(TB) void sid_max_major_kernel(const uint64_t* __restrict__ counts, uint64_t n,
                                                           uint32_t* __restrict__ mx)
{
    uint32_t m = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t f, s, nf, ns, cov;
        sid_major(counts[i], f, s, nf, ns, cov);
        m = max(m, nf + ns);
    }
    for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_down((int)m, off, 64));
    if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}

// host build of the device formatter over an array (tests)
__global__ __launch_bounds__(TB) void sid_fmt_g6_kernel(const double* __restrict__ v, size_t n, char* __restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * TB + threadIdx.x;
    if (i >= n) return;
    char b[SID_FMT_MAX];
    const int l = sid_fmt_g6(v[i], b);
    char* o = out + i * SID_FMT_MAX;
    for (int k = 0; k < SID_FMT_MAX; ++k) o[k] = k < l ? b[k] : 0;
}

}  // namespace

// ============================================================== C ABI ======
// SID_TEXT_TIMING=1: phase times on stderr (measurement only)
static bool text_timing()
{
    static const bool on = std::getenv("SID_TEXT_TIMING") != nullptr;
    return on;
}
static double wall()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct sid_dtext {
    int device = 0;
    int quality = 0;               // parsed for -m quality (7 fields required)
    char* d_text = nullptr;
    uint64_t len = 0;
    uint64_t* d_starts = nullptr;
    uint64_t* d_counts = nullptr;
    uint64_t* d_hdr = nullptr;     // chrom / position per site for the formatter (sid_parse_kernel)
    uint32_t* d_fb = nullptr;      // lines for the general parse routine
    uint64_t nsites = 0;
    uint64_t* d_state = nullptr;   // [0] running site count, [1..2] chunk range, [3] fallback lines
    unsigned long long* d_err = nullptr;
    uint32_t* d_tcnt = nullptr;
    uint64_t* d_toff = nullptr;
    uint64_t tcap = 0;
};

#define TCHECK(x)                                                   \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) return sid_set_hip_error(e_);         \
    } while (0)

extern "C" int sid_dtext_free(sid_dtext* t)
{
    if (!t) return SID_OK;
    (void)hipSetDevice(t->device);
    for (void* p : {(void*)t->d_hdr, (void*)t->d_fb})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)t->d_text, (void*)t->d_starts, (void*)t->d_counts, (void*)t->d_state, (void*)t->d_err,
                    (void*)t->d_tcnt, (void*)t->d_toff})
        if (p) (void)hipFree(p);
    delete t;
    return SID_OK;
}

extern "C" size_t sid_dtext_count(const sid_dtext* t) { return t ? t->nsites : 0; }
extern "C" const uint16_t* sid_dtext_counts(const sid_dtext* t) { return t ? (const uint16_t*)t->d_counts : nullptr; }

static sid_dtext* dtext_alloc(const sid_ctx* ctx, uint64_t len, int* rc)
{
    sid_dtext* T = new sid_dtext();
    T->device = ctx->device;
    T->quality = ctx->opts.method == SID_METHOD_QUALITY;
    T->len = len;
    hipError_t e;
    // padded: 16-B window reads past the end stay inside the allocation
    if ((e = hipMalloc(&T->d_text, ((len + 15) & ~(size_t)15) + 128)) != hipSuccess ||
        (e = hipMalloc(&T->d_state, 4 * sizeof(uint64_t))) != hipSuccess ||
        (e = hipMalloc(&T->d_err, sizeof(unsigned long long))) != hipSuccess) {
        *rc = sid_set_hip_error(e);
        sid_dtext_free(T);
        return nullptr;
    }
    *rc = SID_OK;
    return T;
}

// Line index + parse over the resident text [0, len) (a line start at 0):
// count per tile -> scan -> (sync: the site count) -> line offsets -> parse.
static int dtext_index_parse(sid_dtext* T, hipStream_t st, uint64_t* err_offset)
{
    const uint64_t len = T->len;
    hipError_t e;
    const size_t tiles = std::max<size_t>((len + TILE - 1) / TILE, 1);
    if ((e = hipMalloc(&T->d_tcnt, tiles * 4 + scan_ws_bytes(tiles))) != hipSuccess ||
        (e = hipMalloc(&T->d_toff, tiles * 8)) != hipSuccess)
        return sid_set_hip_error(e);
    T->tcap = tiles;
    if ((e = hipMemsetAsync(T->d_state, 0, 4 * sizeof(uint64_t), st)) != hipSuccess ||
        (e = hipMemsetAsync(T->d_err, 0xFF, sizeof(unsigned long long), st)) != hipSuccess)
        return sid_set_hip_error(e);
    sid_lines_count_kernel<<<(unsigned)tiles, TB, 0, st>>>(T->d_text, 0, 0, len, T->d_tcnt);
    launch_scan(T->d_tcnt, tiles, T->d_toff, T->d_state, T->d_state + 1,
                (uint64_t*)((char*)T->d_tcnt + ((tiles * 4 + 7) & ~(size_t)7)), st);
    if ((e = hipGetLastError()) != hipSuccess) return sid_set_hip_error(e);
    uint64_t total = 0;
    if ((e = hipMemcpyAsync(&total, T->d_state, 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return sid_set_hip_error(e);
    T->nsites = total;
    const size_t m = std::max<uint64_t>(total, 1);
    if ((e = hipMalloc(&T->d_starts, m * 8)) != hipSuccess || (e = hipMalloc(&T->d_counts, m * 8)) != hipSuccess ||
        (e = hipMalloc(&T->d_hdr, m * 16)) != hipSuccess || (e = hipMalloc(&T->d_fb, m * 4)) != hipSuccess)
        return sid_set_hip_error(e);
    sid_lines_emit_kernel<<<(unsigned)tiles, TB, 0, st>>>(T->d_text, 0, 0, len, T->d_toff, T->d_starts);
    launch_parse(T->d_text, len, T->d_starts, T->d_state + 1, total, T->d_counts, T->d_hdr, T->d_fb,
                 (unsigned long long*)(T->d_state + 3), T->d_err, T->quality, st);
    if ((e = hipGetLastError()) != hipSuccess) return sid_set_hip_error(e);
    unsigned long long ek = ~0ull;
    if ((e = hipMemcpyAsync(&ek, T->d_err, 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
        (e = hipStreamSynchronize(st)) != hipSuccess)
        return sid_set_hip_error(e);
    if (ek != ~0ull) {
        if (err_offset) *err_offset = ek >> 3;
        const unsigned kind = (unsigned)(ek & 7);
        return kind == 1 ? SID_EMALFORMED : kind == 2 ? SID_ENULLCHROM : kind == 3 ? SID_EMISSING_MQ : SID_ENOBQ;
    }
    return SID_OK;
}

extern "C" int sid_dtext_parse(sid_ctx* ctx, const char* text, size_t len, size_t chunk, sid_dtext** out,
                               uint64_t* err_offset, void* stream)
{
    if (!ctx || !out || (!text && len)) return SID_EINVAL;
    *out = nullptr;
    const double w0 = wall();
    TCHECK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    int rc;
    sid_dtext* T = dtext_alloc(ctx, len, &rc);
    if (!T) return rc;
    // the padding first, then the text in `chunk`-sized copies.  (Measured on
    // a page-cache file mapping: one stream from a populated mapping beats
    // parallel copies that fault the pages in, and pread() into pinned staging.)
    hipError_t e = hipMemsetAsync(T->d_text + (len & ~(uint64_t)15), 0,
                                  ((len + 15) & ~(uint64_t)15) - (len & ~(uint64_t)15) + 128, st);
    if (chunk == 0) chunk = 256u << 20;
    for (uint64_t off = 0; off < len && e == hipSuccess; off += chunk)
        e = hipMemcpyAsync(T->d_text + off, text + off, std::min<uint64_t>(chunk, len - off), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        sid_dtext_free(T);
        return sid_set_hip_error(e);
    }
    const double w1 = wall();
    rc = dtext_index_parse(T, st, err_offset);
    if (text_timing())
        std::fprintf(stderr, "{\"dtext_parse\": {\"bytes\": %llu, \"upload_s\": %.6f, \"index_parse_s\": %.6f}}\n",
                     (unsigned long long)len, w1 - w0, wall() - w1);
    if (rc != SID_OK) {
        sid_dtext_free(T);
        return rc;
    }
    *out = T;
    return SID_OK;
}

// Text straight from a file descriptor: pread() by `threads` host threads into
// a ring of pinned buffers (context-owned), each DMA'd to HBM as it fills.
// No mapping of the file: no page-table population for gigabytes of page cache.
extern "C" int sid_dtext_parse_fd(sid_ctx* ctx, int fd, uint64_t offset, uint64_t len, int threads, sid_dtext** out,
                                  uint64_t* err_offset, void* stream)
{
    if (!ctx || !out || fd < 0) return SID_EINVAL;
    *out = nullptr;
    const double w0 = wall();
    TCHECK(hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    int rc;
    sid_dtext* T = dtext_alloc(ctx, len, &rc);
    if (!T) return rc;
    const int R = std::max(1, std::min(threads > 0 ? threads : 8, SID_STAGE_N));
    const size_t B = SID_STAGE_BYTES;
    hipError_t e = hipSuccess;
    for (int b = 0; b < R && e == hipSuccess; ++b)
        if (!ctx->in_h[b]) e = hipHostMalloc((void**)&ctx->in_h[b], B, hipHostMallocDefault);
    if (e == hipSuccess)
        e = hipMemsetAsync(T->d_text + (len & ~(uint64_t)15), 0,
                           ((len + 15) & ~(uint64_t)15) - (len & ~(uint64_t)15) + 128, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        sid_dtext_free(T);
        return sid_set_hip_error(e);
    }
    // reader r owns buffer r and chunks r, r+R, r+2R, ...: pread, DMA on its
    // own stream, wait for the DMA before refilling the buffer
    std::vector<int> rcs(R, SID_OK);
    std::vector<std::thread> th;
    const uint64_t nch = (len + B - 1) / B;
    for (int r = 0; r < R; ++r)
        th.emplace_back([&, r] {
            (void)hipSetDevice(T->device);
            hipStream_t rs;
            if (hipStreamCreateWithFlags(&rs, hipStreamNonBlocking) != hipSuccess) {
                rcs[r] = SID_EHIP;
                return;
            }
            char* buf = ctx->in_h[r];
            for (uint64_t c = r; c < nch && rcs[r] == SID_OK; c += R) {
                const uint64_t off = c * B, n = std::min<uint64_t>(B, len - off);
                uint64_t got = 0;
                while (got < n) {
                    const ssize_t k = ::pread(fd, buf + got, n - got, (off_t)(offset + off + got));
                    if (k <= 0) break;
                    got += (uint64_t)k;
                }
                if (got != n) {
                    rcs[r] = SID_EIO;
                    break;
                }
                hipError_t x = hipMemcpyAsync(T->d_text + off, buf, n, hipMemcpyHostToDevice, rs);
                if (x == hipSuccess) x = hipStreamSynchronize(rs);
                if (x != hipSuccess) rcs[r] = sid_set_hip_error(x);
            }
            (void)hipStreamDestroy(rs);
        });
    for (auto& x : th) x.join();
    for (int r : rcs)
        if (r != SID_OK) {
            sid_dtext_free(T);
            return r;
        }
    const double w1 = wall();
    rc = dtext_index_parse(T, st, err_offset);
    if (text_timing())
        std::fprintf(stderr,
                     "{\"dtext_parse_fd\": {\"bytes\": %llu, \"readers\": %d, \"upload_s\": %.6f, \"index_parse_s\": %.6f}}\n",
                     (unsigned long long)len, R, w1 - w0, wall() - w1);
    if (rc != SID_OK) {
        sid_dtext_free(T);
        return rc;
    }
    *out = T;
    return SID_OK;
}

// CSV records of sites [begin, end) (code bit 6: skipped) into pinned staging
// buffers piece by piece; write() receives them in order.
extern "C" int sid_dtext_format(sid_ctx* ctx, const sid_dtext* T, size_t begin, size_t end, const uint8_t* d_code,
                                const double* d_hom, const double* d_het, const char* conf_type,
                                sid_write_fn write, void* user, void* stream)
{
    if (!ctx || !T || !d_code || !d_hom || !d_het || !conf_type || !write) return SID_EINVAL;
    if (end > T->nsites || begin > end) return SID_EINVAL;
    CType ct{};
    ct.len = (int)std::strlen(conf_type);
    if (ct.len >= (int)sizeof ct.s) return SID_EINVAL;
    std::memcpy(ct.s, conf_type, ct.len);
    TCHECK(hipSetDevice(T->device));
    hipStream_t st = (hipStream_t)stream;
    const size_t n = end - begin;
    // blocks (of TB sites) per piece: 256 Ki sites, ~17 MB of records.  The
    // two pinned staging buffers are allocated while the lengths are computed
    // and the allocation holds up the device work: 1 Mi-site pieces cost
    // 33-41 ms before the first write at 50M sites, 256 Ki-site pieces 14-16
    // ms with the same D2H rate; 64 Ki-site pieces D2H slower
    // (round-1 measurement)
    constexpr size_t PB = 1024;
    const size_t nb = (n + TB - 1) / TB;
    uint32_t* d_bsum = nullptr;
    uint64_t* d_boff = nullptr;
    uint64_t* d_base = nullptr;
    int* d_bad = nullptr;
    char** d_out = ctx->fmt_d;   // staging owned by the context
    char** h_out = ctx->fmt_h;
    size_t* cap = ctx->fmt_cap;
    hipEvent_t done[2], written;
    (void)hipEventCreateWithFlags(&done[0], hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&done[1], hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&written, hipEventDisableTiming);
    hipStream_t cs = nullptr;   // D2H of piece k overlaps the formatting of piece k+1
    (void)hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    int rc = SID_OK;
    auto hip = [&](hipError_t x) {
        if (x != hipSuccess && rc == SID_OK) rc = sid_set_hip_error(x);
        return rc == SID_OK;
    };
    double t_wait = 0, t_write = 0, t_size = 0, t_alloc = 0;
    const double f0 = wall();
    // staging for a piece of ~64 B records, pinned on another thread while the
    // lengths are computed (pinning runs at a few GB/s)
    auto stage = [d_out, h_out, cap](size_t need) {
        hipError_t err = hipSuccess;
        for (int b = 0; b < 2 && err == hipSuccess; ++b) {
            if (need <= cap[b]) continue;
            if (d_out[b]) (void)hipFree(d_out[b]);
            if (h_out[b]) (void)hipHostFree(h_out[b]);
            d_out[b] = nullptr;
            h_out[b] = nullptr;
            cap[b] = 0;
            const size_t want = need + need / 8 + 4096;
            if ((err = hipMalloc(&d_out[b], want)) != hipSuccess) break;
            if ((err = hipHostMalloc((void**)&h_out[b], want, hipHostMallocDefault)) != hipSuccess) break;
            cap[b] = want;
        }
        return err;
    };
    hipError_t stage_err = hipSuccess;
    std::thread stager([&, dev = T->device] {
        (void)hipSetDevice(dev);
        stage_err = stage(std::min<size_t>(n, PB * TB) * 64 + 64);
    });
    // record lengths of every site and their block offsets: one pass, one sync
    std::vector<uint64_t> boff(nb + 1, 0);
    hip(hipMalloc(&d_bsum, ((std::max<size_t>(nb, 1) * 4 + 7) & ~(size_t)7) + scan_ws_bytes(nb)));
    hip(hipMalloc(&d_boff, (nb + 1) * 8));
    hip(hipMalloc(&d_base, 8));
    hip(hipMalloc(&d_bad, 4));
    if (rc == SID_OK && nb) {
        hip(hipMemsetAsync(d_bad, 0, 4, st));
        hip(hipMemsetAsync(d_base, 0, 8, st));
        sid_fmt_len_kernel<<<(unsigned)nb, TB, 0, st>>>(T->d_text, T->len, T->d_starts, T->d_hdr, begin, end, d_code, d_hom,
                                                        d_het, ct, d_bsum, d_bad);
        launch_scan(d_bsum, nb, d_boff, d_base, nullptr,
                    (uint64_t*)((char*)d_bsum + ((std::max<size_t>(nb, 1) * 4 + 7) & ~(size_t)7)), st);
        hip(hipGetLastError());
        hip(hipMemcpyAsync(boff.data(), d_boff, nb * 8, hipMemcpyDeviceToHost, st));
        hip(hipMemcpyAsync(&boff[nb], d_base, 8, hipMemcpyDeviceToHost, st));
        hip(hipStreamSynchronize(st));
    }
    t_size = wall() - f0;
    const double al = wall();
    stager.join();
    hip(stage_err);
    // exact size of the largest piece (long chromosome names can exceed the guess)
    size_t need = 64;
    for (size_t b0 = 0; b0 < nb; b0 += PB) need = std::max<size_t>(need, boff[std::min(nb, b0 + PB)] - boff[b0] + 64);
    if (rc == SID_OK) hip(stage(need));
    t_alloc = wall() - al;
    size_t pending_len[2] = {0, 0};
    bool pending[2] = {false, false};
    auto flush = [&](int b) {   // hand piece b to the writer
        if (!pending[b]) return;
        pending[b] = false;
        const double a = wall();
        if (!hip(hipEventSynchronize(done[b]))) return;
        const double m = wall();
        if (pending_len[b] && write(user, h_out[b], pending_len[b]) != 0 && rc == SID_OK) rc = SID_EIO;
        t_wait += m - a;
        t_write += wall() - m;
    };
    int k = 0;
    for (size_t b0 = 0; b0 < nb && rc == SID_OK; b0 += PB, k ^= 1) {
        const size_t b1 = std::min(nb, b0 + PB);
        const size_t s0 = begin + b0 * TB, s1 = std::min(end, begin + b1 * TB);
        const uint64_t bytes = boff[b1] - boff[b0];
        flush(k);   // buffer k is about to be reused
        if (rc != SID_OK) break;
        sid_fmt_write_kernel<<<(unsigned)(b1 - b0), TB, 0, st>>>(T->d_text, T->len, T->d_starts, T->d_hdr, s0, s1, d_code, d_hom,
                                                                 d_het, ct, d_boff + b0, boff[b0], d_out[k]);
        if (!hip(hipGetLastError())) break;
        hip(hipEventRecord(written, st));
        hip(hipStreamWaitEvent(cs, written, 0));
        if (bytes) hip(hipMemcpyAsync(h_out[k], d_out[k], bytes, hipMemcpyDeviceToHost, cs));
        hip(hipEventRecord(done[k], cs));
        pending[k] = true;
        pending_len[k] = bytes;
        flush(k ^ 1);   // the previous piece, while this one copies
    }
    flush(k ^ 1);
    flush(k);
    int bad = 0;
    if (rc == SID_OK && hip(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost)) && bad) rc = SID_ERANGE;
    if (text_timing())
        std::fprintf(stderr,
                     "{\"dtext_format\": {\"sites\": %zu, \"total_s\": %.6f, \"lengths_s\": %.6f, "
                     "\"alloc_s\": %.6f, \"d2h_wait_s\": %.6f, \"write_s\": %.6f}}\n",
                     n, wall() - f0, t_size, t_alloc, t_wait, t_write);
    (void)hipStreamSynchronize(cs);
    for (int b = 0; b < 2; ++b) (void)hipEventDestroy(done[b]);
    (void)hipEventDestroy(written);
    (void)hipStreamDestroy(cs);
    for (void* p : {(void*)d_bsum, (void*)d_boff, (void*)d_base, (void*)d_bad})
        if (p) (void)hipFree(p);
    return rc;
}

extern "C" int sid_format_g6(double v, char* buf, size_t cap)
{
    char tmp[SID_FMT_MAX];
    const sid_g6 g = sid_g6_prep(v);
    const int n = sid_g6_put(g, tmp);
    if (n < 0) return -SID_ERANGE;
    if (sid_g6_len(g) != n) return -SID_EINVAL;   // the length pass must agree with the writer
    if (!buf || cap < (size_t)n + 1) return -(n + 1);
    std::memcpy(buf, tmp, n);
    buf[n] = '\0';
    return n;
}

extern "C" int sid_format_g6_device(sid_ctx* ctx, const double* d_v, size_t n, char* d_out, void* stream)
{
    if (!ctx || (n && (!d_v || !d_out))) return SID_EINVAL;
    if (n == 0) return SID_OK;
    TCHECK(hipSetDevice(ctx->device));
    sid_fmt_g6_kernel<<<(unsigned)((n + TB - 1) / TB), TB, 0, (hipStream_t)stream>>>(d_v, n, d_out);
    TCHECK(hipGetLastError());
    return SID_OK;
}

// call.cpp:291-372 over n sites parsed with the context's method = quality
// (7 fields per line): starts/counts of the sites, text [0, len) resident.
// Host tables: the four per-quality terms (glibc pow/log through volatile
// pointers, so no compiler rewrite of pow(10, x)) and log_gamma up to the
// largest n = count[ref0] + count[ref1] of the sites.
template <class Off>
static int quality_run(sid_ctx* ctx, const char* text, uint64_t len, const Off* starts, const uint64_t* counts,
                       uint64_t n, uint8_t* code, double* hom_conf, double* het_conf, hipStream_t st)
{
    if (n == 0) return SID_OK;
    if (!code || !hom_conf || !het_conf) return SID_EINVAL;
    if (!ctx->d_qtab) {
        double (*volatile powp)(double, double) = pow;
        double (*volatile logp)(double) = log;
        std::vector<double> q(4 * 256);
        for (int v = 0; v < 256; ++v) {
            const double error = powp(10., v / -10.);            // call.cpp:329
            q[v] = logp(1 - error);                              // :331
            q[256 + v] = logp(error);                            // :333
            q[512 + v] = logp(1 - 2. / 3. * error);              // :336
            q[768 + v] = logp(2. / 3. * error);                  // :338
        }
        TCHECK(hipMalloc(&ctx->d_qtab, q.size() * 8));
        TCHECK(hipMemcpy(ctx->d_qtab, q.data(), q.size() * 8, hipMemcpyHostToDevice));
    }
    if (!ctx->d_scratch) TCHECK(hipMalloc(&ctx->d_scratch, 16));
    TCHECK(hipMemsetAsync(ctx->d_scratch, 0, 4, st));
    sid_max_major_kernel<<<(unsigned)std::min<uint64_t>((n + TB - 1) / TB, 2048), TB, 0, st>>>(counts, n,
                                                                                             ctx->d_scratch);
    uint32_t mx = 0;
    TCHECK(hipMemcpyAsync(&mx, ctx->d_scratch, 4, hipMemcpyDeviceToHost, st));
    TCHECK(hipStreamSynchronize(st));
    const size_t need = (size_t)mx + 2;
    if (need > ctx->lg_n) {   // lynch.hpp:11-31 MemoizedLogGamma (x == 0 -> 0)
        const size_t m = std::max<size_t>(need, 1024);
        std::vector<double> lg(m);
        for (size_t x = 0; x < m; ++x) lg[x] = x == 0 ? 0.0 : sid_gsl_lngamma((double)x);
        if (ctx->d_lg) (void)hipFree(ctx->d_lg);
        ctx->d_lg = nullptr;
        ctx->lg_n = 0;
        TCHECK(hipMalloc(&ctx->d_lg, m * 8));
        TCHECK(hipMemcpy(ctx->d_lg, lg.data(), m * 8, hipMemcpyHostToDevice));
        ctx->lg_n = m;
    }
    QParams P{};
    P.sig = ctx->opts.significance_level;
    P.prior = ctx->opts.snp_prior;
    P.prior_on = P.prior > 0;
    P.prior_ld = P.prior_on && P.prior >= 1;
    if (P.prior_on && !P.prior_ld) {
        // pp1 *= (1 - snp_prior): the factor is the double 1 - prior (call.cpp:354-357)
        const long double a = logl((long double)(1.0 - P.prior)), b = logl((long double)P.prior);
        P.lp1 = {(double)a, (double)(a - (long double)(double)a)};
        P.lp2 = {(double)b, (double)(b - (long double)(double)b)};
    }
    P.lg15 = ctx->K.lg15;
    if (n > ctx->qlo_n) {   // phase 1's lo parts, grow-only
        if (ctx->d_qlo) (void)hipFree(ctx->d_qlo);
        ctx->d_qlo = nullptr;
        ctx->qlo_n = 0;
        TCHECK(hipMalloc(&ctx->d_qlo, n * 16));
        ctx->qlo_n = n;
    }
    const unsigned grid = (unsigned)std::min<uint64_t>((n + TB - 1) / TB, 16384);
    sid_quality_sum_kernel<<<grid, TB, 0, st>>>(text, len, starts, counts, n, ctx->d_qtab, hom_conf, het_conf,
                                                (double2*)ctx->d_qlo);
    sid_quality_finish_kernel<<<grid, TB, 0, st>>>(counts, n, ctx->d_lg, P, code, hom_conf, het_conf,
                                                   (const double2*)ctx->d_qlo);
    TCHECK(hipGetLastError());
    return SID_OK;
}

extern "C" int sid_call_quality(sid_ctx* ctx, const sid_dtext* T, uint8_t* code, double* hom_conf,
                                double* het_conf, void* stream)
{
    if (!ctx || !T) return SID_EINVAL;
    if (!T->quality || ctx->opts.method != SID_METHOD_QUALITY) return SID_ESTATE;
    TCHECK(hipSetDevice(T->device));
    return quality_run(ctx, T->d_text, T->len, T->d_starts, T->d_counts, T->nsites, code, hom_conf, het_conf,
                       (hipStream_t)stream);
}

// exclusive scan of m u32 into u64 offsets from *base (*base advances by the
// sum); ws = sid_scan_ws_bytes(m) bytes (synth.hip's text generator)
size_t sid_scan_ws_bytes(uint64_t m) { return scan_ws_bytes(m); }
hipError_t sid_scan_u32(const uint32_t* in, uint64_t m, uint64_t* out, uint64_t* base, uint64_t* ws, hipStream_t st)
{
    launch_scan(in, m, out, base, nullptr, ws, st);
    return hipGetLastError();
}

// ======================================================= chunk pipeline ====
// One line-aligned chunk of text resident on the device (a ring slot, a
// retained buffer or a slice of a resident text), processed in place by the
// streaming engine (run.cpp).  `base` is 16-B aligned; the chunk is bytes
// [c0, c1) of it; every byte past c1 that a 16-B window may touch is readable
// (a zero pad, or the next chunk's text).  Offsets (line starts, the error
// key) are relative to `base`.
#define WCHECK(x)                                                   \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) return sid_set_hip_error(e_);         \
    } while (0)

static uint64_t chunk_tiles(uint64_t c0, uint64_t c1)
{
    const uint64_t t0 = c0 & ~(uint64_t)15;
    return std::max<uint64_t>((c1 - t0 + TILE - 1) / TILE, 1);
}

int sid_chunk_reserve(sid_chunk_ws* W, uint64_t bytes, uint64_t sites)
{
    // grow-only; hipFree waits for the device, so buffers still in use by
    // queued work are not released under it (growth is rare: the first
    // chunks, or a chunk far above the usual lines per byte)
    if (!W->state) WCHECK(hipMalloc(&W->state, 8 * sizeof(uint64_t)));
    const uint64_t tiles = ((bytes + 16 + IX_TILE - 1) / IX_TILE + 1) * IX_SUB;   // 4 KiB tiles, in whole index tiles
    if (tiles > W->tile_cap) {
        const uint64_t t = std::max<uint64_t>(tiles, W->tile_cap + W->tile_cap / 2);
        if (W->tcnt) (void)hipFree(W->tcnt);
        if (W->toff) (void)hipFree(W->toff);
        if (W->masks) (void)hipFree(W->masks);
        W->tcnt = nullptr;
        W->toff = nullptr;
        W->masks = nullptr;
        W->tile_cap = 0;
        WCHECK(hipMalloc(&W->tcnt, ((t * 4 + 7) & ~(size_t)7) + scan_ws_bytes(t)));
        WCHECK(hipMalloc(&W->toff, t * 8));
        WCHECK(hipMalloc(&W->masks, t * TB * sizeof(uint16_t)));   // a u16 per lane per 4 KiB tile
        W->tile_cap = t;
    }
    if (sites > W->site_cap) {
        const uint64_t m = std::max<uint64_t>(sites, W->site_cap + W->site_cap / 2);
        for (void* p : {(void*)W->starts, (void*)W->counts, (void*)W->code, (void*)W->hom, (void*)W->het,
                        (void*)W->bsum, (void*)W->boff, (void*)W->hdr, (void*)W->fb, (void*)W->lb, (void*)W->cls,
                        (void*)W->twv})
            if (p) (void)hipFree(p);
        W->lb = nullptr;
        W->cls = nullptr;
        W->twv = nullptr;
        W->starts = nullptr;
        W->counts = W->hdr = nullptr;
        W->fb = nullptr;
        W->code = nullptr;
        W->hom = W->het = nullptr;
        W->bsum = nullptr;
        W->boff = nullptr;
        W->site_cap = 0;
        const uint64_t nb = (m + TB - 1) / TB + 1;
        WCHECK(hipMalloc(&W->starts, m * sizeof(sid_off_t)));
        WCHECK(hipMalloc(&W->counts, m * 8));
        WCHECK(hipMalloc(&W->cls, m * 4));
        WCHECK(hipMalloc(&W->hdr, m * 16));
        WCHECK(hipMalloc(&W->twv, (m / 32 + 1) * 16));   // the tile parse's wave entries (tile_nwv)
        WCHECK(hipMalloc(&W->fb, m * 12));   // three site lists (sid_chunk_ws::fb)
        WCHECK(hipMalloc(&W->code, m));
        WCHECK(hipMalloc(&W->hom, m * 8));
        WCHECK(hipMalloc(&W->het, m * 8));
        WCHECK(hipMalloc(&W->bsum, ((nb * 4 + 7) & ~(size_t)7) + scan_ws_bytes(nb)));
        WCHECK(hipMalloc(&W->boff, (nb + 1) * 8));
        WCHECK(hipMalloc(&W->lb, std::max<uint64_t>(nb + 5, 8) * 8));
        W->site_cap = m;
    }
    return SID_OK;
}

void sid_chunk_release(sid_chunk_ws* W)
{
    for (void* p : {(void*)W->starts, (void*)W->counts, (void*)W->code, (void*)W->hom, (void*)W->het,
                    (void*)W->bsum, (void*)W->boff, (void*)W->tcnt, (void*)W->toff, (void*)W->state,
                    (void*)W->hdr, (void*)W->fb, (void*)W->masks, (void*)W->lb, (void*)W->cls, (void*)W->twv})
        if (p) (void)hipFree(p);
    *W = sid_chunk_ws{};
}

// blocks of the strided index kernels (count kernel, index stage per 50M
// sites: 512 blocks 1.89, 1024 1.25, 2048 0.99, 4096 0.97 ms)
constexpr unsigned IX_GRID = 4096;

// line starts of [c0, c1): masks and per-tile counts, scan; state[0] = sites
// (the caller reads it back), state[1..2] = [0, sites), state[4] = no error yet
int sid_chunk_index(sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, hipStream_t st)
{
    const uint64_t t0 = c0 & ~(uint64_t)15;
    const uint64_t ntiles = c1 > c0 ? (c1 - t0 + IX_TILE - 1) / IX_TILE : 0;
    if (ntiles * IX_SUB > W->tile_cap) return SID_EINVAL;
    if (c1 > UINT32_MAX) return SID_ELINE;   // line offsets are 32-bit (sid_off_t): a line ran the chunk past 4 GiB
    if (ntiles == 0) {
        WCHECK(hipMemsetAsync(W->state, 0, 4 * sizeof(uint64_t), st));
        WCHECK(hipMemsetAsync(W->state + 4, 0xFF, sizeof(uint64_t), st));
        return SID_OK;
    }
    const unsigned grid = (unsigned)std::min<uint64_t>(ntiles, IX_GRID);
    sid_index_count_kernel<<<grid, TB, 0, st>>>(base, t0, c0, c1, ntiles, W->masks, W->tcnt, W->state);
    launch_scan(W->tcnt, ntiles, W->toff, W->state, W->state + 1,
                (uint64_t*)((char*)W->tcnt + ((ntiles * 4 + 7) & ~(size_t)7)), st);
    WCHECK(hipGetLastError());
    return SID_OK;
}

// line offsets from the index's masks + the two-pass parse of the n sites;
// state[4] = min(offset * 8 + kind) over the malformed lines (all ones: none)
int sid_chunk_parse(sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, uint64_t n, int qmode,
                    hipStream_t st, const sid_ctx* lctx)
{
    W->lens_ready = false;
    W->cls_ready = false;
    if (n > W->site_cap) return SID_EINVAL;
    if (n == 0) return SID_OK;
    const uint64_t t0 = c0 & ~(uint64_t)15;
    const uint64_t ntiles = (c1 - t0 + IX_TILE - 1) / IX_TILE;
    // (not for long lines: at 200x the fused kernel's extra registers and work
    // cost the parse more than the length kernel costs (C5: the per-lane parse
    // on the reduced grid, parse + lengths 145 vs 141 ms; the quad parse with
    // the lengths fused, 71.4 + 1.8 vs 65.9 + 5.4 ms per step)
    const bool lens = lctx && !qmode && n < (1ull << 32) && (c1 - c0) <= 256 * n;
    const uint64_t nb = (n + FTB - 1) / FTB;
    unsigned long long* fbn = (unsigned long long*)(W->state + 6);
    // (with lens the emit kernel also zeroes the formatter's block sums and
    // flags and the fallback counts: three memset launches fewer)
    sid_index_emit_kernel<<<(unsigned)std::min<uint64_t>(ntiles, IX_GRID), TB, 0, st>>>(
        W->masks, t0, ntiles, W->toff, W->starts, lens ? W->bsum : nullptr, lens ? nb : 0, lens ? W->lb : nullptr,
        lens ? fbn : nullptr);
    if (lens) {
        // -m local: the record lengths out of the parse (sid_parse_len_kernel);
        // sid_chunk_local_len then has only the fix-up and the scan left
        // (lb: [0] the miss count, [1] bytes, [2] range flag; zeroed above)
        uint32_t* late = W->fb + W->site_cap;
        const LocalLen LL{lctx->ws.len1, lctx->ws.len2, W->bsum, W->fb + 2 * W->site_cap, W->lb, W->cls};
        const unsigned pg = (unsigned)std::min<uint64_t>((n + TB - 1) / TB, 16384);
        sid_parse_len_kernel<<<line_walk_grid(n, c1 - c0, pg), TB, 0, st>>>(base, c1, W->starts, W->state + 1,
                                                                            W->counts, W->hdr, W->fb, fbn, LL);
        sid_parse_serial_kernel<<<256, TB, 0, st>>>(base, c1, W->starts, W->state + 1, W->counts, W->hdr, W->fb,
                                                    fbn, (unsigned long long*)(W->state + 4), 0, late, fbn + 1);
        sid_local_len_list_kernel<<<64, TB, 0, st>>>(base, c1, W->starts, W->hdr, W->counts, late, fbn + 1, LL);
        W->lens_ready = true;
        W->cls_ready = true;
    } else {
        launch_parse(base, c1, W->starts, W->state + 1, n, W->counts, W->hdr, W->fb,
                     (unsigned long long*)(W->state + 6), (unsigned long long*)(W->state + 4), qmode, st);
    }
    WCHECK(hipGetLastError());
    return SID_OK;
}

static int chunk_ctype(const char* conf_type, CType* ct)
{
    *ct = CType{};
    ct->len = (int)std::strlen(conf_type);
    if (ct->len >= (int)sizeof ct->s) return SID_EINVAL;
    std::memcpy(ct->s, conf_type, ct->len);
    return SID_OK;
}

// a record is its chrom plus at most 64 bytes (call.hpp:29-38: an int
// position of <= 11 characters, two %g fields of <= 13, a conf_type of <= 15,
// six separators and "hom"/"het" + two bases), and the chroms are bytes of
// their lines
uint64_t sid_chunk_fmt_bound(uint64_t n, uint64_t text_bytes) { return 64 * n + text_bytes + 64; }

// the formatter's steps 1-2 (record bytes per block, their offsets); lb[1]
// = the chunk's bytes afterwards
static int fmt_scan(sid_chunk_ws* W, uint64_t nb, hipStream_t st)
{
    launch_scan(W->bsum, nb, W->boff, (uint64_t*)(W->lb + 1), nullptr,
                (uint64_t*)((char*)W->bsum + ((nb * 4 + 7) & ~(size_t)7)), st);
    WCHECK(hipGetLastError());
    return SID_OK;
}

int sid_chunk_fmt_len(sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, const char* conf_type,
                      hipStream_t st)
{
    CType ct;
    if (chunk_ctype(conf_type, &ct)) return SID_EINVAL;
    if (n > W->site_cap) return SID_EINVAL;
    WCHECK(hipMemsetAsync(W->lb, 0, 8 * 8, st));
    const uint64_t nb = (n + FTB - 1) / FTB;
    if (nb) sid_fmt_blen_kernel<<<(unsigned)nb, FTB, 0, st>>>(base, c1, W->starts, W->hdr, n, W->code, W->hom,
                                                              W->het, ct, W->bsum, W->lb);
    WCHECK(hipGetLastError());
    return fmt_scan(W, nb, st);
}

int sid_chunk_fmt_put(sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, const char* conf_type, char* out,
                      hipStream_t st)
{
    CType ct;
    if (chunk_ctype(conf_type, &ct)) return SID_EINVAL;
    const uint64_t nb = (n + FTB - 1) / FTB;
    if (nb == 0) return hipMemcpyAsync(W->lb + 4, W->state + 4, 8, hipMemcpyDeviceToDevice, st) == hipSuccess
                            ? SID_OK : SID_EHIP;
    sid_fmt_put_kernel<<<(unsigned)nb, FTB, 0, st>>>(base, c1, W->starts, W->hdr, n, W->code, W->hom, W->het, ct,
                                                    W->boff, W->state, W->lb, out);
    WCHECK(hipGetLastError());
    return SID_OK;
}

bool sid_chunk_local_ok(const sid_ctx* ctx)
{
    return ctx->opts.method == SID_METHOD_LOCAL && !ctx->K.general && ctx->ws.str1;
}

// the string tables hold -m local's record tails, conf_type "p_value" included
static int local_ctype(const sid_ctx* ctx, const char* conf_type, CType* ct)
{
    if (chunk_ctype(conf_type, ct) || !sid_chunk_local_ok(ctx) || std::strcmp(conf_type, "p_value") != 0)
        return SID_EINVAL;
    return SID_OK;
}

int sid_chunk_local_len(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n,
                        const char* conf_type, hipStream_t st)
{
    CType ct;
    if (local_ctype(ctx, conf_type, &ct)) return SID_EINVAL;
    if (n > W->site_cap || n >= (1ull << 32)) return SID_EINVAL;
    // the fix-up's sites in the third list of W->fb
    uint32_t* miss = W->fb + 2 * W->site_cap;
    const uint64_t nb = (n + FTB - 1) / FTB;
    if (!W->lens_ready) WCHECK(hipMemsetAsync(W->lb, 0, 8 * 8, st));   // [0] the miss count, [1] bytes, [2] range flag
    if (nb) {
        const unsigned grid = (unsigned)((nb + LPB - 1) / LPB);
        if (!W->lens_ready)   // (else the parse computed them: sid_parse_len_kernel)
            sid_local_len_kernel<<<grid, FTB, 0, st>>>(base, c1, W->starts, W->hdr, n, W->counts, ctx->ws.len1,
                                                       ctx->ws.len2, W->bsum, miss, W->lb);
        sid_local_fixlen_kernel<false><<<64, TB, 0, st>>>(base, c1, W->starts, W->hdr, W->counts, miss, W->lb, ctx->K,
                                                   ctx->d_lnt, ct, W->code, W->hom, W->het, W->bsum, W->lb);
    }
    W->lens_ready = false;
    WCHECK(hipGetLastError());
    return fmt_scan(W, nb, st);
}

int sid_chunk_local_put(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n,
                        const char* conf_type, char* out, hipStream_t st)
{
    CType ct;
    if (local_ctype(ctx, conf_type, &ct)) return SID_EINVAL;
    const uint64_t nb = (n + FTB - 1) / FTB;
    if (W->slot_cap) {   // the tile parse's slots
        const uint64_t nbs = (W->slots + FTB - 1) / FTB;
        if (nbs == 0) return hipMemcpyAsync(W->lb + 4, W->state + 4, 8, hipMemcpyDeviceToDevice, st) == hipSuccess
                                 ? SID_OK : SID_EHIP;
        if (W->slots >= SID_SLOTS_MAX) return SID_EINVAL;   // (slot_tile's exact range: a 4 GiB chunk has fewer)
        const SlotDiv cdiv = slot_div(W->slot_cap);
        auto put = W->tile_quad ? sid_local_put_kernel<true, false> : sid_local_put_kernel<true, true>;
        put<<<(unsigned)nbs, FTB, 0, st>>>(base, c1, nullptr, W->hdr, W->slots, W->tcnt, W->slot_cap, cdiv, W->twv,
                                           tile_nwv(W->slot_cap), W->counts, W->cls, ctx->ws.str1, ctx->ws.str2,
                                           W->code, W->hom, W->het, ct, W->boff, W->state, W->lb, out);
        WCHECK(hipGetLastError());
#ifdef SID_TP_STAMP
        {
            const uint64_t m = std::min<uint64_t>(nbs, TP_STAMP_N);
            std::vector<uint32_t> v(m * 4);
            if (hipStreamSynchronize(st) == hipSuccess &&
                hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(put_stamp), m * 16) == hipSuccess && m) {
                double a[4] = {0, 0, 0, 0};
                for (uint64_t k = 0; k < m; ++k)
                    for (int j = 0; j < 4; ++j) a[j] += v[4 * k + j];
                fprintf(stderr, "put_stamp blocks=%llu us/block: loads+len %.2f scan %.2f lds %.2f store %.2f\n",
                        (unsigned long long)m, a[0] / 100.0 / m, a[1] / 100.0 / m, a[2] / 100.0 / m, a[3] / 100.0 / m);
            }
        }
#endif
        return SID_OK;
    }
    if (nb == 0) return hipMemcpyAsync(W->lb + 4, W->state + 4, 8, hipMemcpyDeviceToDevice, st) == hipSuccess
                            ? SID_OK : SID_EHIP;
    if (W->cls_ready)
        sid_local_put_kernel<true><<<(unsigned)nb, FTB, 0, st>>>(base, c1, W->starts, W->hdr, n, nullptr, 0, SlotDiv{0, 0},
                                                                nullptr, 0, W->counts, W->cls,
                                                                ctx->ws.str1, ctx->ws.str2, W->code, W->hom, W->het,
                                                                ct, W->boff, W->state, W->lb, out);
    else
        sid_local_put_kernel<false><<<(unsigned)nb, FTB, 0, st>>>(base, c1, W->starts, W->hdr, n, nullptr, 0,
                                                                 SlotDiv{0, 0}, nullptr, 0, W->counts, nullptr,
                                                                 ctx->ws.str1, ctx->ws.str2, W->code, W->hom, W->het,
                                                                 ct, W->boff, W->state, W->lb, out);
    WCHECK(hipGetLastError());
    return SID_OK;
}

static uint64_t tile_count(uint64_t c0, uint64_t c1, bool quad)
{
    const uint64_t t0 = c0 & ~(uint64_t)15;
    return c1 > c0 ? (c1 - t0 + tp_tile(quad) - 1) / tp_tile(quad) : 0;
}

template <bool LOCAL>
static void launch_tile_parse(bool quad, const char* base, uint64_t c0, uint64_t c1, uint64_t ntp, const TileOut& O,
                              const LocalLen& LL, hipStream_t st)
{
    const uint64_t tb = c0 & ~(uint64_t)15;
    if (quad)
        sid_tile_parse_kernel<true, LOCAL><<<(unsigned)ntp, TB, 0, st>>>(base, tb, c0, c1, O, LL);
    else
        sid_tile_parse_kernel<false, LOCAL><<<(unsigned)ntp, TB, 0, st>>>(base, tb, c0, c1, O, LL);
#ifdef SID_TP_STAMP
    {
        const uint64_t m = std::min<uint64_t>(ntp, TP_STAMP_N);
        std::vector<uint32_t> v(m * 4);
        if (hipStreamSynchronize(st) == hipSuccess &&
            hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(tp_stamp), m * 16) == hipSuccess && m) {
            double a[3] = {0, 0, 0};
            uint32_t lo = UINT32_MAX, hi = 0;
            for (uint64_t k = 0; k < m; ++k) {
                for (int j = 0; j < 3; ++j) a[j] += v[4 * k + j];
                lo = std::min(lo, v[4 * k + 3]);
                hi = std::max(hi, v[4 * k + 3]);
            }
            fprintf(stderr, "tp_stamp quad=%d blocks=%llu us/block: load %.2f index %.2f parse %.2f; starts span %.1f us\n",
                    (int)quad, (unsigned long long)m, a[0] / 100.0 / m, a[1] / 100.0 / m, a[2] / 100.0 / m,
                    (hi - lo) * 0.16);
        }
    }
#endif
}

// the unit of the tile parse's slot layout (bytes of text a tile)
uint32_t sid_tile_unit(bool quad) { return tp_tile(quad); }

uint64_t sid_chunk_tile_slots(uint64_t c0, uint64_t c1, uint32_t cap, bool quad)
{
    return tile_count(c0, c1, quad) * cap;
}

// a record is its chrom plus at most 64 bytes, and the chroms are bytes of
// their lines (sid_chunk_fmt_bound), with at most every slot a site
uint64_t sid_chunk_tile_bound(uint64_t c0, uint64_t c1, uint32_t cap, bool quad)
{
    return sid_chunk_fmt_bound(sid_chunk_tile_slots(c0, c1, cap, quad), c1 - c0);
}

int sid_chunk_tile_local(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, uint32_t cap,
                         bool quad, const char* conf_type, hipStream_t st)
{
    CType ct;
    if (local_ctype(ctx, conf_type, &ct)) return SID_EINVAL;
    if (cap < SID_TILE_CAP_MIN || cap > tp_cap_max(quad) || cap % 16) return SID_EINVAL;
    if (c1 > UINT32_MAX) return SID_ELINE;   // line offsets are 32-bit: a line ran the chunk past 4 GiB
    const uint64_t ntp = tile_count(c0, c1, quad);
    const uint64_t slots = ntp * cap;
    if (slots > W->site_cap || ntp > W->tile_cap || slots >= (1ull << 32)) return SID_EINVAL;
    if (ntp * tile_nwv(cap) > W->site_cap / 32 + 1) return SID_EINVAL;   // (never: cap >= 64)
    W->lens_ready = false;
    W->cls_ready = false;
    W->slot_cap = cap;
    W->slots = slots;
    W->tile_quad = quad;   // (the quad shape stores no compact words: the writer reads every header pair)
    const uint64_t nb = (slots + FTB - 1) / FTB;
    WCHECK(hipMemsetAsync(W->lb, 0, 8 * 8, st));   // [0] fix-up sites [1] bytes [2] range [3] sites [5] max lines [6] [7]
    if (nb) WCHECK(hipMemsetAsync(W->bsum, 0, nb * 4, st));
    if (ntp == 0) {
        WCHECK(hipMemsetAsync(W->state + 4, 0xFF, sizeof(uint64_t), st));
        return fmt_scan(W, nb, st);
    }
    uint32_t* miss = W->fb + 2 * W->site_cap;
    const LocalLen LL{ctx->ws.len1, ctx->ws.len2, W->bsum, miss, W->lb, W->cls};
    const TileOut O{cap, W->tcnt, W->hdr, W->counts, W->fb, W->starts, W->lb, W->state, W->twv, tile_nwv(cap)};
    launch_tile_parse<true>(quad, base, c0, c1, ntp, O, LL, st);
    const LocalFix F{LL, ctx->K, ctx->d_lnt, ct, W->code, W->hom, W->het};
    sid_tile_serial_kernel<true><<<TILE_SERIAL_GRID, TB, 0, st>>>(base, c1, W->fb, W->starts, W->lb, W->tcnt, ntp,
                                                     cap, W->counts, W->hdr,
                                                     (unsigned long long*)(W->state + 4), F);
    WCHECK(hipGetLastError());
    W->cls_ready = true;
    return fmt_scan(W, nb, st);
}

int sid_chunk_tile_counts(sid_chunk_ws* W, const char* base, uint64_t c0, uint64_t c1, uint32_t cap, bool quad,
                          hipStream_t st)
{
    if (cap < SID_TILE_CAP_MIN || cap > tp_cap_max(quad) || cap % 16) return SID_EINVAL;
    if (c1 > UINT32_MAX) return SID_ELINE;   // line offsets are 32-bit: a line ran the chunk past 4 GiB
    const uint64_t ntp = tile_count(c0, c1, quad);
    const uint64_t slots = ntp * cap;
    if (slots > W->site_cap || ntp > W->tile_cap || slots >= (1ull << 32)) return SID_EINVAL;
    W->lens_ready = false;
    W->cls_ready = false;
    W->slot_cap = cap;
    W->slots = slots;
    W->tile_quad = quad;
    W->tile_ntp = ntp;
    WCHECK(hipMemsetAsync(W->lb, 0, 8 * 8, st));
    WCHECK(hipMemsetAsync(W->state, 0, 8, st));   // the scan's running base: the chunk's sites
    if (ntp == 0) {
        WCHECK(hipMemsetAsync(W->state + 4, 0xFF, sizeof(uint64_t), st));
        return SID_OK;
    }
    const LocalLen LL{};
    const TileOut O{cap, W->tcnt, W->hdr, W->counts, W->fb, W->starts, W->lb, W->state, nullptr, 0};
    launch_tile_parse<false>(quad, base, c0, c1, ntp, O, LL, st);
    sid_tile_serial_kernel<false><<<TILE_SERIAL_GRID, TB, 0, st>>>(base, c1, W->fb, W->starts, W->lb, W->tcnt, ntp,
                                                      cap, W->counts, W->hdr,
                                                      (unsigned long long*)(W->state + 4), LocalFix{});
    // the tiles' first sites in file order (state[0]: the chunk's sites; over the cap: void)
    launch_scan(W->tcnt, ntp, W->toff, W->state, nullptr,
                (uint64_t*)((char*)W->tcnt + ((ntp * 4 + 7) & ~(size_t)7)), st);
    WCHECK(hipGetLastError());
    return SID_OK;
}

int sid_chunk_tile_compact(sid_chunk_ws* W, sid_off_t* starts, uint64_t* counts, uint64_t* hdr, hipStream_t st)
{
    if (!W->slot_cap) return SID_ESTATE;
    if (W->slots >= SID_SLOTS_MAX) return SID_EINVAL;   // (slot_tile's exact range: a 4 GiB chunk has fewer)
    const SlotDiv cdiv = slot_div(W->slot_cap);
    const unsigned grid = (unsigned)std::min<uint64_t>(std::max<uint64_t>((W->slots + TB - 1) / TB, 1), 8192);
    sid_tile_compact_kernel<<<grid, TB, 0, st>>>(W->tcnt, W->toff, W->slots, W->slot_cap, cdiv, W->counts, W->hdr,
                                                 starts, counts, hdr);
    W->slot_cap = 0;   // the dense layout again
    WCHECK(hipGetLastError());
    return SID_OK;
}

int sid_chunk_lynch_len(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, hipStream_t st)
{
    sid_lynch_fmt V;
    if (sid_lynch_fmt_view(ctx, &V) != SID_OK) return SID_ESTATE;
    if (n > W->site_cap) return SID_EINVAL;
    WCHECK(hipMemsetAsync(W->lb, 0, 8 * 8, st));   // [1] bytes, [2] range flag
    const uint64_t nb = (n + FTB - 1) / FTB;
    if (nb && V.empty) {   // no class: every site dropped (and no length table)
        WCHECK(hipMemsetAsync(W->bsum, 0, nb * 4, st));
    } else if (nb) {
        sid_lynch_len_kernel<<<(unsigned)((nb + LPB - 1) / LPB), FTB, 0, st>>>(base, c1, W->starts, W->hdr, n,
                                                                                W->counts, V, W->bsum);
    }
    WCHECK(hipGetLastError());
    return fmt_scan(W, nb, st);
}

int sid_chunk_lynch_put(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, char* out,
                        hipStream_t st)
{
    sid_lynch_fmt V;
    if (sid_lynch_fmt_view(ctx, &V) != SID_OK) return SID_ESTATE;
    const uint64_t nb = (n + FTB - 1) / FTB;
    if (nb == 0) return hipMemcpyAsync(W->lb + 4, W->state + 4, 8, hipMemcpyDeviceToDevice, st) == hipSuccess
                            ? SID_OK : SID_EHIP;
    sid_lynch_put_kernel<<<(unsigned)nb, FTB, 0, st>>>(base, c1, W->starts, W->hdr, n, W->counts, V, W->boff,
                                                      W->state, W->lb, out);
    WCHECK(hipGetLastError());
    return SID_OK;
}

hipError_t sid_launch_lynch_str_build(const uint8_t* pcode, const double* cc, uint32_t U, const char* conf_type,
                                      const uint32_t* dense_cidx, char* lstr, uint8_t* dlen, uint32_t* bad,
                                      hipStream_t st)
{
    CType ct;
    if (chunk_ctype(conf_type, &ct)) return hipErrorInvalidValue;
    if (U) sid_lynch_str_kernel<<<(U + 255) / 256, 256, 0, st>>>(pcode, cc, U, ct, lstr, bad);
    sid_lynch_dlen_kernel<<<SID_DENSE_N / 256, 256, 0, st>>>(dense_cidx, lstr, dlen);
    return hipGetLastError();
}

int sid_chunk_quality(sid_ctx* ctx, sid_chunk_ws* W, const char* base, uint64_t c1, uint64_t n, hipStream_t st)
{
    return quality_run(ctx, base, c1, W->starts, W->counts, n, W->code, W->hom, W->het, st);
}
