// synth.h — counter-based synthetic 30x/200x diploid pileup (BASELINE.md
// "Synthetic generator").
//
// Every random draw is a pure function of (seed, global site index, draw
// index), so any site range is generated bit-identically on the host (text)
// and on the device (counts), for any number of GPUs.  Only integer
// arithmetic is used after the Poisson CDF table is built on the host, so the
// host text and the device counts agree exactly (parse(text(i)) == counts(i)).
//
// Per site: ref uniform over ACGT; diploid het with probability 1e-3, alt
// uniform over the other three; depth ~ Poisson(mean).  Per read: allele =
// ref, or ref/alt 50:50 at het sites; sequencing error 1% to a uniform other
// base; strand 50:50 ('.'/',' for ref, upper/lower case otherwise); "^]"
// read start and '$' read end each with probability 1/150; base quality
// uniform Q20..Q40.  Depth 0 prints "*\t*".
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define SID_HD __host__ __device__ __forceinline__
#else
#define SID_HD static inline
#endif

#define SID_SYNTH_MAX_DEPTH_TABLE 1024

// Probabilities as thresholds on a uniform 64-bit draw: P(u < T) = T / 2^64.
#define SID_SYNTH_T_HET 0x004189374BC6A7F0ull   // floor(1e-3 * 2^64)
#define SID_SYNTH_T_ERR 0x028F5C28F5C28F60ull   // floor(1e-2 * 2^64)

SID_HD uint64_t sid_splitmix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

SID_HD uint64_t sid_site_key(uint64_t seed, uint64_t site)
{
    return sid_splitmix64(seed * 0xD1B54A32D192ED03ull ^ sid_splitmix64(site));
}

SID_HD uint64_t sid_draw(uint64_t key, uint32_t j)
{
    return sid_splitmix64(key + (uint64_t)j * 0x9E3779B97F4A7C15ull);
}

// depth = smallest k with u < cdf[k]; cdf[kmax-1] == UINT64_MAX.
SID_HD uint32_t sid_synth_depth(const uint64_t* cdf, uint32_t kmax, uint64_t u)
{
    uint32_t lo = 0, hi = kmax - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

struct sid_synth_site {
    uint32_t ref;    // 0..3
    uint32_t het;    // 0/1
    uint32_t alt;    // 0..3
    uint32_t depth;
    uint64_t key;
};

SID_HD struct sid_synth_site sid_synth_site_header(uint64_t seed, uint64_t site,
                                                   const uint64_t* cdf, uint32_t kmax)
{
    struct sid_synth_site s;
    s.key = sid_site_key(seed, site);
    s.ref = (uint32_t)(sid_draw(s.key, 0) & 3u);
    s.het = sid_draw(s.key, 1) < SID_SYNTH_T_HET ? 1u : 0u;
    s.alt = (s.ref + 1u + (uint32_t)(sid_draw(s.key, 2) % 3u)) & 3u;
    s.depth = sid_synth_depth(cdf, kmax, sid_draw(s.key, 3));
    return s;
}

// Base observed on read r (0..3) and its strand (1 = forward).
SID_HD uint32_t sid_synth_read_base(const struct sid_synth_site* s, uint32_t r, uint32_t* strand)
{
    uint64_t u0 = sid_draw(s->key, 8u + 4u * r);
    uint32_t allele = (s->het && (u0 & 1u)) ? s->alt : s->ref;
    *strand = (uint32_t)((u0 >> 1) & 1u);
    uint64_t u1 = sid_draw(s->key, 8u + 4u * r + 1u);
    if (u1 < SID_SYNTH_T_ERR) {
        uint64_t u2 = sid_draw(s->key, 8u + 4u * r + 2u);
        allele = (allele + 1u + (uint32_t)(u2 % 3u)) & 3u;
    }
    return allele;
}

// Read start / end markers and base quality of read r.
SID_HD void sid_synth_read_marks(const struct sid_synth_site* s, uint32_t r, int* start, int* end,
                                 uint32_t* qual)
{
    uint64_t u3 = sid_draw(s->key, 8u + 4u * r + 3u);
    *start = (u3 & 0xFFFFFu) % 150u == 0u;
    *end = ((u3 >> 20) & 0xFFFFFu) % 150u == 0u;
    *qual = 20u + (uint32_t)((u3 >> 40) % 21u);
}

// Mapping quality of read r (samtools mpileup -s 7th column): uniform 0..60.
SID_HD uint32_t sid_synth_read_mapq(const struct sid_synth_site* s, uint32_t r)
{
    return (uint32_t)(sid_draw(s->key, 0x40000000u + r) % 61u);
}

// Counts (A,C,G,T) packed as profile_t little-endian u64 (pileup.hpp:7).
// Synthetic depth is < 65536, so the per-base 16-bit fields never carry.
SID_HD uint64_t sid_synth_counts(uint64_t seed, uint64_t site, const uint64_t* cdf, uint32_t kmax)
{
    struct sid_synth_site s = sid_synth_site_header(seed, site, cdf, kmax);
    uint64_t packed = 0;
    for (uint32_t r = 0; r < s.depth; ++r) {
        uint32_t strand;
        uint32_t b = sid_synth_read_base(&s, r, &strand);
        packed += 1ull << (16u * b);
    }
    return packed;
}
