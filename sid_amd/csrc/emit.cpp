// emit.cpp — CSV emitter.
//
// Byte-identical to operator<<(OutputRecord) (call.hpp:29-38) as printed by
// sid.cpp:103-105: chrom,pos,label,gt,hom_conf,het_conf,conf_type.  Doubles
// use the iostream default format (%g, precision 6); std::to_chars with
// chars_format::general and precision 6 produces the same bytes (nan/-nan,
// inf/-inf, denormals included; tests/test_emit.py checks against printf).
#include <charconv>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/sid.h"

#include "sites.h"

namespace {
inline char* put_double(char* p, double v)
{
    if (v == 1.0) {   // the most frequent value (one of the two confs is 1)
        *p++ = '1';
        return p;
    }
    auto r = std::to_chars(p, p + 32, v, std::chars_format::general, 6);
    return r.ptr;
}

inline char* put_int(char* p, int32_t v)
{
    auto r = std::to_chars(p, p + 12, v);
    return r.ptr;
}
}  // namespace

extern "C" int sid_format_double(double v, char* buf, size_t cap)
{
    char tmp[40];
    char* e = put_double(tmp, v);
    size_t n = (size_t)(e - tmp);
    if (!buf || cap < n + 1) return -(int)(n + 1);
    std::memcpy(buf, tmp, n);
    buf[n] = '\0';
    return (int)n;
}

extern "C" int sid_format_csv(const sid_sites* s, size_t begin, size_t end, const uint8_t* code,
                              const double* hom_conf, const double* het_conf, const char* conf_type,
                              char* buf, size_t cap, size_t* len)
{
    if (!s || !len || !code || !hom_conf || !het_conf || !conf_type) return SID_EINVAL;
    if (end > s->pos.size() || begin > end) return SID_EINVAL;
    static const char ACGT[] = "ACGT";
    const size_t tlen = std::strlen(conf_type);
    // segment containing `begin`
    size_t k = 0;
    {
        size_t lo = 0, hi = s->seg_start.size();
        while (lo + 1 < hi) {
            size_t mid = (lo + hi) / 2;
            if (s->seg_start[mid] <= begin) lo = mid; else hi = mid;
        }
        k = lo;
    }
    // worst-case size
    size_t maxname = 0;
    for (const auto& n : s->seg_name) maxname = std::max(maxname, n.size());
    const size_t per = maxname + tlen + 12 + 4 + 3 + 2 * 14 + 8;
    const size_t need = (end - begin) * per;
    if (!buf || cap < need) {
        *len = need;
        return SID_ENOMEM;
    }
    char* p = buf;
    size_t next_seg = k + 1 < s->seg_start.size() ? s->seg_start[k + 1] : (size_t)-1;
    const std::string* name = s->seg_name.empty() ? nullptr : &s->seg_name[k];
    for (size_t i = begin; i < end; ++i) {
        while (i >= next_seg) {
            ++k;
            name = &s->seg_name[k];
            next_seg = k + 1 < s->seg_start.size() ? s->seg_start[k + 1] : (size_t)-1;
        }
        const uint8_t c = code[i];
        if (c & 0x40) continue;   // filtered profile: no record (call.cpp:131-140)
        std::memcpy(p, name->data(), name->size());
        p += name->size();
        *p++ = ',';
        p = put_int(p, s->pos[i]);
        *p++ = ',';
        std::memcpy(p, (c & 0x80) ? "het," : "hom,", 4);
        p += 4;
        *p++ = ACGT[c & 3];
        *p++ = ACGT[(c >> 2) & 3];
        *p++ = ',';
        p = put_double(p, hom_conf[i]);
        *p++ = ',';
        p = put_double(p, het_conf[i]);
        *p++ = ',';
        std::memcpy(p, conf_type, tlen);
        p += tlen;
        *p++ = '\n';
    }
    *len = (size_t)(p - buf);
    return SID_OK;
}
