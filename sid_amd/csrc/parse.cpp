// parse.cpp — host pileup parser.
//
// Restates readFile + parsePileupLine + parseReadBases (call.cpp:11-20,
// pileup.cpp:13-153) for streaming, multi-threaded use: the text is split at
// line boundaries, each thread tokenises its lines into SoA columns
// (profile_t counts, int positions, chromosome runs).  Differences from the
// reference are performance-only: no per-site heap objects, a linear (not
// quadratic, pileup.cpp:76) scan of the read-bases field, a class table
// instead of a switch.
//
// Semantics kept exactly:
//   - fields split on runs of ' ' / '\t' (strtok_r, pileup.cpp:11); any other
//     byte, '\r' included, belongs to a token; a NUL byte ends the line;
//   - position = atoi = (int)strtol(tok, 10) (leading isspace, sign,
//     saturation at LONG_MIN/LONG_MAX, then truncation to int);
//   - reference must be exactly one byte; coverage and quality fields are
//     only required to exist as far as the reference requires them;
//   - '.' / ',' stand for toupper(ref) / tolower(ref) and are then classified
//     like any other byte (so a reference of '^', '+' or '-' changes
//     parsing exactly as in pileup.cpp:78-83);
//   - '^' skips one byte; '+'/'-' followed by a digit skip strtol(number)
//     bytes after the number; counts are uint16 and wrap.
#include <algorithm>
#include <climits>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sid.h"

#include "sites.h"

namespace {

enum : uint8_t { C_IGN = 0, C_A = 1, C_C = 2, C_G = 3, C_T = 4, C_CARET = 5, C_INDEL = 6 };

struct ClassTable {
    uint8_t t[256];
    ClassTable()
    {
        std::memset(t, C_IGN, sizeof t);
        t[(uint8_t)'A'] = t[(uint8_t)'a'] = C_A;
        t[(uint8_t)'C'] = t[(uint8_t)'c'] = C_C;
        t[(uint8_t)'G'] = t[(uint8_t)'g'] = C_G;
        t[(uint8_t)'T'] = t[(uint8_t)'t'] = C_T;
        t[(uint8_t)'^'] = C_CARET;
        t[(uint8_t)'+'] = t[(uint8_t)'-'] = C_INDEL;
    }
};
const ClassTable BASE_CLASS;

inline bool is_sep(char c) { return c == ' ' || c == '\t'; }
inline bool is_c_space(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline char c_toupper(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }
inline char c_tolower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

// (int)strtol(s, NULL, 10) over [b, e)
int atoi_like(const char* b, const char* e)
{
    while (b < e && is_c_space(*b)) ++b;
    bool neg = false;
    if (b < e && (*b == '+' || *b == '-')) {
        neg = *b == '-';
        ++b;
    }
    unsigned long long v = 0;
    bool ovf = false;
    while (b < e && is_digit(*b)) {
        unsigned d = (unsigned)(*b - '0');
        if (v > (ULLONG_MAX - d) / 10) ovf = true; else v = v * 10 + d;
        ++b;
    }
    long r;
    if (!neg) {
        r = (ovf || v > (unsigned long long)LONG_MAX) ? LONG_MAX : (long)v;
    } else {
        r = (ovf || v > (unsigned long long)LONG_MAX + 1ull) ? LONG_MIN : (long)(0ull - v);
    }
    return (int)(unsigned)(unsigned long)r;
}

// strtol on a digit run starting at p (first byte is a digit): saturates at LONG_MAX
unsigned long digits_like_strtol(const char* p, const char* e, const char** end)
{
    unsigned long long v = 0;
    bool ovf = false;
    while (p < e && is_digit(*p)) {
        unsigned d = (unsigned)(*p - '0');
        if (!ovf) {
            if (v > ((unsigned long long)LONG_MAX - d) / 10) ovf = true; else v = v * 10 + d;
        }
        ++p;
    }
    *end = p;
    return ovf ? (unsigned long)LONG_MAX : (unsigned long)v;
}

// parseReadBases counts over the token [b, e)
void read_bases(const char* b, const char* e, char ref, uint16_t out[4])
{
    uint8_t cls[256];
    std::memcpy(cls, BASE_CLASS.t, sizeof cls);
    cls[(uint8_t)'.'] = BASE_CLASS.t[(uint8_t)c_toupper(ref)];
    cls[(uint8_t)','] = BASE_CLASS.t[(uint8_t)c_tolower(ref)];
    uint32_t n[5] = {0, 0, 0, 0, 0};
    const size_t len = (size_t)(e - b);
    for (size_t i = 0; i < len; ++i) {
        const uint8_t k = cls[(uint8_t)b[i]];
        if (k <= C_T) {
            n[k]++;   // n[0] collects ignored bytes
        } else if (k == C_CARET) {
            ++i;
        } else {      // C_INDEL
            if (i + 1 < len && is_digit(b[i + 1])) {
                const char* endp;
                unsigned long length = digits_like_strtol(b + i + 1, e, &endp);
                size_t after = (size_t)(endp - b);
                i = after + length - 1;   // cannot wrap: after < 2^32, length <= LONG_MAX
            }
        }
    }
    for (int j = 0; j < 4; ++j) out[j] = (uint16_t)n[j + 1];
}

struct Err {
    uint64_t offset = UINT64_MAX;
    int code = SID_OK;
};

struct Part {
    std::vector<uint16_t> counts;
    std::vector<int32_t> pos;
    std::vector<uint64_t> seg_start;   // local site index
    std::vector<std::string> seg_name;
    Err err;
};

// Parse whole lines in [b, e) (b at a line start).  base = text start.
void parse_range(const char* base, const char* b, const char* e, Part& P)
{
    P.counts.reserve((size_t)(e - b) / 40 * 4 + 16);
    P.pos.reserve((size_t)(e - b) / 40 + 4);
    const char* p = b;
    size_t nsites = 0;
    const char* last_name = nullptr;
    size_t last_len = 0;
    while (p < e) {
        const char* nl = (const char*)std::memchr(p, '\n', (size_t)(e - p));
        const char* le = nl ? nl : e;
        const char* next = nl ? nl + 1 : e;
        if (le == p) {   // empty line (call.cpp:14)
            p = next;
            continue;
        }
        // a NUL ends the C string parsePileupLine sees
        const char* z = (const char*)std::memchr(p, '\0', (size_t)(le - p));
        const char* end = z ? z : le;
        const char* q = p;
        const char* tb[5];
        const char* te[5];
        int nt = 0;
        while (nt < 5) {
            while (q < end && is_sep(*q)) ++q;
            if (q >= end) break;
            tb[nt] = q;
            while (q < end && !is_sep(*q)) ++q;
            te[nt] = q;
            ++nt;
        }
        int code = SID_OK;
        if (nt < 1) code = SID_ENULLCHROM;
        else if (nt < 3 || (te[2] - tb[2]) != 1 || nt < 5) code = SID_EMALFORMED;
        if (code != SID_OK) {
            P.err.offset = (uint64_t)(p - base);
            P.err.code = code;
            return;
        }
        const size_t nlen = (size_t)(te[0] - tb[0]);
        if (!last_name || nlen != last_len || std::memcmp(last_name, tb[0], nlen) != 0) {
            P.seg_start.push_back(nsites);
            P.seg_name.emplace_back(tb[0], nlen);
            last_name = tb[0];
            last_len = nlen;
        }
        P.pos.push_back(atoi_like(tb[1], te[1]));
        uint16_t c[4];
        read_bases(tb[4], te[4], *tb[2], c);
        P.counts.insert(P.counts.end(), c, c + 4);
        ++nsites;
        p = next;
    }
}

}  // namespace

extern "C" int sid_parse_text(const char* text, size_t len, int nthreads, sid_sites** out,
                              uint64_t* err_line)
{
    if (!out || (!text && len)) return SID_EINVAL;
    *out = nullptr;
    int T = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
    if (T > 64) T = 64;
    if (len < (size_t)T * 65536) T = std::max<int>(1, (int)(len / 65536));
    // split at line starts
    std::vector<const char*> cut(T + 1);
    cut[0] = text;
    cut[T] = text + len;
    for (int t = 1; t < T; ++t) {
        const char* c = text + len / T * t;
        if (c < cut[t - 1]) c = cut[t - 1];
        const char* nl = (const char*)std::memchr(c, '\n', (size_t)(text + len - c));
        cut[t] = nl ? nl + 1 : text + len;
    }
    std::vector<Part> parts(T);
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back([&, t] { parse_range(text, cut[t], cut[t + 1], parts[t]); });
    parse_range(text, cut[0], cut[1], parts[0]);
    for (auto& x : th) x.join();
    // first error in file order wins
    Err first;
    for (auto& P : parts)
        if (P.err.code != SID_OK && P.err.offset < first.offset) first = P.err;
    if (first.code != SID_OK) {
        if (err_line) {
            uint64_t lines = 0;
            const char* p = text;
            const char* stop = text + first.offset;
            while (p < stop) {
                const char* nl = (const char*)std::memchr(p, '\n', (size_t)(stop - p));
                if (!nl) break;
                ++lines;
                p = nl + 1;
            }
            *err_line = lines;
        }
        return first.code;
    }
    sid_sites* S = new sid_sites();
    size_t total = 0;
    std::vector<size_t> off(T + 1, 0);
    for (int t = 0; t < T; ++t) {
        off[t] = total;
        total += parts[t].pos.size();
    }
    S->counts.resize(total * 4);
    S->pos.resize(total);
    std::vector<std::thread> cp;
    for (int t = 0; t < T; ++t)
        cp.emplace_back([&, t] {
            if (parts[t].pos.empty()) return;   // (memcpy from a null pointer is undefined, even of 0 bytes)
            std::memcpy(S->counts.data() + 4 * off[t], parts[t].counts.data(), parts[t].counts.size() * 2);
            std::memcpy(S->pos.data() + off[t], parts[t].pos.data(), parts[t].pos.size() * 4);
        });
    for (auto& x : cp) x.join();
    for (int t = 0; t < T; ++t) {
        for (size_t k = 0; k < parts[t].seg_name.size(); ++k) {
            if (!S->seg_name.empty() && S->seg_name.back() == parts[t].seg_name[k]) continue;
            S->seg_start.push_back(off[t] + parts[t].seg_start[k]);
            S->seg_name.push_back(std::move(parts[t].seg_name[k]));
        }
    }
    *out = S;
    return SID_OK;
}

extern "C" void sid_sites_free(sid_sites* s) { delete s; }
extern "C" size_t sid_sites_count(const sid_sites* s) { return s ? s->pos.size() : 0; }
extern "C" const uint16_t* sid_sites_counts(const sid_sites* s) { return s ? s->counts.data() : nullptr; }
extern "C" const int32_t* sid_sites_positions(const sid_sites* s) { return s ? s->pos.data() : nullptr; }
extern "C" size_t sid_sites_chrom_segments(const sid_sites* s) { return s ? s->seg_name.size() : 0; }
extern "C" const char* sid_sites_chrom_name(const sid_sites* s, size_t k, uint64_t* start)
{
    if (!s || k >= s->seg_name.size()) return nullptr;
    if (start) *start = s->seg_start[k];
    return s->seg_name[k].c_str();
}
