// sid_asan — the product's host code (parse.cpp, emit.cpp, fmt.h's host
// build) under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5:
// sanitizers on the host restatement).  TEST INFRASTRUCTURE: driven by
// tests/test_sanitized.py, which compares every output with the unsanitized
// build/libsid.so on the same inputs.
//
//   sid_asan lines FILE          each '\n'-separated line parsed on its own
//                                (sid_parse_text): "OK chrom pos A C G T",
//                                "ERR status", or "NONE" (no site)
//   sid_asan csv FILE THREADS    the whole file parsed with THREADS threads,
//                                then sid_format_csv over every site with
//                                synthetic code / confidences (synth_site)
//   sid_asan g6 FILE             binary f64 values: fmt.h's %g and
//                                sid_format_double, one line each
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fmt.h"
#include "sid.h"

static std::vector<char> slurp(const char* path)
{
    std::vector<char> b;
    FILE* f = std::fopen(path, "rb");
    if (!f) return b;
    char tmp[1 << 16];
    size_t n;
    while ((n = std::fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + n);
    std::fclose(f);
    return b;
}

// the synthetic per-site outputs tests/test_sanitized.py recomputes
static void synth_site(uint64_t i, uint8_t* c, double* h, double* t)
{
    *c = (uint8_t)(((i * 37u) & 0x0Fu) | (i % 5 == 0 ? 0x80u : 0u) | (i % 11 == 3 ? 0x40u : 0u));
    *h = std::ldexp((double)((i * 2654435761ull) % 1000003ull) / 1000003.0, -(int)(i % 60));
    *t = std::ldexp((double)((i * 40503ull + 7) % 999983ull) / 999983.0, -(int)(i % 1075));
}

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    const std::string mode = argv[1];
    std::vector<char> in = slurp(argv[2]);
    if (mode == "lines") {
        size_t at = 0;
        while (at < in.size()) {
            size_t e = at;
            while (e < in.size() && in[e] != '\n') ++e;
            std::vector<char> line(in.begin() + at, in.begin() + e);
            line.push_back('\n');
            sid_sites* s = nullptr;
            uint64_t bad = 0;
            const int rc = sid_parse_text(line.data(), line.size(), 1, &s, &bad);
            if (rc != SID_OK) {
                std::printf("ERR\t%d\n", rc);
            } else if (sid_sites_count(s) == 0) {
                std::printf("NONE\n");
            } else {
                uint64_t start = 0;
                const char* name = sid_sites_chrom_name(s, 0, &start);
                const uint16_t* c = sid_sites_counts(s);
                std::printf("OK\t%s\t%d\t%u\t%u\t%u\t%u\n", name, sid_sites_positions(s)[0], c[0], c[1], c[2], c[3]);
            }
            sid_sites_free(s);
            at = e + 1;
        }
        return 0;
    }
    if (mode == "csv") {
        sid_sites* s = nullptr;
        uint64_t bad = 0;
        const int rc = sid_parse_text(in.data(), in.size(), argc > 3 ? std::atoi(argv[3]) : 4, &s, &bad);
        if (rc != SID_OK) {
            std::printf("ERR\t%d\t%llu\n", rc, (unsigned long long)bad);
            return 0;
        }
        const size_t n = sid_sites_count(s);
        std::vector<uint8_t> code(n + 1);
        std::vector<double> hom(n + 1), het(n + 1);
        for (size_t i = 0; i < n; ++i) synth_site(i, &code[i], &hom[i], &het[i]);
        size_t need = 0;
        sid_format_csv(s, 0, n, code.data(), hom.data(), het.data(), "p_value", nullptr, 0, &need);
        std::vector<char> out(need + 1);
        size_t len = 0;
        if (sid_format_csv(s, 0, n, code.data(), hom.data(), het.data(), "p_value", out.data(), out.size(), &len))
            return 3;
        std::fwrite(out.data(), 1, len, stdout);
        sid_sites_free(s);
        return 0;
    }
    if (mode == "g6") {
        const size_t n = in.size() / 8;
        for (size_t i = 0; i < n; ++i) {
            double v;
            std::memcpy(&v, in.data() + 8 * i, 8);
            char a[SID_FMT_MAX + 1] = {0}, b[64] = {0};
            const int k = sid_fmt_g6(v, a);
            sid_format_double(v, b, sizeof b);
            std::printf("%s\t%s\n", k < 0 ? "RANGE" : a, b);
        }
        return 0;
    }
    return 2;
}
