// ref_pileup_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// Drives the REFERENCE's own pileup.cpp, compiled from /root/reference by
// oracle/Makefile into oracle/_ref/ref_pileup, so the oracle parser and the
// product parser can be pinned against the reference's real code.  This file
// contains no reference source: it only calls the reference's functions
// (pileup.hpp:20,28,30,42,44).
//
//   ref_pileup lines     < text   -> per non-empty line (call.cpp:11-20 loop):
//                                    "OK\t<chrom>\t<pos>\t<A>\t<C>\t<G>\t<T>" or
//                                    "ERR\t<exception type>\t<what()>"
//   ref_pileup profiles  < "A C G T" lines -> countUniqueProfiles + distribution
//   ref_pileup quals     < lines   -> parseQualities values
#include <cstdint>
#include <cstdio>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "pileup.hpp"

int main(int argc, char** argv) {
    std::string mode = argc > 1 ? argv[1] : "lines";
    std::ios::sync_with_stdio(false);
    if (mode == "lines") {
        for (std::string line; std::getline(std::cin, line);) {
            if (line.size() == 0) continue;
            try {
                PileupLine p = parsePileupLine(&line[0u], false, false);
                std::cout << "OK\t" << p.chromosome_name << '\t' << p.position << '\t'
                          << p.base_counts[0] << '\t' << p.base_counts[1] << '\t'
                          << p.base_counts[2] << '\t' << p.base_counts[3] << '\n';
            } catch (const std::invalid_argument& e) {
                std::cout << "ERR\tstd::invalid_argument\t" << e.what() << '\n';
            } catch (const std::logic_error& e) {
                std::cout << "ERR\tstd::logic_error\t" << e.what() << '\n';
            }
        }
    } else if (mode == "profiles") {
        std::vector<PileupLine> lines;
        unsigned a, c, g, t;
        while (std::cin >> a >> c >> g >> t) {
            PileupLine p;
            p.base_counts = {(uint16_t)a, (uint16_t)c, (uint16_t)g, (uint16_t)t};
            lines.push_back(p);
        }
        auto u = countUniqueProfiles(lines);
        for (const auto& x : u)
            std::cout << x.profile[0] << ' ' << x.profile[1] << ' ' << x.profile[2] << ' '
                      << x.profile[3] << ' ' << x.count << ' ' << x.coverage << '\n';
        auto d = computeNucleotideDistribution(u);
        std::printf("dist %.17g %.17g %.17g %.17g\n", d[0], d[1], d[2], d[3]);
    } else if (mode == "quals") {
        for (std::string line; std::getline(std::cin, line);) {
            auto q = parseQualities(line.c_str(), (int)line.size());
            for (size_t i = 0; i < q.size(); ++i) std::cout << (i ? " " : "") << (int)q[i];
            std::cout << '\n';
        }
    } else {
        return 2;
    }
    return 0;
}
