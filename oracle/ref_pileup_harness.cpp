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
//   ref_pileup local FILE [PRIOR ERR SIG]
//                                 -> sid -m local's CSV on stdout, as
//                                    sid.cpp:84-105 prints it (timing only)
//
// `local` is the CPU baseline's "reference sources" leg (bench.py): the
// reference's own per-site work for -m local -- std::ifstream + getline and
// parsePileupLine per line into a std::vector<PileupLine> (the loop of
// call.cpp:11-20), countUniqueProfiles, a std::map from profile to class
// (call.cpp:216-221, 274-285), and the records printed through call.hpp's
// operator<< with iostreams (sid.cpp:102-105).  The one step taken from
// elsewhere is each unique profile's arithmetic (call.cpp:238-273), which
// needs GSL (absent here): oracle_local_profile from the oracle's C
// restatement, once per unique profile (~10^4 of them against 10^6-10^7
// sites, a negligible share of the time).  ORACLE_RANGE=OFF:LEN (as the
// oracle CLI) reads the line-aligned bytes [OFF, OFF+LEN) of FILE.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "call.hpp"
#include "pileup.hpp"
#include "sid_oracle.h"

static int local_mode(int argc, char** argv)
{
    if (argc < 3) return 2;
    const double prior = argc > 3 ? std::atof(argv[3]) : -1.0;
    const double err = argc > 4 ? std::atof(argv[4]) : 0.1;
    const double sig = argc > 5 ? std::atof(argv[5]) : 0.05;
    std::ifstream in(argv[2]);
    if (!in) return 1;
    unsigned long long off = 0, left = ~0ull;
    if (const char* r = std::getenv("ORACLE_RANGE"))
        if (std::sscanf(r, "%llu:%llu", &off, &left) == 2) in.seekg((std::streamoff)off);
    std::vector<PileupLine> sites;
    for (std::string line; left && std::getline(in, line);) {
        left -= std::min<unsigned long long>(left, line.size() + 1);
        if (!line.empty()) sites.push_back(parsePileupLine(&line[0u], false, false));
    }
    const std::vector<UniqueProfile> uniq = countUniqueProfiles(sites);
    std::map<profile_t, size_t> at;
    std::vector<Classification> cls;
    cls.reserve(uniq.size());
    for (const UniqueProfile& u : uniq) {
        at.emplace(u.profile, cls.size());
        uint8_t code = 0;
        double hom = 0, het = 0;
        oracle_local_profile(u.profile.data(), prior, err, sig, &code, &hom, &het);
        Classification c;
        c.label = (code & 0x80) ? "het" : "hom";
        c.genotype = {"ACGT"[code & 3], "ACGT"[(code >> 2) & 3]};
        c.confidence_homozygous = hom;
        c.confidence_heterozygous = het;
        c.confidence_type = "p_value";
        cls.push_back(c);
    }
    std::vector<OutputRecord> out;
    out.reserve(sites.size());
    for (const PileupLine& s : sites) {
        const auto it = at.find(s.base_counts);
        if (it != at.end()) out.push_back({s.chromosome_name, s.position, cls[it->second]});
    }
    std::cout << "chrom,pos,label,gt,hom_conf,het_conf,conf_type" << std::endl;
    for (const OutputRecord& r : out) std::cout << r << '\n';
    return 0;
}

int main(int argc, char** argv) {
    std::string mode = argc > 1 ? argv[1] : "lines";
    if (mode == "local") return local_mode(argc, argv);   // (iostreams synced with stdio, as sid.cpp runs)
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
