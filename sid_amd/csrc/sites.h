// sites.h — parsed-site SoA shared by the parser (parse.cpp) and the CSV
// emitter (emit.cpp).  Opaque to ABI users (sid_sites in include/sid.h).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

struct sid_sites {
    std::vector<uint16_t> counts;        // profile_t per site (pileup.hpp:7)
    std::vector<int32_t> pos;            // PileupLine::position (pileup.hpp:11)
    std::vector<uint64_t> seg_start;     // chromosome runs: first site of run k
    std::vector<std::string> seg_name;   // PileupLine::chromosome_name of run k
};
