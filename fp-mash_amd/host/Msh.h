// Msh.h — Mash .msh (Cap'n Proto MinHash message) writer and reader without capnp.
//
// Replaces Sketch::writeToCapnp (Sketch.cpp:536-642), loadCapnp (:1059-1219) and
// initParametersFromCapnp (:401-470) for capnp/MinHash.capnp:12-59.  The writer
// reproduces capnp's MallocMessageBuilder allocation (first segment 1024 words,
// each new segment max(need, words allocated so far), objects in their pointer's
// segment when they fit, else a far pointer + landing pad in the newest segment)
// so the bytes equal the reference's output.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace fpmhost {

struct MshReference {
    std::string name;
    std::string comment;
    uint64_t length = 0;
    std::vector<uint64_t> hashes;    // hashes64, or hashes32 zero-extended
    std::vector<uint32_t> counts;    // counts32 (may be empty)
    bool countsSorted = false;
};

struct MshHeader {
    uint32_t kmerSize = 0;
    uint32_t windowSize = 0;
    uint32_t minHashesPerWindow = 0;
    bool concatenated = false;
    bool noncanonical = false;
    bool preserveCase = false;
    float error = 0;
    uint32_t hashSeed = 42;
    bool hasAlphabet = false;
    std::string alphabet;
    bool use64 = true;               // hash width of the references
    uint64_t referenceCount = 0;
};

// A reference to serialize without copying its lists (the writer reads them in place).
struct MshRefView {
    const std::string *name;
    const std::string *comment;
    uint64_t length;
    const uint64_t *hashes;
    uint64_t nHashes;
    const uint32_t *counts;
    uint64_t nCounts;
};

// Serialize.  use64 selects hashes64 vs hashes32; counts are written when
// writeCounts and a reference has counts (Sketch.cpp:584-596).
std::string mshSerialize(const MshHeader &h, const std::vector<MshReference> &refs, bool use64,
                         bool writeCounts);

// The same bytes written to the file at `path` (hash lists read in place, parallel writes).
// Returns false if the file cannot be created or written.
bool mshWrite(const std::string &path, const MshHeader &h, const MshRefView *refs, uint64_t n,
              bool use64, bool writeCounts);

// Parse a whole file image.  Hash lists are truncated to maxHashes (loadCapnp's
// truncation to the sketch size, Sketch.cpp:1117-1120, 1135-1138).  use64 picks
// which list is read (the caller's parameters, as loadCapnp does).  Returns false
// with an error message on malformed input.
bool mshParse(const std::string &data, MshHeader &h, std::vector<MshReference> *refs,
              bool use64, uint64_t maxHashes, std::string &err);

}  // namespace fpmhost
