// Sketch.h — host mirror of the reference's Sketch engine (Sketch.h:28-262):
// parameters, references, initFromFiles / initFromFingerprints / writeToCapnp /
// loadCapnp.  The k-mer hashing and bottom-s selection run on the MI355X through
// the C ABI (include/fpmash.h); this layer does file I/O, naming, ordering and
// the .msh format.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace fpmhost {

extern const char *suffixSketch;          // ".msh"
extern const char *alphabetNucleotide;    // "ACGT"
extern const char *alphabetProtein;       // "ACDEFGHIKLMNPQRSTVWY"

struct Parameters {
    int parallelism = 1;
    int kmerSize = 0;
    bool alphabet[256] = {};
    uint32_t alphabetSize = 0;
    bool preserveCase = false;
    bool use64 = false;
    uint32_t seed = 0;
    double error = 0;
    double warning = 0;
    uint64_t minHashesPerWindow = 0;
    uint64_t windowSize = 0;
    bool concatenated = false;
    bool noncanonical = false;
    bool reads = false;
    bool counts = false;
    bool fingerprint = false;
};

struct Reference {
    std::string id;
    std::string name;
    std::string comment;
    uint64_t length = 0;
    std::vector<uint64_t> hashes;   // hashesSorted (u32 values zero-extended when !use64)
    std::vector<uint32_t> counts;   // -M multiplicities (counts32)
    bool countsSorted = false;
    // rows fetched from the device and read in place (Sketch::keepDeviceRows): the sketch
    // command writes them into the .msh without first copying 8 B per hash into `hashes`
    const uint64_t *hashView = nullptr;
    const uint32_t *countView = nullptr;
    uint32_t viewCount = 0;
    size_t hashCount() const { return hashView ? viewCount : hashes.size(); }
    const uint64_t *hashData() const { return hashView ? hashView : hashes.data(); }
    size_t countCount() const { return countView ? viewCount : counts.size(); }
    const uint32_t *countData() const { return countView ? countView : counts.data(); }
};

class Sketch {
public:
    // Sketch::initFromFiles (Sketch.cpp:249-397): .msh inputs are loaded, sequence
    // files are sketched on the GPU (one sketch per file, or per record with -i).
    int initFromFiles(const std::vector<std::string> &files, const Parameters &p,
                      int verbosity = 0, bool enforceParameters = false, bool contain = false);
    // Sketch::initFromFingerprints (Sketch.cpp:56-151)
    void initFromFingerprints(const std::vector<std::string> &files, const Parameters &p);
    // Sketch::initParametersFromCapnp (Sketch.cpp:401-470); returns reference count
    uint64_t initParametersFromMsh(const std::string &file);
    // Sketch::writeToCapnp (Sketch.cpp:536-642)
    int writeToMsh(const std::string &file) const;

    void getAlphabetAsString(std::string &alphabet) const;
    uint32_t getAlphabetSize() const { return parameters.alphabetSize; }
    uint32_t getHashSeed() const { return parameters.seed; }
    int getKmerSize() const { return parameters.kmerSize; }
    double getKmerSpace() const { return kmerSpace; }
    float getMinHashesPerWindow() const { return (float)parameters.minHashesPerWindow; }
    bool getNoncanonical() const { return parameters.noncanonical; }
    bool getPreserveCase() const { return parameters.preserveCase; }
    bool getUse64() const { return parameters.use64; }
    bool getConcatenated() const { return parameters.concatenated; }
    float getError() const { return (float)parameters.error; }
    uint64_t getWindowSize() const { return parameters.windowSize; }
    const Reference &getReference(uint64_t i) const { return references.at(i); }
    uint64_t getReferenceCount() const { return references.size(); }
    double getRandomKmerChance(uint64_t i) const;
    int getMinKmerSize(uint64_t i) const;
    bool hasHashCounts() const { return !references.empty() && references[0].countCount() != 0; }
    // sequence inputs keep their sketch rows in the fetched host arrays (Reference::hashView)
    // instead of per-reference vectors: for a caller that only writes the .msh
    void keepDeviceRows() { rowViews = true; }
    void setReferenceName(int i, const std::string &n) { references[i].name = n; }
    void setReferenceComment(int i, const std::string &c) { references[i].comment = c; }

    Parameters parameters;
    std::vector<Reference> references;
    double kmerSpace = 0;

private:
    void createIndex();
    bool rowViews = false;
    std::vector<std::shared_ptr<void>> rowStores;   // the host arrays the views point into
};

void setAlphabetFromString(Parameters &p, const char *characters);
bool hasSuffix(const std::string &whole, const std::string &suffix);
void splitFile(const std::string &file, std::vector<std::string> &lines);

}  // namespace fpmhost
