// Sketch.cpp — host side of the sketch engine (see Sketch.h).
#include "Sketch.h"

#include "Device.h"
#include "Msh.h"
#include "SeqReader.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>

namespace fpmhost {

const char *suffixSketch = ".msh";
const char *alphabetNucleotide = "ACGT";
const char *alphabetProtein = "ACDEFGHIKLMNPQRSTVWY";

static const uint64_t kLimitReadFingerprint = 1000000;   // Sketch.cpp:37

bool hasSuffix(const std::string &whole, const std::string &suffix)
{
    return whole.size() >= suffix.size() &&
           whole.compare(whole.size() - suffix.size(), suffix.size(), suffix) == 0;
}

void splitFile(const std::string &file, std::vector<std::string> &lines)
{
    std::ifstream in(file);
    if (in.fail()) {
        std::cerr << "ERROR: Could not open " << file << ".\n";
        exit(1);
    }
    std::string line;
    while (std::getline(in, line))
        if (!line.empty()) lines.push_back(line);
}

void setAlphabetFromString(Parameters &p, const char *characters)
{
    p.alphabetSize = 0;
    memset(p.alphabet, 0, sizeof(p.alphabet));
    for (const char *c = characters; *c; c++) {
        char u = *c;
        if (!p.preserveCase && u > 96 && u < 123) u -= 32;
        p.alphabet[(unsigned char)u] = true;
    }
    for (int i = 0; i < 256; i++)
        if (p.alphabet[i]) p.alphabetSize++;
    p.use64 = pow(p.alphabetSize, p.kmerSize) > pow(2, 32);
}

void Sketch::getAlphabetAsString(std::string &alphabet) const
{
    for (int i = 0; i < 256; i++)
        if (parameters.alphabet[i]) alphabet.append(1, (char)i);
}

double Sketch::getRandomKmerChance(uint64_t i) const
{
    return 1. / (kmerSpace / references[i].length + 1.);
}

int Sketch::getMinKmerSize(uint64_t i) const
{
    return (int)ceil(log(references[i].length * (1 - parameters.warning) / parameters.warning) /
                     log(parameters.alphabetSize));
}

void Sketch::createIndex() { kmerSpace = pow(parameters.alphabetSize, parameters.kmerSize); }

static bool readFile(const std::string &path, std::string &out)
{
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    std::ostringstream ss;
    ss << in.rdbuf();
    out = ss.str();
    return true;
}

uint64_t Sketch::initParametersFromMsh(const std::string &file)
{
    std::string data;
    if (!readFile(file, data)) {
        std::cerr << "ERROR: could not open \"" << file << "\" for reading." << std::endl;
        exit(1);
    }
    MshHeader h;
    std::string err;
    if (!mshParse(data, h, nullptr, true, 0, err)) {
        std::cerr << "ERROR: " << file << ": " << err << std::endl;
        exit(1);
    }
    parameters.kmerSize = (int)h.kmerSize;
    parameters.error = h.error;
    parameters.minHashesPerWindow = h.minHashesPerWindow;
    parameters.windowSize = h.windowSize;
    parameters.concatenated = h.concatenated;
    parameters.noncanonical = h.noncanonical;
    parameters.preserveCase = h.preserveCase;
    parameters.seed = h.hashSeed;
    setAlphabetFromString(parameters, h.hasAlphabet ? h.alphabet.c_str() : alphabetNucleotide);
    // counts flag: references[0].hasCounts32 (Sketch.cpp:430)
    std::vector<MshReference> refs;
    if (h.referenceCount && mshParse(data, h, &refs, parameters.use64, 1, err))
        parameters.counts = !refs.empty() && !refs[0].counts.empty();
    return h.referenceCount;
}

// loadCapnp (Sketch.cpp:1059-1219)
static void loadMsh(const std::string &file, const Parameters &p, std::vector<Reference> &out)
{
    std::string data, err;
    if (!readFile(file, data)) return;
    MshHeader h;
    std::vector<MshReference> refs;
    if (!mshParse(data, h, &refs, p.use64, p.minHashesPerWindow, err)) {
        std::cerr << "ERROR: " << file << ": " << err << std::endl;
        exit(1);
    }
    for (auto &m : refs) {
        Reference r;
        r.name = std::move(m.name);
        r.comment = std::move(m.comment);
        r.length = m.length;
        r.hashes = std::move(m.hashes);
        r.counts = std::move(m.counts);
        out.push_back(std::move(r));
    }
}

namespace {

// records and groups collected from all sequence files, sketched in one GPU batch
struct SeqBatch {
    std::string seq;
    std::vector<uint64_t> rec_off{0};
    std::vector<uint32_t> group;
    uint32_t n_groups = 0;
    void add(const std::string &s, uint32_t g)
    {
        seq += s;
        rec_off.push_back(seq.size());
        group.push_back(g);
    }
};

}  // namespace

int Sketch::initFromFiles(const std::vector<std::string> &files, const Parameters &p, int verbosity,
                          bool enforceParameters, bool contain)
{
    parameters = p;
    // output slots in input order: a slot is either loaded references or a GPU group
    struct Slot { bool fromGroup; uint32_t group; Reference ref; };
    std::vector<Slot> slots;
    SeqBatch batch;

    for (size_t i = 0; i < files.size(); i++) {
        const std::string &file = files[i];
        if (hasSuffix(file, suffixSketch)) {
            Sketch test;
            test.initParametersFromMsh(file);
            if (i == 0 && !enforceParameters) initParametersFromMsh(file);
            std::string alphabet, alphabetTest;
            getAlphabetAsString(alphabet);
            test.getAlphabetAsString(alphabetTest);
            if (alphabet != alphabetTest) {
                std::cerr << "\nWARNING: The sketch file " << file << " has different alphabet ("
                          << alphabetTest << ") than the current alphabet (" << alphabet
                          << "). This file will be skipped." << std::endl << std::endl;
                continue;
            }
            if (test.getHashSeed() != parameters.seed) {
                std::cerr << "\nWARNING: The sketch " << file << " has a seed size ("
                          << test.getHashSeed() << ") that does not match the current seed ("
                          << parameters.seed << "). This file will be skipped." << std::endl
                          << std::endl;
                continue;
            }
            if (test.getKmerSize() != parameters.kmerSize) {
                std::cerr << "\nWARNING: The sketch " << file << " has a kmer size ("
                          << test.getKmerSize() << ") that does not match the current kmer size ("
                          << parameters.kmerSize << "). This file will be skipped." << std::endl
                          << std::endl;
                continue;
            }
            if (!contain && test.getMinHashesPerWindow() < parameters.minHashesPerWindow) {
                std::cerr << "\nWARNING: The sketch file " << file << " has a target sketch size ("
                          << test.getMinHashesPerWindow()
                          << ") that is smaller than the current sketch size ("
                          << parameters.minHashesPerWindow << "). This file will be skipped."
                          << std::endl << std::endl;
                continue;
            }
            if (test.getNoncanonical() != parameters.noncanonical) {
                std::cerr << "\nWARNING: The sketch file " << file << " is "
                          << (test.getNoncanonical() ? "noncanonical" : "canonical")
                          << ", which is incompatible with the current setting. This file will be "
                             "skipped." << std::endl << std::endl;
                continue;
            }
            if (test.getMinHashesPerWindow() > parameters.minHashesPerWindow) {
                std::cerr << "\nWARNING: The sketch file " << file << " has a target sketch size ("
                          << test.getMinHashesPerWindow()
                          << ") that is larger than the current sketch size ("
                          << parameters.minHashesPerWindow << "). Its sketches will be reduced."
                          << std::endl << std::endl;
            }
            std::vector<Reference> loaded;
            loadMsh(file, parameters, loaded);
            for (auto &r : loaded) slots.push_back(Slot{false, 0, std::move(r)});
            continue;
        }

        if (verbosity > 0)
            std::cerr << (file == "-" ? std::string("Sketching from stdin...")
                                      : "Sketching " + file + "...") << std::endl;
        if (file != "-") {
            FILE *f = fopen(file.c_str(), "r");
            if (!f) {
                std::cerr << "ERROR: could not open " << file << " for reading." << std::endl;
                exit(1);
            }
            fclose(f);
        }
        SeqReader rd(file);
        if (!rd.ok()) {
            std::cerr << "ERROR: could not open " << file << std::endl;
            exit(1);
        }
        int l;
        if (parameters.concatenated) {
            // sketchFile (Sketch.cpp:1299-1488): one sketch for the whole file
            Reference ref;
            const uint32_t g = batch.n_groups++;
            int count = 0;
            bool skipped = false;
            if (file != "-") ref.name = file;
            while ((l = rd.read()) >= 0) {
                if (l < parameters.kmerSize) { skipped = true; continue; }
                if (count == 0) {
                    if (file == "-") { ref.name = rd.name; ref.comment = rd.comment; }
                    else ref.comment = rd.name + " " + rd.comment;
                }
                count++;
                ref.length += (uint64_t)l;
                batch.add(rd.seq, g);
            }
            if (count > 1) ref.comment = "[" + std::to_string(count) + " seqs] " + ref.comment + " [...]";
            if (l != -1) {
                std::cerr << "\nERROR: reading input files." << std::endl;
                exit(1);
            }
            if (ref.length == 0) {
                if (skipped)
                    std::cerr << "\nWARNING: All fasta records in input files were shorter than the "
                                 "k-mer size (" << parameters.kmerSize << ")." << std::endl;
                else
                    std::cerr << "\nERROR: Did not find fasta records in \"input files\"." << std::endl;
                exit(1);
            }
            slots.push_back(Slot{true, g, std::move(ref)});
        } else {
            // sketchFileBySequence (Sketch.cpp:478-522): one sketch per record >= k
            while ((l = rd.read()) >= 0) {
                if (l < parameters.kmerSize) continue;
                Reference ref;
                ref.name = rd.name;
                ref.comment = rd.comment;
                ref.length = (uint64_t)l;
                const uint32_t g = batch.n_groups++;
                batch.add(rd.seq, g);
                slots.push_back(Slot{true, g, std::move(ref)});
            }
            if (l != -1) {
                std::cerr << "\nERROR: reading " << file << "." << std::endl;
                exit(1);
            }
        }
    }

    if (batch.n_groups) {
        fpm_sketch_params fp{};
        fp.kmer_size = (uint32_t)parameters.kmerSize;
        fp.sketch_size = (uint32_t)parameters.minHashesPerWindow;
        fp.seed = parameters.seed;
        fp.use64 = parameters.use64;
        fp.noncanonical = parameters.noncanonical;
        fp.preserve_case = parameters.preserveCase;
        for (int c = 0; c < 256; c++) fp.alphabet[c] = parameters.alphabet[c] ? 1 : 0;
        const uint64_t s = fp.sketch_size;
        std::vector<uint64_t> out((size_t)batch.n_groups * s);
        std::vector<uint32_t> cnt(batch.n_groups);
        check(fpm_sketch_batch(device(), &fp, batch.seq.data(), batch.rec_off.data(),
                               (uint32_t)batch.group.size(), batch.group.data(), batch.n_groups,
                               out.data(), cnt.data()),
              "sketch");
        for (auto &sl : slots)
            if (sl.fromGroup)
                sl.ref.hashes.assign(out.begin() + (size_t)sl.group * s,
                                     out.begin() + (size_t)sl.group * s + cnt[sl.group]);
    }
    references.clear();
    references.reserve(slots.size());
    for (auto &sl : slots) references.push_back(std::move(sl.ref));
    createIndex();
    return 0;
}

// istream >> unsigned long long, for the cases CFL k-finger files hold
static bool readU64(const char *&p, const char *end, uint64_t &out)
{
    while (p < end && isspace((unsigned char)*p)) p++;
    bool neg = false;
    if (p < end && (*p == '+' || *p == '-')) { neg = *p == '-'; p++; }
    if (p >= end || *p < '0' || *p > '9') return false;
    uint64_t v = 0;
    bool ovf = false;
    while (p < end && *p >= '0' && *p <= '9') {
        uint64_t d = (uint64_t)(*p - '0');
        if (v > (UINT64_MAX - d) / 10) ovf = true;
        v = v * 10 + d;
        p++;
    }
    if (ovf) return false;
    out = neg ? (uint64_t)(0 - v) : v;
    return true;
}

void Sketch::initFromFingerprints(const std::vector<std::string> &files, const Parameters &p)
{
    parameters = p;
    uint64_t counterLine = 0;
    std::string lastID;
    std::cout << "Initializing from fingerprints..." << std::endl;
    for (const std::string &file : files) {
        std::cout << "Processing file: " << file << std::endl;
        std::string text;
        if (!readFile(file, text)) {
            std::cerr << "ERROR: Could not open fingerprint file " << file << " for reading."
                      << std::endl;
            exit(1);
        }
        // parse lines (getline on '\n'; ID token; u64 values) up to the global cap
        std::vector<uint64_t> vals, line_off{0};
        std::vector<std::pair<uint64_t, uint32_t>> ids;
        const char *t = text.data(), *end = text.data() + text.size();
        while (t < end && counterLine < kLimitReadFingerprint) {
            const char *eol = (const char *)memchr(t, '\n', (size_t)(end - t));
            const char *le = eol ? eol : end;
            counterLine++;
            const char *q = t;
            while (q < le && isspace((unsigned char)*q)) q++;
            const char *ib = q;
            while (q < le && !isspace((unsigned char)*q)) q++;
            ids.push_back({(uint64_t)(ib - text.data()), (uint32_t)(q - ib)});
            if (q > ib) {
                uint64_t v;
                while (readU64(q, le, v)) vals.push_back(v);
            }
            line_off.push_back(vals.size());
            t = eol ? eol + 1 : end;
        }
        const uint64_t n = ids.size();
        std::vector<uint32_t> h(n);
        if (n) {
            if (vals.empty()) vals.push_back(0);
            check(fpm_fp_hash_lines(device(), vals.data(), line_off.data(), n, parameters.seed,
                                    parameters.use64, h.data()),
                  "fingerprint hash");
        }
        Reference *cur = nullptr;
        std::vector<Reference> fileRefs;
        for (uint64_t i = 0; i < n; i++) {
            std::string id(text.data() + ids[i].first, ids[i].second);
            const uint64_t nv = line_off[i + 1] - line_off[i];
            if (id != lastID) {
                fileRefs.emplace_back();
                cur = &fileRefs.back();
                cur->id = id;
                cur->length = nv;
                cur->name = id;
                cur->comment = "FingerPrint : " + id;
                lastID = id;
            }
            if (!cur) {
                // the reference dereferences a null Reference here (Sketch.cpp:131-134)
                std::cerr << "ERROR: fingerprint line " << i + 1 << " of " << file
                          << " continues ID \"" << id << "\" from a previous file." << std::endl;
                exit(1);
            }
            cur->hashes.push_back(h[i]);
            cur->length += nv;
        }
        for (auto &r : fileRefs) references.push_back(std::move(r));
    }
    createIndex();
    std::cout << "Initialization complete." << std::endl;
}

int Sketch::writeToMsh(const std::string &file) const
{
    MshHeader h;
    h.kmerSize = (uint32_t)parameters.kmerSize;
    h.hashSeed = parameters.seed;
    h.error = (float)parameters.error;
    h.minHashesPerWindow = (uint32_t)parameters.minHashesPerWindow;
    h.windowSize = (uint32_t)parameters.windowSize;
    h.concatenated = parameters.concatenated;
    h.noncanonical = parameters.noncanonical;
    h.preserveCase = parameters.preserveCase;
    getAlphabetAsString(h.alphabet);
    std::vector<MshReference> refs(references.size());
    for (size_t i = 0; i < references.size(); i++) {
        refs[i].name = references[i].name;
        refs[i].comment = references[i].comment;
        refs[i].length = references[i].length;
        refs[i].hashes = references[i].hashes;
        refs[i].counts = references[i].counts;
    }
    const std::string bytes = mshSerialize(h, refs, parameters.use64, parameters.counts);
    FILE *f = fopen(file.c_str(), "wb");
    if (!f) {
        std::cerr << "ERROR: could not open " << file << " for writing.\n";
        exit(1);
    }
    fwrite(bytes.data(), 1, bytes.size(), f);
    fclose(f);
    return 0;
}

}  // namespace fpmhost
