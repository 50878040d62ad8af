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
        // parse + hash on the device (getline / `iss >> id` / `while (iss >> v)` /
        // getHashFingerPrint per line, Sketch.cpp:82-101, 131), at most the lines left
        // of the global cap
        const uint64_t remaining = kLimitReadFingerprint - counterLine;
        fpm_fptext *job = nullptr;
        uint64_t n = 0;
        check(fpm_fp_text_stage(device(), text.data(), text.size(), remaining, parameters.seed,
                                parameters.use64, &job, &n),
              "fingerprint parse");
        std::vector<uint64_t> idOff(n), h64(parameters.use64 ? n : 0);
        std::vector<uint32_t> idLen(n), nVals(n), h32(parameters.use64 ? 0 : n);
        std::vector<uint8_t> newId(n);
        const int rc = fpm_fp_text_fetch(job, idOff.data(), idLen.data(), nVals.data(),
                                         parameters.use64 ? (void *)h64.data() : (void *)h32.data(),
                                         newId.data());
        fpm_fp_text_free(job);
        check(rc, "fingerprint parse");
        counterLine += n;
        // group lines into References: a new one wherever the ID changes (:104-129)
        Reference *cur = nullptr;
        std::vector<Reference> fileRefs;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t nv = nVals[i];
            const bool isNew = i == 0 ? std::string(text.data() + idOff[0], idLen[0]) != lastID
                                      : newId[i] != 0;
            if (isNew) {
                const std::string id(text.data() + idOff[i], idLen[i]);
                fileRefs.emplace_back();
                cur = &fileRefs.back();
                cur->id = id;
                cur->length = nv;
                cur->name = id;
                cur->comment = "FingerPrint : " + id;
            }
            if (!cur) {
                // the reference dereferences a null Reference here (Sketch.cpp:131-134)
                std::cerr << "ERROR: fingerprint line " << i + 1 << " of " << file
                          << " continues ID \"" << lastID << "\" from a previous file." << std::endl;
                exit(1);
            }
            cur->hashes.push_back(parameters.use64 ? h64[i] : (uint64_t)h32[i]);
            cur->length += nv;
        }
        if (n) lastID.assign(text.data() + idOff[n - 1], idLen[n - 1]);
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
