// Sketch.cpp — host side of the sketch engine (see Sketch.h).
#include "Sketch.h"

#include "Device.h"
#include "Msh.h"
#include "SeqReader.h"
#include "Timing.h"
#include "HostRows.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <algorithm>
#include <sys/stat.h>

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
        fatalExit();
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
    // one sized read (an ostringstream of rdbuf copied the file twice)
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    out.clear();
    if (fseeko(f, 0, SEEK_END) == 0) {
        const off_t n = ftello(f);
        if (n > 0 && fseeko(f, 0, SEEK_SET) == 0) {
            out.resize((size_t)n);
            out.resize(fread(&out[0], 1, (size_t)n, f));
        }
    }
    char buf[1 << 16];   // unsized streams (pipes) or a file that grew
    for (size_t r; (r = fread(buf, 1, sizeof(buf), f)) > 0;) out.append(buf, r);
    fclose(f);
    return true;
}

// The .msh inputs are opened several times (parameters of the first file, the per-file
// compatibility test, the load: Sketch.cpp:257-336): keep the last image read, keyed by path,
// size and modification time, until its load (loadMsh) has parsed it.  One cache per thread
// (thread_local): a Sketch loaded on another thread reads and caches on its own.
static thread_local std::string g_mshPath, g_mshData;
static thread_local struct stat g_mshSt {};

static void releaseMshCache()
{
    g_mshPath.clear();
    std::string().swap(g_mshData);
}

static const std::string *readMshCached(const std::string &path)
{
    std::string &cPath = g_mshPath, &cData = g_mshData;
    struct stat &cSt = g_mshSt;
    struct stat st {};
    if (stat(path.c_str(), &st) != 0) return nullptr;
    if (path == cPath && st.st_size == cSt.st_size && st.st_mtim.tv_sec == cSt.st_mtim.tv_sec &&
        st.st_mtim.tv_nsec == cSt.st_mtim.tv_nsec)
        return &cData;
    cPath.clear();
    if (!readFile(path, cData)) return nullptr;
    cPath = path;
    cSt = st;
    return &cData;
}

uint64_t Sketch::initParametersFromMsh(const std::string &file)
{
    const std::string *img = readMshCached(file);
    if (!img) {
        std::cerr << "ERROR: could not open \"" << file << "\" for reading." << std::endl;
        fatalExit();
    }
    const std::string &data = *img;
    MshHeader h;
    std::string err;
    if (!mshParse(data, h, nullptr, true, 0, err)) {
        std::cerr << "ERROR: " << file << ": " << err << std::endl;
        fatalExit();
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
    std::string err;
    const std::string *img = readMshCached(file);
    if (!img) return;
    const std::string &data = *img;
    MshHeader h;
    std::vector<MshReference> refs;
    if (!mshParse(data, h, &refs, p.use64, p.minHashesPerWindow, err)) {
        std::cerr << "ERROR: " << file << ": " << err << std::endl;
        fatalExit();
    }
    for (auto &m : refs) {
        Reference r;
        r.name = std::move(m.name);
        r.comment = std::move(m.comment);
        r.length = m.length;
        r.hashes = std::move(m.hashes);
        r.counts = std::move(m.counts);
        r.countsSorted = m.countsSorted;
        out.push_back(std::move(r));
    }
    releaseMshCache();   // parsed: the image is not needed past its load
}

namespace {

// one input record as the sketch groups see it
struct SeqRec {
    std::string name, comment;
    uint64_t length = 0;
    uint32_t id = 0;       // record index in the parse (device) or the host batch
};

// host kseq walk of one image (the fallback for FASTQ quality lines): records appended to
// `out`, their bytes to `seq` (record r = seq[off[r] .. off[r + 1])).  Returns kseq_read's
// last status (-1 at a clean end of file, -2 on a truncated quality string).
int hostRecords(const std::string &image, std::vector<SeqRec> &out, std::string &seq,
                std::vector<uint64_t> &off)
{
    SeqReader rd(image.data(), image.size());
    int l;
    while ((l = rd.read()) >= 0) {
        SeqRec r;
        r.name = rd.name;
        r.comment = rd.comment;
        r.length = (uint64_t)l;
        r.id = (uint32_t)(off.size() - 1);
        seq += rd.seq;
        off.push_back(seq.size());
        out.push_back(std::move(r));
    }
    return l;
}

}  // namespace

// Parse and sketch the sequence files [f0, f1) on one device (the reference's per-file work,
// Sketch.cpp:249-397 / 478-522 / 1299-1488): fills fileRefs[f] for those files.
// With `stores`, the references point into the fetched host arrays (Reference::hashView),
// which are appended to *stores (under *storeMu) to keep them alive.
static void sketchFiles(fpm_ctx *ctx, const Parameters &parameters,
                        const std::vector<std::string> &seqFiles, std::vector<std::string> &images,
                        size_t f0, size_t f1, std::vector<std::vector<Reference>> &fileRefs,
                        bool timing, std::vector<std::shared_ptr<void>> *stores = nullptr,
                        std::mutex *storeMu = nullptr)
{
    const size_t nF = f1 - f0;
    auto mark = [&](const char *what) { if (timing) phaseMark(what); };
    // records of each file (kseq rules) parsed on the device
    std::vector<std::vector<SeqRec>> recs(nF);
    fpm_seqtext *parsed = nullptr;
    uint64_t nRec = 0;
    int quality = 0;
    {
        std::vector<const char *> ptr(nF);
        std::vector<uint64_t> len(nF);
        for (size_t f = 0; f < nF; f++) {
            ptr[f] = images[f0 + f].data();
            len[f] = images[f0 + f].size();
        }
        check(fpm_seq_parse(ctx, ptr.data(), len.data(), (uint32_t)nF, &parsed,
                            &nRec, &quality),
              "sequence parse");
    }
    mark("device parse (upload + scan + emit)");
    std::string hostSeq;               // host fallback: the records' bytes
    std::vector<uint64_t> hostOff{0};
    if (!quality) {
        std::vector<uint32_t> seg(nRec);
        std::vector<uint64_t> ho(nRec), hl(nRec), sl(nRec);
        check(fpm_seq_records(parsed, seg.data(), ho.data(), hl.data(), sl.data()),
              "sequence parse");
        for (uint64_t r = 0; r < nRec; r++) {
            const std::string &img = images[f0 + seg[r]];
            // a '>' / '@' as the last byte of a file starts no record (kseq_read returns
            // -1 when the name read hits the end of the stream)
            if (ho[r] + 1 >= img.size()) continue;
            SeqRec x;
            splitHeader(img.data() + ho[r] + 1, hl[r] - 1, x.name, x.comment);
            x.length = sl[r];
            x.id = (uint32_t)r;
            recs[seg[r]].push_back(std::move(x));
        }
    } else {
        // FASTQ quality lines: kseq's record walk on the host
        fpm_seq_free(parsed);
        parsed = nullptr;
        for (size_t f = 0; f < nF; f++) {
            if (hostRecords(images[f0 + f], recs[f], hostSeq, hostOff) != -1) {
                std::cerr << "\nERROR: reading " << (parameters.concatenated ? std::string("input files")
                                                                               : seqFiles[f0 + f])
                          << "." << std::endl;
                fatalExit();
            }
        }
    }
    mark("record headers");

    // sketch groups: one per file (sketchFile, Sketch.cpp:1299-1488) or one per record
    // >= k with -i (sketchFileBySequence, :478-522); records < k are skipped (:488-492)
    const uint64_t nIds = parsed ? nRec : hostOff.size() - 1;
    std::vector<uint32_t> groupOf(nIds, FPM_NO_GROUP);
    uint32_t nGroups = 0;
    std::vector<std::vector<uint32_t>> fileGroups(nF);
    for (size_t f = 0; f < nF; f++) {
        const std::string &file = seqFiles[f0 + f];
        if (parameters.concatenated) {
            Reference ref;
            const uint32_t g = nGroups++;
            int count = 0;
            bool skipped = false;
            if (file != "-") ref.name = file;
            for (const SeqRec &x : recs[f]) {
                if (x.length < (uint64_t)parameters.kmerSize) { skipped = true; continue; }
                if (count == 0) {
                    if (file == "-") { ref.name = x.name; ref.comment = x.comment; }
                    else ref.comment = x.name + " " + x.comment;
                }
                count++;
                ref.length += x.length;
                groupOf[x.id] = g;
            }
            if (count > 1) ref.comment = "[" + std::to_string(count) + " seqs] " + ref.comment + " [...]";
            if (ref.length == 0) {
                if (skipped)
                    std::cerr << "\nWARNING: All fasta records in input files were shorter than the "
                                 "k-mer size (" << parameters.kmerSize << ")." << std::endl;
                else
                    std::cerr << "\nERROR: Did not find fasta records in \"input files\"." << std::endl;
                fatalExit();
            }
            fileRefs[f0 + f].push_back(std::move(ref));
            fileGroups[f].push_back(g);
        } else {
            for (SeqRec &x : recs[f]) {
                if (x.length < (uint64_t)parameters.kmerSize) continue;
                Reference ref;
                ref.name = std::move(x.name);
                ref.comment = std::move(x.comment);
                ref.length = x.length;
                const uint32_t g = nGroups++;
                groupOf[x.id] = g;
                fileRefs[f0 + f].push_back(std::move(ref));
                fileGroups[f].push_back(g);
            }
        }
    }
    for (size_t f = f0; f < f1; f++) {
        images[f].clear();
        images[f].shrink_to_fit();
    }

    if (nGroups) {
        fpm_sketch_params fp{};
        fp.kmer_size = (uint32_t)parameters.kmerSize;
        fp.sketch_size = (uint32_t)parameters.minHashesPerWindow;
        fp.seed = parameters.seed;
        fp.use64 = parameters.use64;
        fp.noncanonical = parameters.noncanonical;
        fp.preserve_case = parameters.preserveCase;
        for (int c = 0; c < 256; c++) fp.alphabet[c] = parameters.alphabet[c] ? 1 : 0;
        const uint64_t s = fp.sketch_size;
        // the output rows' pages (80 MB for C2: ~4 ms of page allocation and zeroing) are
        // populated on a thread beside the staging and the sketch kernels
        auto outp = std::make_shared<HostRows<uint64_t>>((size_t)nGroups * s, false);
        HostRows<uint64_t> &out = *outp;
        std::thread populate([&out] { out.populate(); });
        std::vector<uint32_t> cnt(nGroups);
        fpm_sketch_job *job = nullptr;
        if (parsed) {
            check(fpm_sketch_stage_seq(ctx, &fp, parsed, groupOf.data(), nGroups, &job), "sketch");
        } else {
            // host-parsed records: only those of a group go to the device
            std::vector<uint64_t> off{0};
            std::vector<uint32_t> grp;
            std::string packed;
            for (uint64_t r = 0; r < nIds; r++) {
                if (groupOf[r] == FPM_NO_GROUP) continue;
                packed.append(hostSeq, hostOff[r], hostOff[r + 1] - hostOff[r]);
                off.push_back(packed.size());
                grp.push_back(groupOf[r]);
            }
            check(fpm_sketch_stage(ctx, &fp, packed.data(), off.data(), (uint32_t)grp.size(),
                                   grp.data(), nGroups, &job),
                  "sketch");
        }
        int rc = fpm_sketch_run(job, nullptr);
        populate.join();
        if (rc == FPM_OK) rc = fpm_sketch_fetch(job, out.data(), cnt.data());
        // -M: the heap's multiplicities (Sketch.cpp:584-596)
        auto multp = std::make_shared<std::vector<uint32_t>>();
        std::vector<uint32_t> &mult = *multp;
        if (rc == FPM_OK && parameters.counts) {
            mult.resize((size_t)nGroups * s);
            rc = fpm_sketch_mult(job, nullptr, mult.data());
        }
        fpm_sketch_job_free(job);
        check(rc, "sketch");
        mark("device sketch (stage + run + fetch)");
        if (stores) {
            // views into the fetched arrays (kept alive by the Sketch)
            for (size_t f = 0; f < nF; f++)
                for (size_t i = 0; i < fileRefs[f0 + f].size(); i++) {
                    const uint32_t g = fileGroups[f][i];
                    Reference &ref = fileRefs[f0 + f][i];
                    ref.hashView = out.data() + (size_t)g * s;
                    ref.viewCount = cnt[g];
                    if (!mult.empty()) {
                        ref.countView = mult.data() + (size_t)g * s;
                        ref.countsSorted = true;
                    }
                }
            std::lock_guard<std::mutex> lk(*storeMu);
            stores->push_back(outp);
            if (!mult.empty()) stores->push_back(multp);
            mark("reference lists");
            if (parsed) fpm_seq_free(parsed);
            return;
        }
        // hash lists into the references (threads: the copies are page-fault bound)
        std::vector<std::pair<size_t, size_t>> all;
        for (size_t f = 0; f < nF; f++)
            for (size_t i = 0; i < fileRefs[f0 + f].size(); i++) all.push_back({f, i});
        std::atomic<size_t> nextRef{0};
        auto copyRefs = [&]() {
            for (size_t a; (a = nextRef.fetch_add(256)) < all.size();)
                for (size_t x = a; x < std::min(all.size(), a + 256); x++) {
                    const size_t f = all[x].first, i = all[x].second;
                    const uint32_t g = fileGroups[f][i];
                    Reference &ref = fileRefs[f0 + f][i];
                    ref.hashes.assign(out.begin() + (size_t)g * s, out.begin() + (size_t)g * s + cnt[g]);
                    if (!mult.empty()) {
                        ref.counts.assign(mult.begin() + (size_t)g * s,
                                          mult.begin() + (size_t)g * s + cnt[g]);
                        ref.countsSorted = true;
                    }
                }
        };
        std::vector<std::thread> cp;
        const size_t ncp = all.size() < 1024 ? 0 : std::min(7u, std::thread::hardware_concurrency());
        for (size_t t = 0; t < ncp; t++) cp.emplace_back(copyRefs);
        copyRefs();
        for (auto &t : cp) t.join();
    }
    mark("reference lists");
    if (parsed) fpm_seq_free(parsed);
}

int Sketch::initFromFiles(const std::vector<std::string> &files, const Parameters &p, int verbosity,
                          bool enforceParameters, bool contain)
{
    parameters = p;
    // output slots in input order: loaded references, or one sequence file (index into seqFiles)
    struct Item { bool isSeq; size_t file; std::vector<Reference> refs; };
    std::vector<Item> items;
    std::vector<std::string> seqFiles;

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
            Item it{false, 0, {}};
            loadMsh(file, parameters, it.refs);
            items.push_back(std::move(it));
            continue;
        }
        if (verbosity > 0)
            std::cerr << (file == "-" ? std::string("Sketching from stdin...")
                                      : "Sketching " + file + "...") << std::endl;
        if (file != "-") {
            FILE *f = fopen(file.c_str(), "r");
            if (!f) {
                std::cerr << "ERROR: could not open " << file << " for reading." << std::endl;
                fatalExit();
            }
            fclose(f);
        }
        items.push_back(Item{true, seqFiles.size(), {}});
        seqFiles.push_back(file);
    }

    if (!seqFiles.empty()) {
        // file images: gzip streams inflate on their own threads (one stream inflates
        // serially, several files in parallel)
        std::vector<std::string> images(seqFiles.size());
        {
            std::vector<char> okv(seqFiles.size(), 1);
            std::atomic<size_t> next{0};
            auto work = [&]() {
                for (size_t f; (f = next++) < seqFiles.size();)
                    okv[f] = loadSequenceFile(seqFiles[f], images[f]) ? 1 : 0;
            };
            const size_t nt = std::min<size_t>(seqFiles.size(),
                                               std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
            std::vector<std::thread> pool;
            for (size_t t = 1; t < nt; t++) pool.emplace_back(work);
            work();
            for (auto &t : pool) t.join();
            for (size_t f = 0; f < seqFiles.size(); f++)
                if (!okv[f]) {
                    std::cerr << "ERROR: could not open " << seqFiles[f] << std::endl;
                    fatalExit();
                }
        }
        phaseMark("read input");
        // files over the devices as contiguous ranges balanced by bytes (the reference's -p
        // threads take files in turn, Sketch.cpp:253); one device: every file on device(0)
        std::vector<std::vector<Reference>> fileRefs(seqFiles.size());
        std::mutex storeMu;
        const int nDev = deviceCount();
        const size_t nParts = std::min<size_t>((size_t)std::max(1, nDev), seqFiles.size());
        if (nParts <= 1) {
            fpm_ctx *ctx = device();
            phaseMark("device context");
            sketchFiles(ctx, parameters, seqFiles, images, 0, seqFiles.size(), fileRefs, true,
                        rowViews ? &rowStores : nullptr, &storeMu);
        } else {
            uint64_t tot = 0;
            for (auto &im : images) tot += im.size() + 1;
            std::vector<size_t> cut{0};
            uint64_t acc = 0;
            for (size_t f = 0; f < seqFiles.size(); f++) {
                acc += images[f].size() + 1;
                if (cut.size() < nParts && acc * nParts >= tot * cut.size() && f + 1 < seqFiles.size())
                    cut.push_back(f + 1);
            }
            cut.push_back(seqFiles.size());
            std::vector<std::thread> th;
            for (size_t d = 0; d + 1 < cut.size(); d++)
                th.emplace_back([&, d] {
                    sketchFiles(device((int)d), parameters, seqFiles, images, cut[d], cut[d + 1],
                                fileRefs, false, rowViews ? &rowStores : nullptr, &storeMu);
                });
            for (auto &t : th) t.join();
            phaseMark("device sketch over all devices");
        }
        for (auto &it : items)
            if (it.isSeq) it.refs = std::move(fileRefs[it.file]);
    }
    references.clear();
    for (auto &it : items)
        for (auto &r : it.refs) references.push_back(std::move(r));
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
            fatalExit();
        }
        phaseMark("fingerprint file read");
        // parse + hash on the device (getline / `iss >> id` / `while (iss >> v)` /
        // getHashFingerPrint per line, Sketch.cpp:82-101, 131), at most the lines left
        // of the global cap
        const uint64_t remaining = kLimitReadFingerprint - counterLine;
        fpm_fptext *job = nullptr;
        uint64_t n = 0;
        check(fpm_fp_text_stage(device(), text.data(), text.size(), remaining, parameters.seed,
                                parameters.use64, &job, &n),
              "fingerprint parse");
        // the lines' References grouped on the device (:104-145): their first lines, IDs and
        // lengths; the host fetches those and the line hashes only
        uint64_t nr = 0;
        std::vector<uint64_t> first, idOff, len;
        std::vector<uint32_t> idLen;
        int rc = fpm_fp_text_refs(job, 0, &nr, nullptr, nullptr, nullptr, nullptr);
        if (rc == FPM_OK && nr) {
            first.resize(nr);
            idOff.resize(nr);
            idLen.resize(nr);
            len.resize(nr);
            rc = fpm_fp_text_refs(job, nr, &nr, first.data(), idOff.data(), idLen.data(),
                                  len.data());
        }
        std::vector<uint64_t> h64(parameters.use64 ? n : 0);
        std::vector<uint32_t> h32(parameters.use64 ? 0 : n);
        if (rc == FPM_OK)
            rc = fpm_fp_text_fetch(job, nullptr, nullptr, nullptr,
                                   parameters.use64 ? (void *)h64.data() : (void *)h32.data(),
                                   nullptr);
        fpm_fp_text_free(job);
        check(rc, "fingerprint parse");
        counterLine += n;
        if (nr && std::string(text.data() + idOff[0], idLen[0]) == lastID) {
            // line 0 continues the previous file's last ID: the reference dereferences a null
            // Reference here (Sketch.cpp:131-134, the Reference pointer is reset per file)
            std::cerr << "ERROR: fingerprint line 1 of " << file << " continues ID \"" << lastID
                      << "\" from a previous file." << std::endl;
            fatalExit();
        }
        std::vector<Reference> fileRefs(nr);
        for (uint64_t r = 0; r < nr; r++) {
            Reference &ref = fileRefs[r];
            const std::string id(text.data() + idOff[r], idLen[r]);
            ref.id = id;
            ref.length = len[r];
            ref.name = id;
            ref.comment = "FingerPrint : " + id;
            const uint64_t a = first[r], b = r + 1 < nr ? first[r + 1] : n;
            ref.hashes.resize(b - a);
            for (uint64_t i = a; i < b; i++)
                ref.hashes[i - a] = parameters.use64 ? h64[i] : (uint64_t)h32[i];
        }
        if (nr) lastID.assign(text.data() + idOff[nr - 1], idLen[nr - 1]);
        phaseMark("fingerprint parse + references (device)");
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
    std::vector<MshRefView> refs(references.size());
    for (size_t i = 0; i < references.size(); i++) {
        const Reference &r = references[i];
        refs[i] = MshRefView{&r.name, &r.comment, r.length, r.hashData(), r.hashCount(),
                             r.countData(), r.countCount()};
    }
    if (!mshWrite(file, h, refs.data(), refs.size(), parameters.use64, parameters.counts)) {
        std::cerr << "ERROR: could not open " << file << " for writing.\n";
        fatalExit();
    }
    phaseMark("msh write");
    return 0;
}

}  // namespace fpmhost
