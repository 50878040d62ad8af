// CommandDistance.cpp — `fpmash dist` (CommandDistance.cpp:38-333): same inputs
// (.msh, sequence files, -fp .txt / .msh), same messages, same ordered text
// output.  The shared-hash walk, distance and p-value of every ref x query pair
// run on the MI355X (fpm_dist); the host formats the lines in query-major order.
#include "Command.h"
#include "Device.h"
#include "Sketch.h"
#include "Timing.h"
#include "HostRows.h"

#include <algorithm>
#include <memory>
#include <chrono>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <iostream>
#include <mutex>
#include <thread>

#include <fcntl.h>
#include <climits>
#include <sys/mman.h>
#include <sys/uio.h>
#include <sys/stat.h>
#include <unistd.h>

namespace fpmhost {

CommandDistance::CommandDistance()
{
    name = "dist";
    summary = "Estimate the distance of query sequences to references.";
    description = "Estimate the distance of each query sequence to the reference. Both the "
                  "reference and queries can be fasta or fastq, gzipped or not, or Mash sketch "
                  "files (.msh) with matching k-mer sizes, or (-fp) k-finger fingerprint files. "
                  "The output fields are [reference-ID, query-ID, distance, p-value, "
                  "shared-hashes].";
    argumentString = "<reference> <query> [<query>] ...";
    useOption("help");
    addOption("list", Option(Option::Boolean, "l", "Input",
        "List input. Lines in each <query> specify paths to sequence files, one per line. The "
        "reference file is not affected.", ""));
    addOption("table", Option(Option::Boolean, "t", "Output",
        "Table output (will not report p-values, but fields will be blank if they do not meet "
        "the p-value threshold).", ""));
    addOption("pvalue", Option(Option::Number, "v", "Output", "Maximum p-value to report.",
                               "1.0", 0., 1.));
    addOption("distance", Option(Option::Number, "d", "Output", "Maximum distance to report.",
                                 "1.0", 0., 1.));
    addOption("comment", Option(Option::Boolean, "C", "Output",
        "Show comment fields with reference/query names (denoted with ':').", "1.0", 0., 1.));
    addOption("fingerprint", Option(Option::Boolean, "fp", "Input",
        "Indicates that the input files are fingerprints instead of sequences.", ""));
    useSketchOptions();
}

// containsMSH / containsTXT (CommandDistance.cpp:454-476): substring test on the last file
static bool containsSub(const std::vector<std::string> &v, const char *s)
{
    bool f = false;
    for (const auto &x : v) f = x.find(s) != std::string::npos;
    return f;
}

namespace {

struct Out {
    std::string buf;
    bool autoflush = true;            // false: a formatter piece, written later in order
    void flush() { fwrite(buf.data(), 1, buf.size(), stdout); buf.clear(); }
    void put(const std::string &s) { buf += s; if (autoflush && buf.size() > (1 << 22)) flush(); }
    void put(char c) { buf.push_back(c); }
    void num(double x)   // ostream default: %g, precision 6
    {
        if (x == 1.0) { buf.push_back('1'); return; }     // most cells: no shared hash
        if (x == 0.0 && !std::signbit(x)) { buf.push_back('0'); return; }
        char t[64];
        int n = snprintf(t, sizeof t, "%g", x);
        buf.append(t, n);
    }
    void u(uint64_t x)
    {
        char t[24];
        int n = 0;
        do { t[23 - n++] = (char)('0' + x % 10); x /= 10; } while (x);
        buf.append(t + 24 - n, n);
    }
};

// the same formats into a caller's buffer (the one-append-per-line path): at most
// kLineNums bytes for the two numbers, two counts and four separators of a line
constexpr size_t kLineNums = 2 * 32 + 2 * 20 + 4;
inline char *numTo(char *p, double x)
{
    if (x == 1.0) { *p++ = '1'; return p; }
    if (x == 0.0 && !std::signbit(x)) { *p++ = '0'; return p; }
    return p + snprintf(p, 32, "%g", x);
}
// counts of up to 4 digits (a sketch size of 1000 and below: every count of the C2 text) by
// two-digit table lookups, the rest digit by digit (14.6 against 17.6 ns per list line)
constexpr char kDigits2[] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";
inline char *uTo(char *p, uint64_t x)
{
    if (x < 100) {
        if (x < 10) { *p = (char)('0' + x); return p + 1; }
        memcpy(p, kDigits2 + 2 * x, 2);
        return p + 2;
    }
    if (x < 10000) {
        const uint32_t a = (uint32_t)x / 100, b = (uint32_t)x % 100;
        if (a < 10) {
            *p = (char)('0' + a);
            memcpy(p + 1, kDigits2 + 2 * b, 2);
            return p + 3;
        }
        memcpy(p, kDigits2 + 2 * a, 2);
        memcpy(p + 2, kDigits2 + 2 * b, 2);
        return p + 4;
    }
    char t[20];
    int n = 0;
    do { t[19 - n++] = (char)('0' + x % 10); x /= 10; } while (x);
    memcpy(p, t + 20 - n, n);
    return p + n;
}

// Allocates the output file's pages ahead of the writer: the file's size set to an estimate of
// the text's end, then fallocate (sizes kept) in 64 MB steps from the output position, on a
// thread of its own that starts while the HIP runtime comes up and the rows are packed (idle
// cores).  pwrite into allocated tmpfs pages copies at ~9.7 GB/s against ~6.0 GB/s when every
// page is allocated on the way, and fallocate alone runs at ~18 GB/s (4 GB into /dev/shm on the
// MI355X box, tools/micro/write_rate.cpp).  The file's size stays the caller's to change; the
// pages past the final size are cut by trim().
class Prealloc {
  public:
    void start(int fd, off_t from, off_t upto)
    {
        struct stat st {};
        if (fstat(fd, &st) != 0) return;
        if (st.st_size < upto) {
            fatalCutsOutput(fd, st.st_size);    // an error exit leaves the file as it was
            if (ftruncate(fd, upto) != 0) return;
        }
        fd_ = fd;
        pos_ = from;
        upto_ = upto;
        th_ = std::thread([this] {
            // pwrite mode: only until the writer starts (allocating beside its writes made them
            // queue on the file's inode lock, CLI A/B on the box: 1.0-1.7 s against 1.05-1.28 s);
            // writes through a mapping take no inode lock and run beside it
            while (!stop_.load(std::memory_order_relaxed) && !started_.load(std::memory_order_relaxed)) {
                const off_t n = std::min<off_t>(kStep, upto_ - pos_);
                if (n <= 0 || fallocate(fd_, FALLOC_FL_KEEP_SIZE, pos_, n) != 0) break;
                pos_ += n;
            }
        });
    }
    void writerAt(off_t) { started_.store(true, std::memory_order_relaxed); }
    // stop allocating; the file cut back to `final_size` (fallocate may have extended it)
    bool trim(off_t final_size)
    {
        if (!th_.joinable()) return true;
        stop_ = true;
        th_.join();
        struct stat st {};
        return fstat(fd_, &st) != 0 || st.st_size <= final_size || ftruncate(fd_, final_size) == 0;
    }
    ~Prealloc()
    {
        stop_ = true;
        if (th_.joinable()) th_.join();
    }

  private:
    static constexpr off_t kStep = off_t(64) << 20;
    int fd_ = -1;
    off_t pos_ = 0, upto_ = 0;
    std::atomic<bool> stop_{false}, started_{false};
    std::thread th_;
};

// writes the pieces at `at` in one pwritev() per IOV_MAX pieces (short writes resumed); false on
// an error.  One call per block: the formatter threads keep formatting instead of queueing on
// the file's inode lock, which serialises writes to one file anyway (tmpfs on the MI355X box:
// one stream 5.6-6.1 GB/s; a shared mapping of the file faulted in at 3.5 GB/s and, with the
// pages allocated ahead, still lost to this path in the CLI: tools/micro/write_rate.cpp, DESIGN
// §5).
bool writePieces(int fd, off_t at, const std::vector<std::string> &pieces)
{
    std::vector<struct iovec> iov;
    iov.reserve(pieces.size());
    for (const auto &t : pieces)
        if (!t.empty()) iov.push_back({(void *)t.data(), t.size()});
    size_t i = 0;
    while (i < iov.size()) {
        const int n = (int)std::min<size_t>(iov.size() - i, IOV_MAX);
        const ssize_t w = pwritev(fd, &iov[i], n, at);
        if (w <= 0) return false;
        at += (off_t)w;
        for (size_t left = (size_t)w; left;) {
            if (left >= iov[i].iov_len) {
                left -= iov[i].iov_len;
                i++;
            } else {
                iov[i].iov_base = (char *)iov[i].iov_base + left;
                iov[i].iov_len -= left;
                left = 0;
            }
        }
    }
    return true;
}

}  // namespace

int CommandDistance::run() const
{
    if (arguments.size() < 2 || options.at("help").active) {
        print();
        return 0;
    }
    warmDevices();
    const bool list = options.at("list").active;
    const bool table = options.at("table").active;
    const bool comment = options.at("comment").active;
    const double pValueMax = options.at("pvalue").getArgumentAsNumber();
    const double distanceMax = options.at("distance").getArgumentAsNumber();
    const bool fingerprint = options.at("fingerprint").active;
    Parameters parameters;
    if (sketchParameterSetup(parameters, *this)) return 1;

    Sketch sketchRef;
    uint64_t lengthMax = 0;
    double randomChance = 0;
    int kMin = 0;
    std::string lengthMaxName;
    int warningCount = 0;
    const std::string &fileReference = arguments[0];
    const bool isSketch = hasSuffix(fileReference, suffixSketch);
    if (isSketch) {
        for (const char *o : {"kmer", "noncanonical", "protein", "alphabet"})
            if (options.at(o).active) {
                std::cerr << "ERROR: The option -" << options.at(o).identifier
                          << " cannot be used when a sketch is provided; it is inherited from the "
                             "sketch." << std::endl;
                return 1;
            }
    } else {
        std::cerr << "Sketching " << fileReference
                  << " (provide sketch file made with \"mash sketch\" to skip)...";
    }
    std::vector<std::string> refArg{fileReference};
    const bool tagMSH = containsSub(refArg, ".msh"), tagTXT = containsSub(refArg, ".txt");
    if (fingerprint && tagMSH) sketchRef.initFromFiles(refArg, parameters);
    else if (fingerprint && tagTXT) sketchRef.initFromFingerprints(refArg, parameters);
    else sketchRef.initFromFiles(refArg, parameters);

    phaseMark("reference sketch loaded");
    const double lengthThreshold =
        (parameters.warning * sketchRef.getKmerSpace()) / (1. - parameters.warning);
    if (isSketch) {
        parameters.minHashesPerWindow = (uint64_t)sketchRef.getMinHashesPerWindow();
        parameters.kmerSize = sketchRef.getKmerSize();
        parameters.noncanonical = sketchRef.getNoncanonical();
        parameters.preserveCase = sketchRef.getPreserveCase();
        parameters.seed = sketchRef.getHashSeed();
        std::string alphabet;
        sketchRef.getAlphabetAsString(alphabet);
        setAlphabetFromString(parameters, alphabet.c_str());
    } else {
        for (uint64_t i = 0; i < sketchRef.getReferenceCount(); i++) {
            const uint64_t length = sketchRef.getReference(i).length;
            if (length > lengthThreshold) {
                if (warningCount == 0 || length > lengthMax) {
                    lengthMax = length;
                    lengthMaxName = sketchRef.getReference(i).name;
                    randomChance = sketchRef.getRandomKmerChance(i);
                    kMin = sketchRef.getMinKmerSize(i);
                }
                warningCount++;
            }
        }
        std::cerr << "done.\n";
    }
    Out out;
    if (table) {
        out.put("#query");
        for (uint64_t i = 0; i < sketchRef.getReferenceCount(); i++) {
            out.put('\t');
            out.put(sketchRef.getReference(i).name);
        }
        out.put('\n');
        out.flush();
        fflush(stdout);
    }
    std::vector<std::string> queryFiles;
    for (size_t i = 1; i < arguments.size(); i++) {
        if (list) splitFile(arguments[i], queryFiles);
        else queryFiles.push_back(arguments[i]);
    }
    // `dist X.msh X.msh`: the query set is the reference set (same file, same parameters), so
    // it is parsed and packed once
    const bool sameSet = isSketch && !fingerprint && queryFiles.size() == 1 &&
                         queryFiles[0] == fileReference;
    Sketch sketchQueryOwn;
    if (sameSet) {}
    else if (fingerprint && tagMSH) sketchQueryOwn.initFromFiles(queryFiles, parameters);
    else if (fingerprint && tagTXT) sketchQueryOwn.initFromFingerprints(queryFiles, parameters);
    else sketchQueryOwn.initFromFiles(queryFiles, parameters, 0, true);
    const Sketch &sketchQuery = sameSet ? sketchRef : sketchQueryOwn;

    phaseMark("query sketch loaded");
    const uint64_t nR = sketchRef.getReferenceCount(), nQ = sketchQuery.getReferenceCount();
    const uint64_t sketchSize = (uint64_t)std::min(sketchQuery.getMinHashesPerWindow(),
                                                   sketchRef.getMinHashesPerWindow());
    const bool use64 = sketchRef.getUse64();
    const uint32_t hb = use64 ? 8 : 4;
    // stdout a regular file (not O_APPEND): the text goes in at its offsets, one pwritev() per
    // block; otherwise (pipes, terminals) by fwrite.
    out.flush();
    std::cout.flush();
    fflush(stdout);
    const int ofd = fileno(stdout);
    off_t opos = -1;
    {
        struct stat st {};
        const int fl = fcntl(ofd, F_GETFL);
        if (nR && nQ && fl >= 0 && !(fl & O_APPEND) && fstat(ofd, &st) == 0 && S_ISREG(st.st_mode))
            opos = lseek(ofd, 0, SEEK_CUR);
    }
    const bool direct = opos >= 0;
    // The output file's pages allocated ahead (Prealloc) while the devices come up: the list
    // format and no -d / -v filter, so the text size is about known: every line names its pair
    // and most carry "1\t1\t0/<denom>" (pairs sharing hashes write a few bytes more, past the
    // estimate, into pages allocated on the way)
    Prealloc prealloc;
    const char *pa_env = getenv("FPMASH_DIST_PREALLOC");   // A/B: 0 = pages allocated on the way
    if (direct && !table) {
        const off_t at = opos;
        {
            uint64_t rn = 0, qn = 0;
            for (uint64_t j = 0; j < nR; j++) {
                const Reference &r = sketchRef.getReference(j);
                rn += r.name.size() + (comment ? 1 + r.comment.size() : 0);
            }
            for (uint64_t q = 0; q < nQ; q++) {
                const Reference &r = sketchQuery.getReference(q);
                qn += 2 + r.name.size() + (comment ? 1 + r.comment.size() : 0);
            }
            const uint64_t digits = std::to_string(sketchSize).size();
            const long double est = (long double)nQ * rn + (long double)nR * qn +
                                    (long double)nR * nQ * (7 + digits);
            if (!options.at("distance").active && !options.at("pvalue").active &&
                !(pa_env && strcmp(pa_env, "0") == 0))
                prealloc.start(ofd, at, at + (off_t)std::min<long double>(est, (long double)(1ULL << 46)));
        }
    }
    // dense device layout: one row per sketch
    // (zero pages, populated in one call: a value-initialised vector paid a memset and ~20k
    // page faults on one thread for C2's 80 MB)
    auto pack = [&](const Sketch &sk, std::unique_ptr<HostRows<uint8_t>> &mp,
                    std::vector<uint32_t> &len, std::vector<uint64_t> &L, uint64_t width) {
        const uint64_t n = sk.getReferenceCount();
        mp = std::make_unique<HostRows<uint8_t>>(std::max<uint64_t>(1, n * width) * hb);
        uint8_t *m = mp->data();
        len.resize(n);
        L.resize(n);
        auto rows = [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; i++) {
                const Reference &r = sk.getReference(i);
                len[i] = (uint32_t)r.hashes.size();
                L[i] = r.length;
                if (use64) {
                    memcpy(&m[i * width * 8], r.hashes.data(), r.hashes.size() * 8);
                } else {
                    uint32_t *row = reinterpret_cast<uint32_t *>(&m[i * width * 4]);
                    for (uint64_t j = 0; j < r.hashes.size(); j++) row[j] = (uint32_t)r.hashes[j];
                }
            }
        };
        // several threads past a few thousand rows (C2: 80 MB)
        const uint64_t nt = n >= 4096 ? std::max(1u, std::min(8u, std::thread::hardware_concurrency())) : 1;
        std::vector<std::thread> th;
        for (uint64_t t = 1; t < nt; t++) th.emplace_back(rows, n * t / nt, n * (t + 1) / nt);
        rows(0, n / nt);
        for (auto &x : th) x.join();
    };
    uint64_t width = 1;
    for (uint64_t i = 0; i < nR; i++) width = std::max<uint64_t>(width, sketchRef.getReference(i).hashes.size());
    for (uint64_t i = 0; i < nQ; i++) width = std::max<uint64_t>(width, sketchQuery.getReference(i).hashes.size());
    const int nDev = nR && nQ ? deviceCount() : 0;
    // 1 M pairs per block (16 M-pair slots made pinning and unpinning the slots cost ~0.6 s of
    // the C2 command; C2 `dist` wall: 4 M 1.27 s, 2 M 1.15 s, 1 M 1.06-1.09 s, 512 K 1.50 s)
    uint64_t blockPairs = 1ULL << 20;
    if (const char *bp = getenv("FPMASH_DIST_BLOCK_PAIRS")) blockPairs = std::max(1ULL, strtoull(bp, nullptr, 10));
    const uint64_t block = nR ? std::max<uint64_t>(1, blockPairs / nR) : 1;
    const uint64_t nBlocks = nR ? (nQ + block - 1) / block : 0;
    const int nSlots = std::max(2, 2 * nDev + 1);
    const int nFmt = std::max(1, std::min(parameters.parallelism > 1 ? parameters.parallelism
                                          : (int)std::thread::hardware_concurrency(), 64));
    // A block's results in the compact form (fpm_refset_dist_list): u16 numer / denom of
    // every pair, and distance / p-value / pass of the pairs that share hashes (numer > 0); a
    // pair sharing none has distance 1 (0 for two empty sketches) and p-value 1
    // (CommandDistance.cpp:404-408, 435-437), its line needs nothing else.  4 B per pair over
    // PCIe instead of 21.
    // u16 counts (every count is <= the sketch size), u32 past 65535
    const uint32_t cb = sketchSize <= 65535 ? 2 : 4;
    struct Slot {
        void *nu = nullptr, *de = nullptr;
        uint32_t *lq = nullptr, *lr = nullptr;
        double *ld = nullptr, *lp = nullptr;
        uint8_t *la = nullptr;
        uint64_t cap = 0, nl = 0;           // listed cells: room, count
        std::vector<uint32_t> rowStart;     // per query row of the block: its listed cells,
        std::vector<uint32_t> byRow;        // ordered by reference (indexes into l*)
        int dev = 0;
        uint64_t b = ~0ULL;                 // block held
        std::vector<std::string> text;      // formatted pieces
        int pending = 0;                    // pieces still being formatted
        bool ready = false;
        uint64_t nextB = 0;                 // the next block this slot may take
    };
    std::vector<Slot> slots(nSlots);
    for (int i = 0; i < nSlots; i++) slots[i].nextB = (uint64_t)i;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> tasks;
    bool stop = false;
    auto allocList = [&](Slot &sl, uint64_t cap) {
        fpm_ctx *c = device(0);
        for (void *p : {(void *)sl.lq, (void *)sl.lr, (void *)sl.ld, (void *)sl.lp, (void *)sl.la})
            if (p) fpm_host_free(c, p);
        sl.cap = cap;
        check(fpm_host_alloc(c, (void **)&sl.lq, cap * 4), "pinned buffers");
        check(fpm_host_alloc(c, (void **)&sl.lr, cap * 4), "pinned buffers");
        check(fpm_host_alloc(c, (void **)&sl.ld, cap * 8), "pinned buffers");
        check(fpm_host_alloc(c, (void **)&sl.lp, cap * 8), "pinned buffers");
        check(fpm_host_alloc(c, (void **)&sl.la, cap), "pinned buffers");
    };
    // pinned result buffers (page locking costs ~0.6 ms per MB): one thread per slot, beside
    // the row packing and the reference sets.  The list starts at 1/16 of the block's pairs
    // and grows when a block lists more.
    std::vector<std::thread> pinner;
    for (int i = 0; i < nSlots && nBlocks; i++)
        pinner.emplace_back([&, i] {
            Slot &sl = slots[i];
            const uint64_t np = block * nR;
            fpm_ctx *c = device(0);
            check(fpm_host_alloc(c, &sl.nu, np * cb), "pinned buffers");
            check(fpm_host_alloc(c, &sl.de, np * cb), "pinned buffers");
            allocList(sl, std::max<uint64_t>(4096, np / 16));
        });
    std::unique_ptr<HostRows<uint8_t>> R, Qown;
    std::vector<uint32_t> rl, qlOwn;
    std::vector<uint64_t> rL, qLOwn;
    pack(sketchRef, R, rl, rL, width);
    if (!sameSet) pack(sketchQuery, Qown, qlOwn, qLOwn, width);
    const uint8_t *Q = sameSet ? R->data() : Qown->data();
    const std::vector<uint32_t> &ql = sameSet ? rl : qlOwn;
    const std::vector<uint64_t> &qL = sameSet ? rL : qLOwn;

    // The grid in query blocks (CommandDistance.cpp:224-261 chunks it for the pool): every
    // device holds the reference set with its index built once (fpm_refset_create) and takes
    // blocks in turn; results land in pinned buffers; formatter threads (-p) turn each block
    // into text pieces, which are written strictly in block order (writeOutput, :276-333,
    // consumes the pool's outputs in order).
    std::vector<fpm_refset *> sets(nDev, nullptr);
    for (int d = 0; d < nDev; d++)
        check(fpm_refset_create(device(d), R->data(), rl.data(), rL.data(), width, (uint32_t)nR,
                                hb, (uint32_t)sketchSize, &sets[d]),
              "dist reference set");
    for (auto &t : pinner) t.join();
    phaseMark("rows packed + reference sets on the devices");
    // reference name (+ ":" comment) of each line, built once
    std::vector<std::string> refTag(nR);
    for (uint64_t j = 0; j < nR; j++) {
        const Reference &rr = sketchRef.getReference(j);
        refTag[j] = rr.name;
        if (comment) { refTag[j].push_back(':'); refTag[j] += rr.comment; }
    }
    // the -d / -v filters at the values of a pair sharing no hash (compareSketches, :421-429)
    const bool passNone = !(distanceMax >= 0 && 1.0 > distanceMax) && !(pValueMax >= 0 && 1.0 > pValueMax);
    const bool passEmpty = !(pValueMax >= 0 && 1.0 > pValueMax);   // distance 0: two empty sketches
    auto format = [&](const Slot &sl, uint64_t q0, uint64_t qa, uint64_t qb, std::string &dst) {
        char line[512];
        Out o;
        o.autoflush = false;
        o.buf.swap(dst);                    // the piece's buffer from earlier blocks (no regrowth)
        o.buf.clear();
        for (uint64_t qi = qa; qi < qb; qi++) {
            const Reference &qr = sketchQuery.getReference(q0 + qi);
            if (table) o.put(qr.name);
            std::string qtail;              // "\t<query>[:comment]\t"
            if (!table) {
                qtail.push_back('\t');
                qtail += qr.name;
                if (comment) { qtail.push_back(':'); qtail += qr.comment; }
                qtail.push_back('\t');
            }
            uint32_t cur = sl.rowStart[qi];   // the row's listed cells, in reference order
            for (uint64_t j = 0; j < nR; j++) {
                const uint64_t k = qi * nR + j;
                const uint32_t nm = cb == 2 ? ((const uint16_t *)sl.nu)[k] : ((const uint32_t *)sl.nu)[k];
                const uint32_t dn = cb == 2 ? ((const uint16_t *)sl.de)[k] : ((const uint32_t *)sl.de)[k];
                double di, pv;
                bool pa;
                if (nm == 0) {
                    di = dn == 0 ? 0.0 : 1.0;
                    pv = 1.0;
                    pa = dn == 0 ? passEmpty : passNone;
                } else {
                    const uint32_t e = sl.byRow[cur++];
                    di = sl.ld[e];
                    pv = sl.lp[e];
                    pa = sl.la[e] != 0;
                }
                if (table) {
                    o.put('\t');
                    if (pa) o.num(di);
                } else if (pa) {
                    const std::string &tag = refTag[j];
                    if (tag.size() + qtail.size() + kLineNums <= sizeof(line)) {
                        // one append per line: the line is assembled in a stack buffer
                        char *p = line;
                        memcpy(p, tag.data(), tag.size());
                        p += tag.size();
                        memcpy(p, qtail.data(), qtail.size());
                        p += qtail.size();
                        p = numTo(p, di);
                        *p++ = '\t';
                        p = numTo(p, pv);
                        *p++ = '\t';
                        p = uTo(p, nm);
                        *p++ = '/';
                        p = uTo(p, dn);
                        *p++ = '\n';
                        o.buf.append(line, (size_t)(p - line));
                        continue;
                    }
                    o.put(tag);
                    o.put(qtail);
                    o.num(di);
                    o.put('\t');
                    o.num(pv);
                    o.put('\t');
                    o.u(nm);
                    o.put('/');
                    o.u(dn);
                    o.put('\n');
                }
            }
            if (table) o.put('\n');
        }
        dst.swap(o.buf);
    };
    std::vector<std::thread> fmt;
    for (int t = 0; t < nFmt; t++)
        fmt.emplace_back([&] {
            for (;;) {
                std::function<void()> job;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || !tasks.empty(); });
                    if (tasks.empty()) return;
                    job = std::move(tasks.front());
                    tasks.pop_front();
                }
                job();
            }
        });
    std::atomic<uint64_t> next{0};
    std::atomic<uint64_t> devUs{0};         // device calls + the listed cells' row order
    std::vector<std::thread> gpu;
    for (int d = 0; d < nDev; d++)
        gpu.emplace_back([&, d] {
            for (;;) {
                const uint64_t b = next.fetch_add(1);
                if (b >= nBlocks) return;
                Slot &sl = slots[b % nSlots];
                {
                    // the slot's previous block must be written out first
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return sl.nextB == b; });
                }
                const uint64_t q0 = b * block, nq = std::min(block, nQ - q0);
                const auto tb0 = std::chrono::steady_clock::now();
                for (;;) {
                    check(fpm_refset_dist_list(sets[d], Q + q0 * width * hb, ql.data() + q0,
                                               qL.data() + q0, width, (uint32_t)nq,
                                               (uint32_t)sketchSize,
                                               (uint32_t)sketchRef.getKmerSize(),
                                               sketchRef.getKmerSpace(), distanceMax, pValueMax,
                                               cb, sl.nu, sl.de, sl.lq, sl.lr, sl.ld, sl.lp, sl.la,
                                               sl.cap, &sl.nl),
                          "dist");
                    if (sl.nl <= sl.cap) break;
                    allocList(sl, sl.nl + sl.nl / 4);      // more pairs share hashes: room
                }
                // the listed cells by query row, each row's in reference order (the device
                // lists them unordered)
                sl.rowStart.assign(nq + 1, 0);
                for (uint64_t e = 0; e < sl.nl; e++) sl.rowStart[sl.lq[e] + 1]++;
                for (uint64_t i = 0; i < nq; i++) sl.rowStart[i + 1] += sl.rowStart[i];
                sl.byRow.resize(sl.nl);
                {
                    std::vector<uint32_t> fill(sl.rowStart.begin(), sl.rowStart.end() - 1);
                    for (uint64_t e = 0; e < sl.nl; e++) sl.byRow[fill[sl.lq[e]]++] = (uint32_t)e;
                }
                for (uint64_t i = 0; i < nq; i++)
                    std::sort(sl.byRow.begin() + sl.rowStart[i], sl.byRow.begin() + sl.rowStart[i + 1],
                              [&](uint32_t x, uint32_t y) { return sl.lr[x] < sl.lr[y]; });
                devUs += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::steady_clock::now() - tb0).count();
                // pieces of ~256 K pairs (at least one query row) for the formatter threads:
                // four per block keep the writer fed (C2 command, same box: writer waiting
                // 81-107 -> 24-29 ms, wall 0.93-1.07 -> 0.87-0.92 s against pieces of 1 M; 128 K
                // pieces 0.97-1.06 s)
                const uint64_t per = std::max<uint64_t>(1, (1ULL << 18) / nR);
                const uint64_t parts = (nq + per - 1) / per;
                std::lock_guard<std::mutex> lk(mu);
                sl.b = b;
                sl.dev = d;
                sl.pending = (int)parts;
                sl.ready = false;
                sl.text.resize(parts);
                for (uint64_t p = 0; p < parts; p++) {
                    const uint64_t qa = p * per, qb = std::min(nq, qa + per);
                    tasks.emplace_back([&, q0, qa, qb, p, bslot = &sl] {
                        std::string t;
                        {
                            std::lock_guard<std::mutex> lk2(mu);
                            t.swap(bslot->text[p]);
                        }
                        format(*bslot, q0, qa, qb, t);
                        std::lock_guard<std::mutex> lk2(mu);
                        bslot->text[p].swap(t);
                        if (--bslot->pending == 0) bslot->ready = true;
                        cv.notify_all();
                    });
                }
                cv.notify_all();
            }
        });
    bool writeFailed = false;
    double waitMs = 0, writeMs = 0;
    for (uint64_t b = 0; b < nBlocks; b++) {
        Slot &sl = slots[b % nSlots];
        std::vector<std::string> pieces;
        auto t0 = std::chrono::steady_clock::now();
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return sl.b == b && sl.ready; });
            pieces.swap(sl.text);
        }
        auto t1 = std::chrono::steady_clock::now();
        if (direct) {
            prealloc.writerAt(opos);
            if (!writeFailed && !writePieces(ofd, opos, pieces)) writeFailed = true;
            for (auto &t : pieces) opos += (off_t)t.size();
        } else {
            for (auto &t : pieces) fwrite(t.data(), 1, t.size(), stdout);
        }
        auto t2 = std::chrono::steady_clock::now();
        waitMs += std::chrono::duration<double, std::milli>(t1 - t0).count();
        writeMs += std::chrono::duration<double, std::milli>(t2 - t1).count();
        {
            // the piece buffers go back to the slot for its next block: allocating and
            // unmapping ~40 MB strings per piece cost ~0.4 s of page faults and munmap
            std::lock_guard<std::mutex> lk(mu);
            pieces.swap(sl.text);
            sl.nextB = b + nSlots;
        }
        cv.notify_all();
    }
    if (direct && !prealloc.trim(opos)) writeFailed = true;   // pages allocated past the text
    if (!writeFailed) fatalCutsOutput(-1, 0);                // the text is complete
    if (direct) lseek(ofd, opos, SEEK_SET);   // later output (if any) follows the grid
    if (writeFailed) {
        std::cerr << "ERROR: writing the distance output failed." << std::endl;
        fatalExit();
    }
    if (timingOn())
        fprintf(stderr, "[fpmash] writer waiting for blocks: %.1f ms\n[fpmash] writer copying "
                        "pieces out (%s): %.1f ms\n", waitMs,
                direct ? "pwritev" : "stdout", writeMs);
    if (timingOn())
        fprintf(stderr, "[fpmash] device blocks (compare + fetch + row order, summed): %.1f ms\n",
                devUs.load() / 1e3);
    phaseMark("blocks computed, formatted and written");
    for (auto &t : gpu) t.join();
    {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
    }
    cv.notify_all();
    for (auto &t : fmt) t.join();
    if (cleanExit()) {
        // (the process otherwise leaves by _exit once the output is flushed: unpinning the
        // slots cost ~50 ms of the C2 command)
        for (auto &sl : slots)
            for (void *ptr : {sl.nu, sl.de, (void *)sl.lq, (void *)sl.lr,
                              (void *)sl.ld, (void *)sl.lp, (void *)sl.la})
                if (ptr) fpm_host_free(device(0), ptr);
        for (auto *rs : sets) fpm_refset_free(rs);
    }
    out.flush();
    fflush(stdout);
    if (warningCount > 0 && !parameters.reads)
        warnKmerSize(parameters, *this, lengthMax, lengthMaxName, randomChance, kMin, warningCount);
    if (!cleanExit()) {
        // every output is written: leave before this function's destructors free the ~10^5
        // reference vectors, the row images and the text pieces (~25 ms of the C2 command)
        phaseMark("command done");
        std::cout.flush();
        std::cerr.flush();
        fflush(nullptr);
        _exit(0);
    }
    return 0;
}

}  // namespace fpmhost
