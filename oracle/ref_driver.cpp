// ref_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" driver linked against the reference's OWN hot-path sources,
// compiled unmodified from where they lie (/root/reference/mash/src/mash:
// hash.cpp, MurmurHash3.cpp, MinHashHeap.cpp, HashSet.cpp, HashList.cpp,
// HashPriorityQueue.cpp) by oracle/Makefile into oracle/_ref/libfpmref.so.
// Used only by tests/golden/make_golden.py (in the build container) to generate
// golden vectors and to cross-check the C restatement.  Sketch.cpp itself needs
// Cap'n Proto headers and cannot be compiled here, so the k-mer walk of
// addMinHashes (Sketch.cpp:664-735) is re-driven below around the reference's
// getHash and MinHashHeap.

#include "hash.h"
#include "MinHashHeap.h"

#include "HashList.h"

#include <zlib.h>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

// the reference's own FASTA/FASTQ reader (header-only kseq.h, instantiated as Sketch.cpp:38 does)
#include "kseq.h"
KSEQ_INIT(gzFile, gzread)

extern "C" {

unsigned long long ref_get_hash(const char *seq, int len, unsigned seed, int use64)
{
    hash_u h = getHash(seq, len, seed, use64 != 0);
    return use64 ? h.hash64 : (unsigned long long)h.hash32;
}

unsigned long long ref_get_hash_fp(const unsigned long long *vals, unsigned long long n,
                                   unsigned seed, int use64)
{
    std::vector<uint64_t> v(vals, vals + n);
    hash_u h = getHashFingerPrint(v, (int)(n * sizeof(uint64_t)), seed, use64 != 0);
    return use64 ? h.hash64 : (unsigned long long)h.hash32;
}

// Feed a hash stream through the reference MinHashHeap; return the sorted list.
unsigned long long ref_minhash_stream(const unsigned long long *hashes, unsigned long long n,
                                      int use64, unsigned long long cap,
                                      unsigned long long *out_hashes, unsigned *out_counts)
{
    MinHashHeap heap(use64 != 0, cap, 1, 0);
    for (unsigned long long i = 0; i < n; i++) {
        hash_u h;
        h.hash64 = 0;
        if (use64) h.hash64 = hashes[i]; else h.hash32 = (uint32_t)hashes[i];
        heap.tryInsert(h);
    }
    HashList list(use64 != 0);
    std::vector<uint32_t> counts;
    heap.toHashList(list, counts);
    for (int i = 0; i < list.size(); i++) {
        hash_u h = list.at(i);
        out_hashes[i] = use64 ? h.hash64 : (unsigned long long)h.hash32;
        if (out_counts) out_counts[i] = counts[i];
    }
    return (unsigned long long)list.size();
}

// k-mer walk of addMinHashes (Sketch.cpp:664-735) around reference getHash + MinHashHeap.
// One record or a concatenation (n_rec records streamed into one heap).
static const char kComp[26] = {'T','V','G','H','N','N','C','D','N','N','M','N','K',
                               'N','N','N','N','Y','S','A','A','B','W','N','R','N'};

static void walk(MinHashHeap &heap, char *seq, unsigned long long length, int k,
                 unsigned seed, int use64, int noncanonical, int preserve_case,
                 const unsigned char *alphabet)
{
    if (!preserve_case)
        for (unsigned long long i = 0; i < length; i++)
            if (seq[i] > 96 && seq[i] < 123) seq[i] -= 32;
    std::vector<char> rev(length);
    if (!noncanonical)
        for (unsigned long long i = 0; i < length; i++) {
            int c = (unsigned char)seq[length - i - 1] - 'A';
            rev[i] = (c >= 0 && c < 26) ? kComp[c] : 'N';
        }
    unsigned long long j = 0;
    for (unsigned long long i = 0; i + k <= length; i++) {
        bool bad = false;
        for (; j < i + k; j++)
            if (!alphabet[(unsigned char)seq[j]]) { i = j++; bad = true; break; }
        if (bad) continue;
        const char *f = seq + i, *r = rev.data() + length - i - k;
        const char *km = (noncanonical || memcmp(f, r, k) <= 0) ? f : r;
        heap.tryInsert(getHash(km, k, seed, use64 != 0));
    }
}

unsigned long long ref_sketch_records(const char *seq, const unsigned long long *rec_off,
                                      unsigned n_rec, int k, unsigned long long s,
                                      unsigned seed, int use64, int noncanonical,
                                      int preserve_case, const unsigned char *alphabet,
                                      unsigned long long *out_hashes, unsigned *out_counts)
{
    MinHashHeap heap(use64 != 0, s, 1, 0);
    for (unsigned r = 0; r < n_rec; r++) {
        unsigned long long l = rec_off[r + 1] - rec_off[r];
        if (l < (unsigned long long)k) continue;
        std::vector<char> buf(seq + rec_off[r], seq + rec_off[r] + l);
        walk(heap, buf.data(), l, k, seed, use64, noncanonical, preserve_case, alphabet);
    }
    HashList list(use64 != 0);
    std::vector<uint32_t> counts;
    heap.toHashList(list, counts);
    for (int i = 0; i < list.size(); i++) {
        hash_u h = list.at(i);
        out_hashes[i] = use64 ? h.hash64 : (unsigned long long)h.hash32;
        if (out_counts) out_counts[i] = counts[i];
    }
    return (unsigned long long)list.size();
}

// -i sketches of n_rec records (one heap each) on `threads` std::threads taking records in
// turn (the reference's -p pool hands records to workers one at a time): the reference-heap
// CPU rate without a per-record ctypes hop.  Record r's list lands in out_hashes[r * s ...],
// its size in out_n[r].
void ref_sketch_batch_mt(const char *seq, const unsigned long long *rec_off, unsigned n_rec,
                         int k, unsigned long long s, unsigned seed, int use64, int noncanonical,
                         int preserve_case, const unsigned char *alphabet, int threads,
                         unsigned long long *out_hashes, unsigned long long *out_n)
{
    std::atomic<unsigned> next(0);
    auto work = [&]() {
        for (unsigned r; (r = next.fetch_add(1)) < n_rec;)
            out_n[r] = ref_sketch_records(seq, rec_off + r, 1, k, s, seed, use64, noncanonical,
                                          preserve_case, alphabet, out_hashes + (size_t)r * s,
                                          nullptr);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
}

// kseq_read writes seq.s[seq.l] = 0 after the sequence loop (kseq.h:194) into a buffer it only
// allocates once a base is stored: a stream whose FIRST record has no sequence byte (">x" at
// EOF, ">x\n>y...") dereferences a null pointer there and the reference crashes.  The driver
// pre-sizes the buffers, so such a record reads as an empty sequence -- the definition the
// device parser and tests/seqio.py use.
static kseq_t *presized(kseq_t *seq)
{
    seq->seq.m = 256;
    seq->seq.s = (char *)malloc(seq->seq.m);
    seq->qual.m = 256;
    seq->qual.s = (char *)malloc(seq->qual.m);
    return seq;
}

// kseq_read over a (optionally gzip'd) file, as sketchFileBySequence (Sketch.cpp:478-522)
// reads it: every record's name, comment, sequence and quality strings.  Serialised into one
// malloc'd buffer (free with ref_free): per record u64 lengths then bytes of name, comment,
// seq, qual.  *status = kseq_read's last return (-1: clean end, -2: truncated quality), *n =
// records.  Returns null when the file cannot be opened.
unsigned char *ref_kseq_records(const char *path, unsigned long long *n, int *status,
                                unsigned long long *bytes)
{
    gzFile fp = gzopen(path, "r");
    if (!fp) return nullptr;
    kseq_t *seq = presized(kseq_init(fp));
    std::string out;
    unsigned long long cnt = 0;
    int l;
    auto put = [&](const kstring_t &x) {
        unsigned long long len = x.l;
        out.append((const char *)&len, 8);
        if (len) out.append(x.s, len);
    };
    while ((l = kseq_read(seq)) >= 0) {
        put(seq->name);
        put(seq->comment);
        put(seq->seq);
        put(seq->qual);
        cnt++;
    }
    kseq_destroy(seq);
    gzclose(fp);
    unsigned char *buf = (unsigned char *)malloc(out.size() ? out.size() : 1);
    memcpy(buf, out.data(), out.size());
    *n = cnt;
    *status = l;
    *bytes = out.size();
    return buf;
}

// kseq_read + the per-record sequence copy (Sketch.cpp:502-506) of a file, counting records
// and bases: the reference's input step alone, for the CPU baseline's CLI leg.
static void sink_fn(const char *, size_t) {}
static void (*volatile g_sink)(const char *, size_t) = sink_fn;   // keeps the copy observable

int ref_kseq_scan(const char *path, unsigned long long *n_rec, unsigned long long *n_bases)
{
    gzFile fp = gzopen(path, "r");
    if (!fp) return -3;
    kseq_t *seq = presized(kseq_init(fp));
    unsigned long long c = 0, b = 0;
    int l;
    while ((l = kseq_read(seq)) >= 0) {
        char *copy = new char[l ? l : 1];
        memcpy(copy, seq->seq.s, l);
        g_sink(copy, (size_t)l);
        b += (unsigned long long)l;
        delete[] copy;
        c++;
    }
    kseq_destroy(seq);
    gzclose(fp);
    *n_rec = c;
    *n_bases = b;
    return l;
}

// The per-file work of Sketch::initFromFingerprints (Sketch.cpp:67-145), restated around the
// reference's own getHashFingerPrint (hash.cpp:45-73) and HashList::add (HashList.h:27-33), on
// one thread as the reference runs it: std::getline per line (at most `limit` lines counted
// across the call's files, :37, :82), `istringstream >> id`, `>> number` until it fails (a
// space after a number skipped), a new Reference wherever the ID differs from the previous
// line's, its length the first line's count plus every line's.  For the bench's CPU
// same-work leg of `sketch -fp` (timed, not a parity source: the oracle's C restatement
// pins the parse).  Returns the References made, or -1 when the file cannot be opened;
// *lines_used accumulates, *hash_sum is a checksum over every hash.
long long ref_fp_sketch_file(const char *path, unsigned long long limit,
                             unsigned long long *lines_used, unsigned seed, int use64,
                             unsigned long long *hash_sum)
{
    std::ifstream in(path);
    if (!in) return -1;
    struct Ref { std::string id; unsigned long long length = 0; HashList hashes; };
    std::vector<Ref> refs;
    std::string line, last;
    bool open_ref = false;
    unsigned long long sum = 0;
    while (*lines_used < limit && std::getline(in, line)) {
        ++*lines_used;
        std::istringstream ss(line);
        std::string id;
        ss >> id;
        std::vector<uint64_t> values;
        uint64_t v;
        while (ss >> v) {
            values.push_back(v);
            if (ss.peek() == ' ') ss.ignore();
        }
        if (!open_ref || id != last) {
            refs.emplace_back();
            refs.back().id = id;
            refs.back().length = values.size();
            refs.back().hashes.setUse64(use64 != 0);
            last = id;
            open_ref = true;
        }
        const hash_u h = getHashFingerPrint(values, (int)(values.size() * sizeof(uint64_t)), seed,
                                            use64 != 0);
        refs.back().hashes.add(h);
        refs.back().length += values.size();
        sum += use64 ? h.hash64 : h.hash32;
    }
    *hash_sum += sum;
    return (long long)refs.size();
}

void ref_free(void *p) { free(p); }

}  // extern "C"
