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

#include <cstring>
#include <vector>

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

}  // extern "C"
