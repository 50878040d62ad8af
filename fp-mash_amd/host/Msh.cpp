// Msh.cpp — see Msh.h.  Wire format: Cap'n Proto (segment table + segments of
// 8-byte words; struct / list / far pointers).  Field layout of MinHash.capnp
// follows capnp's ordinal-order slot assignment:
//   MinHash        data 3 words: kmerSize u32@0, windowSize u32@4, minHashesPerWindow
//                  u32@8, concatenated bit 96, noncanonical bit 97, preserveCase bit 98,
//                  error f32@16, hashSeed u32@20 (stored xor its default 42);
//                  pointers: referenceListOld, locusList, alphabet, referenceList
//   ReferenceList  pointers: references (composite list)
//   Reference      data 2 words: length u32@0, counts32Sorted bit 32, length64 u64@8;
//                  pointers: sequence, quality, name, comment, hashes32, hashes64, counts32
//   LocusList      pointers: loci (composite list of 3-data-word Locus structs)
#include "Msh.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

namespace fpmhost {

namespace {

enum : uint64_t { kStruct = 0, kList = 1, kFar = 2 };
enum : uint64_t { kByte = 2, kFour = 4, kEight = 5, kComposite = 7 };

// capnp MallocMessageBuilder + BuilderArena allocation model.  A segment is a run of
// pieces: words the builder owns, or an external block (a reference's hash list, read in
// place when the message is written: the 8 B/hash bulk of a .msh is never copied).
class Builder {
public:
    struct Piece {
        uint64_t off, n;                 // word range in the segment
        std::vector<uint64_t> own;       // owned words (empty for an external block)
        const void *ext = nullptr;
    };
    struct Seg {
        std::vector<Piece> pieces;
        uint64_t used = 0, cap = 0;
    };
    std::vector<Seg> segs;

    // allocate the root pointer (first allocation creates segment 0)
    void allocRootPointer() { arenaAlloc(1, nullptr); }

    // WireHelpers::allocate: an object of n words referenced from (rs, ro).
    // Returns the object's (segment, offset); writes the pointer (or far pointer +
    // landing pad) with the given kind and upper 32 bits.  ext != nullptr: the object's
    // words are n words at ext (written as they are).
    std::pair<int, uint64_t> alloc(int rs, uint64_t ro, uint64_t n, uint64_t kind, uint64_t upper,
                                   const void *ext = nullptr)
    {
        uint64_t off = 0;
        if (tryAlloc(rs, n, off, ext)) {
            word(rs, ro) = pointer(kind, (int64_t)off - (int64_t)(ro + 1), upper);
            return {rs, off};
        }
        auto a = arenaAlloc(n + 1, ext);              // landing pad, then the object
        word(rs, ro) = kFar | (a.second << 3) | ((uint64_t)a.first << 32);
        word(a.first, a.second) = pointer(kind, 0, upper);
        return {a.first, a.second + 1};
    }

    uint64_t &word(int s, uint64_t o)
    {
        auto &P = segs[s].pieces;
        // the piece holding word o (pieces are in offset order; most accesses hit the last)
        size_t lo = 0, hi = P.size();
        if (o >= P.back().off) lo = P.size() - 1;
        else
            while (hi - lo > 1) {
                const size_t m = (lo + hi) / 2;
                if (P[m].off <= o) lo = m; else hi = m;
            }
        return P[lo].own[o - P[lo].off];
    }

    std::vector<uint32_t> segmentTable() const
    {
        const uint32_t n = (uint32_t)segs.size();
        std::vector<uint32_t> table;
        table.push_back(n - 1);
        for (auto &s : segs) table.push_back((uint32_t)s.used);
        if (table.size() % 2) table.push_back(0);
        return table;
    }

    // the message as (pointer, bytes) blocks in file order
    std::vector<std::pair<const char *, size_t>> blocks(const std::vector<uint32_t> &table) const
    {
        std::vector<std::pair<const char *, size_t>> v;
        v.push_back({reinterpret_cast<const char *>(table.data()), table.size() * 4});
        for (auto &s : segs)
            for (auto &p : s.pieces)
                if (p.n)
                    v.push_back({p.ext ? static_cast<const char *>(p.ext)
                                       : reinterpret_cast<const char *>(p.own.data()),
                                 p.n * 8});
        return v;
    }

    std::string serialize() const
    {
        const std::vector<uint32_t> table = segmentTable();
        std::string out;
        for (auto &b : blocks(table)) out.append(b.first, b.second);
        return out;
    }

    // the same bytes as serialize() into a file.  Large messages: space reserved with
    // fallocate, the file mapped, and the blocks copied in by up to 16 threads over disjoint
    // byte ranges (page faults of a shared mapping run in parallel; pwrite calls on one file
    // serialise on its inode lock: 80 MB of a C2 .msh took ~40 ms that way on /dev/shm).
    // Small messages and file systems without fallocate take the pwrite path; a failed reservation never leaves a mapping that could fault past the
    // end of the device.
    bool write(const std::string &path) const
    {
        const std::vector<uint32_t> table = segmentTable();
        const auto B = blocks(table);
        std::vector<uint64_t> at(B.size() + 1, 0);
        for (size_t i = 0; i < B.size(); i++) at[i + 1] = at[i] + B[i].second;
        const uint64_t total = at.back();
        const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0666);
        if (fd < 0) return false;
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const unsigned nt = total < (8u << 20) ? 1u : std::min(16u, hw);
        // blocks overlapping [a, e): fn(block index, first byte, end byte)
        auto forRange = [&](uint64_t a, uint64_t e, auto fn) {
            size_t i = std::upper_bound(at.begin(), at.end(), a) - at.begin() - 1;
            for (uint64_t pos = a; pos < e && i < B.size(); i++) {
                const uint64_t b0 = std::max(pos, at[i]), b1 = std::min(e, at[i + 1]);
                if (b1 > b0 && !fn(i, b0, b1)) return false;
                pos = b1;
            }
            return true;
        };
        auto parallel = [&](auto part) {
            std::atomic<bool> good{true};
            std::vector<std::thread> th;
            for (unsigned t = 1; t < nt; t++)
                th.emplace_back([&, t] { if (!part(t)) good = false; });
            if (!part(0)) good = false;
            for (auto &x : th) x.join();
            return good.load();
        };
        bool ok = false, done = false;
        if (nt > 1 && fallocate(fd, 0, 0, (off_t)total) == 0) {
            void *m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (m != MAP_FAILED) {
                char *dst = static_cast<char *>(m);
                ok = parallel([&](unsigned t) {
                    // 2 MB-aligned ranges: no page is faulted in by two threads
                    const uint64_t a = (total * t / nt) & ~((uint64_t(2) << 20) - 1);
                    const uint64_t e = t + 1 == nt ? total : (total * (t + 1) / nt) & ~((uint64_t(2) << 20) - 1);
#ifdef MADV_POPULATE_WRITE
                    // the range's pages allocated in one call (not one fault per 4 KB page)
                    if (e > a) (void)madvise(dst + a, (size_t)(e - a), MADV_POPULATE_WRITE);
#endif
                    return forRange(a, e, [&](size_t i, uint64_t b0, uint64_t b1) {
                        memcpy(dst + b0, B[i].first + (b0 - at[i]), (size_t)(b1 - b0));
                        return true;
                    });
                });
                if (munmap(m, total) != 0) ok = false;
                done = true;
            }
        }
        if (!done) {
            ok = ftruncate(fd, (off_t)total) == 0 &&
                 parallel([&](unsigned t) {
                     return forRange(total * t / nt, total * (t + 1) / nt,
                                     [&](size_t i, uint64_t b0, uint64_t b1) {
                         for (uint64_t q = b0; q < b1;) {
                             const ssize_t w = pwrite(fd, B[i].first + (q - at[i]),
                                                      (size_t)(b1 - q), (off_t)q);
                             if (w <= 0) return false;
                             q += (uint64_t)w;
                         }
                         return true;
                     });
                 });
        }
        if (close(fd) != 0) ok = false;
        return ok;
    }

private:
    uint64_t nextSize = 1024;   // SUGGESTED_FIRST_SEGMENT_WORDS, GROW_HEURISTICALLY
    int withSpace = -1;

    static uint64_t pointer(uint64_t kind, int64_t offset, uint64_t upper)
    {
        return kind | (((uint64_t)offset & 0x3FFFFFFFULL) << 2) | (upper << 32);
    }

    bool tryAlloc(int s, uint64_t n, uint64_t &off, const void *ext)
    {
        Seg &g = segs[s];
        if (g.used + n > g.cap) return false;
        off = g.used;
        if (ext) {
            g.pieces.push_back(Piece{off, n, {}, ext});
        } else {
            if (g.pieces.empty() || g.pieces.back().ext) g.pieces.push_back(Piece{off, 0, {}, nullptr});
            Piece &p = g.pieces.back();
            p.own.resize(p.own.size() + n, 0);
            p.n += n;
        }
        g.used += n;
        return true;
    }

    // n words in the newest segment with room, else a new one; ext != nullptr: a far
    // pointer's landing pad (1 owned word) followed by the n - 1 external words
    std::pair<int, uint64_t> arenaAlloc(uint64_t n, const void *ext)
    {
        auto place = [&](int sg, uint64_t &off) {
            if (segs[sg].used + n > segs[sg].cap) return false;
            if (!ext) return tryAlloc(sg, n, off, nullptr);
            uint64_t o2 = 0;
            return tryAlloc(sg, 1, off, nullptr) && tryAlloc(sg, n - 1, o2, ext);
        };
        uint64_t off = 0;
        if (withSpace >= 0 && place(withSpace, off)) return {withSpace, off};
        uint64_t size = std::max(n, nextSize);
        if (segs.empty()) nextSize = size;   // after the first segment: total so far
        else nextSize += size;
        segs.push_back(Seg{{}, 0, size});
        withSpace = (int)segs.size() - 1;
        place(withSpace, off);
        return {withSpace, off};
    }
};

uint64_t structUpper(uint64_t dw, uint64_t pw) { return dw | (pw << 16); }
uint64_t listUpper(uint64_t esz, uint64_t count) { return esz | (count << 3); }

void setText(Builder &b, int s, uint64_t ptr, const std::string &t)
{
    const uint64_t bytes = t.size() + 1;
    auto o = b.alloc(s, ptr, (bytes + 7) / 8, kList, listUpper(kByte, bytes));
    char *dst = reinterpret_cast<char *>(&b.word(o.first, o.second));
    memcpy(dst, t.data(), t.size());
}

void setU32(Builder &b, int s, uint64_t w, int byte, uint32_t v)
{
    uint64_t &x = b.word(s, w + byte / 8);
    const int sh = (byte % 8) * 8;
    x = (x & ~(0xFFFFFFFFULL << sh)) | ((uint64_t)v << sh);
}

void setBit(Builder &b, int s, uint64_t w, int bit, bool v)
{
    uint64_t &x = b.word(s, w + bit / 64);
    if (v) x |= 1ULL << (bit % 64);
    else x &= ~(1ULL << (bit % 64));
}

}  // namespace

namespace {

void build(Builder &b, const MshHeader &h, const MshRefView *refs, uint64_t n, bool use64,
           bool writeCounts)
{
    b.allocRootPointer();
    // root struct: 3 data + 4 pointer words, referenced from segment 0 word 0
    auto root = b.alloc(0, 0, 7, kStruct, structUpper(3, 4));
    const int rs = root.first;
    const uint64_t rw = root.second;
    const uint64_t rp = rw + 3;   // pointer section
    // referenceListOld when the seed is the schema default (Sketch.cpp:549)
    const uint64_t listSlot = h.hashSeed == 42 ? rp + 0 : rp + 3;
    auto rl = b.alloc(rs, listSlot, 1, kStruct, structUpper(0, 1));
    auto lst = b.alloc(rl.first, rl.second, 1 + 9 * n, kList, listUpper(kComposite, 9 * n));
    b.word(lst.first, lst.second) = kStruct | ((n & 0x3FFFFFFFULL) << 2) | (structUpper(2, 7) << 32);
    for (uint64_t i = 0; i < n; i++) {
        const int es = lst.first;
        const uint64_t ew = lst.second + 1 + 9 * i;   // element data words
        const uint64_t ep = ew + 2;                   // element pointers
        const MshRefView &r = refs[i];
        setText(b, es, ep + 2, *r.name);
        setText(b, es, ep + 3, *r.comment);
        b.word(es, ew + 1) = r.length;                // length64
        if (r.nHashes) {
            const uint64_t m = r.nHashes;
            if (use64) {
                b.alloc(es, ep + 5, m, kList, listUpper(kEight, m), r.hashes);
            } else {
                auto o = b.alloc(es, ep + 4, (m + 1) / 2, kList, listUpper(kFour, m));
                uint32_t *p = reinterpret_cast<uint32_t *>(&b.word(o.first, o.second));
                for (uint64_t j = 0; j < m; j++) p[j] = (uint32_t)r.hashes[j];
            }
            if (writeCounts && r.nCounts) {
                const uint64_t c = r.nCounts;
                auto o = b.alloc(es, ep + 6, (c + 1) / 2, kList, listUpper(kFour, c));
                memcpy(&b.word(o.first, o.second), r.counts, c * 4);
                setBit(b, es, ew, 32, true);
            }
        }
    }
    // locusList with an empty loci list (Sketch.cpp:606-621)
    auto ll = b.alloc(rs, rp + 1, 1, kStruct, structUpper(0, 1));
    auto loci = b.alloc(ll.first, ll.second, 1, kList, listUpper(kComposite, 0));
    b.word(loci.first, loci.second) = kStruct | (structUpper(3, 0) << 32);
    // scalars (Sketch.cpp:623-630)
    setU32(b, rs, rw, 0, h.kmerSize);
    setU32(b, rs, rw, 20, h.hashSeed ^ 42u);
    uint32_t ebits;
    memcpy(&ebits, &h.error, 4);
    setU32(b, rs, rw, 16, ebits);
    setU32(b, rs, rw, 8, h.minHashesPerWindow);
    setU32(b, rs, rw, 4, h.windowSize);
    setBit(b, rs, rw, 96, h.concatenated);
    setBit(b, rs, rw, 97, h.noncanonical);
    setBit(b, rs, rw, 98, h.preserveCase);
    setText(b, rs, rp + 2, h.alphabet);
}

std::vector<MshRefView> viewsOf(const std::vector<MshReference> &refs)
{
    std::vector<MshRefView> v(refs.size());
    for (size_t i = 0; i < refs.size(); i++)
        v[i] = MshRefView{&refs[i].name, &refs[i].comment, refs[i].length, refs[i].hashes.data(),
                          refs[i].hashes.size(), refs[i].counts.data(), refs[i].counts.size()};
    return v;
}

}  // namespace

std::string mshSerialize(const MshHeader &h, const std::vector<MshReference> &refs, bool use64,
                         bool writeCounts)
{
    const std::vector<MshRefView> v = viewsOf(refs);
    Builder b;
    build(b, h, v.data(), v.size(), use64, writeCounts);
    return b.serialize();
}

bool mshWrite(const std::string &path, const MshHeader &h, const MshRefView *refs, uint64_t n,
              bool use64, bool writeCounts)
{
    Builder b;
    build(b, h, refs, n, use64, writeCounts);
    return b.write(path);
}

// ---------------------------------------------------------------------------
// reader
// ---------------------------------------------------------------------------

namespace {

struct Reader {
    const std::string &d;
    std::vector<std::pair<uint64_t, uint64_t>> segs;   // byte offset, words
    std::string err;

    explicit Reader(const std::string &data) : d(data) {}

    bool init()
    {
        if (d.size() < 8) return fail("file too short for a Cap'n Proto message");
        uint32_t n = rd32(0) + 1;
        uint64_t off = 4 + 4ULL * n;
        off += (8 - off % 8) % 8;
        if (n > (1u << 20) || off > d.size()) return fail("bad segment table");
        for (uint32_t i = 0; i < n; i++) {
            uint64_t w = rd32(4 + 4ULL * i);
            segs.push_back({off, w});
            off += 8 * w;
        }
        if (off > d.size()) return fail("truncated message");
        return true;
    }
    bool fail(const std::string &m) { err = m; return false; }
    uint32_t rd32(uint64_t b) const { uint32_t v; memcpy(&v, d.data() + b, 4); return v; }
    uint64_t word(uint64_t s, uint64_t i) const
    {
        if (s >= segs.size() || i >= segs[s].second) return 0;
        uint64_t v;
        memcpy(&v, d.data() + segs[s].first + 8 * i, 8);
        return v;
    }
    uint64_t addr(uint64_t s, uint64_t i) const { return segs[s].first + 8 * i; }

    // resolve pointer at (s, i) -> target (seg, word, tag-pointer); false if null
    bool resolve(uint64_t s, uint64_t i, uint64_t &ts, uint64_t &tw, uint64_t &p) const
    {
        p = word(s, i);
        if (p == 0) return false;
        if ((p & 3) == kFar) {
            const bool dbl = (p >> 2) & 1;
            const uint64_t off = (p >> 3) & 0x1FFFFFFF, seg = p >> 32;
            if (!dbl) {
                return resolve(seg, off, ts, tw, p);
            }
            const uint64_t pad = word(seg, off), tag = word(seg, off + 1);
            ts = pad >> 32;
            tw = (pad >> 3) & 0x1FFFFFFF;
            p = tag;
            return true;
        }
        int64_t o = (int64_t)((p >> 2) & 0x3FFFFFFF);
        if (o & (1 << 29)) o -= (1LL << 30);
        ts = s;
        tw = (uint64_t)((int64_t)i + 1 + o);
        return true;
    }
};

struct SView {
    const Reader *r = nullptr;
    uint64_t s = 0, w = 0, dw = 0, pw = 0;
    bool ok = false;
    uint32_t u32(int byte) const
    {
        if (!ok || (uint64_t)byte + 4 > 8 * dw) return 0;
        return r->rd32(r->addr(s, w) + byte);
    }
    uint64_t u64(int byte) const
    {
        if (!ok || (uint64_t)byte + 8 > 8 * dw) return 0;
        return r->word(s, w + byte / 8);
    }
    bool bit(int b) const
    {
        if (!ok || (uint64_t)b >= 64 * dw) return false;
        return (r->word(s, w + b / 64) >> (b % 64)) & 1;
    }
    uint64_t ptrw(int i) const { return w + dw + i; }
};

SView structAt(const Reader &r, uint64_t s, uint64_t i)
{
    SView v;
    uint64_t ts, tw, p;
    if (!r.resolve(s, i, ts, tw, p) || (p & 3) != kStruct) return v;
    v.r = &r; v.s = ts; v.w = tw; v.dw = (p >> 32) & 0xFFFF; v.pw = p >> 48; v.ok = true;
    return v;
}

SView structPtr(const SView &v, int i)
{
    if (!v.ok || (uint64_t)i >= v.pw) return SView{};
    return structAt(*v.r, v.s, v.ptrw(i));
}

bool listPtr(const SView &v, int i, uint64_t &ls, uint64_t &lw, uint64_t &esz, uint64_t &cnt)
{
    if (!v.ok || (uint64_t)i >= v.pw) return false;
    uint64_t p;
    if (!v.r->resolve(v.s, v.ptrw(i), ls, lw, p) || (p & 3) != kList) return false;
    esz = (p >> 32) & 7;
    cnt = p >> 35;
    return true;
}

std::string text(const SView &v, int i)
{
    uint64_t s, w, esz, n;
    if (!listPtr(v, i, s, w, esz, n) || esz != kByte || n == 0) return "";
    const char *p = v.r->d.data() + v.r->addr(s, w);
    size_t len = n;
    if (p[len - 1] == 0) len--;
    return std::string(p, len);
}

std::vector<SView> structList(const SView &v, int i)
{
    std::vector<SView> out;
    uint64_t s, w, esz, n;
    if (!listPtr(v, i, s, w, esz, n) || esz != kComposite) return out;
    const uint64_t tag = v.r->word(s, w);
    const uint64_t cnt = (tag >> 2) & 0x3FFFFFFF, dw = (tag >> 32) & 0xFFFF, pw = tag >> 48;
    for (uint64_t j = 0; j < cnt; j++) {
        SView e;
        e.r = v.r; e.s = s; e.w = w + 1 + j * (dw + pw); e.dw = dw; e.pw = pw; e.ok = true;
        out.push_back(e);
    }
    return out;
}

}  // namespace

bool mshParse(const std::string &data, MshHeader &h, std::vector<MshReference> *refs,
              bool use64, uint64_t maxHashes, std::string &err)
{
    Reader r(data);
    if (!r.init()) { err = r.err; return false; }
    SView root = structAt(r, 0, 0);
    if (!root.ok) { err = "missing root struct"; return false; }
    h.kmerSize = root.u32(0);
    h.windowSize = root.u32(4);
    h.minHashesPerWindow = root.u32(8);
    h.concatenated = root.bit(96);
    h.noncanonical = root.bit(97);
    h.preserveCase = root.bit(98);
    uint32_t eb = root.u32(16);
    memcpy(&h.error, &eb, 4);
    h.hashSeed = root.u32(20) ^ 42u;
    {
        uint64_t s, w, esz, n;
        h.hasAlphabet = listPtr(root, 2, s, w, esz, n);
        h.alphabet = text(root, 2);
    }
    // referenceList if it has references, else referenceListOld (Sketch.cpp:427, 1088)
    std::vector<SView> list = structList(structPtr(root, 3), 0);
    if (list.empty()) list = structList(structPtr(root, 0), 0);
    h.referenceCount = list.size();
    h.use64 = use64;
    if (!refs) return true;
    refs->clear();
    refs->resize(list.size());
    // references parsed on several threads past a few thousand (C2's 10,000 x 1,000 hashes:
    // 80 MB copied into per-reference vectors)
    const size_t nt = list.size() >= 4096 ? std::max(1u, std::min(8u, std::thread::hardware_concurrency())) : 1;
    auto parse_one = [&](size_t i) {
        const SView &e = list[i];
        MshReference &m = (*refs)[i];
        m.name = text(e, 2);
        m.comment = text(e, 3);
        const uint64_t l64 = e.u64(8);
        m.length = l64 ? l64 : e.u32(0);
        uint64_t s, w, esz, n;
        if (listPtr(e, use64 ? 5 : 4, s, w, esz, n)) {
            const uint64_t take = std::min<uint64_t>(n, maxHashes);
            m.hashes.resize(take);
            const char *base = data.data() + r.addr(s, w);
            if (use64) {
                memcpy(m.hashes.data(), base, take * 8);
            } else {
                for (uint64_t j = 0; j < take; j++) {
                    uint32_t v;
                    memcpy(&v, base + 4 * j, 4);
                    m.hashes[j] = v;
                }
            }
        }
        if (listPtr(e, 6, s, w, esz, n)) {
            const uint64_t take = std::min<uint64_t>(n, m.hashes.size());
            m.counts.resize(take);
            memcpy(m.counts.data(), data.data() + r.addr(s, w), take * 4);
        }
        m.countsSorted = e.bit(32);
    };
    if (nt == 1) {
        for (size_t i = 0; i < list.size(); i++) parse_one(i);
    } else {
        std::vector<std::thread> th;
        for (size_t t = 0; t < nt; t++)
            th.emplace_back([&, t] {
                for (size_t i = list.size() * t / nt; i < list.size() * (t + 1) / nt; i++) parse_one(i);
            });
        for (auto &x : th) x.join();
    }
    return true;
}

}  // namespace fpmhost
