// SeqReader.cpp — kseq record rules restated (kseq.h:170-208):
//  * skip to the first '>' or '@';
//  * name = bytes up to the first isspace byte; if that byte is not '\n' the
//    comment is the rest of the line (a '\r' of a CRLF file stays in it);
//  * sequence = isgraph bytes until the next '>', '+' or '@' (or EOF);
//  * FASTQ: skip the '+' line, then read quality bytes (33..127) until it is as
//    long as the sequence; one more byte is consumed; shorter quality -> -2;
//  * a 0xff byte reads as end of file in those loops (ks_getc of a signed char buffer).
#include "SeqReader.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <new>
#include <thread>
#include <unistd.h>
#include <vector>

namespace fpmhost {

namespace {

// libdeflate (the image's /lib/x86_64-linux-gnu/libdeflate.so.0; no header in the image, so
// the four entry points are declared here and resolved with dlopen): whole-buffer gzip
// member decoding, ~2-3x zlib's inflate on one thread.  Absent library: zlib's gzread.
enum { kLdOk = 0, kLdBadData = 1, kLdShortOutput = 2, kLdInsufficientSpace = 3 };
struct Deflate {
    void *(*alloc)() = nullptr;
    void (*free_)(void *) = nullptr;
    int (*gunzip_ex)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
    bool ok = false;
    Deflate()
    {
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        free_ = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        gunzip_ex = (int (*)(void *, const void *, size_t, void *, size_t, size_t *, size_t *))
            dlsym(h, "libdeflate_gzip_decompress_ex");
        ok = alloc && free_ && gunzip_ex;
    }
};
const Deflate &deflate()
{
    static const Deflate d;
    return d;
}

inline bool gzipMagic(const unsigned char *p, size_t n) { return n >= 2 && p[0] == 0x1f && p[1] == 0x8b; }

// BGZF (blocked gzip, SAM spec §4.1): every member carries its compressed size in a "BC"
// extra subfield, so the members can be found without inflating and inflated in parallel.
// Returns the member boundaries, or empty when the stream is not BGZF throughout.
std::vector<std::pair<size_t, size_t>> bgzfMembers(const unsigned char *p, size_t n)
{
    std::vector<std::pair<size_t, size_t>> m;
    size_t at = 0;
    while (at < n) {
        if (n - at < 18 || !gzipMagic(p + at, n - at) || p[at + 2] != 8 || !(p[at + 3] & 4)) break;
        const size_t xlen = p[at + 10] | (size_t)p[at + 11] << 8;
        size_t bsize = 0;
        for (size_t x = at + 12; x + 4 <= at + 12 + xlen && x + 4 <= n;) {
            const size_t slen = p[x + 2] | (size_t)p[x + 3] << 8;
            if (p[x] == 'B' && p[x + 1] == 'C' && slen == 2 && x + 6 <= n) {
                bsize = (p[x + 4] | (size_t)p[x + 5] << 8) + 1;
                break;
            }
            x += 4 + slen;
        }
        // a member is at least its 18-byte header + an empty deflate block + the 8-byte trailer,
        // and inflates to at most 64 KiB (SAM spec 4.1): anything else is no BGZF member
        if (bsize < 28 || at + bsize > n) break;
        const unsigned char *t = p + at + bsize - 4;
        if ((t[0] | (size_t)t[1] << 8 | (size_t)t[2] << 16 | (size_t)t[3] << 24) > 65536) break;
        m.push_back({at, bsize});
        at += bsize;
    }
    // a stream that is not BGZF throughout (or has trailing bytes that are no member) takes
    // the sequential path, whose member loop reproduces gzread's treatment of the tail
    if (at != n) m.clear();
    return m;
}

// One gzip member at in[0 .. n) appended to out; *used = its compressed bytes.
bool gunzipMember(void *dec, const unsigned char *in, size_t n, std::string &out, size_t hint,
                  size_t *used)
{
    const Deflate &D = deflate();
    size_t room = std::max<size_t>(hint, std::max<size_t>(n * 4, 1 << 16));
    for (;;) {
        const size_t base = out.size();
        out.resize(base + room);
        size_t in_used = 0, got = 0;
        const int r = D.gunzip_ex(dec, in, n, &out[base], room, &in_used, &got);
        if (r == kLdOk) {
            out.resize(base + got);
            *used = in_used;
            return true;
        }
        out.resize(base);
        if (r != kLdInsufficientSpace) return false;
        room *= 2;
    }
}

// The whole compressed image inflated like gzread: gzip members one after the other; bytes
// after a member that are not a gzip header end the stream (gz_look leaves them unread).
// BGZF members are inflated on several threads.
bool gunzipImage(const unsigned char *p, size_t n, std::string &image)
{
    const Deflate &D = deflate();
    const auto mem = bgzfMembers(p, n);
    try {
    if (mem.size() >= 8) {
        // every BGZF member inflates to at most 64 KiB: slots of ISIZE (its last 4 bytes)
        std::vector<size_t> off(mem.size() + 1, 0);
        for (size_t i = 0; i < mem.size(); i++) {
            const unsigned char *t = p + mem[i].first + mem[i].second - 4;
            off[i + 1] = off[i] + (t[0] | (size_t)t[1] << 8 | (size_t)t[2] << 16 | (size_t)t[3] << 24);
        }
        image.resize(off.back());
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; t++)
            th.emplace_back([&] {
                void *dec = D.alloc();
                if (!dec) { bad = true; return; }
                for (size_t i; !bad && (i = next.fetch_add(1)) < mem.size();) {
                    size_t in_used = 0, got = 0;
                    const size_t want = off[i + 1] - off[i];
                    const int r = D.gunzip_ex(dec, p + mem[i].first, mem[i].second,
                                              want ? &image[off[i]] : nullptr, want, &in_used, &got);
                    if (r != kLdOk || got != want) bad = true;
                }
                D.free_(dec);
            });
        for (auto &x : th) x.join();
        return !bad;
    }
    void *dec = D.alloc();
    if (!dec) return false;
    // released on every path out, the bad_alloc below included
    struct DecGuard {
        const Deflate &lib; void *d;
        ~DecGuard() { lib.free_(d); }
    } guard{D, dec};
    image.clear();
    size_t at = 0;
    bool ok = true;
    while (at < n && gzipMagic(p + at, n - at)) {
        size_t used = 0;
        // ISIZE of a single-member file sizes the output in one go
        size_t hint = 0;
        if (at == 0 && n >= 4)
            hint = p[n - 4] | (size_t)p[n - 3] << 8 | (size_t)p[n - 2] << 16 | (size_t)p[n - 1] << 24;
        // (a corrupt ISIZE must not size the output: deflate expands at most ~1032:1)
        hint = std::min(hint, n * 1032);
        if (!gunzipMember(dec, p + at, n - at, image, hint + 1, &used)) { ok = false; break; }
        at += used;
    }
    return ok;
    } catch (const std::bad_alloc &) {
        // (the caller falls back to zlib's gzread, which grows the image as it inflates)
        image.clear();
        image.shrink_to_fit();
        return false;
    }
}

}  // namespace

bool loadSequenceFile(const std::string &path, std::string &image)
{
    image.clear();
    const bool in = path == "-";
    FILE *f = in ? nullptr : fopen(path.c_str(), "rb");
    if (!in && !f) return false;
    unsigned char magic[2] = {0, 0};
    size_t nm = 0;
    if (f) {
        nm = fread(magic, 1, 2, f);
        if (!(nm == 2 && magic[0] == 0x1f && magic[1] == 0x8b)) {
            // plain file: one sized read
            if (fseeko(f, 0, SEEK_END) == 0) {
                const off_t sz = ftello(f);
                if (sz > 0 && fseeko(f, 0, SEEK_SET) == 0) {
                    image.resize((size_t)sz);
                    image.resize(fread(&image[0], 1, (size_t)sz, f));
                }
            }
            char buf[1 << 16];
            for (size_t r; (r = fread(buf, 1, sizeof(buf), f)) > 0;) image.append(buf, r);
            fclose(f);
            return true;
        }
        // a gzip file: the compressed image in one read, inflated by libdeflate (BGZF members
        // on several threads)
        if (deflate().ok && fseeko(f, 0, SEEK_END) == 0) {
            const off_t sz = ftello(f);
            std::string z;
            if (sz > 0 && fseeko(f, 0, SEEK_SET) == 0) {
                z.resize((size_t)sz);
                z.resize(fread(&z[0], 1, (size_t)sz, f));
            }
            fclose(f);
            f = nullptr;
            if (z.size() == (size_t)sz &&
                gunzipImage((const unsigned char *)z.data(), z.size(), image))
                return true;
            // a stream libdeflate refuses (a truncated or corrupt member): zlib's gzread below,
            // which hands back what it could inflate and ends there, as the reference reads it
        }
        if (f) fclose(f);
    }
    // gzip (or stdin, gzip or not): zlib's transparent reader, as the reference's gzread
    gzFile gz = in ? gzdopen(dup(fileno(stdin)), "r") : gzopen(path.c_str(), "r");
    if (!gz) return false;
    gzbuffer(gz, 1 << 18);
    size_t cap = 1 << 22;
    image.resize(cap);
    size_t len = 0;
    for (;;) {
        if (len == cap) image.resize(cap *= 2);
        const int r = gzread(gz, &image[len], (unsigned)std::min<size_t>(cap - len, 1u << 30));
        if (r < 0) { gzclose(gz); return false; }
        if (r == 0) break;
        len += (size_t)r;
    }
    gzclose(gz);
    image.resize(len);
    return true;
}

void splitHeader(const char *line, size_t n, std::string &name, std::string &comment)
{
    size_t i = 0;
    while (i < n && !isspace((unsigned char)line[i])) i++;
    name.assign(line, i);
    if (i < n && line[i] != '\n') comment.assign(line + i + 1, n - i - 1);
    else comment.clear();
}

int SeqReader::read()
{
    int c;
    if (last_ == 0) {
        while ((c = getc_()) != -1 && c != '>' && c != '@') {}
        if (c == -1) return -1;
        last_ = c;
    }
    name.clear();
    comment.clear();
    seq.clear();
    // name: up to isspace (ks_getuntil KS_SEP_SPACE: -1 only when the stream is at its end)
    if (i_ >= n_) return -1;
    while ((c = raw_()) != -1 && !isspace(c)) name.push_back((char)c);
    if (c != '\n' && c != -1) {
        while ((c = raw_()) != -1 && c != '\n') comment.push_back((char)c);
    }
    while ((c = getc_()) != -1 && c != '>' && c != '+' && c != '@')
        if (isgraph(c)) seq.push_back((char)c);
    // at a -1 (end of file, or a 0xff byte) last_char keeps this record's marker: the next
    // read takes the bytes after it as a header, as kseq_read does
    if (c == '>' || c == '@') last_ = c;
    if (c != '+') return (int)seq.size();
    while ((c = getc_()) != -1 && c != '\n') {}
    if (c == -1) return -2;
    size_t q = 0;
    while ((c = getc_()) != -1 && q < seq.size())
        if (c >= 33 && c <= 127) q++;
    last_ = 0;
    if (q != seq.size()) return -2;
    return (int)seq.size();
}

}  // namespace fpmhost
