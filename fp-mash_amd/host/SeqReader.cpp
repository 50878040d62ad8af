// SeqReader.cpp — kseq record rules restated (kseq.h:170-208):
//  * skip to the first '>' or '@';
//  * name = bytes up to the first isspace byte; if that byte is not '\n' the
//    comment is the rest of the line (a '\r' of a CRLF file stays in it);
//  * sequence = isgraph bytes until the next '>', '+' or '@' (or EOF);
//  * FASTQ: skip the '+' line, then read quality bytes (33..127) until it is as
//    long as the sequence; one more byte is consumed; shorter quality -> -2;
//  * a 0xff byte reads as end of file in those loops (ks_getc of a signed char buffer).
#include "SeqReader.h"

#include <zlib.h>

#include <cctype>
#include <cstdio>
#include <cstring>
#include <unistd.h>

namespace fpmhost {

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
        fclose(f);
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
