// SeqReader.cpp — kseq record rules restated (kseq.h:170-208):
//  * skip to the first '>' or '@';
//  * name = bytes up to the first isspace byte; if that byte is not '\n' the
//    comment is the rest of the line (a '\r' of a CRLF file stays in it);
//  * sequence = isgraph bytes until the next '>', '+' or '@' (or EOF);
//  * FASTQ: skip the '+' line, then read quality bytes (33..127) until it is as
//    long as the sequence; one more byte is consumed; shorter quality -> -2.
#include "SeqReader.h"

#include <cctype>
#include <cstdio>
#include <unistd.h>

namespace fpmhost {

SeqReader::SeqReader(const std::string &path)
{
    fp_ = path == "-" ? gzdopen(dup(fileno(stdin)), "r") : gzopen(path.c_str(), "r");
    if (fp_) gzbuffer(fp_, 1 << 17);
}

SeqReader::~SeqReader()
{
    if (fp_) gzclose(fp_);
}

int SeqReader::getc_()
{
    if (begin_ >= end_) {
        if (eof_) return -1;
        end_ = gzread(fp_, buf_, sizeof(buf_));
        begin_ = 0;
        if (end_ < (int)sizeof(buf_)) eof_ = true;
        if (end_ <= 0) { end_ = 0; return -1; }
    }
    return buf_[begin_++];
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
    // name: up to isspace (ks_getuntil KS_SEP_SPACE)
    bool any = false;
    while ((c = getc_()) != -1 && !isspace(c)) { name.push_back((char)c); any = true; }
    if (c == -1 && !any) return -1;
    if (c != '\n' && c != -1) {
        while ((c = getc_()) != -1 && c != '\n') comment.push_back((char)c);
    }
    while ((c = getc_()) != -1 && c != '>' && c != '+' && c != '@')
        if (isgraph(c)) seq.push_back((char)c);
    if (c == '>' || c == '@') last_ = c;
    if (c != '+') {
        if (c == -1) last_ = 0;
        return (int)seq.size();
    }
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
