// SeqReader.h — FASTA/FASTQ record reader with kseq's rules (kseq.h:170-208),
// gzip-transparent via zlib (gzopen reads plain files too).  Replaces the
// KSEQ_INIT(gzFile, gzread) reader of Sketch.cpp:38.
#pragma once

#include <zlib.h>

#include <cstdint>
#include <string>

namespace fpmhost {

class SeqReader {
public:
    // path "-" reads stdin
    explicit SeqReader(const std::string &path);
    ~SeqReader();
    bool ok() const { return fp_ != nullptr; }
    // >= 0: sequence length; -1: end of file; -2: truncated quality (kseq_read)
    int read();
    std::string name, comment, seq;

private:
    int getc_();
    gzFile fp_ = nullptr;
    unsigned char buf_[1 << 16];
    int begin_ = 0, end_ = 0;
    bool eof_ = false;
    int last_ = 0;
};

}  // namespace fpmhost
