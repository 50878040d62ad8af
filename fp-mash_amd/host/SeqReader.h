// SeqReader.h — FASTA/FASTQ input for sketching.
//
// loadSequenceFile: the whole (inflated) file image — gzip-transparent like the reference's
// gzopen / gzread stream (KSEQ_INIT(gzFile, gzread), Sketch.cpp:38); "-" reads stdin.
// The image normally goes to the device parser (fpm_seq_parse, csrc/seqparse.hip); SeqReader
// walks an image on the host with kseq's record rules (kseq.h:170-208) for the inputs the
// device parser hands back (FASTQ quality lines).
#pragma once

#include <cstdint>
#include <string>

namespace fpmhost {

// false if the file cannot be opened or is a corrupt gzip stream
bool loadSequenceFile(const std::string &path, std::string &image);

class SeqReader {
public:
    SeqReader(const char *data, size_t n) : p_((const unsigned char *)data), n_(n) {}
    // >= 0: sequence length; -1: end of file; -2: truncated quality (kseq_read)
    int read();
    std::string name, comment, seq;

private:
    // ks_getc: (int) of a `char` buffer byte, so 0xff reads as -1 (end of file) on x86; it is
    // consumed and the stream goes on (kseq.h:66-76)
    int getc_()
    {
        if (i_ >= n_) return -1;
        const int c = p_[i_++];
        return c == 0xff ? -1 : c;
    }
    // ks_getuntil's direct buffer scan (name / comment): every byte is data
    int raw_() { return i_ < n_ ? p_[i_++] : -1; }
    const unsigned char *p_;
    size_t n_, i_ = 0;
    int last_ = 0;
};

// kseq's header split of one header line (the bytes after '>' / '@' up to its '\n'): name =
// up to the first isspace byte; if that byte is not '\n' (here: the line continues) the
// comment is the rest of the line (kseq.h:179-180).
void splitHeader(const char *line, size_t n, std::string &name, std::string &comment);

}  // namespace fpmhost
