// seqload — writes the inflated image of a sequence file as `fpmash sketch` loads it
// (host/SeqReader.cpp: loadSequenceFile: plain, gzip through libdeflate with BGZF members
// inflated on several threads, or zlib's gzread) to stdout; exit 1 when it cannot be read.
// CPU-only helper for tests/test_cli.py.
#include "SeqReader.h"

#include <cstdio>
#include <string>

int main(int argc, char **argv)
{
    if (argc != 2) {
        fprintf(stderr, "usage: seqload FILE\n");
        return 2;
    }
    std::string image;
    if (!fpmhost::loadSequenceFile(argv[1], image)) return 1;
    fwrite(image.data(), 1, image.size(), stdout);
    return 0;
}
