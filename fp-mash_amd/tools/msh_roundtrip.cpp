// msh_roundtrip — test tool: parse a .msh (no truncation) and re-serialize it with
// the writer; prints "same" when the bytes are identical.  CPU only.
#include "Msh.h"

#include <cstdio>
#include <unistd.h>
#include <fstream>
#include <iostream>
#include <sstream>

int main(int argc, char **argv)
{
    if (argc < 2) {
        std::cerr << "usage: msh_roundtrip in.msh [out.msh]\n"
                     "       msh_roundtrip --split in.msh out_prefix  (one .msh per sketch)\n";
        return 2;
    }
    const bool split = std::string(argv[1]) == "--split";
    if (split && argc < 4) return 2;
    if (split) { argv++; argc--; }
    std::ifstream in(argv[1], std::ios::binary);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string data = ss.str();
    fpmhost::MshHeader h;
    std::vector<fpmhost::MshReference> r64, r32;
    std::string err;
    if (!fpmhost::mshParse(data, h, &r64, true, ~0ULL, err) ||
        !fpmhost::mshParse(data, h, &r32, false, ~0ULL, err)) { std::cerr << err << "\n"; return 2; }
    bool use64 = false;
    for (auto &r : r64) if (!r.hashes.empty()) use64 = true;
    auto &refs = use64 ? r64 : r32;
    bool counts = false;
    for (auto &r : refs) if (!r.counts.empty()) counts = true;
    if (split) {
        for (size_t i = 0; i < refs.size(); i++) {
            const std::string one = fpmhost::mshSerialize(h, {refs[i]}, use64, counts);
            std::ofstream(std::string(argv[2]) + std::to_string(i) + ".msh", std::ios::binary) << one;
        }
        std::cout << refs.size() << "\n";
        return 0;
    }
    const std::string out = fpmhost::mshSerialize(h, refs, use64, counts);
    // the file writer (hash lists read in place, parallel pwrite) must give the same bytes
    std::vector<fpmhost::MshRefView> views;
    for (auto &r : refs)
        views.push_back(fpmhost::MshRefView{&r.name, &r.comment, r.length, r.hashes.data(),
                                            r.hashes.size(), r.counts.data(), r.counts.size()});
    const std::string path = argc > 2 ? std::string(argv[2]) : "/tmp/msh_roundtrip." + std::to_string(getpid());
    bool fileSame = fpmhost::mshWrite(path, h, views.data(), views.size(), use64, counts);
    if (fileSame) {
        std::ifstream back(path, std::ios::binary);
        std::stringstream bs;
        bs << back.rdbuf();
        fileSame = bs.str() == out;
    }
    if (argc <= 2) std::remove(path.c_str());
    const bool same = out == data && fileSame;
    std::cout << (same ? "same" : "differs") << " " << data.size() << " " << out.size()
              << (fileSame ? "" : " (file writer differs)") << "\n";
    return same ? 0 : 1;
}
