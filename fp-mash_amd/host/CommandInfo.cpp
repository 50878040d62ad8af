// CommandInfo.cpp — `fpmash info` (CommandInfo.cpp:62-346): header (-H), tabular
// (-t) and JSON dump (-d) of a .msh, in the reference's formats (including the
// fork's non-JSON prefix line before -d output, CommandInfo.cpp:148).
#include "Command.h"
#include "Sketch.h"

#include <algorithm>
#include <iostream>
#include <map>

namespace fpmhost {

static const char *kHash = "MurmurHash3_x64_128";

CommandInfo::CommandInfo()
{
    name = "info";
    summary = "Display information about sketch files.";
    description = "Display information about sketch files.";
    argumentString = "<sketch>";
    useOption("help");
    addOption("header", Option(Option::Boolean, "H", "",
        "Only show header info. Do not list each sketch. Incompatible with -d, -t and -c.", ""));
    addOption("tabular", Option(Option::Boolean, "t", "",
        "Tabular output (rather than padded), with no header. Incompatible with -d, -H and -c.", ""));
    addOption("counts", Option(Option::Boolean, "c", "",
        "Show hash count histograms for each sketch. Incompatible with -d, -H and -t.", ""));
    addOption("dump", Option(Option::Boolean, "d", "",
        "Dump sketches in JSON format. Incompatible with -H, -t, and -c.", ""));
}

int CommandInfo::run() const
{
    if (arguments.size() != 1 || options.at("help").active) {
        print();
        return 0;
    }
    const bool header = options.at("header").active, tabular = options.at("tabular").active;
    const bool counts = options.at("counts").active, dump = options.at("dump").active;
    if (header && tabular) { std::cerr << "ERROR: The options -H and -t are incompatible." << std::endl; return 1; }
    if (header && counts) { std::cerr << "ERROR: The options -H and -c are incompatible." << std::endl; return 1; }
    if (tabular && counts) { std::cerr << "ERROR: The options -t and -c are incompatible." << std::endl; return 1; }
    if (dump) {
        if (tabular) { std::cerr << "ERROR: The options -d and -t are incompatible." << std::endl; return 1; }
        if (header) { std::cerr << "ERROR: The options -d and -H are incompatible." << std::endl; return 1; }
        if (counts) { std::cerr << "ERROR: The options -d and -c are incompatible." << std::endl; return 1; }
    }
    const std::string &file = arguments[0];
    if (!hasSuffix(file, suffixSketch)) {
        std::cerr << "ERROR: The file \"" << file << "\" does not look like a sketch." << std::endl;
        return 1;
    }
    Sketch sketch;
    Parameters params;
    uint64_t referenceCount;
    if (header) referenceCount = sketch.initParametersFromMsh(file);
    else {
        sketch.initFromFiles(arguments, params);
        referenceCount = sketch.getReferenceCount();
    }
    if (counts) {
        // printCounts (CommandInfo.cpp:225-262): per sketch, the histogram of its counts
        if (sketch.getReferenceCount() == 0) {
            std::cerr << "ERROR: Sketch file contains no sketches." << std::endl;
            return 1;
        }
        if (!sketch.hasHashCounts()) {
            std::cerr << "ERROR: Sketch file does not have hash counts. Re-sketch with -M to use "
                         "this feature." << std::endl;
            return 1;
        }
        std::cout << "#Sketch\tBin\tFrequency" << std::endl;
        for (uint64_t i = 0; i < sketch.getReferenceCount(); i++) {
            const Reference &r = sketch.getReference(i);
            std::map<uint32_t, uint64_t> histogram;
            for (uint32_t c : r.counts) histogram[c]++;
            for (auto &e : histogram)
                std::cout << r.name << '\t' << e.first << '\t' << e.second << std::endl;
        }
        return 0;
    }
    std::string alphabet;
    sketch.getAlphabetAsString(alphabet);
    const bool use64 = sketch.getUse64();
    if (dump) {
        std::cout << "      \"Write JSON information : " << std::endl;
        std::cout << "{" << std::endl;
        std::cout << "  \"kmer\" : " << sketch.getKmerSize() << ',' << std::endl;
        std::cout << "  \"alphabet\" : \"" << alphabet << "\"," << std::endl;
        std::cout << "  \"preserveCase\" : " << (sketch.getPreserveCase() ? "true" : "false") << ','
                  << std::endl;
        std::cout << "  \"canonical\" : " << (sketch.getNoncanonical() ? "false" : "true") << ','
                  << std::endl;
        std::cout << "  \"sketchSize\" : " << sketch.getMinHashesPerWindow() << ',' << std::endl;
        std::cout << "  \"hashType\" : \"" << kHash << "\"," << std::endl;
        std::cout << "  \"hashBits\" : " << (use64 ? 64 : 32) << ',' << std::endl;
        std::cout << "  \"hashSeed\" : " << sketch.getHashSeed() << ',' << std::endl;
        std::cout << "  \"sketches\" :" << std::endl << "  [" << std::endl;
        for (uint64_t i = 0; i < sketch.getReferenceCount(); i++) {
            const Reference &r = sketch.getReference(i);
            std::cout << "    {" << std::endl;
            std::cout << "      \"name\" : \"" << r.name << "\"," << std::endl;
            std::cout << "      \"length\" : " << r.length << ',' << std::endl;
            std::cout << "      \"comment\" : \"" << r.comment << "\"," << std::endl;
            std::cout << "      \"hashes\" :" << std::endl << "      [" << std::endl;
            for (size_t j = 0; j < r.hashes.size(); j++) {
                std::cout << "        " << (use64 ? r.hashes[j] : (uint32_t)r.hashes[j]);
                if (j + 1 < r.hashes.size()) std::cout << ',';
                std::cout << std::endl;
            }
            std::cout << "      ]" << std::endl;
            if (r.countsSorted) {
                // no comma after the hashes list (CommandInfo.cpp:310-325): not valid JSON
                std::cout << "      \"counts\" :" << std::endl << "      [" << std::endl;
                for (size_t j = 0; j < r.counts.size(); j++) {
                    std::cout << "        " << r.counts[j];
                    if (j + 1 < r.counts.size()) std::cout << ',';
                    std::cout << std::endl;
                }
                std::cout << "      ]" << std::endl;
            }
            std::cout << (i + 1 < sketch.getReferenceCount() ? "    }," : "    }") << std::endl;
        }
        std::cout << "  ]" << std::endl << "}" << std::endl;
        return 0;
    }
    if (tabular) std::cout << "#Hashes\tLength\tID\tComment" << std::endl;
    else {
        std::cout << "Header:" << std::endl;
        std::cout << "  Hash function (seed):          " << kHash << " (" << sketch.getHashSeed()
                  << ")" << std::endl;
        std::cout << "  K-mer size:                    " << sketch.getKmerSize() << " ("
                  << (use64 ? "64" : "32") << "-bit hashes)" << std::endl;
        std::cout << "  Alphabet:                      " << alphabet
                  << (sketch.getNoncanonical() ? "" : " (canonical)")
                  << (sketch.getPreserveCase() ? " (case-sensitive)" : "") << std::endl;
        std::cout << "  Target min-hashes per sketch:  " << sketch.getMinHashesPerWindow() << std::endl;
        std::cout << "  Sketches:                      " << referenceCount << std::endl;
    }
    if (!header) {
        if (!tabular) std::cout << std::endl << "Sketches:" << std::endl;
        std::vector<std::vector<std::string>> cols(4);
        if (!tabular) { cols[0] = {"[Hashes]"}; cols[1] = {"[Length]"}; cols[2] = {"[ID]"}; cols[3] = {"[Comment]"}; }
        for (uint64_t i = 0; i < sketch.getReferenceCount(); i++) {
            const Reference &r = sketch.getReference(i);
            if (tabular)
                std::cout << r.hashes.size() << '\t' << r.length << '\t' << r.name << '\t'
                          << r.comment << std::endl;
            else {
                cols[0].push_back(std::to_string(r.hashes.size()));
                cols[1].push_back(std::to_string(r.length));
                cols[2].push_back(r.name);
                cols[3].push_back(r.comment);
            }
        }
        if (!tabular) {
            std::vector<size_t> w(4, 0);
            for (int c = 0; c < 4; c++)
                for (auto &s : cols[c]) w[c] = std::max(w[c], s.size());
            for (size_t row = 0; row < cols[0].size(); row++) {
                std::cout << "  ";
                for (int c = 0; c < 4; c++) {
                    std::cout << cols[c][row];
                    if (c < 3) std::cout << std::string(w[c] - cols[c][row].size() + 2, ' ');
                }
                std::cout << std::endl;
            }
        }
    }
    return 0;
}

}  // namespace fpmhost
