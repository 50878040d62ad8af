// CommandTriangle.cpp — `fpmash triangle` (CommandTriangle.cpp:18-302): lower-triangular
// distance matrix (relaxed Phylip) or edge list of one set of sketches against itself.
// Rows are emitted in the reference's order (row i = sketch i against sketches 0..i-1).
// k-mer sketches: the whole set goes to the device once (fpm_dist with the same buffers,
// which takes the symmetric self-comparison path); -fp: the positional compare of
// compareFingerprints runs on the device (fpm_fp_positional_grid).
#include "Command.h"
#include "Device.h"
#include "Sketch.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <iostream>

namespace fpmhost {

CommandTriangle::CommandTriangle()
{
    name = "triangle";
    summary = "Estimate a lower-triangular distance matrix.";
    description = "Estimate the distance of each input sequence or fingerprint to every other "
                  "input. Outputs a lower-triangular distance matrix in relaxed Phylip format. "
                  "The input sequences can be fasta or fastq, gzipped or not, or Mash sketch "
                  "files (.msh) with matching k-mer sizes. Input files can also be files of file "
                  "names (see -l). If more than one input file is provided, whole files are "
                  "compared by default (see -i).";
    argumentString = "<seq1> [<seq2>] ...";
    useOption("help");
    addOption("list", Option(Option::Boolean, "l", "Input",
        "List input. Lines in each <query> specify paths to sequence files, one per line. The "
        "reference file is not affected.", ""));
    addOption("comment", Option(Option::Boolean, "C", "Output",
        "Use comment fields for sequence names instead of IDs.", ""));
    addOption("edge", Option(Option::Boolean, "E", "Output",
        "Output edge list instead of Phylip matrix, with fields [seq1, seq2, dist, p-val, "
        "shared-hashes].", ""));
    addOption("pvalue", Option(Option::Number, "v", "Output",
        "Maximum p-value to report in edge list. Implies -E.", "1.0", 0., 1.));
    addOption("distance", Option(Option::Number, "d", "Output",
        "Maximum distance to report in edge list. Implies -E.", "1.0", 0., 1.));
    addOption("fingerprint", Option(Option::Boolean, "fp", "Input",
        "Indicates that the input files are fingerprints instead of sequences.", ""));
    useSketchOptions();
}

// containsExtensionMSH / TXT (CommandTriangle.cpp:...): substring test on the last file
static bool containsSub(const std::vector<std::string> &v, const char *s)
{
    bool f = false;
    for (const auto &x : v) f = x.find(s) != std::string::npos;
    return f;
}

static void putNum(std::string &o, double x)   // ostream default: %g, precision 6
{
    char t[64];
    const int n = snprintf(t, sizeof t, "%g", x);
    o.append(t, n);
}

int CommandTriangle::run() const
{
    if (arguments.empty() || options.at("help").active) {
        print();
        return 0;
    }
    warmDevices();
    const bool list = options.at("list").active;
    const bool comment = options.at("comment").active;
    bool edge = options.at("edge").active;
    const bool fingerprint = options.at("fingerprint").active;
    const double pValueMax = options.at("pvalue").getArgumentAsNumber();
    const double distanceMax = options.at("distance").getArgumentAsNumber();
    double pValuePeak = 0;
    if (options.at("pvalue").active || options.at("distance").active) edge = true;

    Parameters parameters;
    if (sketchParameterSetup(parameters, *this)) return 1;
    if (arguments.size() == 1 && !list) parameters.concatenated = false;

    std::vector<std::string> files;
    for (const auto &a : arguments) {
        if (list) splitFile(a, files);
        else files.push_back(a);
    }
    Sketch sketch;
    if (fingerprint && containsSub(files, ".msh")) sketch.initFromFiles(files, parameters);
    else if (fingerprint) sketch.initFromFingerprints(files, parameters);
    else sketch.initFromFiles(files, parameters);

    const uint64_t n = sketch.getReferenceCount();
    uint64_t lengthMax = 0;
    double randomChance = 0;
    int kMin = 0, warningCount = 0;
    std::string lengthMaxName;
    const double lengthThreshold =
        (parameters.warning * sketch.getKmerSpace()) / (1. - parameters.warning);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t length = sketch.getReference(i).length;
        if (length > lengthThreshold) {
            if (warningCount == 0 || length > lengthMax) {
                lengthMax = length;
                lengthMaxName = sketch.getReference(i).name;
                randomChance = sketch.getRandomKmerChance(i);
                kMin = sketch.getMinKmerSize(i);
            }
            warningCount++;
        }
    }
    auto label = [&](uint64_t i) -> const std::string & {
        return comment ? sketch.getReference(i).comment : sketch.getReference(i).name;
    };
    std::string out;
    if (!edge) {
        out += '\t';
        out += std::to_string(n);
        out += '\n';
        if (n) { out += label(0); out += '\n'; }
    }
    if (n > 1) {
        // the whole set as one dense matrix; row block [q0, q1) x all refs per device call
        const bool use64 = sketch.getUse64();
        const uint32_t hb = use64 ? 8 : 4;
        uint64_t width = 1;
        for (uint64_t i = 0; i < n; i++) width = std::max<uint64_t>(width, sketch.getReference(i).hashes.size());
        std::vector<uint8_t> M(n * width * hb, 0);
        std::vector<uint32_t> len(n);
        std::vector<uint64_t> L(n);
        for (uint64_t i = 0; i < n; i++) {
            const Reference &r = sketch.getReference(i);
            len[i] = (uint32_t)r.hashes.size();
            L[i] = r.length;
            for (uint64_t j = 0; j < r.hashes.size(); j++) {
                if (use64) memcpy(&M[(i * width + j) * 8], &r.hashes[j], 8);
                else { const uint32_t v = (uint32_t)r.hashes[j]; memcpy(&M[(i * width + j) * 4], &v, 4); }
            }
        }
        const uint64_t sketchSize = (uint64_t)sketch.getMinHashesPerWindow();
        std::vector<uint32_t> nu(n * n), de(n * n);
        std::vector<double> di(n * n), pv(n * n);
        std::vector<uint8_t> pa(n * n);
        if (fingerprint)
            check(fpm_fp_positional_grid(device(), M.data(), len.data(), width, (uint32_t)n,
                                         M.data(), len.data(), width, (uint32_t)n, hb, distanceMax,
                                         pValueMax, nu.data(), de.data(), di.data(), pv.data(),
                                         pa.data()),
                  "triangle");
        else
            check(fpm_dist(device(), M.data(), len.data(), L.data(), width, (uint32_t)n, M.data(),
                           len.data(), L.data(), width, (uint32_t)n, hb, (uint32_t)sketchSize,
                           (uint32_t)sketch.getKmerSize(), sketch.getKmerSpace(), distanceMax,
                           pValueMax, nu.data(), de.data(), di.data(), pv.data(), pa.data()),
                  "triangle");
        // writeOutput (CommandTriangle.cpp:200-240): row i vs 0..i-1; compareSketches gets
        // (ref i, ref j), i.e. grid cell query i, ref j
        for (uint64_t i = 1; i < n; i++) {
            if (!edge) out += label(i);
            for (uint64_t j = 0; j < i; j++) {
                const uint64_t k = i * n + j;
                if (edge) {
                    if (pa[k]) {
                        out += label(i); out += '\t'; out += label(j); out += '\t';
                        putNum(out, di[k]); out += '\t'; putNum(out, pv[k]); out += '\t';
                        out += std::to_string(nu[k]); out += '/'; out += std::to_string(de[k]);
                        out += '\n';
                    }
                } else {
                    out += '\t';
                    putNum(out, di[k]);
                }
                if (pv[k] > pValuePeak) pValuePeak = pv[k];
            }
            if (!edge) out += '\n';
            if (out.size() > (1 << 22)) { fwrite(out.data(), 1, out.size(), stdout); out.clear(); }
        }
    }
    fwrite(out.data(), 1, out.size(), stdout);
    fflush(stdout);
    if (!edge) std::cerr << "Max p-value: " << pValuePeak << std::endl;
    if (warningCount > 0 && !parameters.reads)
        warnKmerSize(parameters, *this, lengthMax, lengthMaxName, randomChance, kMin, warningCount);
    return 0;
}

}  // namespace fpmhost
