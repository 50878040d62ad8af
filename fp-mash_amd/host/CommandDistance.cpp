// CommandDistance.cpp — `fpmash dist` (CommandDistance.cpp:38-333): same inputs
// (.msh, sequence files, -fp .txt / .msh), same messages, same ordered text
// output.  The shared-hash walk, distance and p-value of every ref x query pair
// run on the MI355X (fpm_dist); the host formats the lines in query-major order.
#include "Command.h"
#include "Device.h"
#include "Sketch.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <iostream>

namespace fpmhost {

CommandDistance::CommandDistance()
{
    name = "dist";
    summary = "Estimate the distance of query sequences to references.";
    description = "Estimate the distance of each query sequence to the reference. Both the "
                  "reference and queries can be fasta or fastq, gzipped or not, or Mash sketch "
                  "files (.msh) with matching k-mer sizes, or (-fp) k-finger fingerprint files. "
                  "The output fields are [reference-ID, query-ID, distance, p-value, "
                  "shared-hashes].";
    argumentString = "<reference> <query> [<query>] ...";
    useOption("help");
    addOption("list", Option(Option::Boolean, "l", "Input",
        "List input. Lines in each <query> specify paths to sequence files, one per line. The "
        "reference file is not affected.", ""));
    addOption("table", Option(Option::Boolean, "t", "Output",
        "Table output (will not report p-values, but fields will be blank if they do not meet "
        "the p-value threshold).", ""));
    addOption("pvalue", Option(Option::Number, "v", "Output", "Maximum p-value to report.",
                               "1.0", 0., 1.));
    addOption("distance", Option(Option::Number, "d", "Output", "Maximum distance to report.",
                                 "1.0", 0., 1.));
    addOption("comment", Option(Option::Boolean, "C", "Output",
        "Show comment fields with reference/query names (denoted with ':').", "1.0", 0., 1.));
    addOption("fingerprint", Option(Option::Boolean, "fp", "Input",
        "Indicates that the input files are fingerprints instead of sequences.", ""));
    useSketchOptions();
}

// containsMSH / containsTXT (CommandDistance.cpp:454-476): substring test on the last file
static bool containsSub(const std::vector<std::string> &v, const char *s)
{
    bool f = false;
    for (const auto &x : v) f = x.find(s) != std::string::npos;
    return f;
}

namespace {

struct Out {
    std::string buf;
    void flush() { fwrite(buf.data(), 1, buf.size(), stdout); buf.clear(); }
    void put(const std::string &s) { buf += s; if (buf.size() > (1 << 22)) flush(); }
    void put(char c) { buf.push_back(c); }
    void num(double x)   // ostream default: %g, precision 6
    {
        char t[64];
        int n = snprintf(t, sizeof t, "%g", x);
        buf.append(t, n);
    }
    void u(uint64_t x)
    {
        char t[32];
        int n = snprintf(t, sizeof t, "%llu", (unsigned long long)x);
        buf.append(t, n);
    }
};

}  // namespace

int CommandDistance::run() const
{
    if (arguments.size() < 2 || options.at("help").active) {
        print();
        return 0;
    }
    const bool list = options.at("list").active;
    const bool table = options.at("table").active;
    const bool comment = options.at("comment").active;
    const double pValueMax = options.at("pvalue").getArgumentAsNumber();
    const double distanceMax = options.at("distance").getArgumentAsNumber();
    const bool fingerprint = options.at("fingerprint").active;
    Parameters parameters;
    if (sketchParameterSetup(parameters, *this)) return 1;

    Sketch sketchRef;
    uint64_t lengthMax = 0;
    double randomChance = 0;
    int kMin = 0;
    std::string lengthMaxName;
    int warningCount = 0;
    const std::string &fileReference = arguments[0];
    const bool isSketch = hasSuffix(fileReference, suffixSketch);
    if (isSketch) {
        for (const char *o : {"kmer", "noncanonical", "protein", "alphabet"})
            if (options.at(o).active) {
                std::cerr << "ERROR: The option -" << options.at(o).identifier
                          << " cannot be used when a sketch is provided; it is inherited from the "
                             "sketch." << std::endl;
                return 1;
            }
    } else {
        std::cerr << "Sketching " << fileReference
                  << " (provide sketch file made with \"mash sketch\" to skip)...";
    }
    std::vector<std::string> refArg{fileReference};
    const bool tagMSH = containsSub(refArg, ".msh"), tagTXT = containsSub(refArg, ".txt");
    if (fingerprint && tagMSH) sketchRef.initFromFiles(refArg, parameters);
    else if (fingerprint && tagTXT) sketchRef.initFromFingerprints(refArg, parameters);
    else sketchRef.initFromFiles(refArg, parameters);

    const double lengthThreshold =
        (parameters.warning * sketchRef.getKmerSpace()) / (1. - parameters.warning);
    if (isSketch) {
        parameters.minHashesPerWindow = (uint64_t)sketchRef.getMinHashesPerWindow();
        parameters.kmerSize = sketchRef.getKmerSize();
        parameters.noncanonical = sketchRef.getNoncanonical();
        parameters.preserveCase = sketchRef.getPreserveCase();
        parameters.seed = sketchRef.getHashSeed();
        std::string alphabet;
        sketchRef.getAlphabetAsString(alphabet);
        setAlphabetFromString(parameters, alphabet.c_str());
    } else {
        for (uint64_t i = 0; i < sketchRef.getReferenceCount(); i++) {
            const uint64_t length = sketchRef.getReference(i).length;
            if (length > lengthThreshold) {
                if (warningCount == 0 || length > lengthMax) {
                    lengthMax = length;
                    lengthMaxName = sketchRef.getReference(i).name;
                    randomChance = sketchRef.getRandomKmerChance(i);
                    kMin = sketchRef.getMinKmerSize(i);
                }
                warningCount++;
            }
        }
        std::cerr << "done.\n";
    }
    Out out;
    if (table) {
        out.put("#query");
        for (uint64_t i = 0; i < sketchRef.getReferenceCount(); i++) {
            out.put('\t');
            out.put(sketchRef.getReference(i).name);
        }
        out.put('\n');
        out.flush();
        fflush(stdout);
    }
    std::vector<std::string> queryFiles;
    for (size_t i = 1; i < arguments.size(); i++) {
        if (list) splitFile(arguments[i], queryFiles);
        else queryFiles.push_back(arguments[i]);
    }
    Sketch sketchQuery;
    if (fingerprint && tagMSH) sketchQuery.initFromFiles(queryFiles, parameters);
    else if (fingerprint && tagTXT) sketchQuery.initFromFingerprints(queryFiles, parameters);
    else sketchQuery.initFromFiles(queryFiles, parameters, 0, true);

    const uint64_t nR = sketchRef.getReferenceCount(), nQ = sketchQuery.getReferenceCount();
    const uint64_t sketchSize = (uint64_t)std::min(sketchQuery.getMinHashesPerWindow(),
                                                   sketchRef.getMinHashesPerWindow());
    const bool use64 = sketchRef.getUse64();
    const uint32_t hb = use64 ? 8 : 4;
    // dense device layout: one row per sketch
    auto pack = [&](const Sketch &sk, std::vector<uint8_t> &m, std::vector<uint32_t> &len,
                    std::vector<uint64_t> &L, uint64_t width) {
        const uint64_t n = sk.getReferenceCount();
        m.assign(std::max<uint64_t>(1, n * width) * hb, 0);
        len.resize(n);
        L.resize(n);
        for (uint64_t i = 0; i < n; i++) {
            const Reference &r = sk.getReference(i);
            len[i] = (uint32_t)r.hashes.size();
            L[i] = r.length;
            for (uint64_t j = 0; j < r.hashes.size(); j++) {
                if (use64) memcpy(&m[(i * width + j) * 8], &r.hashes[j], 8);
                else { uint32_t v = (uint32_t)r.hashes[j]; memcpy(&m[(i * width + j) * 4], &v, 4); }
            }
        }
    };
    uint64_t width = 1;
    for (uint64_t i = 0; i < nR; i++) width = std::max<uint64_t>(width, sketchRef.getReference(i).hashes.size());
    for (uint64_t i = 0; i < nQ; i++) width = std::max<uint64_t>(width, sketchQuery.getReference(i).hashes.size());
    std::vector<uint8_t> R, Q;
    std::vector<uint32_t> rl, ql;
    std::vector<uint64_t> rL, qL;
    pack(sketchRef, R, rl, rL, width);
    pack(sketchQuery, Q, ql, qL, width);

    // query blocks bound the host buffers (~64 M pairs per block)
    const uint64_t block = nR ? std::max<uint64_t>(1, (64ULL << 20) / nR) : 1;
    std::vector<uint32_t> nu, de;
    std::vector<double> di, pv;
    std::vector<uint8_t> pa;
    for (uint64_t q0 = 0; q0 < nQ && nR; q0 += block) {
        const uint64_t nq = std::min(block, nQ - q0);
        const uint64_t np = nq * nR;
        nu.resize(np); de.resize(np); di.resize(np); pv.resize(np); pa.resize(np);
        check(fpm_dist(device(), R.data(), rl.data(), rL.data(), width, (uint32_t)nR,
                       Q.data() + q0 * width * hb, ql.data() + q0, qL.data() + q0, width,
                       (uint32_t)nq, hb, (uint32_t)sketchSize, (uint32_t)sketchRef.getKmerSize(),
                       sketchRef.getKmerSpace(), distanceMax, pValueMax, nu.data(), de.data(),
                       di.data(), pv.data(), pa.data()),
              "dist");
        // writeOutput (CommandDistance.cpp:276-333), query-major
        for (uint64_t qi = 0; qi < nq; qi++) {
            const Reference &qr = sketchQuery.getReference(q0 + qi);
            if (table) out.put(qr.name);
            for (uint64_t j = 0; j < nR; j++) {
                const uint64_t k = qi * nR + j;
                if (table) {
                    out.put('\t');
                    if (pa[k]) out.num(di[k]);
                } else if (pa[k]) {
                    const Reference &rr = sketchRef.getReference(j);
                    out.put(rr.name);
                    if (comment) { out.put(':'); out.put(rr.comment); }
                    out.put('\t');
                    out.put(qr.name);
                    if (comment) { out.put(':'); out.put(qr.comment); }
                    out.put('\t');
                    out.num(di[k]);
                    out.put('\t');
                    out.num(pv[k]);
                    out.put('\t');
                    out.u(nu[k]);
                    out.put('/');
                    out.u(de[k]);
                    out.put('\n');
                }
            }
            if (table) out.put('\n');
        }
    }
    out.flush();
    fflush(stdout);
    if (warningCount > 0 && !parameters.reads)
        warnKmerSize(parameters, *this, lengthMax, lengthMaxName, randomChance, kMin, warningCount);
    return 0;
}

}  // namespace fpmhost
