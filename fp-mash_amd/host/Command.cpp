// Command.cpp — option registry and argv parsing with the reference's semantics
// (Command.cpp:31-427): numbers parse with stof (float precision, as the reference),
// ranges and integer-ness are checked, Size accepts k/M/G/T suffixes, unknown
// options are an error, everything that is not an option is an argument.
#include "Command.h"

#include "Sketch.h"

#include <cstdint>
#include <cstdio>
#include <iostream>
#include <sstream>

namespace fpmhost {

static const char *kVersion = "2.3";   // the reference's SOFTWARE_VERSION (version.h:8)

Command::Option::Option(Type t, const std::string &id, const std::string &cat,
                        const std::string &desc, const std::string &def, double mn, double mx)
    : type(t), identifier(id), category(cat), description(desc), argumentDefault(def),
      argumentMin(mn), argumentMax(mx)
{
    setArgument(def);
}

static double g_num_dummy;

void Command::Option::setArgument(const std::string &a)
{
    argument = a;
    (void)g_num_dummy;
    if (type == Number || type == Integer) {
        if (argument.empty()) return;
        bool failed = false;
        double v = 0;
        try {
            v = std::stof(argument);
            if (argumentMin != argumentMax && (v < argumentMin || v > argumentMax)) failed = true;
            else if (type == Integer && (double)(uint64_t)v != v) failed = true;
        } catch (const std::exception &) {
            failed = true;
        }
        if (failed) {
            std::cerr << "ERROR: Argument to -" << identifier << " must be a"
                      << (type == Integer ? "n integer" : " number");
            if (argumentMin != argumentMax)
                std::cerr << " between " << argumentMin << " and " << argumentMax;
            std::cerr << " (" << argument << " given)" << std::endl;
            exit(1);
        }
    } else if (type == Size) {
        if (argument.empty()) return;
        char suffix = argument.back();
        uint64_t factor = 1;
        std::string body = argument;
        if (suffix < '0' || suffix > '9') {
            switch (suffix) {
            case 'k': case 'K': factor = 1000ULL; break;
            case 'm': case 'M': factor = 1000000ULL; break;
            case 'g': case 'G': factor = 1000000000ULL; break;
            case 't': case 'T': factor = 1000000000000ULL; break;
            default:
                std::cerr << "ERROR: Unrecognized unit (\"" << suffix << "\") in argument to -"
                          << identifier << ". If specified, unit must be one of [kKmMgGtT]."
                          << std::endl;
                exit(1);
            }
            body.pop_back();
        }
        bool fail = false;
        double v = 0;
        try { v = std::stof(body); } catch (const std::exception &) { fail = true; }
        if (v <= 0 || (double)(uint64_t)v != v) fail = true;
        if (fail) {
            std::cerr << "ERROR: Argument to -" << identifier
                      << " must be a whole number, optionally followed by one of [kKmMgGtT]."
                      << std::endl;
            exit(1);
        }
        (void)factor;
    }
}

double Command::Option::getArgumentAsNumber() const
{
    if (argument.empty()) return 0;
    if (type == Size) {
        std::string body = argument;
        double factor = 1;
        char suffix = body.back();
        if (suffix < '0' || suffix > '9') {
            switch (suffix) {
            case 'k': case 'K': factor = 1e3; break;
            case 'm': case 'M': factor = 1e6; break;
            case 'g': case 'G': factor = 1e9; break;
            case 't': case 'T': factor = 1e12; break;
            }
            body.pop_back();
        }
        return (double)std::stof(body) * factor;
    }
    if (type == Number || type == Integer) return (double)std::stof(argument);
    return 0;
}

Command::Command()
{
    addAvailableOption("help", Option(Option::Boolean, "h", "", "Help", ""));
    addAvailableOption("kmer", Option(Option::Integer, "k", "Sketch",
        "K-mer size. Hashes will be based on strings of this many nucleotides. Canonical "
        "nucleotides are used by default (see Alphabet options below).", "21", 1, 32));
    addAvailableOption("sketchSize", Option(Option::Integer, "s", "Sketch",
        "Sketch size. Each sketch will have at most this many non-redundant min-hashes.", "1000"));
    addAvailableOption("individual", Option(Option::Boolean, "i", "Sketch",
        "Sketch individual sequences, rather than whole files, e.g. for multi-fastas of "
        "single-chromosome genomes or pair-wise gene comparisons.", ""));
    addAvailableOption("warning", Option(Option::Number, "w", "Sketch",
        "Probability threshold for warning about low k-mer size.", "0.01", 0, 1));
    addAvailableOption("reads", Option(Option::Boolean, "r", "Sketch",
        "Input is a read set. See Reads options below. Implies -M. Incompatible with -i.", ""));
    addAvailableOption("seed", Option(Option::Integer, "S", "Sketch",
        "Seed to provide to the hash function.", "42", 0, 0xFFFFFFFF));
    addAvailableOption("memory", Option(Option::Size, "b", "Reads",
        "Use a Bloom filter of this size (raw bytes or with K/M/G/T) to filter out unique "
        "k-mers. Implies -r."));
    addAvailableOption("minCov", Option(Option::Integer, "m", "Reads",
        "Minimum copies of each k-mer required to pass noise filter for reads. Implies -r.", "1"));
    addAvailableOption("targetCov", Option(Option::Number, "c", "Reads",
        "Target coverage. Sketching will conclude if this coverage is reached before the end of "
        "the input file (estimated by average k-mer multiplicity). Implies -r."));
    addAvailableOption("genome", Option(Option::Size, "g", "Reads",
        "Genome size (raw bases or with K/M/G/T). If specified, will be used for p-value "
        "calculation instead of an estimated size from k-mer content. Implies -r."));
    addAvailableOption("noncanonical", Option(Option::Boolean, "n", "Alphabet",
        "Preserve strand (by default, strand is ignored by using canonical DNA k-mers, which are "
        "alphabetical minima of forward-reverse pairs). Implied if an alphabet is specified with "
        "-a or -z.", ""));
    addAvailableOption("protein", Option(Option::Boolean, "a", "Alphabet",
        "Use amino acid alphabet (A-Z, except BJOUXZ). Implies -n, -k 9.", ""));
    addAvailableOption("alphabet", Option(Option::String, "z", "Alphabet",
        "Alphabet to base hashes on (case ignored by default; see -Z). K-mers with other "
        "characters will be ignored. Implies -n.", ""));
    addAvailableOption("case", Option(Option::Boolean, "Z", "Alphabet",
        "Preserve case in k-mers and alphabet (case is ignored by default). Sequence letters "
        "whose case is not in the current alphabet will be skipped when sketching.", ""));
    addAvailableOption("threads", Option(Option::Integer, "p", "",
        "Parallelism. This many threads will be spawned for processing (accepted; the MI355X "
        "path runs on the device).", "1"));
    addCategory("", "");
    addCategory("Input", "Input");
    addCategory("Output", "Output");
    addCategory("Sketch", "Sketching");
    addCategory("Reads", "Sketching (reads)");
    addCategory("Alphabet", "Sketching (alphabet)");
}

void Command::addOption(const std::string &n, const Option &o)
{
    options[n] = o;
    optionNamesByCategory[o.category].push_back(n);
    optionNamesByIdentifier[o.identifier] = n;
}

void Command::useOption(const std::string &n) { addOption(n, optionsAvailable.at(n)); }

void Command::addAvailableOption(const std::string &n, const Option &o) { optionsAvailable[n] = o; }

void Command::addCategory(const std::string &n, const std::string &d)
{
    if (!categoryDisplayNames.count(n)) {
        categories.push_back(n);
        categoryDisplayNames[n] = d;
        optionNamesByCategory[n] = {};
    }
}

// useSketchOptions (Command.cpp:385-410, COMMAND_FIND off)
void Command::useSketchOptions()
{
    for (const char *n : {"threads", "kmer", "noncanonical", "protein", "alphabet", "case",
                          "sketchSize", "individual", "seed", "warning", "reads", "memory",
                          "minCov", "targetCov", "genome"})
        useOption(n);
}

int Command::run(int argc, const char **argv)
{
    for (int i = 0; i < argc; i++) {
        if (argv[i][0] == '-' && argv[i][1] != 0) {
            auto it = optionNamesByIdentifier.find(argv[i] + 1);
            if (it == optionNamesByIdentifier.end()) {
                std::cerr << "ERROR: Unrecognized option: " << argv[i] << std::endl;
                return 1;
            }
            Option &o = options.at(it->second);
            o.active = true;
            if (o.type != Option::Boolean) {
                i++;
                if (i == argc) {
                    std::cerr << "ERROR: -" << o.identifier << " requires an argument" << std::endl;
                    return 1;
                }
                o.setArgument(argv[i]);
            }
        } else {
            arguments.push_back(argv[i]);
        }
    }
    return run();
}

void Command::print() const
{
    std::cout << std::endl << "Version: " << kVersion << std::endl << std::endl;
    std::cout << "Usage:" << std::endl << std::endl;
    std::cout << "  fpmash " << name << " [options] " << argumentString << std::endl << std::endl;
    std::cout << "Description:" << std::endl << std::endl << "  " << description << std::endl
              << std::endl;
    if (options.empty()) return;
    std::cout << "Options:" << std::endl << std::endl;
    for (const auto &cat : categories) {
        auto it = optionNamesByCategory.find(cat);
        if (it == optionNamesByCategory.end() || it->second.empty()) continue;
        if (!cat.empty()) std::cout << "  ..." << categoryDisplayNames.at(cat) << "..." << std::endl;
        for (const auto &on : it->second) {
            const Option &o = options.at(on);
            std::string s = "-" + o.identifier;
            switch (o.type) {
            case Option::Number: s += " <num>"; break;
            case Option::Integer: s += " <int>"; break;
            case Option::Size: s += " <size>"; break;
            case Option::File: s += " <path>"; break;
            case Option::String: s += " <text>"; break;
            default: break;
            }
            std::string d = o.description;
            if (!o.argumentDefault.empty()) d += " [" + o.argumentDefault + "]";
            char buf[32];
            snprintf(buf, sizeof buf, "  %-16s ", s.c_str());
            std::cout << buf << d << std::endl;
        }
    }
    std::cout << std::endl;
}

CommandList::~CommandList()
{
    for (auto &c : commands) delete c.second;
}

void CommandList::print() const
{
    std::cout << std::endl << "fpmash (MI355X sketch + dist, Mash " << kVersion
              << " compatible)" << std::endl << std::endl << "Usage:" << std::endl << std::endl
              << "  " << name << " <command> [options] [arguments ...]" << std::endl << std::endl
              << "Commands:" << std::endl << std::endl;
    for (const auto &c : commands) {
        char buf[32];
        snprintf(buf, sizeof buf, "  %-10s ", c.first.c_str());
        std::cout << buf << c.second->summary << std::endl;
    }
    std::cout << std::endl;
}

int CommandList::run(int argc, const char **argv)
{
    if (argc > 1 && std::string(argv[1]) == "--version") {
        std::cout << kVersion << std::endl;
        return 0;
    }
    if (argc < 2 || !commands.count(argv[1])) {
        print();
        return 0;
    }
    return commands.at(argv[1])->run(argc - 2, argv + 2);
}

int sketchParameterSetup(Parameters &p, const Command &c)
{
    p.kmerSize = (int)c.getOption("kmer").getArgumentAsNumber();
    p.minHashesPerWindow = (uint64_t)c.getOption("sketchSize").getArgumentAsNumber();
    p.concatenated = !c.getOption("individual").active;
    p.noncanonical = c.getOption("noncanonical").active;
    p.seed = (uint32_t)(uint64_t)c.getOption("seed").getArgumentAsNumber();
    p.reads = c.getOption("reads").active;
    p.fingerprint = c.hasOption("fingerprint") && c.getOption("fingerprint").active;
    p.parallelism = (int)c.getOption("threads").getArgumentAsNumber();
    p.preserveCase = c.getOption("case").active;
    if (c.hasOption("warning")) p.warning = c.getOption("warning").getArgumentAsNumber();
    if (c.getOption("memory").active || c.getOption("minCov").active ||
        c.getOption("targetCov").active || c.getOption("genome").active)
        p.reads = true;
    if (p.reads) {
        // reads mode (Bloom / minCov / targetCov / genome size) is outside the MI355X hot path
        std::cerr << "ERROR: reads mode (-r/-b/-m/-c/-g) is not supported by fpmash; sketch "
                     "assemblies or -fp k-finger files." << std::endl;
        return 1;
    }
    if (p.fingerprint) {
        p.kmerSize = 1;
        p.noncanonical = true;
        setAlphabetFromString(p, "0123456789");
    } else if (c.getOption("protein").active) {
        p.noncanonical = true;
        setAlphabetFromString(p, alphabetProtein);
        if (!c.getOption("kmer").active) p.kmerSize = 9;
        setAlphabetFromString(p, alphabetProtein);
    } else if (c.getOption("alphabet").active) {
        p.noncanonical = true;
        setAlphabetFromString(p, c.getOption("alphabet").argument.c_str());
    } else {
        setAlphabetFromString(p, alphabetNucleotide);
    }
    return 0;
}

void warnKmerSize(const Parameters &p, const Command &c, uint64_t lengthMax,
                  const std::string &lengthMaxName, double randomChance, int kMin,
                  int warningCount)
{
    std::cerr << "\nWARNING: For the k-mer size used (" << p.kmerSize
              << "), the random match probability (" << randomChance
              << ") is above the specified warning threshold (" << p.warning
              << ") for the sequence \"" << lengthMaxName << "\" of size " << lengthMax;
    if (warningCount > 1) std::cerr << " (and " << (warningCount - 1) << " others)";
    std::cerr << ". Distances to " << (warningCount == 1 ? "this sequence" : "these sequences")
              << " may be underestimated as a result. To meet the threshold of " << p.warning
              << ", a k-mer size of at least " << kMin << " is required. See: -"
              << c.getOption("kmer").identifier << ", -" << c.getOption("warning").identifier
              << "." << std::endl << std::endl;
}

}  // namespace fpmhost
