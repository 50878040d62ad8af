// CommandSketch.cpp — `fpmash sketch` (CommandSketch.cpp:19-122): same options,
// messages and .msh output; sketching runs on the MI355X.
#include "Command.h"
#include "Timing.h"
#include "Device.h"
#include "Sketch.h"

#include <cstdlib>
#include <iostream>
#include <memory>

namespace fpmhost {

CommandSketch::CommandSketch()
{
    name = "sketch";
    summary = "Create sketches (reduced representations for fast operations).";
    description = "Create a sketch file, which is a reduced representation of a sequence or set "
                  "of sequences (based on min-hashes) that can be used for fast distance "
                  "estimations. Inputs can be fasta or fastq files (gzipped or not), and \"-\" can "
                  "be given to read from standard input. With -fp the inputs are k-finger "
                  "fingerprint files.";
    argumentString = "<input> [<input>] ...";
    useOption("help");
    addOption("list", Option(Option::Boolean, "l", "Input",
        "List input. Lines in each <input> specify paths to sequence files, one per line.", ""));
    addOption("prefix", Option(Option::File, "o", "Output",
        "Output prefix (first input file used if unspecified). The suffix '.msh' will be "
        "appended.", ""));
    addOption("id", Option(Option::File, "I", "Sketch",
        "ID field for sketch of reads (instead of first sequence ID).", ""));
    addOption("comment", Option(Option::File, "C", "Sketch",
        "Comment for a sketch of reads (instead of first sequence comment).", ""));
    addOption("counts", Option(Option::Boolean, "M", "Sketch",
        "Store multiplicity of each k-mer in each sketch.", ""));
    addOption("fingerprint", Option(Option::Boolean, "fp", "Input",
        "Indicates that the input files are fingerprints instead of sequences.", ""));
    useSketchOptions();
}

int CommandSketch::run() const
{
    if (arguments.empty() || options.at("help").active) {
        print();
        return 0;
    }
    warmDevices();
    const int verbosity = 1;
    const bool list = options.at("list").active;
    const bool fingerprint = options.at("fingerprint").active;
    Parameters parameters;
    parameters.counts = options.at("counts").active;
    if (sketchParameterSetup(parameters, *this)) return 1;
    std::vector<std::string> files;
    for (const auto &a : arguments) {
        if (list) splitFile(a, files);
        else files.push_back(a);
    }
    // heap-held: main leaves with _exit once the .msh is written, so the 80 MB of rows and the
    // per-reference strings of a C2 sketch are returned with the process (~3 ms of frees)
    // instead of one by one; FPMASH_CLEAN_EXIT=1 destroys it
    std::unique_ptr<Sketch> owned(new Sketch());
    Sketch &sketch = *owned;
    sketch.keepDeviceRows();   // the rows are only written to the .msh
    if (fingerprint) sketch.initFromFingerprints(files, parameters);
    else sketch.initFromFiles(files, parameters, verbosity);
    if (getOption("id").active) sketch.setReferenceName(0, getOption("id").argument);
    if (getOption("comment").active) sketch.setReferenceComment(0, getOption("comment").argument);
    std::string prefix;
    if (!options.at("prefix").argument.empty()) prefix = options.at("prefix").argument;
    else prefix = arguments[0] == "-" ? "stdin" : arguments[0];
    if (!hasSuffix(prefix, suffixSketch)) prefix += suffixSketch;
    std::cerr << "Writing to " << prefix << "..." << std::endl;
    sketch.writeToMsh(prefix);
    if (!cleanExit()) (void)owned.release();
    return 0;
}

}  // namespace fpmhost
