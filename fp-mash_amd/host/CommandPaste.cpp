// CommandPaste.cpp — `fpmash paste` (CommandPaste.cpp:12-214): one .msh from several.
// Same argument conventions as the fork: the output prefix comes first, or last with
// -o; -fp accepts <x>.txt (replaced by its sketch <x>.msh, which must exist) and
// <x>.msh (whose <x>.txt must exist); -l and no option take .msh files as given (the
// fork's -l list reading is a TODO that keeps the arguments, :77-80).  The sketches
// are loaded and written by the same host code as `sketch` (no device work).
#include "Command.h"
#include "Sketch.h"

#include <iostream>
#include <unistd.h>

namespace fpmhost {

static const char *suffixFingerprint = ".txt";   // Sketch.h:29

CommandPaste::CommandPaste()
{
    name = "paste";
    summary = "Create a single sketch file from multiple sketch files.";
    description = "Create a single sketch file from multiple sketch files.";
    argumentString = "<out_prefix> <sketch> [<sketch>] ...";
    useOption("help");
    addOption("list", Option(Option::Boolean, "l", "", "Input files are lists of file names.", ""));
    addOption("fingerPrint", Option(Option::Boolean, "fp", "",
        "Insert fingerprint files are lists of file names.", ""));
    addOption("output", Option(Option::Boolean, "o", "",
        "Insert -o to indicate the name and path for the output file. Take this option as the "
        "last one after -fp or -l ", ""));
}

static bool fileExists(const std::string &f) { return access(f.c_str(), F_OK) != -1; }

int CommandPaste::run() const
{
    const bool output = options.at("output").active;
    const bool list = options.at("list").active;
    const bool fingerPrint = options.at("fingerPrint").active;
    if (list && fingerPrint) {
        std::cerr << "ERROR: The options -l and -fp are incompatible." << std::endl;
        return 1;
    }
    if (arguments.size() < 2 || options.at("help").active) {
        print();
        return 0;
    }
    std::vector<std::string> files;
    std::string out;
    if (output) {
        files.assign(arguments.begin(), arguments.end() - 1);
        out = arguments.back();
    } else {
        files.assign(arguments.begin() + 1, arguments.end());
        out = arguments[0];
    }
    std::vector<std::string> filesGood;
    for (std::string file : files) {
        if (fingerPrint) {
            if (!hasSuffix(file, suffixFingerprint) && !hasSuffix(file, suffixSketch)) {
                std::cerr << "ERROR: The file \"" << file
                          << "\" does not look like a fingerprint or sketch." << std::endl;
                return 1;
            }
            if (hasSuffix(file, ".txt")) {
                const std::string msh = file.substr(0, file.size() - 4) + ".msh";
                if (!fileExists(msh)) {
                    std::cerr << "ERROR: The file \"" << msh
                              << "\" does not exist but is required. Do the command sketch "
                                 "before doing this operation " << std::endl;
                    return 1;
                }
                file = msh;
            } else if (hasSuffix(file, ".msh")) {
                const std::string txt = file.substr(0, file.size() - 4) + ".txt";
                if (!fileExists(txt)) {
                    std::cerr << "ERROR: The file \"" << txt << "\" does not exist but is required."
                              << std::endl;
                    return 1;
                }
            }
        } else if (!hasSuffix(file, suffixSketch)) {
            std::cerr << "ERROR: The file \"" << file << "\" does not look like a sketch."
                      << std::endl;
            return 1;
        }
        filesGood.push_back(file);
    }
    Parameters parameters;
    parameters.parallelism = 1;
    Sketch sketch;
    sketch.initFromFiles(filesGood, parameters);
    if (!hasSuffix(out, suffixSketch)) out += suffixSketch;
    if (fileExists(out)) {
        std::cerr << "ERROR: \"" << out << "\" exists; remove to write." << std::endl;
        exit(1);
    }
    std::cerr << "Writing " << out << "..." << std::endl;
    sketch.writeToMsh(out);
    return 0;
}

}  // namespace fpmhost
