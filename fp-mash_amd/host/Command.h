// Command.h — the reference's plugin surface (Command.h:26-136, CommandList.cpp:88-109):
// a Command owns an option registry, parses argv, and runs.  Commands register
// in main.cpp exactly as mash.cpp:23-37 does for the hot-path verbs.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace fpmhost {

class Command {
public:
    struct Option {
        enum Type { Boolean, Number, Integer, Size, File, String };
        Type type = Boolean;
        std::string identifier, category, description, argument, argumentDefault;
        double argumentMin = 0, argumentMax = 0;
        bool active = false;
        bool changed = false;
        Option() = default;
        Option(Type t, const std::string &id, const std::string &cat, const std::string &desc,
               const std::string &def = "", double mn = 0, double mx = 0);
        void setArgument(const std::string &a);
        double getArgumentAsNumber() const;
    };

    Command();
    virtual ~Command() = default;
    int run(int argc, const char **argv);
    virtual int run() const = 0;
    void print() const;
    const Option &getOption(const std::string &name) const { return options.at(name); }
    bool hasOption(const std::string &name) const { return options.count(name) > 0; }

    std::string name, summary, description, argumentString;

protected:
    void addOption(const std::string &name, const Option &o);
    void useOption(const std::string &name);
    void useSketchOptions();

    std::map<std::string, Option> options;
    std::map<std::string, Option> optionsAvailable;
    std::map<std::string, std::string> optionNamesByIdentifier;
    std::map<std::string, std::vector<std::string>> optionNamesByCategory;
    std::vector<std::string> categories;
    std::map<std::string, std::string> categoryDisplayNames;
    std::vector<std::string> arguments;

private:
    void addAvailableOption(const std::string &name, const Option &o);
    void addCategory(const std::string &name, const std::string &display);
};

class CommandList {
public:
    explicit CommandList(const std::string &name) : name(name) {}
    ~CommandList();
    void addCommand(Command *c) { commands[c->name] = c; }
    int run(int argc, const char **argv);

private:
    void print() const;
    std::string name;
    std::map<std::string, Command *> commands;
};

class CommandSketch : public Command {
public:
    CommandSketch();
    int run() const override;
};

class CommandDistance : public Command {
public:
    CommandDistance();
    int run() const override;
};

class CommandInfo : public Command {
public:
    CommandInfo();
    int run() const override;
};

class CommandPaste : public Command {
public:
    CommandPaste();
    int run() const override;
};

class CommandTriangle : public Command {
public:
    CommandTriangle();
    int run() const override;
};

// sketchParameterSetup (sketchParameterSetup.cpp:9-126)
struct Parameters;
int sketchParameterSetup(Parameters &p, const Command &c);
void warnKmerSize(const Parameters &p, const Command &c, uint64_t lengthMax,
                  const std::string &lengthMaxName, double randomChance, int kMin,
                  int warningCount);

}  // namespace fpmhost
