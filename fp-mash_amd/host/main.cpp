// main.cpp — `fpmash`: the reference's CLI entry (mash.cpp:19-40) for the hot-path
// verbs.  `fpmash sketch|dist [-fp] ...` is a drop-in for `mash sketch|dist [-fp] ...`.
#include "Command.h"

int main(int argc, const char **argv)
{
    fpmhost::CommandList commandList("fpmash");
    commandList.addCommand(new fpmhost::CommandSketch());
    commandList.addCommand(new fpmhost::CommandDistance());
    commandList.addCommand(new fpmhost::CommandInfo());
    return commandList.run(argc, argv);
}
