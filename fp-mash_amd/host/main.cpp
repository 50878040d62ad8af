// main.cpp — `fpmash`: the reference's CLI entry (mash.cpp:19-40) for the hot-path
// verbs.  `fpmash sketch|dist|info|paste|triangle [-fp] ...` is a drop-in for the same
// `mash` verbs.
#include "Command.h"
#include "Timing.h"

int main(int argc, const char **argv)
{
    fpmhost::phaseMark("start");
    fpmhost::CommandList commandList("fpmash");
    commandList.addCommand(new fpmhost::CommandSketch());
    commandList.addCommand(new fpmhost::CommandDistance());
    commandList.addCommand(new fpmhost::CommandInfo());
    commandList.addCommand(new fpmhost::CommandPaste());
    commandList.addCommand(new fpmhost::CommandTriangle());
    const int rc = commandList.run(argc, argv);
    fpmhost::phaseMark("command done");
    return rc;
}
