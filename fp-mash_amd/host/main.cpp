// main.cpp — `fpmash`: the reference's CLI entry (mash.cpp:19-40) for the hot-path
// verbs.  `fpmash sketch|dist|info|paste|triangle [-fp] ...` is a drop-in for the same
// `mash` verbs.
#include "Command.h"
#include "Timing.h"

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <unistd.h>

int main(int argc, const char **argv)
{
    fpmhost::phaseMark("start");
    // Host<->device copies by blit kernels on the compute queue instead of the SDMA engines
    // (set before the HIP runtime starts, unless the caller chose): a process's first SDMA copy
    // brings up the engine's queue, ~10 ms of the CLI's start-up (staging ring + first copy
    // 16.8 -> 7.0 ms, `sketch -fp` median call 0.137-0.147 -> 0.115-0.117 s, `dist c2.msh
    // c2.msh` unchanged, same box, profiles/r06/cli_sdma_ab.txt).  The CLI's copies are a few
    // MB each way per command; the library itself leaves the setting to its host process.
    setenv("HSA_ENABLE_SDMA", "0", 0);
    fpmhost::CommandList commandList("fpmash");
    commandList.addCommand(new fpmhost::CommandSketch());
    commandList.addCommand(new fpmhost::CommandDistance());
    commandList.addCommand(new fpmhost::CommandInfo());
    commandList.addCommand(new fpmhost::CommandPaste());
    commandList.addCommand(new fpmhost::CommandTriangle());
    const int rc = commandList.run(argc, argv);
    fpmhost::phaseMark("command done");
    // Every output is written and the device work is complete (results were fetched): leave
    // without the HIP runtime's teardown (context, stream and code-object release run from
    // atexit and the library destructors), which the kernel driver does with the process
    // anyway.  FPMASH_CLEAN_EXIT=1 keeps the full teardown.
    if (!fpmhost::cleanExit()) {
        std::cout.flush();
        std::cerr.flush();
        fflush(nullptr);
        _exit(rc);
    }
    return rc;
}
