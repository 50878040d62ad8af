// Timing.h — FPMASH_TIMING=1 prints the wall time of each host phase to stderr
// ("[fpmash] phase: ms"), so the end-to-end CLI walls in the bench can be split into
// process start, input parsing, device work and output.  Off by default: no output change.
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace fpmhost {

inline bool timingOn()
{
    static const bool on = [] {
        const char *v = getenv("FPMASH_TIMING");
        return v && *v && *v != '0';
    }();
    return on;
}

// FPMASH_CLEAN_EXIT=1: the full teardown at exit (contexts, pinned buffers); otherwise a
// command leaves by _exit once its outputs are flushed (main.cpp)
inline bool cleanExit()
{
    static const bool on = [] {
        const char *v = getenv("FPMASH_CLEAN_EXIT");
        return v && *v && *v != '0';
    }();
    return on;
}

// prints the time since the previous mark (or since the first call) under `what`
inline void phaseMark(const char *what)
{
    using clk = std::chrono::steady_clock;
    static clk::time_point last = clk::now();
    if (!timingOn()) return;
    const clk::time_point now = clk::now();
    fprintf(stderr, "[fpmash] %s: %.3f ms\n", what,
            std::chrono::duration<double, std::milli>(now - last).count());
    last = now;
}

}  // namespace fpmhost
