// Device.h — the host's gfx950 contexts.  Every call goes through the C ABI
// (include/fpmash.h); a non-zero status prints "ERROR: ..." and exit(1)s, the
// reference's failure convention on this path (Sketch.cpp:75-76, 1446-1463).
//
// Devices used: FPMASH_DEVICE=i pins one device; otherwise every visible device (at most
// FPMASH_DEVICES=n of them).  device(0) is the default context; the dist and sketch
// commands spread query blocks / sketch groups over device(0..deviceCount()-1), the way
// the reference spreads them over its -p threads (CommandDistance.cpp:191, Sketch.cpp:253).
#pragma once
#include <sys/types.h>

#include "fpmash.h"

namespace fpmhost {

int deviceCount();
// start creating every context on a background thread (the first device() call joins it)
void warmDevices();
fpm_ctx *device(int i = 0);
void check(int rc, const char *what);
// exit status 1 after flushing stdout / stderr, without the atexit context teardown (safe from
// any thread: other threads may still be using the contexts)
[[noreturn]] void fatalExit();
// fatalExit first cuts file `fd` back to `at` bytes (an output sized ahead of its text)
void fatalCutsOutput(int fd, off_t at);

}  // namespace fpmhost
