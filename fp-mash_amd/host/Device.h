// Device.h — the host's single gfx950 context.  Every call goes through the C ABI
// (include/fpmash.h); a non-zero status prints "ERROR: ..." and exit(1)s, the
// reference's failure convention on this path (Sketch.cpp:75-76, 1446-1463).
#pragma once

#include "fpmash.h"

namespace fpmhost {

fpm_ctx *device();
void check(int rc, const char *what);

}  // namespace fpmhost
