#include "Device.h"

#include <cstdlib>
#include <iostream>

namespace fpmhost {

namespace {
fpm_ctx *g_ctx = nullptr;
void release() { if (g_ctx) { fpm_ctx_destroy(g_ctx); g_ctx = nullptr; } }
}  // namespace

void check(int rc, const char *what)
{
    if (rc != FPM_OK) {
        std::cerr << "ERROR: " << what << ": " << fpm_last_error() << std::endl;
        exit(1);
    }
}

fpm_ctx *device()
{
    if (!g_ctx) {
        const char *dev = getenv("FPMASH_DEVICE");
        check(fpm_ctx_create(dev ? atoi(dev) : 0, &g_ctx), "MI355X device");
        atexit(release);
    }
    return g_ctx;
}

}  // namespace fpmhost
