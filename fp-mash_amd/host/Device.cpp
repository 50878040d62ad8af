#include "Device.h"

#include <cstdlib>
#include <iostream>
#include <mutex>
#include <vector>

namespace fpmhost {

namespace {
std::vector<fpm_ctx *> g_ctx;
std::vector<int> g_ids;
std::once_flag g_once;
std::mutex g_mu;

void release()
{
    for (auto *c : g_ctx)
        if (c) fpm_ctx_destroy(c);
    g_ctx.clear();
}

void init_ids()
{
    if (const char *dev = getenv("FPMASH_DEVICE")) {
        g_ids.push_back(atoi(dev));
    } else {
        int n = 0;
        if (fpm_device_count(&n) != FPM_OK) n = 0;
        if (const char *lim = getenv("FPMASH_DEVICES")) n = std::min(n, std::max(1, atoi(lim)));
        for (int i = 0; i < n; i++) g_ids.push_back(i);
        if (g_ids.empty()) g_ids.push_back(0);   // fpm_ctx_create reports the missing device
    }
    g_ctx.assign(g_ids.size(), nullptr);
    atexit(release);
}
}  // namespace

void check(int rc, const char *what)
{
    if (rc != FPM_OK) {
        std::cerr << "ERROR: " << what << ": " << fpm_last_error() << std::endl;
        exit(1);
    }
}

int deviceCount()
{
    std::call_once(g_once, init_ids);
    return (int)g_ids.size();
}

fpm_ctx *device(int i)
{
    std::call_once(g_once, init_ids);
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ctx[i]) check(fpm_ctx_create(g_ids[i], &g_ctx[i]), "MI355X device");
    return g_ctx[i];
}

}  // namespace fpmhost
