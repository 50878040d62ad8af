#include "Device.h"
#include "Timing.h"

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <mutex>
#include <unistd.h>
#include <cstdio>
#include <thread>
#include <vector>

namespace fpmhost {

namespace {
std::vector<fpm_ctx *> g_ctx;
std::vector<int> g_ids;
std::unique_ptr<std::once_flag[]> g_ctx_once;   // one context creation per device slot
std::once_flag g_once;
std::mutex g_mu;
std::thread g_warm;
std::once_flag g_warm_join;

double g_warm_ms[3] = {-1, -1, -1};

// FPMASH_TIMING=1: the warm-up thread's own steps, on lines of their own ("[fpmash-warm]":
// not main-thread phases; the main thread's wait for them is its "device context" phase)
void join_warm()
{
    if (!g_warm.joinable()) return;
    g_warm.join();
    if (timingOn() && g_warm_ms[0] >= 0)
        fprintf(stderr,
                "[fpmash-warm] runtime start + device enumeration: %.3f ms\n"
                "[fpmash-warm] context (stream): %.3f ms\n"
                "[fpmash-warm] staging ring + first copy: %.3f ms\n",
                g_warm_ms[0], g_warm_ms[1], g_warm_ms[2]);
}

void release()
{
    for (auto *c : g_ctx)
        if (c) fpm_ctx_destroy(c);
    g_ctx.clear();
}

std::once_flag g_exit_once;

void shutdown()
{
    join_warm();
    release();
}

// one exit handler, registered on the main thread before any context exists
void ensure_exit_handler()
{
    std::call_once(g_exit_once, [] { atexit(shutdown); });
}

void init_ids()
{
    if (const char *list = getenv("FPMASH_DEVICE_LIST")) {
        // explicit ordinals, e.g. "0,0" runs two contexts on one GPU (the tests' stand-in for
        // a multi-GPU node)
        for (const char *c = list; *c;) {
            g_ids.push_back(atoi(c));
            while (*c && *c != ',') c++;
            if (*c == ',') c++;
        }
        if (g_ids.empty()) g_ids.push_back(0);
    } else if (const char *dev = getenv("FPMASH_DEVICE")) {
        g_ids.push_back(atoi(dev));
    } else {
        int n = 0;
        if (fpm_device_count(&n) != FPM_OK) n = 0;
        if (const char *lim = getenv("FPMASH_DEVICES")) n = std::min(n, std::max(1, atoi(lim)));
        for (int i = 0; i < n; i++) g_ids.push_back(i);
        if (g_ids.empty()) g_ids.push_back(0);   // fpm_ctx_create reports the missing device
    }
    g_ctx.assign(g_ids.size(), nullptr);
    g_ctx_once.reset(new std::once_flag[g_ids.size()]);
    ensure_exit_handler();
}
}  // namespace

// Errors end the process the reference's way (message, status 1), from whichever thread
// meets them: GPU, pinner and formatter threads may still be running, so the process leaves
// with _exit after flushing, without the atexit teardown that would destroy the contexts
// those threads are using.
static std::atomic<int> g_cut_fd{-1};
static std::atomic<long long> g_cut_at{0};
void fatalCutsOutput(int fd, off_t at)
{
    g_cut_at = (long long)at;
    g_cut_fd = fd;
}

void fatalExit()
{
    // an output file sized ahead of its text (the dist writer) goes back to what was there
    const int cfd = g_cut_fd.exchange(-1);
    if (cfd >= 0 && ftruncate(cfd, (off_t)g_cut_at.load()) != 0) {}
    std::cout.flush();
    std::cerr.flush();
    fflush(stdout);
    fflush(stderr);
    _exit(1);
}

void check(int rc, const char *what)
{
    if (rc != FPM_OK) {
        std::cerr << "ERROR: " << what << ": " << fpm_last_error() << std::endl;
        fatalExit();
    }
}

int deviceCount()
{
    std::call_once(g_warm_join, join_warm);
    std::call_once(g_once, init_ids);
    return (int)g_ids.size();
}

void warmDevices()
{
    ensure_exit_handler();
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_warm.joinable()) return;
    // HIP runtime start-up (device enumeration + the first context's streams: ~0.1-0.25 s)
    // runs beside the caller's input reading.  Only the first device is warmed: the others
    // are created on first use (device(i)), once the command knows how many parts it spreads,
    // so a single-file sketch on an 8-GPU node does not bring up 8 contexts.  A context that
    // fails to come up is reported by the first device() call.
    g_warm = std::thread([] {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        std::call_once(g_once, init_ids);
        const auto t1 = clk::now();
        std::call_once(g_ctx_once[0], [] {
            if (fpm_ctx_create(g_ids[0], &g_ctx[0]) != FPM_OK) g_ctx[0] = nullptr;
        });
        const auto t2 = clk::now();
        // the staging ring and the first DMA, before the first upload needs them
        if (g_ctx[0]) (void)fpm_ctx_warm(g_ctx[0]);
        const auto t3 = clk::now();
        auto ms = [](clk::time_point a, clk::time_point b) {
            return std::chrono::duration<double, std::milli>(b - a).count();
        };
        g_warm_ms[0] = ms(t0, t1);
        g_warm_ms[1] = ms(t1, t2);
        g_warm_ms[2] = ms(t2, t3);
    });
}

fpm_ctx *device(int i)
{
    std::call_once(g_warm_join, join_warm);
    std::call_once(g_once, init_ids);
    // per-device creation (device threads bring their contexts up in parallel); a failed
    // warm-up of device 0 is retried here and reported
    std::call_once(g_ctx_once[i], [i] {
        if (fpm_ctx_create(g_ids[i], &g_ctx[i]) != FPM_OK) g_ctx[i] = nullptr;
    });
    if (!g_ctx[i]) {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_ctx[i]) check(fpm_ctx_create(g_ids[i], &g_ctx[i]), "MI355X device");
    }
    return g_ctx[i];
}

}  // namespace fpmhost
