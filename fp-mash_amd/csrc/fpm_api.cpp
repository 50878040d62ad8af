// fpm_api.cpp — implementation of the C ABI declared in include/fpmash.h.
//
// Host-side staging (record packing, tile plan, merge schedule) and kernel
// launches for the gfx950 kernels in sketch.hip / fingerprint.hip / dist.hip.
// There is deliberately no CPU compute path here: without a usable device every
// compute entry point returns FPM_ENODEV.
#include "fpm_kernels.hpp"
#include "../../include/fpmash.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <array>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdio>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <string>
#include <system_error>
#include <vector>

using namespace fpm;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(FPM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

// Reference complement table for 'A'..'Z' (Sketch.cpp:1223-1250); other bytes 'N'.
const char kComplAZ[26] = {'T', 'V', 'G', 'H', 'N', 'N', 'C', 'D', 'N', 'N', 'M', 'N', 'K',
                           'N', 'N', 'N', 'N', 'Y', 'S', 'A', 'A', 'B', 'W', 'N', 'R', 'N'};

// Tile sizing: small records are packed up to kPackKmers k-mer starts per tile,
// long records are cut into kChunkKmers-start chunks (k-1 bytes of halo).
constexpr uint32_t kPackKmers = 2048;
// (2048-start chunks: the tile kernel 1.3 ms faster on C5, the group selection 1.3 ms slower)
constexpr uint32_t kChunkKmers = 4096;

int tile_class(uint32_t nstarts)
{
    for (int c = 0; c < kTileClasses; c++)
        if (nstarts <= kTileCap[c]) return c;
    return -1;
}

}  // namespace

// merge rounds whose estimated input lists are at most merge_small_cap() long use
// merge_small_kernel; FPM_MERGE_SMALL=0 turns it off (A/B), =2 uses it for every round
// (tests: its global-memory search past the LDS cap)
static const int g_merge_small_env = [] {
    const char *v = getenv("FPM_MERGE_SMALL");
    return v ? atoi(v) : 1;
}();

// Host memcpy split over a few persistent threads: the pinned ring's copies of pageable caller
// memory ran at one thread's ~8 GB/s, below the DMA behind them (C3's 301 MB of -fp text:
// ~40 ms of the parse wall).  Parts of >= 1 MB; the caller copies the first part itself.
class CopyPool {
  public:
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void copy(void *dst, const void *src, size_t n)
    {
        constexpr size_t kPart = size_t(1) << 20;
        const unsigned want = (unsigned)std::min<size_t>(kMaxThreads + 1, n / kPart);
        if (want <= 1) { memcpy(dst, src, n); return; }
        std::unique_lock<std::mutex> lk(mu_);
        while (th_.size() + 1 < want && th_.size() < threads()) {
            // (at the process's thread limit: fewer parts, never an exception through the C ABI)
            try {
                th_.emplace_back([this] { work(); });
            } catch (const std::system_error &) {
                break;
            }
        }
        const unsigned parts = (unsigned)std::min<size_t>(want, th_.size() + 1);
        const size_t per = (n + parts - 1) / parts;
        char *d = static_cast<char *>(dst);
        const char *sp = static_cast<const char *>(src);
        for (unsigned i = 1; i < parts; i++) {
            const size_t a = i * per, b = std::min(n, a + per);
            if (a < b) { q_.push_back({d + a, sp + a, b - a}); pending_++; }
        }
        lk.unlock();
        cv_.notify_all();
        memcpy(d, sp, std::min(n, per));
        lk.lock();
        done_.wait(lk, [this] { return pending_ == 0; });
    }

  private:
    static constexpr unsigned kMaxThreads = 7;
    static unsigned threads()
    {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        return std::min(kMaxThreads, std::max(1u, hw / 2));
    }
    struct Task { char *d; const char *s; size_t n; };
    void work()
    {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
            if (q_.empty()) return;
            const Task t = q_.back();
            q_.pop_back();
            lk.unlock();
            memcpy(t.d, t.s, t.n);
            lk.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    std::vector<Task> q_;
    size_t pending_ = 0;
    bool stop_ = false;
};

struct fpm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[FPM_K_COUNT];
    // grow-only device scratch, one buffer per named slot (no allocation in steady state)
    struct Slot { void *p = nullptr; size_t bytes = 0; };
    Slot scratch[22];
    unsigned long long *host_counters = nullptr;   // pinned + mapped, for the events read-back
    unsigned long long *dev_counters = nullptr;    // its device-side address
    unsigned long long pub_seq = 0;                // last sequence number published into it
    int dist_mode = FPM_DIST_AUTO;
    int fill_counts = -1;      // the side-stream fill also writes the numer / denom defaults
                               // (-1: for grids of >= 2^28 pairs; FPM_FILL_COUNTS=0/1 forces)
    int last_sparse = 0;
    uint64_t last_events = 0, last_cand = 0;
    const unsigned long long *last_cand_dev = nullptr;   // the last sparse call's counter
    hipStream_t last_cand_stream = nullptr;
    // side stream for the sparse dist's fill (a pure write stream that runs beside the
    // latency-bound candidate compare); ev_in / ev_fill order it against `stream`
    hipStream_t aux = nullptr;
    hipEvent_t ev_in = nullptr, ev_fill = nullptr;
    // a compact grid's counts written ahead on `aux` (fpm_dist_list_prefill), until the dist
    // call on that grid takes it over (or any other dist call waits for it): ev_prefill
    struct Prefill {
        const void *numer = nullptr, *denom = nullptr;
        uint32_t n_ref = 0, n_qry = 0, S = 0;
        bool pending = false;
    } prefill;
    hipEvent_t ev_prefill = nullptr;
    // pinned staging ring for host -> device copies of pageable caller memory
    static constexpr int kRing = 4;
    static constexpr size_t kRingBytes = 8u << 20;
    void *ring[kRing] = {};
    hipEvent_t ring_ev[kRing] = {};
    CopyPool copier;                       // the ring's host-side copies
    // device buffers of released -fp text jobs, reused by the next jobs: a fresh hipMalloc of
    // tens of MB is cleared by the driver before first use, and a kernel writing it could wait
    // ~27 ms for that (tools/micro/fp_text_time.py under rocprofv3: fp_line_kernel 0.06 ms,
    // now and then 27 ms)
    static constexpr size_t kPoolBytes = size_t(2) << 30;
    uint64_t idx_rebuilds = 0;             // one-pass index builds that overflowed a slot
    // The last sparse rank-kernel call's shape and candidate capacity: a call of the same
    // shape enqueues its probe right behind the index build, before the host reads the
    // build's counters (compare_impl), and checks afterwards that the path and the capacity
    // held; otherwise the probe's output is dropped and the call proceeds as without it.
    struct SpecProfile {
        bool valid = false;
        uint32_t n_ref = 0, n_qry = 0, S = 0;
        uint64_t ref_stride = 0, qry_stride = 0, cap = 0;
        bool self_set = false, defaults = false;
    } spec;
    uint64_t spec_hits = 0, spec_misses = 0;
    std::vector<std::pair<void *, size_t>> pool;
    size_t pool_bytes = 0;
    std::mutex pool_mu;
};

// smallest pooled buffer of >= bytes (and at most 4x: a 1 GB buffer is not kept busy by a
// 1 KB request), else a new one
static hipError_t pool_alloc(fpm_ctx *ctx, void **p, size_t bytes)
{
    {
        std::lock_guard<std::mutex> g(ctx->pool_mu);
        size_t best = SIZE_MAX, bi = 0;
        for (size_t i = 0; i < ctx->pool.size(); i++) {
            const size_t b = ctx->pool[i].second;
            if (b >= bytes && b <= 4 * bytes + 4096 && b < best) { best = b; bi = i; }
            if (best == bytes) break;
        }
        if (best != SIZE_MAX) {
            *p = ctx->pool[bi].first;
            ctx->pool_bytes -= best;
            ctx->pool[bi] = ctx->pool.back();
            ctx->pool.pop_back();
            return hipSuccess;
        }
    }
    return hipMalloc(p, bytes);
}

// back to the pool (the caller's stream work on it is complete), or freed past kPoolBytes
static void pool_free(fpm_ctx *ctx, void *p, size_t bytes)
{
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(ctx->pool_mu);
        if (ctx->pool_bytes + bytes <= fpm_ctx::kPoolBytes) {
            ctx->pool.push_back({p, bytes});
            ctx->pool_bytes += bytes;
            return;
        }
    }
    (void)hipFree(p);
}

// Synchronous copies and memsets run on the context stream, after the work queued there, and
// never on the null stream: the null stream's first use in a process creates one more
// hardware queue (~9 ms in the CLI's trace), and a separate copy stream cost another ~8 ms of
// start-up for no overlap the synchronous copies could use.
static hipError_t ensure_ring(fpm_ctx *ctx)
{
    hipError_t e = hipSuccess;
    if (ctx->ring_ev[fpm_ctx::kRing - 1]) return e;
    for (int i = 0; e == hipSuccess && i < fpm_ctx::kRing; i++) {
        if (!ctx->ring[i]) e = hipHostMalloc(&ctx->ring[i], fpm_ctx::kRingBytes, hipHostMallocDefault);
        if (e == hipSuccess && !ctx->ring_ev[i])
            e = hipEventCreateWithFlags(&ctx->ring_ev[i], hipEventDisableTiming);
    }
    return e;
}

// synchronous copy on the context stream (ordered after the work queued there)
static hipError_t copy_sync(fpm_ctx *ctx, void *dst, const void *src, size_t bytes,
                            hipMemcpyKind kind)
{
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e;
}

static hipError_t memset_sync(fpm_ctx *ctx, void *dst, int v, size_t bytes)
{
    hipError_t e = hipMemsetAsync(dst, v, bytes, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    return e;
}

// Host -> device copy of pageable memory through the context's pinned ring: the caller's
// thread memcpy's piece i into a pinned buffer while the DMA engine moves piece i - 1
// (hipMemcpy from pageable memory stages through the runtime's own buffers one piece at a
// time: ~3.8 GB/s measured on the -fp text).  Synchronous on return.
static hipError_t h2d_staged(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!bytes) return hipSuccess;
    if (bytes < (1u << 20)) return copy_sync(ctx, dst, src, bytes, hipMemcpyHostToDevice);
    hipError_t e = ensure_ring(ctx);
    if (e != hipSuccess) return e;
    const char *s = static_cast<const char *>(src);
    char *d = static_cast<char *>(dst);
    bool used[fpm_ctx::kRing] = {};
    for (size_t off = 0, i = 0; off < bytes; off += fpm_ctx::kRingBytes, i++) {
        const int slot = (int)(i % fpm_ctx::kRing);
        const size_t n = std::min(fpm_ctx::kRingBytes, bytes - off);
        if (used[slot] && (e = hipEventSynchronize(ctx->ring_ev[slot])) != hipSuccess) return e;
        ctx->copier.copy(ctx->ring[slot], s + off, n);
        if ((e = hipMemcpyAsync(d + off, ctx->ring[slot], n, hipMemcpyHostToDevice, ctx->stream)) !=
            hipSuccess)
            return e;
        if ((e = hipEventRecord(ctx->ring_ev[slot], ctx->stream)) != hipSuccess) return e;
        used[slot] = true;
    }
    return hipStreamSynchronize(ctx->stream);
}

static hipError_t ensure_ring(fpm_ctx *ctx);

// Device -> host copy into pageable caller memory through the same pinned ring: the DMA of
// piece i overlaps the caller thread's memcpy of piece i - 1 out of the ring.
static hipError_t d2h_staged(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!bytes) return hipSuccess;
    if (bytes < (64u << 10)) return copy_sync(ctx, dst, src, bytes, hipMemcpyDeviceToHost);
    hipError_t e = ensure_ring(ctx);
    if (e != hipSuccess) return e;
    const char *s = static_cast<const char *>(src);
    char *d = static_cast<char *>(dst);
    const size_t R = fpm_ctx::kRingBytes;
    const size_t n_pieces = (bytes + R - 1) / R;
    auto issue = [&](size_t i) -> hipError_t {
        const int slot = (int)(i % fpm_ctx::kRing);
        const size_t off = i * R, n = std::min(R, bytes - off);
        hipError_t x = hipMemcpyAsync(ctx->ring[slot], s + off, n, hipMemcpyDeviceToHost, ctx->stream);
        if (x == hipSuccess) x = hipEventRecord(ctx->ring_ev[slot], ctx->stream);
        return x;
    };
    for (size_t i = 0; i < std::min<size_t>(n_pieces, fpm_ctx::kRing); i++)
        if ((e = issue(i)) != hipSuccess) return e;
    for (size_t i = 0; i < n_pieces; i++) {
        const int slot = (int)(i % fpm_ctx::kRing);
        const size_t off = i * R, n = std::min(R, bytes - off);
        if ((e = hipEventSynchronize(ctx->ring_ev[slot])) != hipSuccess) return e;
        ctx->copier.copy(d + off, ctx->ring[slot], n);
        if (i + fpm_ctx::kRing < n_pieces && (e = issue(i + fpm_ctx::kRing)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// Caller memory that is not page-locked goes through the context's pinned ring (d2h_staged)
// and is never handed to hipMemcpy directly: the runtime locks a large pageable buffer for the
// DMA (a userptr mapping), and when the caller later frees it (numpy / malloc give such
// buffers back with munmap) the kernel driver evicts and restores the process's GPU queues,
// which stalled whatever ran on the GPU for ~20-30 ms (tools/micro/fp_clock.hip: a ticker
// wave on its own stream saw a 26 ms gap next to the -fp text fetch into freshly malloc'd
// arrays).

static bool host_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// device -> caller host memory, synchronous; the caller has ordered `src`'s producers
static hipError_t copy_out(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!bytes) return hipSuccess;
    if (bytes < (64u << 10) || host_pinned(dst))
        return copy_sync(ctx, dst, src, bytes, hipMemcpyDeviceToHost);
    return d2h_staged(ctx, dst, src, bytes);
}

// caller host memory -> device, synchronous
static hipError_t copy_in(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (!bytes) return hipSuccess;
    if (host_pinned(src)) return copy_sync(ctx, dst, src, bytes, hipMemcpyHostToDevice);
    return h2d_staged(ctx, dst, src, bytes);
}

static hipError_t ensure_aux(fpm_ctx *ctx)
{
    if (ctx->aux) return hipSuccess;
    // default priority: a low-priority side stream (or a high-priority main one) measured
    // slower, the fill then trails the candidate compare instead of sharing its CUs; so did
    // CU-masked streams splitting the CUs between the fill and the compare
    hipError_t e = hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_in, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_fill, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_prefill, hipEventDisableTiming);
    return e;
}

// Device counters -> host (the index build's posting events and sortedness flags, read
// mid-call to pick the path): publish_kernel copies them into the context's mapped pinned
// block and then bumps a sequence word, which the host spins on.  A D2H copy + stream sync
// left the GPU idle ~45 us per call (the sync's wake-up, then the next launch).
// The two halves: publish_counters enqueues the copy (returns its sequence number), and
// wait_counters spins until it has landed, so work enqueued between them runs while the host
// waits (the speculated rank kernel of a resident set's block, compare_impl).
static int publish_counters(fpm_ctx *ctx, const unsigned long long *d_src, uint32_t n,
                            hipStream_t st, unsigned long long *seq_out)
{
    if (!ctx->host_counters) {
        HIP_TRY(hipHostMalloc((void **)&ctx->host_counters, kPubWords * 8,
                              hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer((void **)&ctx->dev_counters, ctx->host_counters, 0));
        memset(ctx->host_counters, 0, kPubWords * 8);
    }
    const unsigned long long seq = ++ctx->pub_seq;
    HIP_TRY(launch_publish(d_src, n, ctx->dev_counters, seq, st));
    *seq_out = seq;
    return FPM_OK;
}

static int wait_counters(fpm_ctx *ctx, unsigned long long seq, hipStream_t st)
{
    volatile unsigned long long *flag = ctx->host_counters + kPubWords - 1;
    for (uint64_t spin = 1;; spin++) {
        if (*flag == seq) break;
        if ((spin & 1023) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q != hipSuccess && q != hipErrorNotReady) return fail(FPM_EHIP, hipGetErrorString(q));
            if (q == hipSuccess && *flag != seq) {
                std::atomic_thread_fence(std::memory_order_seq_cst);
                if (*flag != seq) return fail(FPM_EHIP, "counter publish did not land");
            }
        }
        __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return FPM_OK;
}

static int read_counters(fpm_ctx *ctx, const unsigned long long *d_src, uint32_t n,
                         hipStream_t st)
{
    unsigned long long seq;
    if (int rc = publish_counters(ctx, d_src, n, st, &seq)) return rc;
    return wait_counters(ctx, seq, st);
}

// the dist counters (scratch slot 7): [0] events, [1..64] per-block partials, [65] candidates,
// [66] unsorted flag, [68] largest indexed key; [72..73] idx_kmax_kernel's accumulator
constexpr size_t kCtrWords = 80;

// returns a device buffer of at least `bytes` for scratch slot `id`
static hipError_t scratch(fpm_ctx *ctx, int id, size_t bytes, void **out)
{
    auto &s = ctx->scratch[id];
    if (s.bytes < bytes) {
        if (s.p) { hipError_t e = hipFree(s.p); if (e != hipSuccess) return e; }
        s.p = nullptr;
        s.bytes = 0;
        size_t b = bytes + bytes / 8 + 256;
        hipError_t e = hipMalloc(&s.p, b);
        if (e != hipSuccess) return e;
        s.bytes = b;
        // small buffers (the counters) start zeroed: some words are kept at zero between
        // calls by the kernels themselves (idx_kmax_kernel's accumulator)
        if (b <= 4096) {
            if ((e = memset_sync(ctx, s.p, 0, b)) != hipSuccess) return e;
        }
    }
    *out = s.p;
    return hipSuccess;
}

// RAII-free event bracket: records start before and stop after a launch.
struct TimedLaunch {
    fpm_ctx *ctx; int kid; hipStream_t st; hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(fpm_ctx *c, int k, hipStream_t s) : ctx(c), kid(k), st(s)
    {
        if (ctx->timing) {
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a, st);
        }
    }
    void done()
    {
        if (ctx->timing) {
            (void)hipEventRecord(b, st);
            ctx->ev[kid].push_back({a, b});
        }
    }
};

// errors of fpm_comm.cpp, reported through the same fpm_last_error() text
__attribute__((visibility("hidden"))) int fpm_detail_fail(int code, const std::string &msg)
{
    return fail(code, msg);
}

static int set_device(fpm_ctx *ctx)
{
    if (!ctx) return fail(FPM_EINVAL, "null context");
    HIP_TRY(hipSetDevice(ctx->device));
    return FPM_OK;
}

static hipStream_t pick_stream(fpm_ctx *ctx, void *stream)
{
    return stream ? (hipStream_t)stream : ctx->stream;
}

extern "C" {

int fpm_abi_version(void) { return FPM_ABI_VERSION; }

const char *fpm_last_error(void) { return g_err.c_str(); }

int fpm_device_count(int *count)
{
    if (!count) return fail(FPM_EINVAL, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return FPM_OK;
}

int fpm_ctx_create(int device, fpm_ctx **out)
{
    if (!out) return fail(FPM_EINVAL, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(FPM_ENODEV, "no HIP device visible (fpmash has no CPU fallback)");
    if (device < 0 || device >= n) return fail(FPM_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
        return fail(FPM_ENODEV, std::string("device is ") + prop.gcnArchName +
                                    ", fpmash kernels are built for gfx950 only");
    fpm_ctx *ctx = new fpm_ctx();
    ctx->device = device;
    if (const char *v = getenv("FPM_FILL_COUNTS")) ctx->fill_counts = atoi(v) != 0 ? 1 : 0;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return fail(FPM_EHIP, std::string("context init: ") + hipGetErrorString(e));
    }
    *out = ctx;
    return FPM_OK;
}

void fpm_ctx_destroy(fpm_ctx *ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    fpm_ctx_reset_timing(ctx);
    for (auto &s : ctx->scratch)
        if (s.p) (void)hipFree(s.p);
    if (ctx->host_counters) (void)hipHostFree(ctx->host_counters);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->ev_in) (void)hipEventDestroy(ctx->ev_in);
    if (ctx->ev_fill) (void)hipEventDestroy(ctx->ev_fill);
    if (ctx->ev_prefill) (void)hipEventDestroy(ctx->ev_prefill);
    for (int i = 0; i < fpm_ctx::kRing; i++) {
        if (ctx->ring[i]) (void)hipHostFree(ctx->ring[i]);
        if (ctx->ring_ev[i]) (void)hipEventDestroy(ctx->ring_ev[i]);
    }
    for (auto &b : ctx->pool) (void)hipFree(b.first);
    delete ctx;
}

int fpm_ctx_warm(fpm_ctx *ctx)
{
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(ensure_ring(ctx));
    // one 1 MB copy each way between the ring and the device: the first DMA of a process
    // sets up its copy path (~8-11 ms inside the first staged upload in the CLI's trace)
    constexpr size_t kWarm = 1u << 20;
    void *d = nullptr;
    HIP_TRY(hipMalloc(&d, kWarm));
    hipError_t e = hipMemcpyAsync(d, ctx->ring[0], kWarm, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ctx->ring[1], d, kWarm, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    const hipError_t f = hipFree(d);
    HIP_TRY(e);
    HIP_TRY(f);
    return FPM_OK;
}

void *fpm_ctx_stream(fpm_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int fpm_stream_create(fpm_ctx *ctx, void **stream)
{
    if (!stream) return fail(FPM_EINVAL, "null stream");
    if (int rc = set_device(ctx)) return rc;
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return FPM_OK;
}

int fpm_stream_destroy(fpm_ctx *ctx, void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    if (stream) HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return FPM_OK;
}

int fpm_event_create(fpm_ctx *ctx, void **event)
{
    if (!event) return fail(FPM_EINVAL, "null event");
    if (int rc = set_device(ctx)) return rc;
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *event = e;
    return FPM_OK;
}

int fpm_event_destroy(fpm_ctx *ctx, void *event)
{
    if (int rc = set_device(ctx)) return rc;
    if (event) HIP_TRY(hipEventDestroy((hipEvent_t)event));
    return FPM_OK;
}

int fpm_event_record(fpm_ctx *ctx, void *event, void *stream)
{
    if (!event) return fail(FPM_EINVAL, "null event");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipEventRecord((hipEvent_t)event, pick_stream(ctx, stream)));
    return FPM_OK;
}

int fpm_stream_wait_event(fpm_ctx *ctx, void *stream, void *event)
{
    if (!event) return fail(FPM_EINVAL, "null event");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipStreamWaitEvent(pick_stream(ctx, stream), (hipEvent_t)event, 0));
    return FPM_OK;
}

int fpm_ctx_synchronize(fpm_ctx *ctx)
{
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipDeviceSynchronize());
    return FPM_OK;
}

int fpm_malloc(fpm_ctx *ctx, void **dptr, size_t bytes)
{
    if (int rc = set_device(ctx)) return rc;
    if (!dptr) return fail(FPM_EINVAL, "null dptr");
    hipError_t e = hipMalloc(dptr, bytes ? bytes : 1);
    if (e != hipSuccess) return fail(FPM_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return FPM_OK;
}

int fpm_free(fpm_ctx *ctx, void *dptr)
{
    if (int rc = set_device(ctx)) return rc;
    if (dptr) HIP_TRY(hipFree(dptr));
    return FPM_OK;
}

int fpm_memcpy_h2d(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));   // earlier work on dst is ordered before
    if (bytes) HIP_TRY(h2d_staged(ctx, dst, src, bytes));
    return FPM_OK;
}

int fpm_memcpy_d2h(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(copy_out(ctx, dst, src, bytes));
    return FPM_OK;
}

int fpm_memcpy_d2d(fpm_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    if (int rc = set_device(ctx)) return rc;
    if (bytes) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return FPM_OK;
}

int fpm_memset(fpm_ctx *ctx, void *dptr, int value, size_t bytes)
{
    if (int rc = set_device(ctx)) return rc;
    if (bytes) HIP_TRY(hipMemsetAsync(dptr, value, bytes, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return FPM_OK;
}

int fpm_ctx_set_dist_mode(fpm_ctx *ctx, int mode)
{
    if (!ctx || mode < FPM_DIST_AUTO || mode > FPM_DIST_SPARSE) return fail(FPM_EINVAL, "bad dist mode");
    ctx->dist_mode = mode;
    return FPM_OK;
}

int fpm_ctx_last_dist_stats(fpm_ctx *ctx, int *sparse, uint64_t *events, uint64_t *candidates)
{
    if (!ctx) return fail(FPM_EINVAL, "null context");
    if (sparse) *sparse = ctx->last_sparse;
    if (events) *events = ctx->last_events;
    if (ctx->last_cand == (uint64_t)-1) {
        if (int rc = set_device(ctx)) return rc;
        HIP_TRY(hipStreamSynchronize(ctx->last_cand_stream));
        unsigned long long v = 0;
        HIP_TRY(hipMemcpy(&v, ctx->last_cand_dev, 8, hipMemcpyDeviceToHost));
        ctx->last_cand = v;
    }
    if (candidates) *candidates = ctx->last_cand;
    return FPM_OK;
}

int fpm_ctx_index_rebuilds(fpm_ctx *ctx, uint64_t *count)
{
    if (!ctx || !count) return fail(FPM_EINVAL, "null argument");
    *count = ctx->idx_rebuilds;
    return FPM_OK;
}

int fpm_ctx_spec_stats(fpm_ctx *ctx, uint64_t *hits, uint64_t *misses)
{
    if (!ctx || !hits || !misses) return fail(FPM_EINVAL, "null argument");
    *hits = ctx->spec_hits;
    *misses = ctx->spec_misses;
    return FPM_OK;
}

int fpm_ctx_set_timing(fpm_ctx *ctx, int enable)
{
    if (!ctx) return fail(FPM_EINVAL, "null context");
    ctx->timing = enable != 0;
    return FPM_OK;
}

int fpm_ctx_reset_timing(fpm_ctx *ctx)
{
    if (!ctx) return fail(FPM_EINVAL, "null context");
    for (auto &v : ctx->ev) {
        for (auto &pr : v) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
        v.clear();
    }
    return FPM_OK;
}

int fpm_ctx_kernel_time(fpm_ctx *ctx, int kernel, double *total_ms, uint64_t *launches)
{
    if (!ctx || kernel < 0 || kernel >= FPM_K_COUNT) return fail(FPM_EINVAL, "bad kernel id");
    if (int rc = set_device(ctx)) return rc;
    double t = 0;
    for (auto &pr : ctx->ev[kernel]) {
        HIP_TRY(hipEventSynchronize(pr.second));
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
        t += ms;
    }
    if (total_ms) *total_ms = t;
    if (launches) *launches = ctx->ev[kernel].size();
    return FPM_OK;
}

}  // extern "C"

// ----------------------------------------------------------------------------
// Sketch job: packing + tile plan + merge schedule
// ----------------------------------------------------------------------------
// Rows of one device matrix d_rows[n_rows][s]: rows [0, n_groups) are the final
// sketches, rows >= n_groups hold per-tile / intermediate lists of groups whose
// records span several tiles; those are reduced by pairwise merge rounds.

struct fpm_sketch_job {
    fpm_ctx *ctx = nullptr;
    SketchKParams kp{};
    uint32_t n_groups = 0;
    uint32_t n_rows = 0;
    uint64_t seq_bytes = 0;
    uint64_t n_kmers = 0;
    uint64_t n_tiles = 0;
    uint8_t *d_seq = nullptr;
    TileDesc *d_tiles = nullptr;
    uint64_t *d_rows = nullptr;
    uint32_t *d_count = nullptr;
    MergeDesc *d_merge = nullptr;
    uint32_t class_begin[kTileClasses + 1] = {0};
    std::vector<uint32_t> round_begin;
    std::vector<uint8_t> round_small, sround_small;   // per round: merge_small_kernel
    // long groups: a 1-in-kSampleEvery sample of their tiles is sketched first; its s-th
    // smallest hash bounds what every tile of the group keeps
    uint32_t n_slots = 0;
    TileDesc *d_stiles = nullptr;
    MergeDesc *d_smerge = nullptr;
    uint32_t *d_srow = nullptr;
    uint64_t *d_thr = nullptr;
    uint32_t sclass_begin[kTileClasses + 1] = {0};
    std::vector<uint32_t> sround_begin;
    // sampled groups: one-workgroup selection from their bounded tile lists
    // (group_select_kernel); a pairwise merge plan of the same lists is kept as the fallback
    // for groups whose keys below the cut do not fit in LDS
    uint32_t n_sel = 0;
    SelDesc *d_sel = nullptr;
    uint32_t *d_sel_rows = nullptr, *d_sel_failed = nullptr, *h_sel_failed = nullptr;
    MergeDesc *d_fmerge = nullptr;
    std::vector<uint32_t> fround_begin;
    std::vector<uint8_t> fround_small;
    uint32_t n_ssel = 0;                      // sample selections (first n_ssel of d_sel)
    std::vector<uint32_t> ssel_begin, sel_begin;   // d_sel offsets of each level
    // fallback merge plans (rows >= n_rows live in d_fb_rows, allocated on first use)
    std::vector<std::array<uint32_t, 3>> fplan, sfplan;
    uint32_t n_fb_rows = 0;
    uint64_t *d_fb_rows = nullptr;
    uint32_t *d_fb_count = nullptr;
    MergeDesc *d_sfmerge = nullptr;
    std::vector<uint32_t> sfround_begin;
    std::vector<uint8_t> sfround_small;
    // class-4 tiles all bounded (C5's genomes): the survivors-only tile kernel, whose
    // overflowing tiles (d_redo, count d_redo_n) run again through the plain one
    bool thr4 = false;
    TileDesc *d_redo = nullptr;
    uint32_t *d_redo_n = nullptr;
    uint32_t n4 = 0;                 // class-4 tiles (the redo list's capacity)
    // tight bounds (groups with a selection): each slot's bound is the sample's kt-th smallest
    // hash instead of its s-th (d_kt), the s-th kept as d_thr_safe; a group left with fewer
    // than s hashes (sketch_short_kernel: d_short = count, then the slots) is redone with the
    // safe bound: its tiles and selections again, from the host copies below
    bool tight = false;
    uint32_t *d_kt = nullptr, *d_slot_group = nullptr, *d_short = nullptr;
    uint64_t *d_thr_safe = nullptr;
    std::vector<TileDesc> h_tiles;          // the main tiles by class (class_begin)
    std::vector<SelDesc> h_sel;             // the selections (sample levels, then main)
    TileDesc *d_rtiles = nullptr;           // the redo's subsets (allocated on first use)
    SelDesc *d_rsel = nullptr;
    int32_t last_short = -1;                // groups redone by the last run (-1: no tight bounds)
    // a-priori sample bounds (d_thr[n_slots ..]): a sample left short is redone unbounded
    bool sbounded = false;
    uint32_t *d_sshort = nullptr;           // count, then the slots
    uint64_t *d_sbound0 = nullptr;          // the a-priori sample bounds as staged: restored
                                            // into d_thr at every run (a short sample's redo
                                            // lifts its bound in d_thr)
    std::vector<TileDesc> h_stiles;         // the sample tiles by class (sclass_begin)
    std::vector<uint32_t> h_ssel_tag;       // each sample selection's slot
    int32_t last_sample_short = -1;
    // -M pass (allocated on first use)
    uint32_t *d_mult = nullptr;
    unsigned long long *d_first = nullptr;
    uint64_t *d_ttop = nullptr;
};

static void job_release(fpm_sketch_job *j)
{
    if (!j) return;
    (void)hipSetDevice(j->ctx->device);
    (void)hipFree(j->d_seq); (void)hipFree(j->d_tiles); (void)hipFree(j->d_rows); (void)hipFree(j->d_count);
    (void)hipFree(j->d_merge);
    (void)hipFree(j->d_stiles); (void)hipFree(j->d_smerge); (void)hipFree(j->d_srow);
    (void)hipFree(j->d_thr);
    (void)hipFree(j->d_redo); (void)hipFree(j->d_redo_n);
    (void)hipFree(j->d_kt); (void)hipFree(j->d_slot_group); (void)hipFree(j->d_short);
    (void)hipFree(j->d_thr_safe); (void)hipFree(j->d_rtiles); (void)hipFree(j->d_rsel);
    (void)hipFree(j->d_sshort); (void)hipFree(j->d_sbound0);
    (void)hipFree(j->d_sel); (void)hipFree(j->d_sel_rows); (void)hipFree(j->d_sel_failed);
    (void)hipFree(j->d_fmerge);
    (void)hipFree(j->d_sfmerge);
    (void)hipFree(j->d_fb_rows); (void)hipFree(j->d_fb_count);
    (void)hipFree(j->d_mult); (void)hipFree(j->d_first); (void)hipFree(j->d_ttop);
    if (j->h_sel_failed) (void)hipHostFree(j->h_sel_failed);
}

extern "C" {

}  // extern "C"

// Records to sketch, in the order their groups stream them: `rec_len(r)` bytes at `rec_pos(r)`
// of the device sequence buffer.  Host path: fpm_sketch_stage packs the records itself
// (host_packed); device path: fpm_sketch_stage_seq adopts the buffer seqparse.hip packed.
struct StageRecords {
    std::vector<uint32_t> order;        // records in group order (records of no group left out)
    std::vector<uint64_t> pos, len;     // per record (indexed by record id)
    std::vector<uint32_t> group;        // per record
    uint32_t n_groups = 0;
    const char *host_seq = nullptr;     // host path: record r is host_seq[pos..pos+len)
    uint8_t *d_seq = nullptr;           // device path: packed buffer (ownership moves to the job)
    uint64_t d_seq_bytes = 0;
};

static int stage_core(fpm_ctx *ctx, const fpm_sketch_params *p, StageRecords &R,
                      fpm_sketch_job **job_out);

extern "C" {

int fpm_sketch_stage(fpm_ctx *ctx, const fpm_sketch_params *p, const char *seq,
                     const uint64_t *rec_off, uint32_t n_rec, const uint32_t *group_of_rec,
                     uint32_t n_groups, fpm_sketch_job **job_out)
{
    if (int rc = set_device(ctx)) return rc;
    if (!p || !job_out || (n_rec && (!seq || !rec_off))) return fail(FPM_EINVAL, "null argument");
    *job_out = nullptr;
    if (!group_of_rec) n_groups = n_rec;
    for (uint32_t r = 0; r < n_rec; r++)
        if (rec_off[r + 1] < rec_off[r]) return fail(FPM_EINVAL, "record offsets must be non-decreasing");
    if (group_of_rec)
        for (uint32_t r = 0; r < n_rec; r++)
            if (group_of_rec[r] >= n_groups) return fail(FPM_EINVAL, "group id out of range");
    StageRecords R;
    R.n_groups = n_groups;
    R.host_seq = seq;
    R.pos.resize(n_rec);
    R.len.resize(n_rec);
    R.group.resize(n_rec);
    R.order.resize(n_rec);
    for (uint32_t r = 0; r < n_rec; r++) {
        R.pos[r] = rec_off[r];
        R.len[r] = rec_off[r + 1] - rec_off[r];
        R.group[r] = group_of_rec ? group_of_rec[r] : r;
        R.order[r] = r;
    }
    // records of a group in stream order, groups ascending
    if (group_of_rec)
        std::stable_sort(R.order.begin(), R.order.end(),
                         [&](uint32_t a, uint32_t b) { return R.group[a] < R.group[b]; });
    return stage_core(ctx, p, R, job_out);
}

}  // extern "C"

static int stage_core(fpm_ctx *ctx, const fpm_sketch_params *p, StageRecords &R,
                      fpm_sketch_job **job_out)
{
    if (p->kmer_size < 1 || p->kmer_size > 32) return fail(FPM_EINVAL, "kmer_size must be 1..32");
    if (p->sketch_size < 1) return fail(FPM_EINVAL, "sketch_size must be >= 1");
    const uint32_t k = p->kmer_size, s = p->sketch_size;
    const uint32_t n_groups = R.n_groups;
    const std::vector<uint32_t> &order = R.order;
    SketchKParams kp{};
    kp.k = k; kp.s = s; kp.seed = p->seed; kp.use64 = p->use64 ? 1 : 0;
    kp.canonical = p->noncanonical ? 0 : 1; kp.preserve_case = p->preserve_case ? 1 : 0;
    for (int c = 0; c < 256; c++) {
        kp.alphabet[c] = p->alphabet[c] ? 1 : 0;
        kp.complement[c] = (c >= 'A' && c <= 'Z') ? (uint8_t)kComplAZ[c - 'A'] : (uint8_t)'N';
    }
    kp.alphabet[0] = 0;   // the separator byte is never a k-mer byte
    kp.compl_acgt = 1;
    for (int c = 0; c < 256; c++)
        if (kp.alphabet[c] && c != 'A' && c != 'C' && c != 'G' && c != 'T') kp.compl_acgt = 0;

    // host path: pack records >= k (each followed by 0x00) in group order
    std::vector<uint8_t> packed;
    if (R.host_seq) {
        uint64_t total = 0;
        for (uint32_t r : order)
            if (R.len[r] >= k) total += R.len[r] + 1;
        packed.resize(total);
        uint64_t at = 0;
        for (uint32_t r : order) {
            if (R.len[r] < k) continue;
            memcpy(packed.data() + at, R.host_seq + R.pos[r], R.len[r]);
            packed[at + R.len[r]] = 0;
            R.pos[r] = at;                      // now the packed offset
            at += R.len[r] + 1;
        }
    }
    // cut tiles: a tile covers [byte_off, byte_off + n_bytes) of the packed buffer, records of
    // one group only; short records share a tile while its k-mer starts fit (bytes between
    // them, separators or records shorter than k, hold no valid window)
    std::vector<TileDesc> tiles;
    std::vector<uint32_t> tile_group;
    uint64_t n_kmers = 0;
    uint32_t cur_group = UINT32_MAX;
    bool open = false;
    TileDesc cur{};
    auto close = [&]() {
        if (open) { tiles.push_back(cur); tile_group.push_back(cur_group); open = false; }
    };
    for (uint32_t r : order) {
        const uint64_t l = R.len[r];
        const uint32_t g = R.group[r];
        if (g != cur_group) { close(); cur_group = g; }
        if (l < k) continue;
        const uint64_t poff = R.pos[r];
        const uint64_t nk = l - k + 1;
        n_kmers += nk;
        if (nk > kPackKmers) {
            close();
            for (uint64_t c0 = 0; c0 < nk; c0 += kChunkKmers) {
                uint64_t cn = std::min<uint64_t>(kChunkKmers, nk - c0);
                tiles.push_back(TileDesc{poff + c0, (uint32_t)(cn + k - 1), 0});
                tile_group.push_back(g);
            }
        } else if (open && poff > cur.byte_off + cur.n_bytes &&
                   poff + l - cur.byte_off - k + 1 <= kPackKmers) {
            cur.n_bytes = (uint32_t)(poff + l - cur.byte_off);   // through this record
        } else {
            close();
            cur = TileDesc{poff, (uint32_t)l, 0};
            open = true;
        }
    }
    close();
    for (size_t t = 0; t < tiles.size(); t++) tiles[t].pad = tile_group[t];

    // rows: single-tile groups write their final row, others get temp rows
    std::vector<uint32_t> ntile_of(n_groups, 0);
    for (uint32_t g : tile_group) ntile_of[g]++;
    std::vector<std::vector<uint32_t>> lists(n_groups);
    uint32_t n_rows = n_groups;
    for (size_t t = 0; t < tiles.size(); t++) {
        uint32_t g = tile_group[t];
        if (ntile_of[g] == 1) tiles[t].out_row = g;
        else { tiles[t].out_row = n_rows; lists[g].push_back(n_rows); n_rows++; }
    }
    // long groups (many 4096-k-mer chunks: C5 genomes): every kSampleEvery-th tile is also
    // sketched in a sample pass (own temp rows and merge plan); the sample's s-th smallest
    // hash is >= the group's s-th smallest, so the full pass drops every hash above it and
    // its merges move ~kSampleEvery*s hashes per group instead of every tile's bottom-s.
    // The sample rate per group: every E-th tile, E = the group's k-mers / 8 s within
    // [16, 64], so a sample holds ~8 s k-mers: enough for its s-th smallest (the safe bound)
    // and a tight kt-th one.  C5's 5 Mb genomes: E = 61, C5 23.6 -> 21.9 ms against E = 16
    // (22.8 ms at 16 s k-mers, E = 31), same box, r05x / r05y.
    constexpr uint32_t kSampleEvery = 16;
    std::vector<uint32_t> every(n_groups, kSampleEvery);
    for (uint32_t g = 0; g < n_groups; g++)
        every[g] = (uint32_t)std::min<uint64_t>(
            64, std::max<uint64_t>(kSampleEvery, (uint64_t)ntile_of[g] * kChunkKmers / (8ULL * s)));
    std::vector<uint32_t> slot_of(n_groups, 0);          // 0: not sampled, else slot + 1
    std::vector<TileDesc> stiles;
    std::vector<std::vector<uint32_t>> slists(n_groups);
    std::vector<uint32_t> srow, sgroup;                  // sgroup: each sample tile's group
    {
        std::vector<uint32_t> seen(n_groups, 0);
        for (size_t t = 0; t < tiles.size(); t++) {
            const uint32_t g = tile_group[t];
            const uint64_t sample_kmers = (uint64_t)(ntile_of[g] / every[g]) * kChunkKmers;
            if (ntile_of[g] < 2 * every[g] || sample_kmers < 4ULL * s) continue;
            if (!slot_of[g]) { srow.push_back(0); slot_of[g] = (uint32_t)srow.size(); }
            if (seen[g]++ % every[g] == 0) {
                TileDesc st = tiles[t];
                st.out_row = n_rows;
                st.thr_slot = 0;
                slists[g].push_back(n_rows++);
                stiles.push_back(st);
                sgroup.push_back(g);
            }
        }
        for (size_t t = 0; t < tiles.size(); t++) tiles[t].thr_slot = slot_of[tile_group[t]];
    }
    // list-length estimate per row (steers merge_small_kernel only; results do not depend
    // on it): a tile keeps at most its k-mers and s; a tile of a sampled (thresholded) group
    // keeps ~kSampleEvery * s / tiles of the group's hashes (2x margin)
    std::vector<uint64_t> est(n_rows, s);
    for (size_t t = 0; t < tiles.size(); t++) {
        const uint32_t g = tile_group[t];
        uint64_t e = std::min<uint64_t>(s, tiles[t].n_bytes >= k ? tiles[t].n_bytes - k + 1 : 0);
        if (slot_of[g]) e = std::min<uint64_t>(e, 2ULL * every[g] * s / ntile_of[g] + 64);
        if (tiles[t].out_row < est.size()) est[tiles[t].out_row] = e;
    }
    for (auto &st : stiles)
        if (st.out_row < est.size())
            est[st.out_row] = std::min<uint64_t>(s, st.n_bytes >= k ? st.n_bytes - k + 1 : 0);
    struct Plan { uint32_t a, b, c; };
    // pairwise merge rounds of each group's lists; the last merge writes final_row(g)
    auto plan_rounds = [&](std::vector<std::vector<uint32_t>> &L_of, auto final_row,
                           std::vector<Plan> &plan, std::vector<uint32_t> &rounds,
                           std::vector<uint8_t> &small) {
        rounds.assign(1, 0);
        small.clear();
        for (;;) {
            bool any = false;
            uint64_t round_max = 0;
            for (uint32_t g = 0; g < n_groups; g++) {
                auto &L = L_of[g];
                if (L.size() < 2) continue;
                any = true;
                std::vector<uint32_t> next;
                for (size_t i = 0; i + 1 < L.size(); i += 2) {
                    uint32_t c = (L.size() == 2) ? final_row(g) : n_rows++;
                    plan.push_back({L[i], L[i + 1], c});
                    next.push_back(c);
                    if (est.size() <= c) est.resize(c + 1, s);
                    const uint64_t ea = est[L[i]], eb = est[L[i + 1]];
                    est[c] = std::min<uint64_t>(s, ea + eb);
                    round_max = std::max(round_max, std::max(ea, eb));
                }
                if (L.size() % 2) next.push_back(L.back());
                if (next.size() == 1) next.clear();   // reached the final row
                L.swap(next);
            }
            if (!any) break;
            rounds.push_back((uint32_t)plan.size());
            small.push_back(round_max <= merge_small_cap() ? 1 : 0);
        }
    };
    std::vector<Plan> splan, mplan, fplan;
    std::vector<uint32_t> srb, rb, frb;
    std::vector<uint8_t> ssmall, msmall, fsmall;
    for (uint32_t g = 0; g < n_groups; g++)
        if (slot_of[g]) srow[slot_of[g] - 1] = slists[g].size() == 1 ? slists[g][0] : 0;
    // sampled groups select their sketch (and their sample's) with group_select_kernel; their
    // lists leave the merge plans for fallback plans (pairwise merges only: C5 17.6 vs 2.6 ms).
    // A group with more keys than one workgroup should read (~2^19: a 1 Gb genome's sample
    // holds 62 M) is split into chunks of rows selected in parallel, then the chunks' sketches
    // are selected again (a tree of levels, one launch per level).
    std::vector<uint32_t> sel_rows;
    std::vector<std::vector<SelDesc>> ssel_lv, sel_lv;
    const bool use_sel = (uint64_t)s + s / 8 + 64 <= group_select_cap();
    // A sample's tiles keep only the hashes below an a-priori bound: hash values are uniform,
    // so of a sample's N windows ~frac N lie below frac of the hash range, and frac =
    // (1.25 s + 16 sqrt(s)) / N leaves >= s of them (C5: ~14k of a sample's 82k) with ~40
    // standard deviations to spare.  The sample's selection then reads ~6x fewer keys.  A
    // sample left with fewer than s (values repeated across its tiles) gives its group no
    // bound, as a sample shorter than s always did (the sketches do not depend on it).
    std::vector<uint64_t> sbound(srow.size(), ~0ULL);
    if (use_sel && !srow.empty()) {
        std::vector<uint64_t> ns(srow.size(), 0);
        for (size_t i = 0; i < stiles.size(); i++)
            ns[slot_of[sgroup[i]] - 1] += stiles[i].n_bytes >= k ? stiles[i].n_bytes - k + 1 : 0;
        const double range = kp.use64 ? 18446744073709551616.0 : 4294967296.0;
        for (size_t i = 0; i < srow.size(); i++) {
            const double frac = (1.25 * s + 16.0 * std::sqrt((double)s)) / std::max<double>(1, ns[i]);
            if (frac < 0.5) sbound[i] = (uint64_t)(frac * range);
        }
        const uint32_t n_sl = (uint32_t)srow.size();
        for (size_t i = 0; i < stiles.size(); i++) {
            const uint32_t sl = slot_of[sgroup[i]];
            if (sbound[sl - 1] != ~0ULL) {
                stiles[i].thr_slot = n_sl + sl;              // d_thr[n_slots + slot]
                if (stiles[i].out_row < est.size())
                    est[stiles[i].out_row] = std::min<uint64_t>(
                        est[stiles[i].out_row], (uint64_t)(2.0 * (double)sbound[sl - 1] / range *
                                                           stiles[i].n_bytes) + 64);
            }
        }
    }
    // tags (optional): per level, the slot of each descriptor (sample selections carry slot
    // 0xFFFFFFFF on the device; the host finds a group's descriptors by the tag)
    auto build_sel = [&](const std::vector<uint32_t> &rows0, uint32_t final_row, uint32_t slot,
                         std::vector<std::vector<SelDesc>> &lv,
                         std::vector<std::vector<uint32_t>> *tags = nullptr, uint32_t tag = 0) {
        constexpr uint64_t kKeysPerWG = 1u << 19;
        constexpr size_t kRowsPerWG = 4096;
        std::vector<uint32_t> cur = rows0;
        for (size_t level = 0;; level++) {
            if (lv.size() <= level) lv.resize(level + 1);
            if (tags && tags->size() <= level) tags->resize(level + 1);
            std::vector<std::pair<size_t, size_t>> ch;
            size_t a = 0;
            uint64_t acc = 0;
            for (size_t i = 0; i < cur.size(); i++) {
                const uint64_t e = est[cur[i]];
                if (i > a && (acc + e > kKeysPerWG || i - a >= kRowsPerWG)) {
                    ch.push_back({a, i});
                    a = i;
                    acc = 0;
                }
                acc += e;
            }
            ch.push_back({a, cur.size()});
            if (ch.size() == 1) {
                lv[level].push_back(SelDesc{(uint32_t)sel_rows.size(), (uint32_t)cur.size(),
                                            final_row, slot});
                if (tags) (*tags)[level].push_back(tag);
                sel_rows.insert(sel_rows.end(), cur.begin(), cur.end());
                return;
            }
            std::vector<uint32_t> next;
            for (auto &c : ch) {
                const uint32_t r = n_rows++;
                if (est.size() <= r) est.resize(r + 1, s);
                uint64_t sum = 0;
                for (size_t i = c.first; i < c.second; i++) sum += est[cur[i]];
                est[r] = std::min<uint64_t>(s, sum);
                lv[level].push_back(SelDesc{(uint32_t)sel_rows.size(),
                                            (uint32_t)(c.second - c.first), r, slot});
                if (tags) (*tags)[level].push_back(tag);
                sel_rows.insert(sel_rows.end(), cur.begin() + c.first, cur.begin() + c.second);
                next.push_back(r);
            }
            cur.swap(next);
        }
    };
    std::vector<Plan> sfplan;
    std::vector<uint32_t> sfrb;
    std::vector<uint8_t> sfsmall;
    std::vector<std::vector<uint32_t>> sflists(n_groups), flists(n_groups);
    std::vector<std::vector<uint32_t>> ssel_tag_lv;
    if (use_sel)
        for (uint32_t g = 0; g < n_groups; g++) {
            if (!slot_of[g] || slists[g].size() < 2) continue;
            const uint32_t r = n_rows++;                    // the sample's sketch row
            srow[slot_of[g] - 1] = r;
            build_sel(slists[g], r, 0xFFFFFFFFu, ssel_lv, &ssel_tag_lv, slot_of[g] - 1);
            sflists[g].swap(slists[g]);
        }
    plan_rounds(slists, [&](uint32_t g) {
        const uint32_t r = n_rows++;
        srow[slot_of[g] - 1] = r;
        return r;
    }, splan, srb, ssmall);
    if (use_sel)
        for (uint32_t g = 0; g < n_groups; g++) {
            if (!slot_of[g] || lists[g].size() < 2) continue;
            build_sel(lists[g], g, slot_of[g] - 1, sel_lv);
            flists[g].swap(lists[g]);
        }
    plan_rounds(lists, [](uint32_t g) { return g; }, mplan, rb, msmall);
    // d_sel: the sample levels, then the main levels; level boundaries for the launches
    std::vector<SelDesc> sel;
    std::vector<uint32_t> ssel_begin{0}, sel_begin, ssel_tag;
    for (auto &l : ssel_lv) {
        sel.insert(sel.end(), l.begin(), l.end());
        ssel_begin.push_back((uint32_t)sel.size());
    }
    for (auto &l : ssel_tag_lv) ssel_tag.insert(ssel_tag.end(), l.begin(), l.end());
    sel_begin.push_back((uint32_t)sel.size());
    for (auto &l : sel_lv) {
        sel.insert(sel.end(), l.begin(), l.end());
        sel_begin.push_back((uint32_t)sel.size());
    }
    // the fallback plans' intermediate rows come last: they are allocated only if a selection
    // fails (a C5 share holds ~1.2 M tile rows of s u64: the fallback rows would double that)
    const uint32_t n_core = n_rows;
    if (use_sel) {
        plan_rounds(sflists, [&](uint32_t g) { return srow[slot_of[g] - 1]; }, sfplan, sfrb,
                    sfsmall);
        plan_rounds(flists, [](uint32_t g) { return g; }, fplan, frb, fsmall);
    }

    // tiles ordered by capacity class
    auto order_by_class = [&](const std::vector<TileDesc> &in, std::vector<TileDesc> &out,
                              uint32_t *begin) {
        out.clear();
        out.reserve(in.size());
        begin[0] = 0;
        for (int c = 0; c < kTileClasses; c++) {
            for (auto &t : in)
                if (tile_class(t.n_bytes - k + 1) == c) out.push_back(t);
            begin[c + 1] = (uint32_t)out.size();
        }
        return out.size() == in.size();
    };
    std::vector<TileDesc> by_class, sby_class;
    uint32_t class_begin[kTileClasses + 1] = {0}, sclass_begin[kTileClasses + 1] = {0};
    if (!order_by_class(tiles, by_class, class_begin) ||
        !order_by_class(stiles, sby_class, sclass_begin))
        return fail(FPM_EINVAL, "internal: tile exceeds capacity");

    auto *job = new fpm_sketch_job();
    job->ctx = ctx;
    job->kp = kp;
    job->n_groups = n_groups;
    job->n_rows = n_core;
    job->n_fb_rows = n_rows - n_core;
    for (auto &pl : fplan) job->fplan.push_back({pl.a, pl.b, pl.c});
    for (auto &pl : sfplan) job->sfplan.push_back({pl.a, pl.b, pl.c});
    job->seq_bytes = R.host_seq ? packed.size() : R.d_seq_bytes;
    job->n_kmers = n_kmers;
    job->n_tiles = tiles.size();
    memcpy(job->class_begin, class_begin, sizeof(class_begin));
    memcpy(job->sclass_begin, sclass_begin, sizeof(sclass_begin));
    job->round_begin = rb;
    job->sround_begin = srb;
    job->round_small = msmall;
    job->sround_small = ssmall;
    job->n_slots = (uint32_t)srow.size();
    job->ssel_begin = ssel_begin;
    job->sel_begin = sel_begin;
    job->n_ssel = ssel_begin.back();
    job->n_sel = sel_begin.back() - sel_begin.front();
    job->sfround_begin = sfrb;
    job->sfround_small = sfsmall;
    job->fround_begin = frb;
    job->fround_small = fsmall;

    hipError_t e = hipSuccess;
    auto alloc = [&](void **ptr, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(ptr, bytes ? bytes : 16);
    };
    if (R.host_seq) alloc((void **)&job->d_seq, packed.size() + 64);
    else { job->d_seq = R.d_seq; R.d_seq = nullptr; }   // the parse's packed records
    alloc((void **)&job->d_tiles, by_class.size() * sizeof(TileDesc));
    alloc((void **)&job->d_rows, (size_t)n_core * s * sizeof(uint64_t));
    alloc((void **)&job->d_count, (size_t)n_core * sizeof(uint32_t));
    // groups without any k-mer keep count 0: zeroed once here (every run rewrites the count
    // of each group that has tiles: the tile kernel or the last merge of its group)
    if (e == hipSuccess) e = memset_sync(ctx, job->d_count, 0, (size_t)n_core * sizeof(uint32_t));
    alloc((void **)&job->d_merge, mplan.size() * sizeof(MergeDesc));
    alloc((void **)&job->d_stiles, sby_class.size() * sizeof(TileDesc));
    alloc((void **)&job->d_smerge, splan.size() * sizeof(MergeDesc));
    alloc((void **)&job->d_srow, srow.size() * sizeof(uint32_t));
    alloc((void **)&job->d_thr, 2 * srow.size() * sizeof(uint64_t));   // main, then sample bounds
    alloc((void **)&job->d_sel, sel.size() * sizeof(SelDesc));
    alloc((void **)&job->d_sel_rows, sel_rows.size() * sizeof(uint32_t));
    alloc((void **)&job->d_sel_failed, (sel.size() + 2) * sizeof(uint32_t));
    if (e == hipSuccess && !sel.empty())
        e = hipHostMalloc((void **)&job->h_sel_failed, 3 * sizeof(uint32_t), hipHostMallocDefault);
    // tight bounds where every sampled group has a selection: kt = f s + 8 sqrt(f s) + 32 of
    // the sample's hashes (f = the group's sampled share of tiles), so ~kt / f >= s of the
    // group's distinct hashes lie below it with ~8 standard deviations to spare (C5 at E = 61:
    // ~300 of the sample's 10,000; the group keeps ~18k hashes instead of ~160k)
    std::vector<uint32_t> kt, slot_group;
    if (use_sel && !srow.empty() && !sel.empty()) {
        kt.assign(srow.size(), s);
        slot_group.assign(srow.size(), 0);
        for (uint32_t g = 0; g < n_groups; g++) {
            if (!slot_of[g]) continue;
            const uint32_t i = slot_of[g] - 1;
            slot_group[i] = g;
            const double f = (double)((ntile_of[g] + every[g] - 1) / every[g]) / ntile_of[g];
            const double fs = f * s;
            kt[i] = (uint32_t)std::min<double>(s, std::ceil(fs + 8.0 * std::sqrt(fs) + 32.0));
        }
        job->tight = true;
        alloc((void **)&job->d_kt, kt.size() * sizeof(uint32_t));
        alloc((void **)&job->d_slot_group, slot_group.size() * sizeof(uint32_t));
        alloc((void **)&job->d_short, (srow.size() + 1) * sizeof(uint32_t));
        alloc((void **)&job->d_thr_safe, srow.size() * sizeof(uint64_t));
        job->h_tiles = by_class;
        job->h_sel = sel;
        job->last_short = 0;
        bool any_sb = false;
        for (uint64_t b : sbound) any_sb = any_sb || b != ~0ULL;
        if (any_sb) {
            job->sbounded = true;
            job->h_stiles = sby_class;
            job->h_ssel_tag = ssel_tag;
            job->last_sample_short = 0;
            alloc((void **)&job->d_sshort, (srow.size() + 1) * sizeof(uint32_t));
            alloc((void **)&job->d_sbound0, srow.size() * sizeof(uint64_t));
        }
    }
    {
        // the survivors-only tile kernel for the class-4 tiles when every one carries its
        // group's bound and that bound leaves few survivors per tile: a group's main pass keeps
        // about kSampleEvery * s of its hashes (the sample's s-th smallest bounds them), so a
        // tile keeps ~kSampleEvery * s / (the group's tiles); est (2x margin + 64, above) must
        // stay within half of what one tile holds, or most tiles would be hashed twice (their
        // survivors overflow and the plain kernel redoes them).  (C5 one GPU: 31.2 -> 25.8 ms,
        // same box, r04; C5 tiles: est 326 of 1,024)
        const uint32_t b4 = class_begin[4], n4 = class_begin[5] - b4;
        // (tight bounds: ~kt / f survivors per group; a short group's redo under the safe bound
        // keeps ~E s per group, and its tiles that overflow are redone by the plain kernel)
        std::vector<uint64_t> slot_est(srow.size() + 1, ~0ULL);
        for (uint32_t g = 0; g < n_groups; g++) {
            if (!slot_of[g]) continue;
            const double f = (double)((ntile_of[g] + every[g] - 1) / every[g]) / ntile_of[g];
            slot_est[slot_of[g]] = job->tight
                                       ? (uint64_t)(2.0 * kt[slot_of[g] - 1] / f / ntile_of[g]) + 64
                                       : 2ULL * every[g] * s / ntile_of[g] + 64;
        }
        bool all = n4 > 0;
        for (uint32_t i = 0; all && i < n4; i++) {
            const uint32_t sl = by_class[b4 + i].thr_slot;
            all = sl != 0 && slot_est[sl] <= kThrTileKeys / 2;
        }
        job->thr4 = all;
        job->n4 = n4;
        if (all) {
            alloc((void **)&job->d_redo, (size_t)n4 * sizeof(TileDesc));
            alloc((void **)&job->d_redo_n, sizeof(uint32_t));
        }
    }
    if (e != hipSuccess) {
        job_release(job);
        delete job;
        return fail(FPM_ENOMEM, std::string("sketch staging alloc: ") + hipGetErrorString(e));
    }
    auto descs = [&](const std::vector<Plan> &plan) {
        std::vector<MergeDesc> md(plan.size());
        for (size_t i = 0; i < plan.size(); i++) {
            md[i].a = job->d_rows + (uint64_t)plan[i].a * s;
            md[i].alen = job->d_count + plan[i].a;
            md[i].b = job->d_rows + (uint64_t)plan[i].b * s;
            md[i].blen = job->d_count + plan[i].b;
            md[i].c = job->d_rows + (uint64_t)plan[i].c * s;
            md[i].clen = job->d_count + plan[i].c;
        }
        return md;
    };
    const std::vector<MergeDesc> md = descs(mplan), smd = descs(splan);
    if (!packed.empty()) e = h2d_staged(ctx, job->d_seq, packed.data(), packed.size());
    if (e == hipSuccess && !by_class.empty())
        e = copy_in(ctx, job->d_tiles, by_class.data(), by_class.size() * sizeof(TileDesc));
    if (e == hipSuccess && !md.empty())
        e = copy_in(ctx, job->d_merge, md.data(), md.size() * sizeof(MergeDesc));
    if (e == hipSuccess && !sby_class.empty())
        e = copy_in(ctx, job->d_stiles, sby_class.data(), sby_class.size() * sizeof(TileDesc));
    if (e == hipSuccess && !smd.empty())
        e = copy_in(ctx, job->d_smerge, smd.data(), smd.size() * sizeof(MergeDesc));
    if (e == hipSuccess && !srow.empty())
        e = copy_in(ctx, job->d_srow, srow.data(), srow.size() * sizeof(uint32_t));
    if (e == hipSuccess && !sel.empty())
        e = copy_in(ctx, job->d_sel, sel.data(), sel.size() * sizeof(SelDesc));
    if (e == hipSuccess && !sel_rows.empty())
        e = copy_in(ctx, job->d_sel_rows, sel_rows.data(), sel_rows.size() * sizeof(uint32_t));
    if (e == hipSuccess && !sbound.empty())
        e = copy_in(ctx, job->d_thr + srow.size(), sbound.data(), sbound.size() * sizeof(uint64_t));
    if (e == hipSuccess && job->d_sbound0)
        e = copy_in(ctx, job->d_sbound0, sbound.data(), sbound.size() * sizeof(uint64_t));
    if (e == hipSuccess && !kt.empty())
        e = copy_in(ctx, job->d_kt, kt.data(), kt.size() * sizeof(uint32_t));
    if (e == hipSuccess && !slot_group.empty())
        e = copy_in(ctx, job->d_slot_group, slot_group.data(), slot_group.size() * sizeof(uint32_t));
    if (e != hipSuccess) {
        job_release(job);
        delete job;
        return fail(FPM_EHIP, std::string("sketch staging copy: ") + hipGetErrorString(e));
    }
    *job_out = job;
    return FPM_OK;
}

// the fallback merge plans' descriptors (first failure of a selection): intermediate rows in
// a buffer of their own
static int fallback_descs(fpm_sketch_job *job)
{
    if (job->d_fmerge || job->d_sfmerge) return FPM_OK;
    const uint64_t s = job->kp.s;
    if (job->n_fb_rows) {
        HIP_TRY(hipMalloc(&job->d_fb_rows, (size_t)job->n_fb_rows * s * sizeof(uint64_t)));
        HIP_TRY(hipMalloc(&job->d_fb_count, (size_t)job->n_fb_rows * sizeof(uint32_t)));
    }
    auto row = [&](uint32_t r) { return r < job->n_rows ? job->d_rows + r * s
                                                       : job->d_fb_rows + (r - job->n_rows) * s; };
    auto cnt = [&](uint32_t r) { return r < job->n_rows ? job->d_count + r
                                                       : job->d_fb_count + (r - job->n_rows); };
    auto upload = [&](const std::vector<std::array<uint32_t, 3>> &plan, MergeDesc **dst) -> int {
        std::vector<MergeDesc> md(plan.size());
        for (size_t i = 0; i < plan.size(); i++)
            md[i] = MergeDesc{row(plan[i][0]), cnt(plan[i][0]), row(plan[i][1]), cnt(plan[i][1]),
                              row(plan[i][2]), cnt(plan[i][2])};
        HIP_TRY(hipMalloc(dst, std::max<size_t>(1, md.size()) * sizeof(MergeDesc)));
        if (!md.empty())
            HIP_TRY(copy_in(job->ctx, *dst, md.data(), md.size() * sizeof(MergeDesc)));
        return FPM_OK;
    };
    if (int rc = upload(job->fplan, &job->d_fmerge)) return rc;
    return upload(job->sfplan, &job->d_sfmerge);
}

// device room for a redo's tile and selection subsets (allocated on first use)
static int redo_buffers(fpm_sketch_job *job)
{
    if (!job->d_rtiles)
        HIP_TRY(hipMalloc((void **)&job->d_rtiles,
                          std::max<size_t>(1, std::max(job->h_tiles.size(), job->h_stiles.size())) *
                              sizeof(TileDesc)));
    if (!job->d_rsel)
        HIP_TRY(hipMalloc((void **)&job->d_rsel, std::max<size_t>(1, job->h_sel.size()) * sizeof(SelDesc)));
    return FPM_OK;
}

// The samples an a-priori bound left short (slots in d_sshort[1 ..], bounds lifted by
// sketch_sample_short_kernel): their sample tiles and sample selections once more
template <typename TilesPass>
static int redo_sample_short(fpm_sketch_job *job, uint32_t n_short, hipStream_t st,
                             TilesPass &tiles_pass)
{
    fpm_ctx *ctx = job->ctx;
    std::vector<uint32_t> slots(n_short);
    HIP_TRY(hipMemcpyAsync(slots.data(), job->d_sshort + 1, n_short * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<uint8_t> is_short(job->n_slots + 1, 0);
    for (uint32_t i : slots)
        if (i < job->n_slots) is_short[i] = 1;
    std::vector<TileDesc> sub;
    uint32_t begin[kTileClasses + 1] = {0};
    for (int c = 0; c < kTileClasses; c++) {
        for (uint32_t t = job->sclass_begin[c]; t < job->sclass_begin[c + 1]; t++) {
            const TileDesc &td = job->h_stiles[t];
            if (td.thr_slot > job->n_slots && is_short[td.thr_slot - job->n_slots - 1]) sub.push_back(td);
        }
        begin[c + 1] = (uint32_t)sub.size();
    }
    std::vector<SelDesc> rsel;
    std::vector<uint32_t> rbegin{0};
    for (size_t l = 0; l + 1 < job->ssel_begin.size(); l++) {
        for (uint32_t i = job->ssel_begin[l]; i < job->ssel_begin[l + 1]; i++)
            if (i < job->h_ssel_tag.size() && job->h_ssel_tag[i] < job->n_slots &&
                is_short[job->h_ssel_tag[i]])
                rsel.push_back(job->h_sel[i]);
        rbegin.push_back((uint32_t)rsel.size());
    }
    if (int rc = redo_buffers(job)) return rc;
    if (!sub.empty()) HIP_TRY(copy_in(ctx, job->d_rtiles, sub.data(), sub.size() * sizeof(TileDesc)));
    if (!rsel.empty()) HIP_TRY(copy_in(ctx, job->d_rsel, rsel.data(), rsel.size() * sizeof(SelDesc)));
    if (int rc = tiles_pass(job->d_rtiles, begin, false)) return rc;
    for (size_t l = 0; l + 1 < rbegin.size(); l++) {
        const uint32_t b = rbegin[l], n = rbegin[l + 1] - b;
        if (!n) continue;
        TimedLaunch tl(ctx, FPM_K_MERGE, st);
        HIP_TRY(launch_group_select(job->d_rsel + b, n, job->d_sel_rows, job->d_rows, job->d_count,
                                    job->kp.s, job->d_thr, job->d_sel_failed + 1, st));
        tl.done();
    }
    return FPM_OK;
}

// The groups a tight bound left short (their slots in d_short[1 ..], bounds already raised
// to the safe ones by sketch_short_kernel): their main tiles and selections once more
template <typename TilesPass>
static int redo_short(fpm_sketch_job *job, uint32_t n_short, hipStream_t st, TilesPass &tiles_pass)
{
    fpm_ctx *ctx = job->ctx;
    std::vector<uint32_t> slots(n_short);
    HIP_TRY(hipMemcpyAsync(slots.data(), job->d_short + 1, n_short * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<uint8_t> is_short(job->n_slots + 1, 0);
    for (uint32_t i : slots)
        if (i < job->n_slots) is_short[i] = 1;
    std::vector<TileDesc> sub;
    uint32_t begin[kTileClasses + 1] = {0};
    for (int c = 0; c < kTileClasses; c++) {
        for (uint32_t t = job->class_begin[c]; t < job->class_begin[c + 1]; t++) {
            const TileDesc &td = job->h_tiles[t];
            if (td.thr_slot && is_short[td.thr_slot - 1]) sub.push_back(td);
        }
        begin[c + 1] = (uint32_t)sub.size();
    }
    std::vector<SelDesc> rsel;
    std::vector<uint32_t> rbegin{0};
    for (size_t l = 0; l + 1 < job->sel_begin.size(); l++) {
        for (uint32_t i = job->sel_begin[l]; i < job->sel_begin[l + 1]; i++) {
            const SelDesc &d = job->h_sel[i];
            if (d.slot != 0xFFFFFFFFu && d.slot < job->n_slots && is_short[d.slot]) rsel.push_back(d);
        }
        rbegin.push_back((uint32_t)rsel.size());
    }
    if (int rc = redo_buffers(job)) return rc;
    if (!sub.empty()) HIP_TRY(copy_in(ctx, job->d_rtiles, sub.data(), sub.size() * sizeof(TileDesc)));
    if (!rsel.empty()) HIP_TRY(copy_in(ctx, job->d_rsel, rsel.data(), rsel.size() * sizeof(SelDesc)));
    if (int rc = tiles_pass(job->d_rtiles, begin, true)) return rc;
    for (size_t l = 0; l + 1 < rbegin.size(); l++) {
        const uint32_t b = rbegin[l], n = rbegin[l + 1] - b;
        if (!n) continue;
        TimedLaunch tl(ctx, FPM_K_MERGE, st);
        HIP_TRY(launch_group_select(job->d_rsel + b, n, job->d_sel_rows, job->d_rows, job->d_count,
                                    job->kp.s, job->d_thr, job->d_sel_failed, st));
        tl.done();
    }
    return FPM_OK;
}

extern "C" {

int fpm_sketch_run(fpm_sketch_job *job, void *stream)
{
    if (!job) return fail(FPM_EINVAL, "null job");
    fpm_ctx *ctx = job->ctx;
    if (int rc = set_device(ctx)) return rc;
    hipStream_t st = pick_stream(ctx, stream);
    auto tiles_pass = [&](const TileDesc *d_t, const uint32_t *begin, bool main) -> int {
        for (int c = 0; c < kTileClasses; c++) {
            uint32_t b = begin[c], n = begin[c + 1] - b;
            if (!n) continue;
            TimedLaunch tl(ctx, FPM_K_SKETCH, st);
            if (main && c == 4 && job->thr4) {
                HIP_TRY(hipMemsetAsync(job->d_redo_n, 0, sizeof(uint32_t), st));
                HIP_TRY(launch_sketch_tiles_thr(job->d_seq, d_t + b, n, job->kp, job->d_thr,
                                                job->d_rows, job->d_count, job->d_redo,
                                                job->d_redo_n, st));
                // the tiles whose survivors did not fit, again through the plain kernel; the
                // count stays on the device (the list holds at most n: one entry per tile)
                HIP_TRY(launch_sketch_redo(job->d_seq, job->d_redo, job->d_redo_n, n, job->kp,
                                           job->d_thr, job->d_rows, job->d_count, st));
            } else {
                HIP_TRY(launch_sketch_tiles(c, job->d_seq, d_t + b, n, job->kp, job->d_thr,
                                            job->d_rows, job->d_count, st));
            }
            tl.done();
        }
        return FPM_OK;
    };
    auto merge_pass = [&](const MergeDesc *d_m, const std::vector<uint32_t> &rounds,
                          const std::vector<uint8_t> &small) -> int {
        for (size_t r = 0; r + 1 < rounds.size(); r++) {
            uint32_t b = rounds[r], n = rounds[r + 1] - b;
            TimedLaunch tl(ctx, FPM_K_MERGE, st);
            const bool sm = g_merge_small_env == 2 ||
                            (g_merge_small_env != 0 && r < small.size() && small[r]);
            HIP_TRY(launch_merge(d_m + b, n, job->kp.s, sm, st));
            tl.done();
        }
        return FPM_OK;
    };
    // failure flags: [0] main selections, [1] sample selections, [2..] per selection
    uint32_t *fail_main = job->d_sel_failed, *fail_samp = job->d_sel_failed + 1;
    if (job->n_ssel + job->n_sel)
        HIP_TRY(hipMemsetAsync(job->d_sel_failed, 0, (job->n_ssel + job->n_sel + 2) * sizeof(uint32_t),
                               st));
    if (job->n_slots) {   // sample pass of long groups -> per-group hash bounds
        if (job->sbounded)   // the bounds as staged (a previous run's redo lifted some)
            HIP_TRY(hipMemcpyAsync(job->d_thr + job->n_slots, job->d_sbound0,
                                   job->n_slots * sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
        if (int rc = tiles_pass(job->d_stiles, job->sclass_begin, false)) return rc;
        if (job->n_ssel) {
            for (size_t l = 0; l + 1 < job->ssel_begin.size(); l++) {
                const uint32_t b = job->ssel_begin[l], n = job->ssel_begin[l + 1] - b;
                TimedLaunch tl(ctx, FPM_K_MERGE, st);
                HIP_TRY(launch_group_select(job->d_sel + b, n, job->d_sel_rows, job->d_rows,
                                            job->d_count, job->kp.s, job->d_thr, fail_samp, st));
                tl.done();
            }
            HIP_TRY(hipMemcpyAsync(job->h_sel_failed + 1, fail_samp, sizeof(uint32_t),
                                   hipMemcpyDeviceToHost, st));
        }
        if (int rc = merge_pass(job->d_smerge, job->sround_begin, job->sround_small)) return rc;
        if (job->n_ssel) {
            auto sample_fallback = [&]() -> int {
                if (int rc = fallback_descs(job)) return rc;
                return merge_pass(job->d_sfmerge, job->sfround_begin, job->sfround_small);
            };
            // samples their a-priori bound left short, counted before the one host read that
            // also fetches the selections' failure flag (a listing without `raise` changes
            // nothing but the list, so a count stale from a failed selection is harmless: after
            // the fallback the samples are counted again); a redo lists them again with their
            // bounds lifted
            auto list_sample_short = [&](bool raise) -> int {
                HIP_TRY(hipMemsetAsync(job->d_sshort, 0, sizeof(uint32_t), st));
                HIP_TRY(launch_sketch_sample_short(job->d_srow, job->n_slots, job->d_count,
                                                   job->kp.s, job->d_thr + job->n_slots,
                                                   job->d_sshort, job->d_sshort + 1, raise, st));
                HIP_TRY(hipMemcpyAsync(job->h_sel_failed + 2, job->d_sshort, sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, st));
                return FPM_OK;
            };
            if (job->sbounded)
                if (int rc = list_sample_short(false)) return rc;
            HIP_TRY(hipStreamSynchronize(st));
            if (job->h_sel_failed[1]) {
                if (int rc = sample_fallback()) return rc;
                if (job->sbounded) {
                    if (int rc = list_sample_short(false)) return rc;
                    HIP_TRY(hipStreamSynchronize(st));
                }
            }
            if (job->sbounded) {
                // samples left short: redone unbounded
                const uint32_t n_ss = job->h_sel_failed[2];
                job->last_sample_short = (int32_t)n_ss;
                if (n_ss) {
                    if (int rc = list_sample_short(true)) return rc;   // the same list, lifted
                    HIP_TRY(hipMemsetAsync(fail_samp, 0, sizeof(uint32_t), st));
                    if (int rc = redo_sample_short(job, n_ss, st, tiles_pass)) return rc;
                    HIP_TRY(hipMemcpyAsync(job->h_sel_failed + 1, fail_samp, sizeof(uint32_t),
                                           hipMemcpyDeviceToHost, st));
                    HIP_TRY(hipStreamSynchronize(st));
                    if (job->h_sel_failed[1])
                        if (int rc = sample_fallback()) return rc;
                }
            }
        }
        HIP_TRY(launch_sketch_threshold(job->d_srow, job->n_slots, job->d_rows, job->d_count,
                                        job->kp.s, job->tight ? job->d_kt : nullptr, job->d_thr,
                                        job->tight ? job->d_thr_safe : nullptr, st));
    }
    // (the selections of each batch of genomes on a side stream beside the next batch's
    // tiles measured a wash on C5: the 120 KB-LDS selection workgroups take the tiles' CUs)
    if (int rc = tiles_pass(job->d_tiles, job->class_begin, true)) return rc;
    const bool tight = job->tight && job->n_slots;
    if (job->n_sel) {
        for (size_t l = 0; l + 1 < job->sel_begin.size(); l++) {
            const uint32_t b = job->sel_begin[l], n = job->sel_begin[l + 1] - b;
            TimedLaunch tl(ctx, FPM_K_MERGE, st);
            HIP_TRY(launch_group_select(job->d_sel + b, n, job->d_sel_rows, job->d_rows,
                                        job->d_count, job->kp.s, job->d_thr, fail_main, st));
            tl.done();
        }
        HIP_TRY(hipMemcpyAsync(job->h_sel_failed, fail_main, sizeof(uint32_t),
                               hipMemcpyDeviceToHost, st));
    }
    if (int rc = merge_pass(job->d_merge, job->round_begin, job->round_small)) return rc;
    if (job->n_sel) {
        // a selection that did not fit (more repeated values below the cut than LDS holds):
        // the pairwise merges of every sampled group's lists (rare; one host round trip)
        auto fallback = [&]() -> int {
            if (int rc = fallback_descs(job)) return rc;
            return merge_pass(job->d_fmerge, job->fround_begin, job->fround_small);
        };
        // the groups the tight bound left short, counted before the one host read that also
        // fetches the selections' failure flag (a listing without `raise` changes nothing but
        // the list, so a count stale from a failed selection is harmless: after the fallback
        // the groups are counted again); a redo lists them again with their bounds raised
        auto list_short = [&](bool raise) -> int {
            HIP_TRY(hipMemsetAsync(job->d_short, 0, sizeof(uint32_t), st));
            HIP_TRY(launch_sketch_short(job->d_slot_group, job->n_slots, job->d_count, job->kp.s,
                                        job->d_thr, job->d_thr_safe, job->d_short, job->d_short + 1,
                                        raise, st));
            HIP_TRY(hipMemcpyAsync(job->h_sel_failed + 2, job->d_short, sizeof(uint32_t),
                                   hipMemcpyDeviceToHost, st));
            return FPM_OK;
        };
        if (tight)
            if (int rc = list_short(false)) return rc;
        HIP_TRY(hipStreamSynchronize(st));
        if (*job->h_sel_failed) {
            if (int rc = fallback()) return rc;
            if (tight) {
                if (int rc = list_short(false)) return rc;
                HIP_TRY(hipStreamSynchronize(st));
            }
        }
        if (tight) {
            // their tiles and selections run again
            const uint32_t n_short = job->h_sel_failed[2];
            job->last_short = (int32_t)n_short;
            if (n_short) {
                if (int rc = list_short(true)) return rc;   // the same list, raised
                HIP_TRY(hipMemsetAsync(fail_main, 0, sizeof(uint32_t), st));
                if (int rc = redo_short(job, n_short, st, tiles_pass)) return rc;
                HIP_TRY(hipMemcpyAsync(job->h_sel_failed, fail_main, sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                if (*job->h_sel_failed)
                    if (int rc = fallback()) return rc;
            }
        }
    }
    return FPM_OK;
}

int fpm_sketch_job_short_groups(fpm_sketch_job *job, int32_t *n_short)
{
    if (!job || !n_short) return fail(FPM_EINVAL, "null argument");
    *n_short = job->last_short;
    return FPM_OK;
}

int fpm_sketch_job_sample_short(fpm_sketch_job *job, int32_t *n_short)
{
    if (!job || !n_short) return fail(FPM_EINVAL, "null argument");
    *n_short = job->sbounded ? job->last_sample_short : -1;
    return FPM_OK;
}

int fpm_merge_small_spills(fpm_ctx *ctx, uint64_t *count)
{
    if (!count) return fail(FPM_EINVAL, "null argument");
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(merge_small_spills(count));
    return FPM_OK;
}

int fpm_sketch_device_output(fpm_sketch_job *job, uint64_t **d_hashes, uint32_t **d_count,
                             uint32_t *n_groups, uint32_t *row_stride)
{
    if (!job) return fail(FPM_EINVAL, "null job");
    if (d_hashes) *d_hashes = job->d_rows;
    if (d_count) *d_count = job->d_count;
    if (n_groups) *n_groups = job->n_groups;
    if (row_stride) *row_stride = job->kp.s;
    return FPM_OK;
}

int fpm_sketch_fetch(fpm_sketch_job *job, uint64_t *out_hashes, uint32_t *out_count)
{
    if (!job) return fail(FPM_EINVAL, "null job");
    fpm_ctx *ctx = job->ctx;
    if (int rc = set_device(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipDeviceSynchronize());
    if (out_hashes && job->n_groups)
        HIP_TRY(d2h_staged(ctx, out_hashes, job->d_rows,
                           (size_t)job->n_groups * job->kp.s * sizeof(uint64_t)));
    if (out_count && job->n_groups)
        HIP_TRY(copy_out(ctx, out_count, job->d_count, (size_t)job->n_groups * sizeof(uint32_t)));
    return FPM_OK;
}

int fpm_sketch_mult(fpm_sketch_job *job, void *stream, uint32_t *out_mult)
{
    if (!job) return fail(FPM_EINVAL, "null job");
    fpm_ctx *ctx = job->ctx;
    if (int rc = set_device(ctx)) return rc;
    hipStream_t st = pick_stream(ctx, stream);
    const uint64_t s = job->kp.s, ng = job->n_groups;
    if (!ng) return FPM_OK;
    if (!job->d_mult) {
        HIP_TRY(hipMalloc(&job->d_mult, ng * s * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&job->d_first, ng * s * sizeof(unsigned long long)));
        HIP_TRY(hipMalloc(&job->d_ttop, ng * sizeof(uint64_t)));
    }
    HIP_TRY(hipMemsetAsync(job->d_mult, 0, ng * s * sizeof(uint32_t), st));
    HIP_TRY(hipMemsetAsync(job->d_first, 0xff, ng * s * sizeof(unsigned long long), st));
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1)
            HIP_TRY(launch_mult_ttop(job->d_count, job->n_groups, job->kp.s, job->d_first,
                                     job->d_ttop, st));
        for (int c = 0; c < kTileClasses; c++) {
            const uint32_t b = job->class_begin[c], n = job->class_begin[c + 1] - b;
            if (!n) continue;
            TimedLaunch tl(ctx, FPM_K_SKETCH, st);
            HIP_TRY(launch_sketch_mult(c, pass, job->d_seq, job->d_tiles + b, n, job->kp,
                                       job->d_rows, job->d_count, job->d_mult, job->d_first,
                                       job->d_ttop, st));
            tl.done();
        }
    }
    if (out_mult) {
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(d2h_staged(ctx, out_mult, job->d_mult, ng * s * sizeof(uint32_t)));
    }
    return FPM_OK;
}

int fpm_sketch_job_info(fpm_sketch_job *job, uint64_t *seq_bytes, uint64_t *n_tiles,
                        uint64_t *n_kmers)
{
    if (!job) return fail(FPM_EINVAL, "null job");
    if (seq_bytes) *seq_bytes = job->seq_bytes;
    if (n_tiles) *n_tiles = job->n_tiles;
    if (n_kmers) *n_kmers = job->n_kmers;
    return FPM_OK;
}

int fpm_sketch_job_redo_tiles(fpm_sketch_job *job, int32_t *n_redo)
{
    if (!job || !n_redo) return fail(FPM_EINVAL, "null argument");
    *n_redo = -1;
    if (!job->thr4 || !job->d_redo_n) return FPM_OK;
    if (int rc = set_device(job->ctx)) return rc;
    uint32_t v = 0;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&v, job->d_redo_n, sizeof v, hipMemcpyDeviceToHost));
    *n_redo = (int32_t)v;
    return FPM_OK;
}

void fpm_sketch_job_free(fpm_sketch_job *job)
{
    if (!job) return;
    job_release(job);
    delete job;
}

int fpm_sketch_merge_dev(fpm_ctx *ctx, const uint64_t *d_lists, const uint32_t *d_counts,
                         uint32_t n_lists, uint32_t s, uint64_t *d_out, uint32_t *d_out_count,
                         void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    if ((n_lists && (!d_lists || !d_counts)) || !d_out || !d_out_count || s == 0)
        return fail(FPM_EINVAL, "sketch_merge_dev: bad argument");
    hipStream_t st = pick_stream(ctx, stream);
    if (n_lists == 0) {
        HIP_TRY(hipMemsetAsync(d_out_count, 0, 4, st));
        return FPM_OK;
    }
    if (n_lists == 1) {
        HIP_TRY(hipMemcpyAsync(d_out, d_lists, (size_t)s * 8, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipMemcpyAsync(d_out_count, d_counts, 4, hipMemcpyDeviceToDevice, st));
        return FPM_OK;
    }
    // pairwise rounds (the bottom s of a union = the bottom s of the union of the parts'
    // bottom s); intermediate lists in scratch rows, the last merge writes d_out
    void *tmp, *tcnt, *dd;
    HIP_TRY(scratch(ctx, 16, (size_t)(n_lists - 1) * s * 8, &tmp));
    HIP_TRY(scratch(ctx, 17, (size_t)(n_lists - 1) * 4, &tcnt));
    struct L { const uint64_t *p; const uint32_t *c; };
    std::vector<L> cur(n_lists);
    for (uint32_t i = 0; i < n_lists; i++) cur[i] = L{d_lists + (uint64_t)i * s, d_counts + i};
    std::vector<MergeDesc> md;
    std::vector<uint32_t> rounds{0};
    uint32_t used = 0;
    while (cur.size() > 1) {
        std::vector<L> nxt;
        for (size_t i = 0; i + 1 < cur.size(); i += 2) {
            uint64_t *c = cur.size() == 2 ? d_out : (uint64_t *)tmp + (uint64_t)used * s;
            uint32_t *cc = cur.size() == 2 ? d_out_count : (uint32_t *)tcnt + used;
            if (cur.size() != 2) used++;
            md.push_back(MergeDesc{cur[i].p, cur[i].c, cur[i + 1].p, cur[i + 1].c, c, cc});
            nxt.push_back(L{c, cc});
        }
        if (cur.size() % 2) nxt.push_back(cur.back());
        cur.swap(nxt);
        rounds.push_back((uint32_t)md.size());
    }
    HIP_TRY(scratch(ctx, 18, md.size() * sizeof(MergeDesc), &dd));
    HIP_TRY(hipStreamSynchronize(st));   // the descriptor buffer may still be read by a prior call
    HIP_TRY(copy_in(ctx, dd, md.data(), md.size() * sizeof(MergeDesc)));
    for (size_t r = 0; r + 1 < rounds.size(); r++) {
        TimedLaunch tl(ctx, FPM_K_MERGE, st);
        HIP_TRY(launch_merge((const MergeDesc *)dd + rounds[r], rounds[r + 1] - rounds[r], s, false,
                             st));
        tl.done();
    }
    return FPM_OK;
}

int fpm_sketch_batch(fpm_ctx *ctx, const fpm_sketch_params *p, const char *seq,
                     const uint64_t *rec_off, uint32_t n_rec, const uint32_t *group_of_rec,
                     uint32_t n_groups, uint64_t *out_hashes, uint32_t *out_count)
{
    fpm_sketch_job *job = nullptr;
    int rc = fpm_sketch_stage(ctx, p, seq, rec_off, n_rec, group_of_rec, n_groups, &job);
    if (rc) return rc;
    rc = fpm_sketch_run(job, nullptr);
    if (!rc) rc = fpm_sketch_fetch(job, out_hashes, out_count);
    fpm_sketch_job_free(job);
    return rc;
}

// ----------------------------------------------------------------------------
// -fp line hashing
// ----------------------------------------------------------------------------

int fpm_fp_hash_lines_dev(fpm_ctx *ctx, const uint64_t *d_vals, const uint64_t *d_line_off,
                          uint64_t n_lines, uint32_t seed, uint32_t use64, void *d_out,
                          void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    hipStream_t st = pick_stream(ctx, stream);
    TimedLaunch tl(ctx, FPM_K_FPHASH, st);
    HIP_TRY(launch_fp_hash(d_vals, d_line_off, n_lines, seed, use64, d_out, st));
    tl.done();
    return FPM_OK;
}

int fpm_fp_hash_lines(fpm_ctx *ctx, const uint64_t *vals, const uint64_t *line_off,
                      uint64_t n_lines, uint32_t seed, uint32_t use64, void *out)
{
    if (int rc = set_device(ctx)) return rc;
    if (!line_off || (n_lines && !out)) return fail(FPM_EINVAL, "null argument");
    if (n_lines == 0) return FPM_OK;
    const uint64_t nv = line_off[n_lines];
    const size_t ob = (use64 ? 8 : 4) * n_lines;
    uint64_t *dv = nullptr, *doff = nullptr;
    void *dout = nullptr;
    hipError_t e = hipMalloc((void **)&dv, (nv ? nv : 1) * 8);
    if (e == hipSuccess) e = hipMalloc((void **)&doff, (n_lines + 1) * 8);
    if (e == hipSuccess) e = hipMalloc(&dout, ob);
    if (e == hipSuccess && nv) e = copy_in(ctx, dv, vals, nv * 8);
    if (e == hipSuccess) e = copy_in(ctx, doff, line_off, (n_lines + 1) * 8);
    int rc = FPM_OK;
    if (e != hipSuccess) rc = fail(FPM_EHIP, std::string("fp staging: ") + hipGetErrorString(e));
    if (!rc) rc = fpm_fp_hash_lines_dev(ctx, dv, doff, n_lines, seed, use64, dout, nullptr);
    if (!rc) {
        e = hipStreamSynchronize(ctx->stream);
        if (e == hipSuccess) e = copy_out(ctx, out, dout, ob);
        if (e != hipSuccess) rc = fail(FPM_EHIP, std::string("fp fetch: ") + hipGetErrorString(e));
    }
    (void)hipFree(dv); (void)hipFree(doff); (void)hipFree(dout);
    return rc;
}

// ----------------------------------------------------------------------------
// -fp text
// ----------------------------------------------------------------------------

}  // extern "C"

struct fpm_fptext {
    fpm_ctx *ctx = nullptr;
    uint64_t n_lines = 0;
    uint32_t use64 = 0;
    uint8_t *d_text = nullptr;
    uint64_t *d_line_start = nullptr;
    uint32_t *d_blk = nullptr;
    uint64_t *d_id_off = nullptr;
    uint32_t *d_id_len = nullptr, *d_n_vals = nullptr;
    void *d_hash = nullptr;
    uint8_t *d_new_id = nullptr;
    // the file's References (fpm_fp_text_refs), computed on the first call
    bool refs_done = false;
    uint64_t n_refs = 0;
    uint64_t *d_first = nullptr, *d_length = nullptr, *d_ref_id_off = nullptr;
    uint32_t *d_ref_id_len = nullptr;
    std::vector<std::pair<void *, size_t>> bufs;   // every buffer above, with its size
    template <typename T> hipError_t alloc(T **p, size_t bytes)
    {
        void *q = nullptr;
        const hipError_t e = pool_alloc(ctx, &q, bytes);
        if (e == hipSuccess) { bufs.push_back({q, bytes}); *p = static_cast<T *>(q); }
        return e;
    }
};

static void fptext_release(fpm_fptext *j)
{
    if (!j) return;
    (void)hipSetDevice(j->ctx->device);
    // the job's kernels ran on the context stream: done before its buffers are handed out again
    (void)hipStreamSynchronize(j->ctx->stream);
    for (auto &b : j->bufs) pool_free(j->ctx, b.first, b.second);
}

extern "C" {

int fpm_fp_text_stage(fpm_ctx *ctx, const char *text, uint64_t text_len, uint64_t max_lines,
                      uint32_t seed, uint32_t use64, fpm_fptext **job, uint64_t *n_lines)
{
    if (!job || !n_lines) return fail(FPM_EINVAL, "fp_text_stage: null output");
    *job = nullptr;
    *n_lines = 0;
    if (int rc = set_device(ctx)) return rc;
    std::unique_ptr<fpm_fptext, void (*)(fpm_fptext *)> j(new fpm_fptext,
        [](fpm_fptext *p) { fptext_release(p); delete p; });
    j->ctx = ctx;
    j->use64 = use64;
    hipStream_t st = ctx->stream;
    const uint32_t nb = text_blocks(text_len);
    const uint64_t scan_w = scan_scratch_words(nb ? nb : 1);
    HIP_TRY(j->alloc(&j->d_text, text_len + 16));
    HIP_TRY(j->alloc(&j->d_blk, ((size_t)2 * nb + 2 + scan_w) * 4));
    if (text_len) HIP_TRY(h2d_staged(ctx, j->d_text, text, text_len));
    uint32_t *blk_cnt = j->d_blk, *blk_off = j->d_blk + nb, *scan_s = j->d_blk + 2 * nb + 2;
    // newline count first: it sizes the line index
    uint64_t n_nl = 0;
    if (nb) {
        {
            TimedLaunch tl(ctx, FPM_K_FPTEXT, st);
            HIP_TRY(launch_fp_nl_count(j->d_text, text_len, blk_cnt, blk_off, scan_s, st));
            tl.done();
        }
        // the total (blk_off[nb], 8-B aligned: blk_off starts nb words into an aligned block)
        // through the mapped counter block: no copy + stream sync round trip
        if (int rc = read_counters(ctx, (const unsigned long long *)(blk_off + nb), 1, st)) return rc;
        const uint32_t tot = (uint32_t)ctx->host_counters[0];
        n_nl = tot;
    }
    HIP_TRY(j->alloc(&j->d_line_start, (n_nl + 1) * 8));
    HIP_TRY(hipMemsetAsync(j->d_line_start, 0, 8, st));
    if (n_nl) {
        TimedLaunch tl(ctx, FPM_K_FPTEXT, st);
        HIP_TRY(launch_fp_nl_scatter(j->d_text, text_len, blk_off, j->d_line_start, st));
        tl.done();
    }
    const uint64_t total = n_nl + ((text_len && text[text_len - 1] != '\n') ? 1 : 0);
    const uint64_t nl = std::min(total, max_lines);
    j->n_lines = nl;
    if (nl) {
        HIP_TRY(j->alloc(&j->d_id_off, nl * 8));
        HIP_TRY(j->alloc(&j->d_id_len, nl * 4));
        HIP_TRY(j->alloc(&j->d_n_vals, nl * 4));
        HIP_TRY(j->alloc(&j->d_hash, nl * (use64 ? 8 : 4)));
        HIP_TRY(j->alloc(&j->d_new_id, nl));
        TimedLaunch tl(ctx, FPM_K_FPTEXT, st);
        HIP_TRY(launch_fp_lines(j->d_text, text_len, j->d_line_start, n_nl, nl, seed, use64,
                                j->d_id_off, j->d_id_len, j->d_n_vals, j->d_hash, j->d_new_id, st));
        tl.done();
    }
    *n_lines = nl;
    *job = j.release();
    return FPM_OK;
}

int fpm_fp_text_fetch(fpm_fptext *j, uint64_t *id_off, uint32_t *id_len, uint32_t *n_vals,
                      void *hash, uint8_t *new_id)
{
    if (!j) return fail(FPM_EINVAL, "fp_text_fetch: null job");
    if (int rc = set_device(j->ctx)) return rc;
    hipStream_t st = j->ctx->stream;
    const uint64_t n = j->n_lines;
    HIP_TRY(hipStreamSynchronize(st));
    if (n) {
        fpm_ctx *ctx = j->ctx;
        if (id_off) HIP_TRY(copy_out(ctx, id_off, j->d_id_off, n * 8));
        if (id_len) HIP_TRY(copy_out(ctx, id_len, j->d_id_len, n * 4));
        if (n_vals) HIP_TRY(copy_out(ctx, n_vals, j->d_n_vals, n * 4));
        if (hash) HIP_TRY(copy_out(ctx, hash, j->d_hash, n * (j->use64 ? 8 : 4)));
        if (new_id) HIP_TRY(copy_out(ctx, new_id, j->d_new_id, n));
    }
    return FPM_OK;
}

int fpm_fp_text_refs(fpm_fptext *j, uint64_t cap, uint64_t *n_refs, uint64_t *first_line,
                     uint64_t *id_off, uint32_t *id_len, uint64_t *length)
{
    if (!j || !n_refs) return fail(FPM_EINVAL, "fp_text_refs: null argument");
    if (int rc = set_device(j->ctx)) return rc;
    fpm_ctx *ctx = j->ctx;
    hipStream_t st = ctx->stream;
    const uint64_t n = j->n_lines;
    if (!j->refs_done && n) {
        const uint32_t nb = fp_head_blocks(n);
        uint32_t *blk;
        HIP_TRY(j->alloc(&blk, ((size_t)2 * nb + 2 + scan_scratch_words(nb)) * 4));
        uint32_t *blk_cnt = blk, *blk_off = blk + nb, *scan_s = blk + 2 * nb + 2;
        {
            TimedLaunch tl(ctx, FPM_K_FPTEXT, st);
            HIP_TRY(launch_fp_heads(j->d_new_id, n, blk_cnt, blk_off, scan_s, st));
            tl.done();
        }
        // the total (blk_off[nb], 8-B aligned: blk_off starts nb words into an aligned block)
        // through the mapped counter block: no copy + stream sync round trip
        if (int rc = read_counters(ctx, (const unsigned long long *)(blk_off + nb), 1, st)) return rc;
        const uint32_t tot = (uint32_t)ctx->host_counters[0];
        j->n_refs = tot;
        uint64_t *blk4;
        HIP_TRY(j->alloc(&blk4, (size_t)tot * 28 + 32));
        j->d_first = blk4;
        j->d_ref_id_off = blk4 + tot;
        j->d_length = blk4 + 2 * (size_t)tot;
        j->d_ref_id_len = reinterpret_cast<uint32_t *>(blk4 + 3 * (size_t)tot);
        TimedLaunch tl(ctx, FPM_K_FPTEXT, st);
        HIP_TRY(launch_fp_refs(j->d_new_id, n, blk_off, tot, j->d_n_vals, j->d_id_off,
                               j->d_id_len, j->d_first, j->d_length, j->d_ref_id_off,
                               j->d_ref_id_len, st));
        tl.done();
    }
    j->refs_done = true;
    *n_refs = j->n_refs;
    if (cap < j->n_refs || !j->n_refs) return FPM_OK;     // sized by this call
    const uint64_t m = j->n_refs;
    // the four arrays are one device block (first, ID offset, length: u64; ID length: u32):
    // one copy into the pinned ring and one wait, then spread into the caller's arrays
    const size_t bytes = m * 28;
    if (bytes <= fpm_ctx::kRingBytes) {
        HIP_TRY(ensure_ring(ctx));
        HIP_TRY(hipMemcpyAsync(ctx->ring[0], j->d_first, bytes, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        const char *r = static_cast<const char *>(ctx->ring[0]);
        if (first_line) memcpy(first_line, r, m * 8);
        if (id_off) memcpy(id_off, r + m * 8, m * 8);
        if (length) memcpy(length, r + m * 16, m * 8);
        if (id_len) memcpy(id_len, r + m * 24, m * 4);
        return FPM_OK;
    }
    HIP_TRY(hipStreamSynchronize(st));
    if (first_line) HIP_TRY(copy_out(ctx, first_line, j->d_first, m * 8));
    if (id_off) HIP_TRY(copy_out(ctx, id_off, j->d_ref_id_off, m * 8));
    if (id_len) HIP_TRY(copy_out(ctx, id_len, j->d_ref_id_len, m * 4));
    if (length) HIP_TRY(copy_out(ctx, length, j->d_length, m * 8));
    return FPM_OK;
}

void fpm_fp_text_free(fpm_fptext *j)
{
    fptext_release(j);
    delete j;
}

}  // extern "C"

// ----------------------------------------------------------------------------
// FASTA text -> packed records on the device (seqparse.hip)
// ----------------------------------------------------------------------------

struct fpm_seqtext {
    fpm_ctx *ctx = nullptr;
    std::vector<uint64_t> seg_off, seg_len;     // each file's offset in the device text
    uint64_t n_rec = 0, total_kept = 0;
    uint8_t *d_text = nullptr, *d_reset = nullptr, *d_out = nullptr;
    void *d_xf = nullptr, *d_cin = nullptr;
    uint64_t *d_rec = nullptr;                  // hdr_pos | hdr_end | kept_at | seq_off | seq_len
    uint64_t *d_totals = nullptr;
};

static void seqtext_release(fpm_seqtext *j)
{
    if (!j) return;
    (void)hipSetDevice(j->ctx->device);
    for (void *p : {(void *)j->d_text, (void *)j->d_reset, (void *)j->d_out, j->d_xf, j->d_cin,
                    (void *)j->d_rec, (void *)j->d_totals})
        if (p) (void)hipFree(p);
}

extern "C" {

}  // extern "C"

// The FASTQ path of fpm_seq_parse (seqparse.hip: 4-line records verified against kseq_read):
// newline index, lines per file, record table + packed bases.  *ok = false when a record does
// not read the 4-line way (nothing of the job changed then).
namespace {
// device scratch freed on every return path
struct TmpBufs {
    std::vector<void *> p;
    ~TmpBufs() { for (void *x : p) (void)hipFree(x); }
    template <typename T> hipError_t get(T **out, size_t bytes)
    {
        void *q = nullptr;
        const hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
        if (e == hipSuccess) { p.push_back(q); *out = static_cast<T *>(q); }
        return e;
    }
};
}  // namespace

static int fastq_parse(fpm_ctx *ctx, fpm_seqtext *j, uint64_t text_bytes, hipStream_t st, bool *ok)
{
    *ok = false;
    const uint32_t n_seg = (uint32_t)j->seg_off.size();
    TmpBufs tmp;
    const uint32_t nb = text_blocks(text_bytes);
    const uint64_t scan_w = scan_scratch_words(nb ? nb : 1);
    uint32_t *blk;
    HIP_TRY(tmp.get(&blk, ((size_t)2 * nb + 2 + scan_w) * 4));
    uint32_t *blk_cnt = blk, *blk_off = blk + nb, *scan_s = blk + 2 * nb + 2;
    TimedLaunch tl(ctx, FPM_K_SEQPARSE, st);
    HIP_TRY(launch_fp_nl_count(j->d_text, text_bytes, blk_cnt, blk_off, scan_s, st));
    uint32_t n_nl = 0;
    HIP_TRY(hipMemcpyAsync(&n_nl, blk_off + nb, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    uint64_t *line_start, *d_seg, *file_lines;
    HIP_TRY(tmp.get(&line_start, ((size_t)n_nl + 1) * 8));
    HIP_TRY(hipMemsetAsync(line_start, 0, 8, st));
    HIP_TRY(launch_fp_nl_scatter(j->d_text, text_bytes, blk_off, line_start, st));
    std::vector<uint64_t> seg(2 * (size_t)n_seg), fl(2 * (size_t)n_seg);
    for (uint32_t f = 0; f < n_seg; f++) {
        seg[2 * f] = j->seg_off[f];
        seg[2 * f + 1] = j->seg_len[f];
    }
    HIP_TRY(tmp.get(&d_seg, seg.size() * 8));
    HIP_TRY(tmp.get(&file_lines, seg.size() * 8));
    if (n_seg) HIP_TRY(hipMemcpyAsync(d_seg, seg.data(), seg.size() * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(launch_fq_files(line_start, (uint64_t)n_nl + 1, d_seg, n_seg, file_lines, st));
    if (n_seg) HIP_TRY(hipMemcpyAsync(fl.data(), file_lines, fl.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<uint64_t> base(n_seg ? n_seg : 1, 0);
    uint64_t n_rec = 0;
    for (uint32_t f = 0; f < n_seg; f++) {
        base[f] = n_rec;
        n_rec += fl[2 * f + 1] / 4;
    }
    uint64_t *d_base, *d_rec, *d_scan, *d_total;
    uint32_t *d_fail;
    HIP_TRY(tmp.get(&d_base, base.size() * 8));
    HIP_TRY(hipMalloc((void **)&d_rec, (size_t)(n_rec ? n_rec : 1) * 5 * 8));
    tmp.p.push_back(d_rec);
    HIP_TRY(tmp.get(&d_scan, ((n_rec + 1023) / 1024 + 1) * 8));
    HIP_TRY(tmp.get(&d_total, 16));
    HIP_TRY(tmp.get(&d_fail, 4));
    HIP_TRY(hipMemcpyAsync(d_base, base.data(), base.size() * 8, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetAsync(d_fail, 0, 4, st));
    HIP_TRY(hipMemsetAsync(d_total, 0, 16, st));
    HIP_TRY(launch_fq_records(j->d_text, line_start, d_seg, file_lines, d_base, n_seg, n_rec, d_rec,
                              d_scan, d_total, d_fail, nullptr, st));
    uint64_t total = 0;
    uint32_t failed = 0;
    HIP_TRY(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipMemcpyAsync(&failed, d_fail, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (failed) {
        tl.done();
        return FPM_OK;
    }
    uint8_t *d_out;
    HIP_TRY(hipMalloc((void **)&d_out, total + n_rec + 64));
    if (hipError_t e = launch_fq_emit(j->d_text, n_rec, d_rec, d_out, st)) {
        (void)hipFree(d_out);
        return fail(FPM_EHIP, std::string("fastq emit: ") + hipGetErrorString(e));
    }
    tl.done();
    if (hipError_t e = hipStreamSynchronize(st)) {
        (void)hipFree(d_out);
        return fail(FPM_EHIP, std::string("fastq emit: ") + hipGetErrorString(e));
    }
    tmp.p.erase(std::find(tmp.p.begin(), tmp.p.end(), (void *)d_rec));   // the job keeps it
    j->d_rec = d_rec;
    j->d_out = d_out;
    j->n_rec = n_rec;
    j->total_kept = total;
    *ok = true;
    return FPM_OK;
}

extern "C" {

int fpm_seq_parse(fpm_ctx *ctx, const char *const *seg_text, const uint64_t *seg_len,
                  uint32_t n_seg, fpm_seqtext **job, uint64_t *n_records, int *quality_lines)
{
    if (!job || !n_records || (n_seg && (!seg_text || !seg_len)))
        return fail(FPM_EINVAL, "seq_parse: null argument");
    *job = nullptr;
    *n_records = 0;
    if (quality_lines) *quality_lines = 0;
    if (int rc = set_device(ctx)) return rc;
    std::unique_ptr<fpm_seqtext, void (*)(fpm_seqtext *)> j(new fpm_seqtext,
        [](fpm_seqtext *p) { seqtext_release(p); delete p; });
    j->ctx = ctx;
    // each file from a chunk boundary, at least one '\n' after it
    uint64_t at = 0;
    for (uint32_t i = 0; i < n_seg; i++) {
        j->seg_off.push_back(at);
        j->seg_len.push_back(seg_len[i]);
        at = (at + seg_len[i] + 1 + kSpChunk - 1) / kSpChunk * kSpChunk;
    }
    const uint64_t text_bytes = at;
    const uint64_t n_chunks64 = text_bytes / kSpChunk;
    if (n_chunks64 > 0xFFFFFFFFull) return fail(FPM_EINVAL, "seq_parse: input too large");
    const uint32_t n_chunks = (uint32_t)n_chunks64;
    hipStream_t st = ctx->stream;
    // 64 bytes of slack: the FASTQ emit reads whole 64-byte windows past a sequence line
    HIP_TRY(hipMalloc(&j->d_text, text_bytes + 64));
    HIP_TRY(hipMalloc(&j->d_reset, n_chunks ? n_chunks : 1));
    HIP_TRY(hipMalloc(&j->d_xf, (size_t)(n_chunks ? n_chunks : 1) * seq_xf_bytes()));
    HIP_TRY(hipMalloc(&j->d_cin, (size_t)(n_chunks ? n_chunks : 1) * seq_cin_bytes()));
    HIP_TRY(hipMalloc(&j->d_totals, 3 * sizeof(uint64_t)));
    std::vector<uint8_t> reset(n_chunks ? n_chunks : 1, 0);
    for (uint32_t i = 0; i < n_seg; i++)
        if (j->seg_off[i] / kSpChunk < n_chunks) reset[j->seg_off[i] / kSpChunk] = 1;
    HIP_TRY(hipMemsetAsync(j->d_text, '\n', text_bytes, st));
    HIP_TRY(hipMemcpyAsync(j->d_reset, reset.data(), n_chunks, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < n_seg; i++)
        HIP_TRY(h2d_staged(ctx, j->d_text + j->seg_off[i], seg_text[i], seg_len[i]));
    uint64_t tot[3] = {0, 0, 0};
    if (n_chunks) {
        TimedLaunch tl(ctx, FPM_K_SEQPARSE, st);
        HIP_TRY(launch_seq_scan(j->d_text, j->d_reset, n_chunks, j->d_xf, j->d_cin, j->d_totals, st));
        tl.done();
        HIP_TRY(hipMemcpyAsync(tot, j->d_totals, sizeof(tot), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (tot[2]) {
        // a '+' in sequence text: FASTQ.  The 4-line layout is parsed on the device and every
        // record verified against kseq_read's quality rules; a file that does not read that way
        // leaves *quality_lines set and the caller walks the files on the host
        bool parsed = false;
        if (int rc = fastq_parse(ctx, j.get(), text_bytes, st, &parsed)) return rc;
        if (parsed) {
            for (void **p : {(void **)&j->d_text, (void **)&j->d_xf, (void **)&j->d_cin})
                if (*p) { (void)hipFree(*p); *p = nullptr; }
            *n_records = j->n_rec;
            *job = j.release();
            return FPM_OK;
        }
    }
    j->n_rec = tot[0];
    j->total_kept = tot[1];
    if (quality_lines) *quality_lines = tot[2] ? 1 : 0;
    HIP_TRY(hipMalloc(&j->d_out, j->total_kept + j->n_rec + 64));
    HIP_TRY(hipMalloc(&j->d_rec, (size_t)(j->n_rec ? j->n_rec : 1) * 5 * sizeof(uint64_t)));
    if (n_chunks) {
        const uint64_t n = j->n_rec ? j->n_rec : 1;
        TimedLaunch tl(ctx, FPM_K_SEQPARSE, st);
        HIP_TRY(launch_seq_emit(j->d_text, n_chunks, j->d_cin, j->n_rec, j->total_kept, j->d_rec,
                                j->d_rec + n, j->d_rec + 2 * n, j->d_rec + 3 * n, j->d_rec + 4 * n,
                                j->d_out, st));
        tl.done();
    }
    // the text image and scan scratch are not needed past this point
    HIP_TRY(hipStreamSynchronize(st));
    for (void **p : {(void **)&j->d_text, (void **)&j->d_xf, (void **)&j->d_cin})
        if (*p) { (void)hipFree(*p); *p = nullptr; }
    *n_records = j->n_rec;
    *job = j.release();
    return FPM_OK;
}

int fpm_seq_records(fpm_seqtext *j, uint32_t *seg_of_rec, uint64_t *hdr_off, uint64_t *hdr_len,
                    uint64_t *seq_len)
{
    if (!j) return fail(FPM_EINVAL, "seq_records: null job");
    if (int rc = set_device(j->ctx)) return rc;
    const uint64_t n = j->n_rec;
    if (!n) return FPM_OK;
    std::vector<uint64_t> rec((size_t)n * 5);
    HIP_TRY(d2h_staged(j->ctx, rec.data(), j->d_rec, rec.size() * 8));
    const uint64_t *pos = rec.data(), *end = pos + n, *len = pos + 4 * n;
    for (uint64_t r = 0; r < n; r++) {
        // the file holding the header: the last segment starting at or before it
        const uint32_t sg = (uint32_t)(std::upper_bound(j->seg_off.begin(), j->seg_off.end(), pos[r]) -
                                       j->seg_off.begin()) - 1;
        const uint64_t o = pos[r] - j->seg_off[sg];
        // the header's '\n', or the end of its file (the '\n' bytes after a file are padding)
        const uint64_t e = std::min(end[r] - j->seg_off[sg], j->seg_len[sg]);
        if (seg_of_rec) seg_of_rec[r] = sg;
        if (hdr_off) hdr_off[r] = o;
        if (hdr_len) hdr_len[r] = e - o;
        if (seq_len) seq_len[r] = len[r];
    }
    return FPM_OK;
}

void fpm_seq_free(fpm_seqtext *j)
{
    seqtext_release(j);
    delete j;
}

int fpm_sketch_stage_seq(fpm_ctx *ctx, const fpm_sketch_params *p, fpm_seqtext *seq,
                         const uint32_t *group_of_rec, uint32_t n_groups, fpm_sketch_job **job_out)
{
    if (int rc = set_device(ctx)) return rc;
    if (!p || !seq || !job_out || (seq->n_rec && !group_of_rec))
        return fail(FPM_EINVAL, "sketch_stage_seq: null argument");
    if (seq->ctx != ctx) return fail(FPM_EINVAL, "sketch_stage_seq: records parsed on another context");
    if (!seq->d_out) return fail(FPM_EINVAL, "sketch_stage_seq: records already staged");
    *job_out = nullptr;
    const uint64_t n = seq->n_rec;
    if (n > 0xFFFFFFFFull) return fail(FPM_EINVAL, "sketch_stage_seq: too many records");
    StageRecords R;
    R.n_groups = n_groups;
    R.pos.resize(n);
    R.len.resize(n);
    R.group.assign(group_of_rec, group_of_rec + n);
    const uint64_t nn = n ? n : 1;
    HIP_TRY(d2h_staged(ctx, R.pos.data(), seq->d_rec + 3 * nn, n * 8));
    HIP_TRY(d2h_staged(ctx, R.len.data(), seq->d_rec + 4 * nn, n * 8));
    for (uint64_t r = 0; r < n; r++) {
        if (group_of_rec[r] == FPM_NO_GROUP) continue;
        if (group_of_rec[r] >= n_groups) return fail(FPM_EINVAL, "group id out of range");
        R.order.push_back((uint32_t)r);
    }
    std::stable_sort(R.order.begin(), R.order.end(),
                     [&](uint32_t a, uint32_t b) { return R.group[a] < R.group[b]; });
    R.d_seq = seq->d_out;
    R.d_seq_bytes = seq->total_kept + seq->n_rec;
    const int rc = stage_core(ctx, p, R, job_out);
    if (!R.d_seq) seq->d_out = nullptr;   // the job owns the packed records now
    return rc;
}

}  // extern "C"

extern "C" {

// ----------------------------------------------------------------------------
// dist
// ----------------------------------------------------------------------------

}  // extern "C"

// One grid's outputs: the counts, and either the full per-cell distance / p-value / pass
// (fpm_dist_dev*) or the compact list of the cells with numer > 0 (fpm_dist_list_dev*).
struct DistOut {
    Counts cnt;
    double *dist = nullptr, *pval = nullptr;
    uint8_t *pass = nullptr;
    CellList list{};
};

// The outputs handed to compare_impl, so the sparse path can finalize in place: the probe (or
// the side fill) writes every cell's no-shared-hash values and a candidate kernel rewrites
// (or lists) the candidates, with no dense pass re-reading the grid.
struct DistFinal {
    const uint64_t *ref_length, *qry_length;
    uint32_t kmer_size;
    double kmer_space, max_dist, max_pvalue;
    DistOut prim;
    // the transposed grid too (fpm_refset_dist_mirror_dev*): filled beside the primary grid and
    // its candidate cells scattered by the candidate finalize; compare_impl sets *mirrored
    // when it wrote it (the sorted sparse path), else dist_dev_impl computes it by a second,
    // swapped call
    DistOut mir;
    bool *mirrored = nullptr;
    // the grid's counts were prefilled (fpm_dist_list_prefill): no defaults of its own, the
    // short pairs corrected after ev_prefill, before the first cell write
    bool prefilled = false;
    bool compact() const { return prim.list.count != nullptr; }
    bool has_mirror() const { return mir.cnt.numer != nullptr; }
};

// bucket index geometry for E entries over n_ref rows: ~2.4 entries per bucket (2^nbits >=
// E/4, at most 2^24 buckets); entries are u32 (ref id in rbits, key fingerprint in the other
// >= 8 bits).  4K level-2 counters (16 KiB of LDS) and a 16 MB directory at the bench's
// E = 1e7.  Same-box A/B: E/2 buckets cost 0.04 ms more in the bucket pass than the extra
// probe events saved; E/8 a wash.
// FPM_IDX_ONEPASS=0: always the exact two-pass index build (A/B)
static const bool g_idx_one_pass = [] {
    const char *v = getenv("FPM_IDX_ONEPASS");
    return !(v && v[0] == '0');
}();

static IdxGeom make_geom(uint32_t n_ref, uint64_t E)
{
    IdxGeom geom{};
    uint32_t rbits = 1, lg = 1;
    while (rbits < 32 && (1ULL << rbits) < n_ref) rbits++;
    while (lg < 40 && (1ULL << lg) < E) lg++;
    geom.l2 = lg > kIdxL1 + 2 ? std::min<uint32_t>(lg - 2 - kIdxL1, 14) : 1;
    geom.nbits = kIdxL1 + geom.l2;
    geom.rbits = rbits;
    geom.fbits = 32 - rbits;
    // level-1 tiles (one 1024-thread workgroup per CU: their LDS staging holds 8 B per cell)
    // in whole rounds of 256: the cells per tile trimmed so that the last round is not a
    // fraction of the chip (C2's 1e7 cells: 752 tiles of 13,312 instead of 611 of 16,384)
    {
        const uint64_t rounds = std::max<uint64_t>(1, (E + 256ULL * kIdxTile - 1) / (256ULL * kIdxTile));
        uint64_t tile = (E + 256 * rounds - 1) / (256 * rounds);
        tile = std::min<uint64_t>(kIdxTile, std::max<uint64_t>(1024, (tile + 1023) / 1024 * 1024));
        geom.tile = (uint32_t)tile;
        geom.ntiles = (uint32_t)((E + tile - 1) / tile);
    }
    // one-pass level 1: each partition's slot holds 1.5 x the mean + 6 sigma + 64 entries.
    // Bottom-s sketch values are uniform below each row's own maximum, and the rows' maxima
    // differ, so the density over the indexed range [0, kmax] tapers towards kmax and the low
    // partitions run ~10 % above the mean (C2: a 6-sigma slot overflowed on every build);
    // skewed keys (repeated -fp values) overflow and take the exact build
    const double mean = (double)E / (double)(1u << kIdxL1);
    geom.cap = g_idx_one_pass
                   ? (uint32_t)(((uint64_t)(1.5 * mean + 6.0 * std::sqrt(mean)) + 64 + 63) & ~63ull)
                   : 0u;
    return geom;
}

// One index build (launch_idx_build) and the read-back of its counters (events, sortedness,
// the one-pass overflow flag at word 67), after `then` (work queued behind the build, e.g.
// the query side's probe count).  The one-pass build first; if a level-1 partition overflowed
// its slot, the exact two-pass build (g.cap = 0) replaces it.
template <typename Then>
// raw_of_unsorted: the caller re-indexes unsorted rows over their records, so when the rows
// turn out unsorted an overflowed one-pass build is left as it is (its flags and counters
// are all the caller reads) instead of being rebuilt exactly.
static int build_index(fpm_ctx *ctx, const void *rows, const uint32_t *len, uint64_t stride,
                       uint32_t n_ref, uint32_t hash_bytes, IdxGeom &g, uint32_t *dir,
                       uint32_t *entries, unsigned long long *ctr, bool self_events,
                       hipStream_t st, Then then, bool raw_of_unsorted = false,
                       const std::function<int()> &before_read = nullptr,
                       unsigned long long *zero_x = nullptr)
{
    for (;;) {
        const uint64_t E = (uint64_t)n_ref * stride;
        const uint64_t nh = (uint64_t)(1u << kIdxL1) * g.ntiles;
        void *tile_hist, *tile_off, *tent, *scan_s, *part_fill;
        HIP_TRY(scratch(ctx, 0, nh * 4, &tile_hist));
        HIP_TRY(scratch(ctx, 1, (nh + 1) * 4, &tile_off));
        HIP_TRY(scratch(ctx, 2, idx_tent_words(g, E) * 8, &tent));
        HIP_TRY(scratch(ctx, 6, scan_scratch_words(nh) * 4, &scan_s));
        HIP_TRY(scratch(ctx, 16, (size_t)(1u << kIdxL1) * 4, &part_fill));
        uint32_t *unsorted = (uint32_t *)(ctr + 66), *overflow = (uint32_t *)(ctr + 67);
        {
            TimedLaunch tl(ctx, FPM_K_INDEX, st);
            HIP_TRY(launch_idx_build(rows, len, stride, n_ref, hash_bytes, g,
                                     (uint32_t *)tile_hist, (uint32_t *)tile_off,
                                     (uint32_t *)scan_s, (uint64_t *)tent, dir, entries, unsorted,
                                     self_events ? ctr : nullptr, ctr, 72, ctr + 72,
                                     (uint32_t *)part_fill, overflow, st, zero_x));
            if (int rc = then()) return rc;
            tl.done();
        }
        // the counters' copy first, then the work enqueued behind it before the host waits for
        // them (the speculated probe: the GPU runs it while the host reads and enqueues the
        // rest; enqueued before the copy, it would hold the copy, and the host, until it ends)
        unsigned long long seq;
        if (int rc = publish_counters(ctx, ctr, 68, st, &seq)) return rc;
        if (before_read)
            if (int rc = before_read()) return rc;
        if (int rc = wait_counters(ctx, seq, st)) return rc;
        if (g.cap && ((const uint32_t *)(ctx->host_counters + 67))[0] != 0) {
            if (raw_of_unsorted && ((const uint32_t *)(ctx->host_counters + 66))[0] != 0)
                return FPM_OK;
            g.cap = 0;
            ctx->idx_rebuilds++;
            continue;
        }
        return FPM_OK;
    }
}

// A reference set resident on the device with its bucket index built once (fpm_refset_*):
// query blocks probe it without re-uploading the references or rebuilding the index.
struct fpm_refset {
    fpm_ctx *ctx = nullptr;
    // reference rows (owned when uploaded from host buffers)
    const void *ref = nullptr;
    const uint32_t *ref_len = nullptr;
    const uint64_t *ref_length = nullptr;
    uint64_t ref_stride = 0;
    uint32_t n_ref = 0, hash_bytes = 0, sketch_size = 0;
    void *own[3] = {nullptr, nullptr, nullptr};
    // index buffers (slot ids as in compare_impl), the largest indexed key, host state
    fpm_ctx::Slot slot[16];
    unsigned long long *kmax = nullptr;
    IdxGeom geom{};
    bool sparse_ok = false;       // the index exists (the sparse path is possible)
    bool ref_unsorted = false;    // some reference row is unsorted / carries duplicates
    bool recorded = false;        // the index holds launch_record_rows copies (slots 10, 11)
    uint64_t mr = 0;              // their row stride
    uint64_t self_events = 0;     // sum_b |b|^2: the posting events of the set against itself
    // per-query-block host buffers (fpm_refset_dist): pinned staging + device copies
    void *h_stage = nullptr;
    size_t h_stage_bytes = 0;
    fpm_ctx::Slot qslot[16];
    uint64_t list_cap = 0;        // entries the device list slots (qslot 10-15) hold
};

static hipError_t slot_buf(fpm_ctx::Slot &s, size_t bytes, void **out)
{
    if (s.bytes < bytes) {
        if (s.p) { hipError_t e = hipFree(s.p); if (e != hipSuccess) return e; }
        s.p = nullptr;
        s.bytes = 0;
        size_t b = bytes + bytes / 8 + 256;
        hipError_t e = hipMalloc(&s.p, b);
        if (e != hipSuccess) return e;
        s.bytes = b;
    }
    *out = s.p;
    return hipSuccess;
}

// Build the reference index of a resident set (once): over the raw rows, or, when a row is
// unsorted / carries duplicates (-fp lists), over their records (launch_record_rows: only
// pairs sharing a record value can count anything in the literal walk).
static int refset_build_index(fpm_refset *rs, hipStream_t st)
{
    fpm_ctx *ctx = rs->ctx;
    const uint64_t E = (uint64_t)rs->n_ref * rs->ref_stride;
    IdxGeom geom = make_geom(rs->n_ref, E);
    rs->sparse_ok = E > 0 && geom.rbits <= 24 && E < (1ULL << 31);
    if (!rs->sparse_ok) return FPM_OK;
    void *ctr;
    HIP_TRY(scratch(ctx, 7, kCtrWords * 8, &ctr));
    if (!rs->kmax) HIP_TRY(hipMalloc((void **)&rs->kmax, 8));
    auto build = [&](const void *rows, const uint32_t *len, uint64_t stride, IdxGeom &g,
                     bool raw) -> int {
        const uint64_t En = (uint64_t)rs->n_ref * stride;
        void *dir, *entries;
        HIP_TRY(slot_buf(rs->slot[4], ((1ULL << g.nbits) + 1) * 4, &dir));
        HIP_TRY(slot_buf(rs->slot[5], En * 4, &entries));
        // the bucket pass also sums the self events (a query block that is the set itself
        // then needs no probe count)
        return build_index(ctx, rows, len, stride, rs->n_ref, rs->hash_bytes, g, (uint32_t *)dir,
                           (uint32_t *)entries, (unsigned long long *)ctr, true, st,
                           [] { return FPM_OK; }, raw);
    };
    geom.kmax = rs->kmax;
    if (int rc = build(rs->ref, rs->ref_len, rs->ref_stride, geom, true)) return rc;
    rs->ref_unsorted = ((const uint32_t *)(ctx->host_counters + 66))[0] != 0;
    rs->self_events = ctx->host_counters[0];
    rs->mr = std::min<uint64_t>(rs->ref_stride, rs->sketch_size);
    rs->recorded = rs->ref_unsorted;
    if (rs->recorded) {
        void *dref, *dref_len, *dref_pos;
        HIP_TRY(slot_buf(rs->slot[10], (size_t)rs->n_ref * rs->mr * rs->hash_bytes, &dref));
        HIP_TRY(slot_buf(rs->slot[11], (size_t)rs->n_ref * 4, &dref_len));
        HIP_TRY(slot_buf(rs->slot[12], (size_t)rs->n_ref * rs->mr * 4, &dref_pos));
        {
            TimedLaunch tl(ctx, FPM_K_INDEX, st);
            HIP_TRY(launch_record_rows(rs->ref, rs->ref_len, rs->ref_stride, rs->n_ref,
                                       rs->hash_bytes, rs->sketch_size, dref, (uint32_t *)dref_pos,
                                       (uint32_t *)dref_len, rs->mr, st));
            tl.done();
        }
        geom = make_geom(rs->n_ref, (uint64_t)rs->n_ref * rs->mr);
        geom.kmax = rs->kmax;
        if (int rc = build(dref, (const uint32_t *)dref_len, rs->mr, geom, false)) return rc;
    }
    rs->geom = geom;
    return FPM_OK;
}

// The grid compare: dense walk, or bucket index + probe + candidate kernel (sparse).
// With `fin`, a sparse run also finalizes (full outputs, or the compact list) and sets
// *finalized.  With `rs`, the references are that resident set and its index is reused.
static int compare_impl(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                        uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                        const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                        uint32_t hash_bytes, uint32_t sketch_size, Counts cnt,
                        void *stream, const DistFinal *fin = nullptr,
                        bool *finalized = nullptr, fpm_refset *rs = nullptr)
{
    if (finalized) *finalized = false;
    if (int rc = set_device(ctx)) return rc;
    if (hash_bytes != 4 && hash_bytes != 8) return fail(FPM_EINVAL, "hash_bytes must be 4 or 8");
    hipStream_t st = pick_stream(ctx, stream);
    if (ctx->prefill.pending) {
        // a prefill this call does not take over: nothing here may run beside it
        HIP_TRY(hipStreamWaitEvent(st, ctx->ev_prefill, 0));
        ctx->prefill.pending = false;
    }
    const uint64_t n_pairs = (uint64_t)n_ref * n_qry;
    ctx->last_sparse = 0;
    ctx->last_events = 0;
    ctx->last_cand = 0;
    if (n_pairs == 0) {
        if (fin && fin->compact()) HIP_TRY(hipMemsetAsync(fin->prim.list.count, 0, 8, st));
        return FPM_OK;
    }
    const uint64_t E = (uint64_t)n_ref * ref_stride;   // index entries (upper bound)
    bool try_sparse = ctx->dist_mode == FPM_DIST_SPARSE ||
                      (ctx->dist_mode == FPM_DIST_AUTO && n_pairs >= 4096 && E > 0);
    if (E == 0) try_sparse = false;
    IdxGeom geom = make_geom(n_ref, E);
    if (geom.rbits > 24 || E >= (1ULL << 31)) try_sparse = false;
    if (rs && !rs->sparse_ok) try_sparse = false;
    const bool self_set = d_ref == d_qry && d_ref_len == d_qry_len && ref_stride == qry_stride &&
                          n_ref == n_qry;
    const bool compact = fin && fin->compact();
    const bool want_mir = fin && fin->has_mirror() && !self_set;
    // the compact output's list count starts at zero: cleared by the index build's first
    // kernel when this call builds an index (no memset launch), else here before the first
    // kernel that appends to the list
    unsigned long long *const list_cnt =
        compact ? reinterpret_cast<unsigned long long *>(fin->prim.list.count) : nullptr;
    bool list_zeroed = !compact;
    auto zero_list = [&]() -> int {
        if (!list_zeroed) HIP_TRY(hipMemsetAsync(list_cnt, 0, 8, st));
        list_zeroed = true;
        return FPM_OK;
    };
    // The side-stream fill writes every cell's no-shared-hash values (full output: distance /
    // p-value / pass, 17 B per cell), and with fill_cnt the numer / denom defaults too, which
    // the probe then leaves out: the probe (event reads, latency-bound, slowed ~3x by any write
    // stream beside it) gets shorter and the bytes move beside the rank kernel.  Measured
    // (same box, full output): C4's 2.5e9-pair grid 16.7 -> 15.4 ms; C2's 1e8 pairs +1 %, so
    // by grid size.  A transposed grid's defaults are written by the fill only.  The compact
    // output needs a fill only for the counts.
    const bool prefilled = fin && fin->prefilled;
    const bool fill_cnt = fin && !prefilled &&
                          (want_mir || (ctx->fill_counts < 0 ? n_pairs >= (1ULL << 28)
                                                             : ctx->fill_counts != 0));
    const bool need_fill = fin && (!compact || fill_cnt);
    bool fill_pending = false;
    // a prefilled grid: wait for the prefill, then correct the pairs whose lists hold fewer
    // than S hashes together, before the first write of a cell (once)
    bool prefill_done = !prefilled;
    auto settle_prefill = [&]() -> int {
        if (prefill_done) return FPM_OK;
        prefill_done = true;
        HIP_TRY(hipStreamWaitEvent(st, ctx->ev_prefill, 0));
        HIP_TRY(launch_dist_counts_fixup(d_ref_len, n_ref, d_qry_len, n_qry, sketch_size,
                                         (uint16_t *)cnt.denom, st));
        return FPM_OK;
    };
    // record_in = false: the caller recorded ev_in on `st` already (at the point the fill may
    // start) and submits the fill after later work on `st`
    auto launch_fill = [&](bool record_in) -> int {
        PairFill fill;
        fill.dist = compact ? nullptr : fin->prim.dist;
        fill.pval = compact ? nullptr : fin->prim.pval;
        fill.pass = compact ? nullptr : fin->prim.pass;
        fill.max_dist = fin->max_dist;
        fill.max_pvalue = fin->max_pvalue;
        HIP_TRY(ensure_aux(ctx));
        if (record_in) HIP_TRY(hipEventRecord(ctx->ev_in, st));
        HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_in, 0));
        TimedLaunch tl(ctx, FPM_K_FILL, ctx->aux);
        // the flattened fill runs ~35 % faster alone but slows a rank kernel beside it more
        // (C2, 1e8 cells / 2.3e8 events: rank 0.66 -> 0.70 ms while the fill shrank 0.63 ->
        // 0.57; C4, 2.5e9 cells: 14.1 -> 12.8-13.3 ms).  The fill is the long pole when its
        // cells outweigh the posting events (the rank kernel's work): flattened when the cells
        // written (both grids with a transpose) times 1.6 exceed the events
        const long double cells_w = (long double)n_pairs * (want_mir ? 2 : 1);
        const bool flat = cells_w * 1.6L > (long double)ctx->last_events;
        HIP_TRY(launch_dist_fill(d_ref_len, n_ref, d_qry_len, n_qry, sketch_size,
                                 fill_cnt ? cnt : Counts{}, fill, ctx->aux, flat));
        if (want_mir) {
            // the transposed grid: the ref rows as queries against the query rows
            PairFill mf = fill;
            mf.dist = compact ? nullptr : fin->mir.dist;
            mf.pval = compact ? nullptr : fin->mir.pval;
            mf.pass = compact ? nullptr : fin->mir.pass;
            HIP_TRY(launch_dist_fill(d_qry_len, n_qry, d_ref_len, n_ref, sketch_size,
                                     fin->mir.cnt, mf, ctx->aux, flat));
        }
        tl.done();
        HIP_TRY(hipEventRecord(ctx->ev_fill, ctx->aux));
        fill_pending = true;
        return FPM_OK;
    };
    if (try_sparse) {
        const uint64_t NB = 1ULL << geom.nbits;
        void *ctr;
        HIP_TRY(scratch(ctx, 7, kCtrWords * 8, &ctr));
        // ctr: [0] events, [1..64] per-block partial events, [65] candidates, [66] unsorted flag,
        // [67] the one-pass index build's overflow flag,
        // [68] the largest indexed key (the bucket scale)
        unsigned long long *events = (unsigned long long *)ctr, *n_cand = events + 65;
        uint32_t *unsorted = (uint32_t *)(events + 66);
        // [69]: a probe ran past its candidate buffer (only a speculated probe can)
        uint32_t *cand_over = (uint32_t *)(events + 69);
        bool spec_probe = false;            // the probe is enqueued already (speculated)
        const void *p_qry = d_qry;                  // the rows the probe reads
        const uint32_t *p_qry_it = nullptr;         // and their lengths (null: d_qry_len)
        uint64_t p_qry_stride = qry_stride;
        const uint32_t *dir = nullptr, *entries = nullptr;
        uint64_t ev = 0;
        bool all_sorted = true;
        RecRows rec_r{}, rec_q{};                   // record rows (unsorted lists) for the walk
        // A resident sorted set against another block of sorted rows (the C4 block pairs, the
        // CLI's query blocks): no probe count.  The count pass reads every query hash's
        // bucket bounds at random (~0.27 ms for 2.2e7 hashes at N = 8, as long as the index
        // rebuild), and the probe reads them again; instead the probe reports the row's
        // posting events and whether the query rows are sorted, and the candidate compare is
        // chosen after it (rank kernel, or the literal walk for unsorted rows: the candidates
        // are the same).  Taken in the forced sparse mode, and in AUTO when the set's own
        // density (its self events per row) says the block is far from the dense regime.
        const long double ev_est =
            rs ? (long double)rs->self_events * n_qry / std::max<uint32_t>(1, rs->n_ref) : 0.0L;
        const bool skip_count = rs && !self_set && !rs->recorded && !rs->ref_unsorted &&
                                hash_bytes == 8 &&
                                (ctx->dist_mode == FPM_DIST_SPARSE ||
                                 (ctx->dist_mode == FPM_DIST_AUTO &&
                                  ev_est * 16.0L <= (long double)n_pairs * sketch_size));
        if (rs && self_set && !rs->recorded) {
            // the resident set against itself: its posting events and sortedness are the
            // index build's (sum_b |b|^2, the reference flag), no probe count
            geom = rs->geom;
            dir = (const uint32_t *)rs->slot[4].p;
            entries = (const uint32_t *)rs->slot[5].p;
            ev = rs->self_events;
            all_sorted = !rs->ref_unsorted;
            HIP_TRY(hipMemsetAsync(ctr, 0, 67 * 8, st));   // the candidate counter among them
        } else if (skip_count) {
            geom = rs->geom;
            dir = (const uint32_t *)rs->slot[4].p;
            entries = (const uint32_t *)rs->slot[5].p;
            ev = (uint64_t)ev_est;          // replaced by the probe's own count
            all_sorted = true;              // verified by the probe
            HIP_TRY(hipMemsetAsync(ctr, 0, 67 * 8, st));
        } else if (rs) {
            // resident index: count this block's posting events (and its sortedness)
            geom = rs->geom;
            dir = (const uint32_t *)rs->slot[4].p;
            entries = (const uint32_t *)rs->slot[5].p;
            TimedLaunch tl(ctx, FPM_K_INDEX, st);
            HIP_TRY(hipMemsetAsync(ctr, 0, 67 * 8, st));
            if (rs->recorded) {
                const uint64_t mq = std::min<uint64_t>(qry_stride, sketch_size);
                void *dqry, *dqry_len, *dqry_pos;
                HIP_TRY(scratch(ctx, 12, (size_t)n_qry * mq * hash_bytes, &dqry));
                HIP_TRY(scratch(ctx, 13, (size_t)n_qry * 4, &dqry_len));
                HIP_TRY(scratch(ctx, 20, (size_t)n_qry * mq * 4, &dqry_pos));
                HIP_TRY(launch_record_rows(d_qry, d_qry_len, qry_stride, n_qry, hash_bytes,
                                           sketch_size, dqry, (uint32_t *)dqry_pos,
                                           (uint32_t *)dqry_len, mq, st));
                rec_r = RecRows{rs->slot[10].p, (const uint32_t *)rs->slot[12].p,
                                (const uint32_t *)rs->slot[11].p, rs->mr};
                rec_q = RecRows{dqry, (const uint32_t *)dqry_pos, (const uint32_t *)dqry_len, mq};
                p_qry = dqry;
                p_qry_it = (const uint32_t *)dqry_len;
                p_qry_stride = mq;
            }
            HIP_TRY(launch_probe_count(p_qry, p_qry_it ? p_qry_it : d_qry_len, p_qry_stride, n_qry,
                                       hash_bytes, geom, dir, events, unsorted, st));
            tl.done();
            if (int rc = read_counters(ctx, (const unsigned long long *)events, 67, st)) return rc;
            ev = ctx->host_counters[0];
            const bool q_unsorted = ((const uint32_t *)(ctx->host_counters + 66))[0] != 0;
            // record rows are sorted by construction: the query's own order is what the walk
            // needs, so the walk is literal whenever the index holds records
            all_sorted = !rs->ref_unsorted && (rs->recorded ? false : !q_unsorted);
        } else {
            void *dir_, *entries_;
            HIP_TRY(scratch(ctx, 4, (NB + 1) * 4, &dir_));
            HIP_TRY(scratch(ctx, 5, E * 4, &entries_));
            dir = (const uint32_t *)dir_;
            entries = (const uint32_t *)entries_;
            // Unsorted lists (-fp): the index runs over each row's records among its first
            // min(len, S) entries (launch_record_rows): ~ln(S) values per row instead of every
            // distinct one, and only pairs sharing a record can count anything.  The
            // candidates are walked on the original lists.
            const uint64_t mr = std::min<uint64_t>(ref_stride, sketch_size);
            const uint64_t mq = std::min<uint64_t>(qry_stride, sketch_size);
            void *dref = nullptr, *dref_len = nullptr, *dref_pos = nullptr, *dqry = nullptr,
                 *dqry_len = nullptr, *dqry_pos = nullptr;
            // the record rows of both sides; flag: also test every row's order into `unsorted`
            auto records = [&](uint32_t *flag) -> int {
                HIP_TRY(scratch(ctx, 10, (size_t)n_ref * mr * hash_bytes, &dref));
                HIP_TRY(scratch(ctx, 11, (size_t)n_ref * 4, &dref_len));
                HIP_TRY(scratch(ctx, 19, (size_t)n_ref * mr * 4, &dref_pos));
                if (!self_set) {
                    HIP_TRY(scratch(ctx, 12, (size_t)n_qry * mq * hash_bytes, &dqry));
                    HIP_TRY(scratch(ctx, 13, (size_t)n_qry * 4, &dqry_len));
                    HIP_TRY(scratch(ctx, 20, (size_t)n_qry * mq * 4, &dqry_pos));
                }
                TimedLaunch tl(ctx, FPM_K_INDEX, st);
                HIP_TRY(launch_record_rows(d_ref, d_ref_len, ref_stride, n_ref, hash_bytes,
                                           sketch_size, dref, (uint32_t *)dref_pos,
                                           (uint32_t *)dref_len, mr, st, flag));
                if (!self_set)
                    HIP_TRY(launch_record_rows(d_qry, d_qry_len, qry_stride, n_qry, hash_bytes,
                                               sketch_size, dqry, (uint32_t *)dqry_pos,
                                               (uint32_t *)dqry_len, mq, st, flag));
                tl.done();
                return FPM_OK;
            };
            // the index over the record rows (after records())
            auto record_index = [&]() -> int {
                rec_r = RecRows{dref, (const uint32_t *)dref_pos, (const uint32_t *)dref_len, mr};
                rec_q = self_set ? rec_r
                                 : RecRows{dqry, (const uint32_t *)dqry_pos,
                                           (const uint32_t *)dqry_len, mq};
                p_qry = self_set ? dref : dqry;
                p_qry_it = (const uint32_t *)(self_set ? dref_len : dqry_len);
                p_qry_stride = self_set ? mr : mq;
                geom = make_geom(n_ref, (uint64_t)n_ref * mr);
                geom.kmax = events + 68;
                if (int rc = build_index(ctx, dref, (const uint32_t *)dref_len, mr, n_ref, hash_bytes,
                                         geom, (uint32_t *)dir_, (uint32_t *)entries_, events,
                                         self_set, st, [&]() -> int {
                                             if (!self_set)
                                                 HIP_TRY(launch_probe_count(
                                                     p_qry, p_qry_it, p_qry_stride, n_qry,
                                                     hash_bytes, geom, (const uint32_t *)dir_,
                                                     events, unsorted, st));
                                             return FPM_OK;
                                         }, false, nullptr, list_zeroed ? nullptr : list_cnt))
                    return rc;
                list_zeroed = true;
                all_sorted = false;
                ev = ctx->host_counters[0];
                return FPM_OK;
            };
            bool indexed = false;
            if (hash_bytes == 4) {
                // u32 rows (the -fp lists; k <= 16 sketches): their order is tested with the
                // records, and unsorted rows go straight to the record index (C3: the raw
                // index built only to learn the order cost ~0.2 ms of 1.45)
                HIP_TRY(hipMemsetAsync(unsorted, 0, sizeof(uint32_t), st));
                if (int rc = records(unsorted)) return rc;
                if (int rc = read_counters(ctx, (const unsigned long long *)events, 67, st)) return rc;
                if (((const uint32_t *)(ctx->host_counters + 66))[0] != 0) {
                    if (int rc = record_index()) return rc;
                    indexed = true;
                }
            }
            if (!indexed) {
                geom.kmax = events + 68;
                // A call of the last sparse rank-kernel call's shape (the bench's steps, a
                // pipeline's batches) enqueues its probe behind the index build before the
                // host reads the build's counters, so the GPU is not idle while the host
                // waits for them and launches (14-20 us per call); the probe's
                // candidates are kept when the counters confirm the path (sorted rows, sparse)
                // and the capacity (candidates <= min(events, pairs) <= cap).
                const fpm_ctx::SpecProfile &pf = ctx->spec;
#ifdef FPM_NO_SPEC
                const bool can_spec = false && pf.valid;   // (same-box A/B builds only)
#else
                const bool can_spec = pf.valid && hash_bytes == 8 && pf.n_ref == n_ref &&
                                      pf.n_qry == n_qry && pf.S == sketch_size &&
                                      pf.ref_stride == ref_stride && pf.qry_stride == qry_stride &&
                                      pf.self_set == self_set &&
                                      pf.defaults == (!fill_cnt && !prefilled) &&
                                      ctx->dist_mode != FPM_DIST_DENSE && n_ref <= (1u << 19) &&
                                      std::max(ref_stride, qry_stride) <= 2048;
#endif
                auto speculate = [&]() -> int {
                    spec_probe = false;
                    if (!can_spec) return FPM_OK;
                    void *cand, *row_seg;
                    HIP_TRY(scratch(ctx, 8, pf.cap * 8, &cand));
                    HIP_TRY(scratch(ctx, 9, (size_t)n_qry * 8, &row_seg));
                    TimedLaunch tl(ctx, FPM_K_PROBE, st);
                    HIP_TRY(launch_probe_rows(d_qry, d_qry_len, qry_stride, n_qry, n_ref,
                                              hash_bytes, geom, (const uint32_t *)dir_,
                                              (const uint32_t *)entries_, d_ref_len, sketch_size,
                                              self_set, pf.defaults, self_set, cnt,
                                              (uint64_t *)cand, n_cand, (uint64_t *)row_seg,
                                              nullptr, nullptr, nullptr, pf.cap, cand_over, st));
                    tl.done();
                    spec_probe = true;
                    return FPM_OK;
                };
                // one set against itself: the query side is the ref side, so its sortedness
                // is the ref flag and its posting events are sum_b |b|^2 from the bucket pass.
                // The counters are zeroed by the first index kernel.
                if (int rc = build_index(ctx, d_ref, d_ref_len, ref_stride, n_ref, hash_bytes,
                                         geom, (uint32_t *)dir_, (uint32_t *)entries_, events,
                                         self_set, st,
                                         [&]() -> int {
                                             if (!self_set)
                                                 HIP_TRY(launch_probe_count(
                                                     d_qry, d_qry_len, qry_stride, n_qry,
                                                     hash_bytes, geom, (const uint32_t *)dir_,
                                                     events, unsorted, st));
                                             return FPM_OK;
                                         }, true, speculate, list_zeroed ? nullptr : list_cnt))
                    return rc;
                list_zeroed = true;
                ev = ctx->host_counters[0];
                all_sorted = ((const uint32_t *)(ctx->host_counters + 66))[0] == 0;
                if (!all_sorted) {
                    if (hash_bytes != 4)
                        if (int rc = records(nullptr)) return rc;
                    if (int rc = record_index()) return rc;
                }
            }
        }
        ctx->last_events = ev;
        // Unsorted lists: a candidate costs a literal walk of ~S steps from global memory,
        // and whether the walk ever meets a shared value depends on the order, so a pair
        // sharing values rarely shares a counted one (C3: every pair shares the frequent
        // k-fingers, 4 % have numer > 0).  Take the index path only when the events say
        // most pairs share nothing (fewer events than half the pairs).
        const bool sparse = ctx->dist_mode == FPM_DIST_SPARSE ||
                            ((long double)ev * 4.0L <= (long double)n_pairs * sketch_size &&
                             (all_sorted || 2 * ev <= n_pairs));
        const uint64_t lcap = std::max(ref_stride, qry_stride);
        bool rows_merge = sparse && all_sorted && hash_bytes == 8 && n_ref <= (1u << 19) &&
                          lcap <= 2048;
        // without a count the candidates are bounded by the pairs only
        uint64_t cap = std::max<uint64_t>(1, skip_count ? n_pairs : std::min<uint64_t>(ev, n_pairs));
        if (spec_probe) {
            // the speculated probe stands when it took this call's path and its buffer held
            // every candidate: sparse, rank kernel (sorted rows), the symmetric choice it made
            // (self_set), candidates <= min(events, pairs) <= its capacity
            if (rows_merge && cap <= ctx->spec.cap) {
                cap = ctx->spec.cap;
                ctx->spec_hits++;
            } else {
                spec_probe = false;
                ctx->spec_misses++;
                HIP_TRY(hipMemsetAsync(n_cand, 0, 8, st));
                HIP_TRY(hipMemsetAsync(cand_over, 0, 4, st));
            }
        }
        if (rows_merge && !skip_count) {
            // the profile of this shape for the next call (capacity grow-only)
            fpm_ctx::SpecProfile &pf = ctx->spec;
            const bool same = pf.valid && pf.n_ref == n_ref && pf.n_qry == n_qry &&
                              pf.S == sketch_size && pf.ref_stride == ref_stride &&
                              pf.qry_stride == qry_stride && pf.self_set == self_set;
            const uint64_t keep = same ? std::max(pf.cap, cap) : cap;
            pf = fpm_ctx::SpecProfile{true, n_ref, n_qry, sketch_size, ref_stride, qry_stride,
                                      keep, self_set, !fill_cnt && !prefilled};
        }
        if (sparse) {
            void *cand, *row_seg;
            HIP_TRY(scratch(ctx, 8, cap * 8, &cand));
            HIP_TRY(scratch(ctx, 9, (size_t)n_qry * 8, &row_seg));
            // one sorted set against itself: (numer, denom) of sorted distinct lists is
            // symmetric in the two sets, so each unordered pair is ranked once (by the row the
            // probe gives it: pair parity) and each result is written to both cells (q, r) and
            // (r, q)
            const bool sym = rows_merge && self_set;
            if (!spec_probe) {
                TimedLaunch tl(ctx, FPM_K_PROBE, st);
                HIP_TRY(launch_probe_rows(p_qry, d_qry_len, p_qry_stride, n_qry, n_ref, hash_bytes,
                                          geom, dir, entries, d_ref_len, sketch_size, sym,
                                          !fill_cnt && !prefilled, self_set, cnt,
                                          (uint64_t *)cand, n_cand,
                                          (uint64_t *)row_seg, p_qry_it,
                                          skip_count ? unsorted : nullptr,
                                          skip_count ? events : nullptr, cap, cand_over, st));
                tl.done();
            }
            // A resident sorted set against a block without a count (skip_count): the rank
            // kernel is enqueued behind the probe before the host waits for the probe's
            // sortedness flag (the block's rows are sorted in every bench / CLI use; a row
            // that is not makes its rank workgroup exit, and the results are then dropped for
            // the literal walk), so the GPU does not idle while the host reads and launches.
            // The fill may start where the probe ends (ev_in) and is submitted after the read.
            bool rank_done = false;
            if (skip_count) {
                unsigned long long seq;
                if (int rc = publish_counters(ctx, (const unsigned long long *)events, 67, st, &seq))
                    return rc;
#ifdef FPM_NO_SPEC
                const bool spec_rank = false;   // (same-box A/B builds only)
#else
                const bool spec_rank = fin && rows_merge;
#endif
                if (spec_rank) {
                    void *cres;
                    HIP_TRY(scratch(ctx, 3, cap * 8, &cres));
                    if (need_fill) {
                        HIP_TRY(ensure_aux(ctx));
                        HIP_TRY(hipEventRecord(ctx->ev_in, st));
                    }
                    TimedLaunch tl(ctx, FPM_K_COMPARE, st);
                    HIP_TRY(launch_merge_rows((const uint64_t *)cand, (const uint64_t *)row_seg,
                                              n_qry, (const uint64_t *)d_ref, d_ref_len,
                                              ref_stride, n_ref, (const uint64_t *)d_qry,
                                              d_qry_len, qry_stride, sketch_size, sym, cnt,
                                              (uint32_t *)cres, (uint32_t *)cres + cap, st));
                    tl.done();
                    rank_done = true;
                }
                if (int rc = wait_counters(ctx, seq, st)) return rc;
                ctx->last_events = ctx->host_counters[0];
                if (((const uint32_t *)(ctx->host_counters + 66))[0] != 0) {
                    all_sorted = false;         // unsorted query rows: the literal walk
                    rows_merge = false;
                    rank_done = false;          // (its per-candidate slots are not read)
                }
            }
            // The rank kernel keeps its results in per-candidate slots (cnum / cden) and leaves
            // the grid alone, so the fill (needing only the list lengths) runs beside it on the
            // side stream, and the candidate finalize scatters the results after both.  The
            // literal walk writes cells in place, so it waits for the fill instead.  (Beside the
            // index build or the probe the fill slowed both: they move as many bytes as it does.)
            uint32_t *cnum = nullptr, *cden = nullptr;
            if (fin && rows_merge) {
                void *cres;
                HIP_TRY(scratch(ctx, 3, cap * 8, &cres));
                cnum = (uint32_t *)cres;
                cden = cnum + cap;
            }
            // (Submitted before the probe instead, the fill slows the probe more than it gains:
            // C4 one GPU 6.66 -> 6.80-6.86 ms, same box, r04.  Written by the rank kernel's own
            // row workgroups after their candidates instead of beside them: rank 2.7 -> 3.3 ms
            // with the fill inside, C4 6.48-6.55 -> 6.69-6.72 ms, same box, r04.)
            // After the host read of the probe's counters the GPU is idle: a fill submitted
            // first would take every CU before the rank kernel's workgroups arrive (rank +
            // fill 0.39 + 1.51 -> 0.55 + 1.67 ms at N = 8).  The fill may start where the probe
            // ends (ev_in recorded here) but is submitted after the candidate compare.
            const bool defer_fill = need_fill && skip_count && rows_merge;
            if (defer_fill) {
                HIP_TRY(ensure_aux(ctx));
                if (!rank_done) HIP_TRY(hipEventRecord(ctx->ev_in, st));
            } else if (need_fill) {
                if (int rc = launch_fill(true)) return rc;
            }
            if (fill_pending && !cnum) HIP_TRY(hipStreamWaitEvent(st, ctx->ev_fill, 0));
            if (!cnum)                              // the literal walk writes cells in place
                if (int rc = settle_prefill()) return rc;
            if (!rank_done) {
                TimedLaunch tl(ctx, FPM_K_COMPARE, st);
                if (rows_merge)
                    HIP_TRY(launch_merge_rows((const uint64_t *)cand, (const uint64_t *)row_seg, n_qry,
                                              (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                                              (const uint64_t *)d_qry, d_qry_len, qry_stride,
                                              sketch_size, sym, cnt, cnum, cden, st));
                else
                    HIP_TRY(launch_walk_candidates((const uint64_t *)cand, n_cand, cap, d_ref,
                                                   d_ref_len, ref_stride, n_ref, d_qry, d_qry_len,
                                                   qry_stride, hash_bytes, sketch_size, cnt,
                                                   rec_r, rec_q, st));
                tl.done();
            }
            if (defer_fill)
                if (int rc = launch_fill(false)) return rc;
            if (fill_pending && cnum) HIP_TRY(hipStreamWaitEvent(st, ctx->ev_fill, 0));
            if (int rc = settle_prefill()) return rc;
            if (fin) {
                if (int rc = zero_list()) return rc;
                TimedLaunch tl(ctx, FPM_K_FINALIZE, st);
                if (compact) {
                    const CellList none{};
                    HIP_TRY(launch_dist_cand_list((const uint64_t *)cand, n_cand, cap, sym, cnum,
                                                  cden, cnt, fin->ref_length, fin->qry_length,
                                                  n_ref, fin->kmer_size, fin->kmer_space,
                                                  fin->max_dist, fin->max_pvalue, fin->prim.list,
                                                  want_mir && cnum ? fin->mir.cnt : Counts{}, n_qry,
                                                  want_mir && cnum ? fin->mir.list : none, st));
                } else {
                    MirrorOut mir{};
                    if (want_mir && cnum) {
                        mir.cnt = fin->mir.cnt;
                        mir.dist = fin->mir.dist;
                        mir.pval = fin->mir.pval;
                        mir.pass = fin->mir.pass;
                        mir.n_qry = n_qry;
                    }
                    HIP_TRY(launch_dist_cand_finalize((const uint64_t *)cand, n_cand, cap, sym, cnum,
                                                      cden, cnt, fin->ref_length,
                                                      fin->qry_length, n_ref, fin->kmer_size,
                                                      fin->kmer_space, fin->max_dist,
                                                      fin->max_pvalue, fin->prim.dist,
                                                      fin->prim.pval, fin->prim.pass, mir, st));
                }
                tl.done();
                if (want_mir && cnum && fin->mirrored) *fin->mirrored = true;
                *finalized = true;
            }
            ctx->last_sparse = rows_merge ? 2 : 1;
            ctx->last_cand = (uint64_t)-1;   // read by fpm_ctx_last_dist_stats (sync + copy)
            ctx->last_cand_dev = n_cand;
            ctx->last_cand_stream = st;
            return FPM_OK;
        }
    }
    // (dist_dev_impl lists the cells of the dense grid afterwards)
    if (int rc = zero_list()) return rc;
    // the dense compare writes every cell: after a prefill, not beside it
    if (prefilled && !prefill_done) {
        HIP_TRY(hipStreamWaitEvent(st, ctx->ev_prefill, 0));
        prefill_done = true;
    }
    if (compare_grid_img_ok(hash_bytes, sketch_size, ref_stride, qry_stride)) {
        size_t ub, bb;
        compare_grid_img_scratch(n_qry, sketch_size, ref_stride, qry_stride, &ub, &bb);
        void *ublk, *bimg;
        HIP_TRY(scratch(ctx, 14, ub, &ublk));
        HIP_TRY(scratch(ctx, 15, bb, &bimg));
        TimedLaunch tl(ctx, FPM_K_COMPARE, st);
        HIP_TRY(launch_compare_grid_img(d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len,
                                        qry_stride, n_qry, sketch_size, ublk, bimg, cnt, st));
        tl.done();
        ctx->last_cand = n_pairs;
        return FPM_OK;
    }
    TimedLaunch tl(ctx, FPM_K_COMPARE, st);
    HIP_TRY(launch_compare_grid(d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len, qry_stride,
                                n_qry, hash_bytes, sketch_size, cnt, st));
    tl.done();
    ctx->last_cand = n_pairs;
    return FPM_OK;
}

extern "C" {

int fpm_compare_grid_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                         uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                         const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                         uint32_t hash_bytes, uint32_t sketch_size, uint32_t *d_numer,
                         uint32_t *d_denom, void *stream)
{
    return compare_impl(ctx, d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len, qry_stride,
                        n_qry, hash_bytes, sketch_size, Counts{d_numer, d_denom, false}, stream);
}

}  // extern "C"

// compare + finalize on device buffers (fpm_dist_dev* and fpm_dist_list_dev*)
static int dist_dev_impl(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                         const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                         const void *d_qry, const uint32_t *d_qry_len,
                         const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                         uint32_t hash_bytes, uint32_t sketch_size, uint32_t kmer_size,
                         double kmer_space, double max_dist, double max_pvalue, const DistOut &out,
                         void *stream, const char *who, fpm_refset *rs = nullptr,
                         const DistOut *mirror = nullptr)
{
    const bool compact = out.list.count != nullptr;
    if (!d_ref_length || !d_qry_length)
        return fail(FPM_EINVAL, std::string(who) + ": lengths required");
    if (!out.cnt.numer || !out.cnt.denom)
        return fail(FPM_EINVAL, std::string(who) + ": numer / denom buffers required");
    if (compact ? (!out.list.qry || !out.list.ref || !out.list.dist || !out.list.pval)
                : (!out.dist || !out.pval))
        return fail(FPM_EINVAL, std::string(who) +
                                    (compact ? ": list qry / ref / distance / p-value buffers required"
                                             : ": distance and p-value buffers required"));
    hipStream_t st = pick_stream(ctx, stream);
    // the prefill of this very grid (fpm_dist_list_prefill) is taken over; any other waits in
    // compare_impl
    bool prefilled = false;
    if (ctx->prefill.pending) {
        const fpm_ctx::Prefill &pf = ctx->prefill;
        prefilled = compact && out.cnt.c16 && !mirror && !rs && pf.numer == out.cnt.numer &&
                    pf.denom == out.cnt.denom && pf.n_ref == n_ref && pf.n_qry == n_qry &&
                    pf.S == sketch_size;
        if (prefilled) ctx->prefill.pending = false;
    }
    // (the list count is cleared inside compare_impl: by the index build, else a memset)
    DistFinal fin{d_ref_length, d_qry_length, kmer_size, kmer_space, max_dist, max_pvalue, out};
    fin.prefilled = prefilled;
    bool finalized = false, mirrored = false;
    if (mirror) {
        fin.mir = *mirror;
        fin.mirrored = &mirrored;
        if (compact) HIP_TRY(hipMemsetAsync(mirror->list.count, 0, 8, st));
    }
    if (int rc = compare_impl(ctx, d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len,
                              qry_stride, n_qry, hash_bytes, sketch_size, out.cnt, stream, &fin,
                              &finalized, rs)) {
        // an error before the compare ordered itself after a taken-over prefill: the side
        // stream may still be writing the caller's counts, so wait for it before returning
        if (prefilled) (void)hipEventSynchronize(ctx->ev_prefill);
        return rc;
    }
    // the transposed grid, when the compare could not scatter it (dense path, unsorted lists:
    // their literal walk is not symmetric): the swapped call, ref and query sets exchanged
    auto mirror_swapped = [&]() -> int {
        if (!mirror || mirrored) return FPM_OK;
        return dist_dev_impl(ctx, d_qry, d_qry_len, d_qry_length, qry_stride, n_qry, d_ref,
                             d_ref_len, d_ref_length, ref_stride, n_ref, hash_bytes, sketch_size,
                             kmer_size, kmer_space, max_dist, max_pvalue, *mirror, stream, who);
    };
    if (finalized) return mirror_swapped();
    TimedLaunch tl(ctx, FPM_K_FINALIZE, st);
    if (compact)
        HIP_TRY(launch_dist_grid_list(out.cnt, n_ref, n_qry, d_ref_length, d_qry_length, kmer_size,
                                      kmer_space, max_dist, max_pvalue, out.list, st));
    else
        HIP_TRY(launch_dist_finalize(out.cnt, d_ref_length, d_qry_length, n_ref, n_qry, kmer_size,
                                     kmer_space, max_dist, max_pvalue, out.dist, out.pval,
                                     out.pass, st));
    tl.done();
    return mirror_swapped();
}

static DistOut full_out(void *numer, void *denom, bool c16, double *dist, double *pval,
                        uint8_t *pass)
{
    DistOut o;
    o.cnt = Counts{numer, denom, c16};
    o.dist = dist;
    o.pval = pval;
    o.pass = pass;
    return o;
}

static int list_out(void *numer, void *denom, bool c16, const fpm_cell_list *l, DistOut &o,
                    const char *who)
{
    if (!l || !l->count) return fail(FPM_EINVAL, std::string(who) + ": cell list with a count required");
    o.cnt = Counts{numer, denom, c16};
    o.list.qry = l->qry;
    o.list.ref = l->ref;
    o.list.dist = l->dist;
    o.list.pval = l->pvalue;
    o.list.pass = l->pass;
    o.list.count = (unsigned long long *)l->count;
    o.list.cap = l->cap;
    return FPM_OK;
}

extern "C" {

int fpm_dist_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                 const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                 const void *d_qry, const uint32_t *d_qry_len, const uint64_t *d_qry_length,
                 uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes, uint32_t sketch_size,
                 uint32_t kmer_size, double kmer_space, double max_dist, double max_pvalue,
                 uint32_t *d_numer, uint32_t *d_denom, double *d_dist, double *d_pvalue,
                 uint8_t *d_pass, void *stream)
{
    return dist_dev_impl(ctx, d_ref, d_ref_len, d_ref_length, ref_stride, n_ref, d_qry, d_qry_len,
                         d_qry_length, qry_stride, n_qry, hash_bytes, sketch_size, kmer_size,
                         kmer_space, max_dist, max_pvalue,
                         full_out(d_numer, d_denom, false, d_dist, d_pvalue, d_pass), stream,
                         "fpm_dist_dev");
}

int fpm_dist_dev16(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                   const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                   const void *d_qry, const uint32_t *d_qry_len, const uint64_t *d_qry_length,
                   uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes, uint32_t sketch_size,
                   uint32_t kmer_size, double kmer_space, double max_dist, double max_pvalue,
                   uint16_t *d_numer, uint16_t *d_denom, double *d_dist, double *d_pvalue,
                   uint8_t *d_pass, void *stream)
{
    if (sketch_size > 65535)
        return fail(FPM_EINVAL, "fpm_dist_dev16: sketch_size must be <= 65535 (u16 counts)");
    return dist_dev_impl(ctx, d_ref, d_ref_len, d_ref_length, ref_stride, n_ref, d_qry, d_qry_len,
                         d_qry_length, qry_stride, n_qry, hash_bytes, sketch_size, kmer_size,
                         kmer_space, max_dist, max_pvalue,
                         full_out(d_numer, d_denom, true, d_dist, d_pvalue, d_pass), stream,
                         "fpm_dist_dev16");
}

int fpm_dist_list_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                      const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                      const void *d_qry, const uint32_t *d_qry_len, const uint64_t *d_qry_length,
                      uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes,
                      uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                      double max_dist, double max_pvalue, uint16_t *d_numer, uint16_t *d_denom,
                      const fpm_cell_list *list, void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    if (sketch_size > 65535)
        return fail(FPM_EINVAL, "fpm_dist_list_dev: sketch_size must be <= 65535 (u16 counts)");
    DistOut o;
    if (int rc = list_out(d_numer, d_denom, true, list, o, "fpm_dist_list_dev")) return rc;
    return dist_dev_impl(ctx, d_ref, d_ref_len, d_ref_length, ref_stride, n_ref, d_qry, d_qry_len,
                         d_qry_length, qry_stride, n_qry, hash_bytes, sketch_size, kmer_size,
                         kmer_space, max_dist, max_pvalue, o, stream, "fpm_dist_list_dev");
}

int fpm_dist_list_prefill(fpm_ctx *ctx, uint16_t *d_numer, uint16_t *d_denom, uint32_t n_ref,
                          uint32_t n_qry, uint32_t sketch_size, void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    if (!d_numer || !d_denom) return fail(FPM_EINVAL, "fpm_dist_list_prefill: numer / denom buffers required");
    if (sketch_size > 65535)
        return fail(FPM_EINVAL, "fpm_dist_list_prefill: sketch_size must be <= 65535 (u16 counts)");
    hipStream_t st = pick_stream(ctx, stream);
    HIP_TRY(ensure_aux(ctx));
    // one prefill at a time: an earlier one nobody took over is waited for by `stream` first
    if (ctx->prefill.pending) HIP_TRY(hipStreamWaitEvent(st, ctx->ev_prefill, 0));
    HIP_TRY(hipEventRecord(ctx->ev_in, st));
    HIP_TRY(hipStreamWaitEvent(ctx->aux, ctx->ev_in, 0));
    {
        TimedLaunch tl(ctx, FPM_K_FILL, ctx->aux);
        HIP_TRY(launch_dist_counts_const(d_numer, d_denom, (uint64_t)n_ref * n_qry, sketch_size,
                                         ctx->aux));
        tl.done();
    }
    HIP_TRY(hipEventRecord(ctx->ev_prefill, ctx->aux));
    ctx->prefill = fpm_ctx::Prefill{d_numer, d_denom, n_ref, n_qry, sketch_size, true};
    return FPM_OK;
}

int fpm_dist_finalize_dev(fpm_ctx *ctx, const uint32_t *d_numer, const uint32_t *d_denom,
                          const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                          uint32_t n_ref, uint32_t n_qry, uint32_t kmer_size,
                          double kmer_space, double max_dist, double max_pvalue,
                          double *d_dist, double *d_pvalue, uint8_t *d_pass, void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    hipStream_t st = pick_stream(ctx, stream);
    TimedLaunch tl(ctx, FPM_K_FINALIZE, st);
    HIP_TRY(launch_dist_finalize(Counts{(void *)d_numer, (void *)d_denom, false}, d_ref_length,
                                 d_qry_length, n_ref, n_qry, kmer_size, kmer_space, max_dist,
                                 max_pvalue, d_dist, d_pvalue, d_pass, st));
    tl.done();
    return FPM_OK;
}

int fpm_pvalue_batch_dev(fpm_ctx *ctx, const void *d_numer, const void *d_denom,
                         uint32_t count_bytes, const uint64_t *d_len_ref,
                         const uint64_t *d_len_qry, uint64_t n, uint32_t kmer_size,
                         double kmer_space, double *d_dist, double *d_pvalue, void *stream)
{
    if (int rc = set_device(ctx)) return rc;
    if (count_bytes != 2 && count_bytes != 4) return fail(FPM_EINVAL, "count_bytes must be 2 or 4");
    if (n && (!d_numer || !d_denom || !d_len_ref || !d_len_qry))
        return fail(FPM_EINVAL, "null input");
    hipStream_t st = pick_stream(ctx, stream);
    TimedLaunch tl(ctx, FPM_K_FINALIZE, st);
    HIP_TRY(launch_pvalue_batch(d_numer, d_denom, count_bytes, d_len_ref, d_len_qry, n, kmer_size,
                                kmer_space, d_dist, d_pvalue, st));
    tl.done();
    return FPM_OK;
}

namespace {
struct DevBuf {
    void *p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
};
}  // namespace

int fpm_dist(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len, const uint64_t *ref_length,
             uint64_t ref_stride, uint32_t n_ref, const void *qry, const uint32_t *qry_len,
             const uint64_t *qry_length, uint64_t qry_stride, uint32_t n_qry,
             uint32_t hash_bytes, uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
             double max_dist, double max_pvalue, uint32_t *out_numer, uint32_t *out_denom,
             double *out_dist, double *out_pvalue, uint8_t *out_pass)
{
    if (int rc = set_device(ctx)) return rc;
    if (hash_bytes != 4 && hash_bytes != 8) return fail(FPM_EINVAL, "hash_bytes must be 4 or 8");
    const uint64_t np = (uint64_t)n_ref * n_qry;
    if (np == 0) return FPM_OK;
    const bool fin = out_dist || out_pvalue || out_pass;
    if (fin && (!ref_length || !qry_length)) return fail(FPM_EINVAL, "lengths required for distance");
    DevBuf r, rl, rL, q, ql, qL, nu, de, di, pv, pa;
    hipError_t e = hipSuccess;
    auto up = [&](DevBuf &b, const void *h, size_t bytes) {
        if (e != hipSuccess) return;
        e = hipMalloc(&b.p, bytes ? bytes : 16);
        if (e == hipSuccess && h && bytes) e = copy_in(ctx, b.p, h, bytes);
    };
    // one set against itself (dist X.msh X.msh): upload once; the grid call then sees
    // identical device inputs and may use the pair symmetry
    const bool same = ref == qry && ref_len == qry_len && ref_stride == qry_stride &&
                      n_ref == n_qry;
    up(r, ref, (size_t)n_ref * ref_stride * hash_bytes);
    up(rl, ref_len, (size_t)n_ref * 4);
    if (!same) {
        up(q, qry, (size_t)n_qry * qry_stride * hash_bytes);
        up(ql, qry_len, (size_t)n_qry * 4);
    }
    up(nu, nullptr, np * 4);
    up(de, nullptr, np * 4);
    if (fin) {
        up(rL, ref_length, (size_t)n_ref * 8);
        up(qL, qry_length, (size_t)n_qry * 8);
        up(di, nullptr, np * 8);
        up(pv, nullptr, np * 8);
        up(pa, nullptr, np);
    }
    if (e != hipSuccess) return fail(FPM_ENOMEM, std::string("dist staging: ") + hipGetErrorString(e));
    const void *dq = same ? r.p : q.p;
    const uint32_t *dql = (const uint32_t *)(same ? rl.p : ql.p);
    int rc = fin ? fpm_dist_dev(ctx, r.p, (const uint32_t *)rl.p, (const uint64_t *)rL.p,
                                ref_stride, n_ref, dq, dql, (const uint64_t *)qL.p, qry_stride,
                                n_qry, hash_bytes, sketch_size, kmer_size, kmer_space, max_dist,
                                max_pvalue, (uint32_t *)nu.p, (uint32_t *)de.p, (double *)di.p,
                                (double *)pv.p, (uint8_t *)pa.p, nullptr)
                 : fpm_compare_grid_dev(ctx, r.p, (const uint32_t *)rl.p, ref_stride, n_ref, dq,
                                        dql, qry_stride, n_qry, hash_bytes, sketch_size,
                                        (uint32_t *)nu.p, (uint32_t *)de.p, nullptr);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (out_numer) HIP_TRY(copy_out(ctx, out_numer, nu.p, np * 4));
    if (out_denom) HIP_TRY(copy_out(ctx, out_denom, de.p, np * 4));
    if (out_dist) HIP_TRY(copy_out(ctx, out_dist, di.p, np * 8));
    if (out_pvalue) HIP_TRY(copy_out(ctx, out_pvalue, pv.p, np * 8));
    if (out_pass) HIP_TRY(copy_out(ctx, out_pass, pa.p, np));
    return FPM_OK;
}

// ---- resident reference set ----------------------------------------------------------

int fpm_host_alloc(fpm_ctx *ctx, void **p, size_t bytes)
{
    if (!p) return fail(FPM_EINVAL, "host_alloc: null output");
    *p = nullptr;
    if (int rc = set_device(ctx)) return rc;
    if (hipHostMalloc(p, bytes ? bytes : 16) != hipSuccess)
        return fail(FPM_ENOMEM, "host_alloc: pinned allocation failed");
    return FPM_OK;
}

int fpm_host_free(fpm_ctx *ctx, void *p)
{
    if (int rc = set_device(ctx)) return rc;
    if (p) HIP_TRY(hipHostFree(p));
    return FPM_OK;
}

static int refset_init(fpm_refset *rs)
{
    hipStream_t st = rs->ctx->stream;
    if (int rc = refset_build_index(rs, st)) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    return FPM_OK;
}

int fpm_refset_create_dev(fpm_ctx *ctx, const void *d_ref, const uint32_t *d_ref_len,
                          const uint64_t *d_ref_length, uint64_t ref_stride, uint32_t n_ref,
                          uint32_t hash_bytes, uint32_t sketch_size, fpm_refset **out)
{
    if (!out) return fail(FPM_EINVAL, "refset_create: null output");
    *out = nullptr;
    if (int rc = set_device(ctx)) return rc;
    if (hash_bytes != 4 && hash_bytes != 8) return fail(FPM_EINVAL, "hash_bytes must be 4 or 8");
    std::unique_ptr<fpm_refset, void (*)(fpm_refset *)> rs(new fpm_refset, fpm_refset_free);
    rs->ctx = ctx;
    rs->ref = d_ref;
    rs->ref_len = d_ref_len;
    rs->ref_length = d_ref_length;
    rs->ref_stride = ref_stride;
    rs->n_ref = n_ref;
    rs->hash_bytes = hash_bytes;
    rs->sketch_size = sketch_size;
    if (int rc = refset_init(rs.get())) return rc;
    *out = rs.release();
    return FPM_OK;
}

int fpm_refset_create(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len,
                      const uint64_t *ref_length, uint64_t ref_stride, uint32_t n_ref,
                      uint32_t hash_bytes, uint32_t sketch_size, fpm_refset **out)
{
    if (!out) return fail(FPM_EINVAL, "refset_create: null output");
    *out = nullptr;
    if (int rc = set_device(ctx)) return rc;
    if (hash_bytes != 4 && hash_bytes != 8) return fail(FPM_EINVAL, "hash_bytes must be 4 or 8");
    std::unique_ptr<fpm_refset, void (*)(fpm_refset *)> rs(new fpm_refset, fpm_refset_free);
    rs->ctx = ctx;
    const size_t mb = std::max<size_t>(16, (size_t)n_ref * ref_stride * hash_bytes);
    HIP_TRY(hipMalloc(&rs->own[0], mb));
    HIP_TRY(hipMalloc(&rs->own[1], std::max<size_t>(16, (size_t)n_ref * 4)));
    HIP_TRY(hipMalloc(&rs->own[2], std::max<size_t>(16, (size_t)n_ref * 8)));
    if ((size_t)n_ref * ref_stride)
        HIP_TRY(copy_in(ctx, rs->own[0], ref, (size_t)n_ref * ref_stride * hash_bytes));
    if (n_ref) {
        HIP_TRY(copy_in(ctx, rs->own[1], ref_len, (size_t)n_ref * 4));
        if (ref_length) HIP_TRY(copy_in(ctx, rs->own[2], ref_length, (size_t)n_ref * 8));
    }
    rs->ref = rs->own[0];
    rs->ref_len = (const uint32_t *)rs->own[1];
    rs->ref_length = (const uint64_t *)rs->own[2];
    rs->ref_stride = ref_stride;
    rs->n_ref = n_ref;
    rs->hash_bytes = hash_bytes;
    rs->sketch_size = sketch_size;
    if (int rc = refset_init(rs.get())) return rc;
    *out = rs.release();
    return FPM_OK;
}

static int refset_check(fpm_refset *rs, uint32_t sketch_size, uint32_t count_bytes,
                        const char *who)
{
    if (!rs) return fail(FPM_EINVAL, std::string(who) + ": null set");
    if (sketch_size != rs->sketch_size)
        return fail(FPM_EINVAL, std::string(who) + ": sketch_size differs from the set's");
    if (count_bytes != 2 && count_bytes != 4) return fail(FPM_EINVAL, "count_bytes must be 2 or 4");
    if (count_bytes == 2 && sketch_size > 65535)
        return fail(FPM_EINVAL, std::string(who) + ": u16 counts need sketch_size <= 65535");
    return set_device(rs->ctx);
}

int fpm_refset_dist_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                        const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                        uint32_t sketch_size, uint32_t count_bytes, uint32_t kmer_size,
                        double kmer_space, double max_dist, double max_pvalue, void *d_numer,
                        void *d_denom, double *d_dist, double *d_pvalue, uint8_t *d_pass,
                        void *stream)
{
    if (int rc = refset_check(rs, sketch_size, count_bytes, "fpm_refset_dist_dev")) return rc;
    return dist_dev_impl(rs->ctx, rs->ref, rs->ref_len, rs->ref_length, rs->ref_stride, rs->n_ref,
                         d_qry, d_qry_len, d_qry_length, qry_stride, n_qry, rs->hash_bytes,
                         sketch_size, kmer_size, kmer_space, max_dist, max_pvalue,
                         full_out(d_numer, d_denom, count_bytes == 2, d_dist, d_pvalue, d_pass),
                         stream, "fpm_refset_dist_dev", rs);
}

}  // extern "C"

static int refset_list_impl(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                            const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                            uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                            double max_dist, double max_pvalue, uint32_t count_bytes,
                            void *d_numer, void *d_denom, const fpm_cell_list *list, void *stream,
                            const char *who)
{
    if (int rc = refset_check(rs, sketch_size, count_bytes, who)) return rc;
    DistOut o;
    if (int rc = list_out(d_numer, d_denom, count_bytes == 2, list, o, who)) return rc;
    return dist_dev_impl(rs->ctx, rs->ref, rs->ref_len, rs->ref_length, rs->ref_stride, rs->n_ref,
                         d_qry, d_qry_len, d_qry_length, qry_stride, n_qry, rs->hash_bytes,
                         sketch_size, kmer_size, kmer_space, max_dist, max_pvalue, o, stream, who,
                         rs);
}

extern "C" {

int fpm_refset_dist_list_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                             const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                             uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                             double max_dist, double max_pvalue, uint16_t *d_numer,
                             uint16_t *d_denom, const fpm_cell_list *list, void *stream)
{
    return refset_list_impl(rs, d_qry, d_qry_len, d_qry_length, qry_stride, n_qry, sketch_size,
                            kmer_size, kmer_space, max_dist, max_pvalue, 2, d_numer, d_denom,
                            list, stream, "fpm_refset_dist_list_dev");
}

static int mirror_check(fpm_refset *rs, const void *d_qry, const char *who)
{
    if (d_qry == rs->ref)
        return fail(FPM_EINVAL, std::string(who) + ": the query rows are the reference rows "
                                                   "(use the non-mirror call: that grid is its "
                                                   "own transpose)");
    return FPM_OK;
}

int fpm_refset_dist_mirror_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                               const uint64_t *d_qry_length, uint64_t qry_stride, uint32_t n_qry,
                               uint32_t sketch_size, uint32_t count_bytes, uint32_t kmer_size,
                               double kmer_space, double max_dist, double max_pvalue,
                               void *d_numer, void *d_denom, double *d_dist, double *d_pvalue,
                               uint8_t *d_pass, void *m_numer, void *m_denom, double *m_dist,
                               double *m_pvalue, uint8_t *m_pass, void *stream)
{
    const char *who = "fpm_refset_dist_mirror_dev";
    if (int rc = refset_check(rs, sketch_size, count_bytes, who)) return rc;
    if (!m_numer || !m_denom || !m_dist || !m_pvalue)
        return fail(FPM_EINVAL, "refset_dist_mirror: mirror numer / denom / distance / p-value required");
    if (int rc = mirror_check(rs, d_qry, who)) return rc;
    const DistOut mir = full_out(m_numer, m_denom, count_bytes == 2, m_dist, m_pvalue, m_pass);
    return dist_dev_impl(rs->ctx, rs->ref, rs->ref_len, rs->ref_length, rs->ref_stride, rs->n_ref,
                         d_qry, d_qry_len, d_qry_length, qry_stride, n_qry, rs->hash_bytes,
                         sketch_size, kmer_size, kmer_space, max_dist, max_pvalue,
                         full_out(d_numer, d_denom, count_bytes == 2, d_dist, d_pvalue, d_pass),
                         stream, who, rs, &mir);
}

int fpm_refset_dist_mirror_list_dev(fpm_refset *rs, const void *d_qry, const uint32_t *d_qry_len,
                                    const uint64_t *d_qry_length, uint64_t qry_stride,
                                    uint32_t n_qry, uint32_t sketch_size, uint32_t kmer_size,
                                    double kmer_space, double max_dist, double max_pvalue,
                                    uint16_t *d_numer, uint16_t *d_denom,
                                    const fpm_cell_list *list, uint16_t *m_numer,
                                    uint16_t *m_denom, const fpm_cell_list *m_list, void *stream)
{
    const char *who = "fpm_refset_dist_mirror_list_dev";
    if (int rc = refset_check(rs, sketch_size, 2, who)) return rc;
    if (int rc = mirror_check(rs, d_qry, who)) return rc;
    DistOut o, m;
    if (int rc = list_out(d_numer, d_denom, true, list, o, who)) return rc;
    if (int rc = list_out(m_numer, m_denom, true, m_list, m, who)) return rc;
    if (!m_numer || !m_denom) return fail(FPM_EINVAL, std::string(who) + ": mirror numer / denom required");
    return dist_dev_impl(rs->ctx, rs->ref, rs->ref_len, rs->ref_length, rs->ref_stride, rs->n_ref,
                         d_qry, d_qry_len, d_qry_length, qry_stride, n_qry, rs->hash_bytes,
                         sketch_size, kmer_size, kmer_space, max_dist, max_pvalue, o, stream, who,
                         rs, &m);
}

int fpm_refset_reindex(fpm_refset *rs, void *stream)
{
    if (!rs) return fail(FPM_EINVAL, "refset_reindex: null set");
    if (int rc = set_device(rs->ctx)) return rc;
    return refset_build_index(rs, pick_stream(rs->ctx, stream));
}

int fpm_refset_dist(fpm_refset *rs, const void *qry, const uint32_t *qry_len,
                    const uint64_t *qry_length, uint64_t qry_stride, uint32_t n_qry,
                    uint32_t sketch_size, uint32_t kmer_size, double kmer_space, double max_dist,
                    double max_pvalue, uint32_t *out_numer, uint32_t *out_denom, double *out_dist,
                    double *out_pvalue, uint8_t *out_pass)
{
    if (!rs) return fail(FPM_EINVAL, "refset_dist: null set");
    fpm_ctx *ctx = rs->ctx;
    if (int rc = set_device(ctx)) return rc;
    const uint64_t np = (uint64_t)rs->n_ref * n_qry;
    if (np == 0) return FPM_OK;
    hipStream_t st = ctx->stream;
    void *q, *ql, *qL, *nu, *de, *di, *pv, *pa;
    const size_t qb = std::max<size_t>(16, (size_t)n_qry * qry_stride * rs->hash_bytes);
    HIP_TRY(slot_buf(rs->qslot[0], qb, &q));
    HIP_TRY(slot_buf(rs->qslot[1], (size_t)n_qry * 4, &ql));
    HIP_TRY(slot_buf(rs->qslot[2], (size_t)n_qry * 8, &qL));
    HIP_TRY(slot_buf(rs->qslot[3], np * 4, &nu));
    HIP_TRY(slot_buf(rs->qslot[4], np * 4, &de));
    HIP_TRY(slot_buf(rs->qslot[5], np * 8, &di));
    HIP_TRY(slot_buf(rs->qslot[6], np * 8, &pv));
    HIP_TRY(slot_buf(rs->qslot[7], np, &pa));
    HIP_TRY(hipStreamSynchronize(st));            // the query slots are free to overwrite
    HIP_TRY(copy_in(ctx, q, qry, (size_t)n_qry * qry_stride * rs->hash_bytes));
    HIP_TRY(copy_in(ctx, ql, qry_len, (size_t)n_qry * 4));
    if (qry_length)
        HIP_TRY(copy_in(ctx, qL, qry_length, (size_t)n_qry * 8));
    else
        HIP_TRY(hipMemsetAsync(qL, 0, (size_t)n_qry * 8, st));
    if (int rc = fpm_refset_dist_dev(rs, q, (const uint32_t *)ql, (const uint64_t *)qL, qry_stride,
                                     n_qry, sketch_size, 4, kmer_size, kmer_space, max_dist,
                                     max_pvalue, nu, de, (double *)di, (double *)pv,
                                     (uint8_t *)pa, st))
        return rc;
    // results: caller memory (pinned from fpm_host_alloc copies at full PCIe rate, pageable
    // memory through the context's pinned ring)
    HIP_TRY(hipStreamSynchronize(st));
    if (out_numer) HIP_TRY(copy_out(ctx, out_numer, nu, np * 4));
    if (out_denom) HIP_TRY(copy_out(ctx, out_denom, de, np * 4));
    if (out_dist) HIP_TRY(copy_out(ctx, out_dist, di, np * 8));
    if (out_pvalue) HIP_TRY(copy_out(ctx, out_pvalue, pv, np * 8));
    if (out_pass) HIP_TRY(copy_out(ctx, out_pass, pa, np));
    return FPM_OK;
}

int fpm_refset_dist_list(fpm_refset *rs, const void *qry, const uint32_t *qry_len,
                         const uint64_t *qry_length, uint64_t qry_stride, uint32_t n_qry,
                         uint32_t sketch_size, uint32_t kmer_size, double kmer_space,
                         double max_dist, double max_pvalue, uint32_t count_bytes,
                         void *out_numer, void *out_denom, uint32_t *l_qry, uint32_t *l_ref,
                         double *l_dist, double *l_pvalue, uint8_t *l_pass, uint64_t cap,
                         uint64_t *n_listed)
{
    if (!rs) return fail(FPM_EINVAL, "refset_dist_list: null set");
    if (count_bytes != 2 && count_bytes != 4) return fail(FPM_EINVAL, "count_bytes must be 2 or 4");
    if (!n_listed) return fail(FPM_EINVAL, "refset_dist_list: null n_listed");
    *n_listed = 0;
    fpm_ctx *ctx = rs->ctx;
    if (int rc = set_device(ctx)) return rc;
    const uint64_t np = (uint64_t)rs->n_ref * n_qry;
    if (np == 0) return FPM_OK;
    hipStream_t st = ctx->stream;
    void *q, *ql, *qL, *nu, *de;
    const size_t qb = std::max<size_t>(16, (size_t)n_qry * qry_stride * rs->hash_bytes);
    HIP_TRY(slot_buf(rs->qslot[0], qb, &q));
    HIP_TRY(slot_buf(rs->qslot[1], (size_t)n_qry * 4, &ql));
    HIP_TRY(slot_buf(rs->qslot[2], (size_t)n_qry * 8, &qL));
    HIP_TRY(slot_buf(rs->qslot[3], np * count_bytes, &nu));
    HIP_TRY(slot_buf(rs->qslot[4], np * count_bytes, &de));
    HIP_TRY(hipStreamSynchronize(st));            // the query slots are free to overwrite
    HIP_TRY(copy_in(ctx, q, qry, (size_t)n_qry * qry_stride * rs->hash_bytes));
    HIP_TRY(copy_in(ctx, ql, qry_len, (size_t)n_qry * 4));
    if (qry_length)
        HIP_TRY(copy_in(ctx, qL, qry_length, (size_t)n_qry * 8));
    else
        HIP_TRY(hipMemsetAsync(qL, 0, (size_t)n_qry * 8, st));
    // the device list: grown (and the call repeated) when the cells sharing hashes outnumber it
    uint64_t want = std::max<uint64_t>(rs->list_cap, std::max<uint64_t>(4096, np / 32));
    for (;;) {
        fpm_cell_list L{};
        void *p[6];
        const size_t eb[6] = {4, 4, 8, 8, 1, 0};
        for (int i = 0; i < 5; i++) HIP_TRY(slot_buf(rs->qslot[10 + i], want * eb[i], &p[i]));
        HIP_TRY(slot_buf(rs->qslot[15], 8, &p[5]));
        rs->list_cap = want;
        L.qry = (uint32_t *)p[0];
        L.ref = (uint32_t *)p[1];
        L.dist = (double *)p[2];
        L.pvalue = (double *)p[3];
        L.pass = (uint8_t *)p[4];
        L.cap = want;
        L.count = (uint64_t *)p[5];
        if (int rc = refset_list_impl(rs, q, (const uint32_t *)ql, (const uint64_t *)qL,
                                      qry_stride, n_qry, sketch_size, kmer_size, kmer_space,
                                      max_dist, max_pvalue, count_bytes, nu, de, &L, st,
                                      "fpm_refset_dist_list"))
            return rc;
        uint64_t cnt = 0;
        HIP_TRY(hipMemcpyAsync(&cnt, L.count, 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        if (cnt > want) {
            want = cnt + cnt / 8;
            continue;
        }
        *n_listed = cnt;
        const uint64_t m = std::min<uint64_t>(cnt, cap);
        if (out_numer) HIP_TRY(copy_out(ctx, out_numer, nu, np * count_bytes));
        if (out_denom) HIP_TRY(copy_out(ctx, out_denom, de, np * count_bytes));
        if (m) {
            if (l_qry) HIP_TRY(copy_out(ctx, l_qry, L.qry, m * 4));
            if (l_ref) HIP_TRY(copy_out(ctx, l_ref, L.ref, m * 4));
            if (l_dist) HIP_TRY(copy_out(ctx, l_dist, L.dist, m * 8));
            if (l_pvalue) HIP_TRY(copy_out(ctx, l_pvalue, L.pvalue, m * 8));
            if (l_pass) HIP_TRY(copy_out(ctx, l_pass, L.pass, m));
        }
        return FPM_OK;
    }
}

void fpm_refset_free(fpm_refset *rs)
{
    if (!rs) return;
    if (rs->ctx) (void)hipSetDevice(rs->ctx->device);
    for (auto &sl : rs->slot)
        if (sl.p) (void)hipFree(sl.p);
    for (auto &sl : rs->qslot)
        if (sl.p) (void)hipFree(sl.p);
    for (void *o : rs->own)
        if (o) (void)hipFree(o);
    if (rs->kmax) (void)hipFree(rs->kmax);
    delete rs;
}

int fpm_fp_positional_grid(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len,
                           uint64_t ref_stride, uint32_t n_ref, const void *qry,
                           const uint32_t *qry_len, uint64_t qry_stride, uint32_t n_qry,
                           uint32_t hash_bytes, double max_dist, double max_pvalue,
                           uint32_t *out_numer, uint32_t *out_denom, double *out_dist,
                           double *out_pvalue, uint8_t *out_pass)
{
    if (int rc = set_device(ctx)) return rc;
    if (hash_bytes != 4 && hash_bytes != 8) return fail(FPM_EINVAL, "hash_bytes must be 4 or 8");
    if (n_qry > 65535) return fail(FPM_EINVAL, "positional grid: at most 65535 queries per call");
    const uint64_t np = (uint64_t)n_ref * n_qry;
    if (np == 0) return FPM_OK;
    DevBuf r, rl, q, ql, nu, de, di, pv, pa;
    hipError_t e = hipSuccess;
    auto up = [&](DevBuf &b, const void *h, size_t bytes) {
        if (e != hipSuccess) return;
        e = hipMalloc(&b.p, bytes ? bytes : 16);
        if (e == hipSuccess && h && bytes) e = copy_in(ctx, b.p, h, bytes);
    };
    up(r, ref, (size_t)n_ref * ref_stride * hash_bytes);
    up(rl, ref_len, (size_t)n_ref * 4);
    up(q, qry, (size_t)n_qry * qry_stride * hash_bytes);
    up(ql, qry_len, (size_t)n_qry * 4);
    up(nu, nullptr, np * 4);
    up(de, nullptr, np * 4);
    up(di, nullptr, np * 8);
    up(pv, nullptr, np * 8);
    up(pa, nullptr, np);
    if (e != hipSuccess) return fail(FPM_ENOMEM, std::string("positional staging: ") + hipGetErrorString(e));
    hipStream_t st = ctx->stream;
    HIP_TRY(launch_positional_grid(r.p, (const uint32_t *)rl.p, ref_stride, n_ref, q.p,
                                   (const uint32_t *)ql.p, qry_stride, n_qry, hash_bytes, max_dist,
                                   max_pvalue, (uint32_t *)nu.p, (uint32_t *)de.p, (double *)di.p,
                                   (double *)pv.p, (uint8_t *)pa.p, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (out_numer) HIP_TRY(copy_out(ctx, out_numer, nu.p, np * 4));
    if (out_denom) HIP_TRY(copy_out(ctx, out_denom, de.p, np * 4));
    if (out_dist) HIP_TRY(copy_out(ctx, out_dist, di.p, np * 8));
    if (out_pvalue) HIP_TRY(copy_out(ctx, out_pvalue, pv.p, np * 8));
    if (out_pass) HIP_TRY(copy_out(ctx, out_pass, pa.p, np));
    return FPM_OK;
}

int fpm_compare_grid(fpm_ctx *ctx, const void *ref, const uint32_t *ref_len,
                     uint64_t ref_stride, uint32_t n_ref, const void *qry,
                     const uint32_t *qry_len, uint64_t qry_stride, uint32_t n_qry,
                     uint32_t hash_bytes, uint32_t sketch_size, uint32_t *out_numer,
                     uint32_t *out_denom)
{
    return fpm_dist(ctx, ref, ref_len, nullptr, ref_stride, n_ref, qry, qry_len, nullptr,
                    qry_stride, n_qry, hash_bytes, sketch_size, 0, 0.0, -1.0, -1.0, out_numer,
                    out_denom, nullptr, nullptr, nullptr);
}

}  // extern "C"
