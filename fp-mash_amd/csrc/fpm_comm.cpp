// fpm_comm.cpp — RCCL over xGMI inside libfpmash (include/fpmash.h, "communicator").
//
// The one exchange the north-star path has: the bottom-s MIN-MERGE of one sketch computed in
// parts on several GPUs (a genome's k-mer ranges, or a reference set larger than one GPU's
// HBM).  The reference has no collective at all: one process, one pthreads pool
// (ThreadPool.h:13-61) feeding one MinHashHeap per genome (Sketch.cpp:1354-1422, MinHashHeap.cpp:
// 68-146).  Here every rank's bottom-s row (s hashes + its count) is all-gathered by RCCL into
// library-owned buffers on the context's device and stream, and merged there by
// fpm_sketch_merge_dev: the s smallest distinct of a union are the s smallest of the union of
// the parts' s smallest.
//
// The communicator runs on the SAME HIP runtime as the kernels (system ROCm), so its buffers,
// streams and ordering are the library's own: no second runtime in the process, no host sync
// between the gather and the merge.  librccl (~570 MB) is loaded with dlopen on first use,
// so processes that never build a communicator (the CLI) do not pay for mapping it.  The
// unique id travels over the caller's host channel (fpm_comm_unique_id on one rank, then any
// broadcast of its 128 bytes), as ncclGetUniqueId's contract asks.
#include "../../include/fpmash.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

namespace {

// the subset of RCCL this file calls, resolved from the system librccl
struct Rccl {
    void *h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    std::string why;
};

Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char *n : names)
            if ((r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!r.h) {
            const char *e = dlerror();
            r.why = std::string("librccl not loadable: ") + (e ? e : "?");
            return;
        }
        auto sym = [&](const char *s) {
            void *p = dlsym(r.h, s);
            if (!p && r.why.empty()) r.why = std::string("librccl lacks ") + s;
            return p;
        };
        r.get_unique_id = (decltype(r.get_unique_id))sym("ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))sym("ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))sym("ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather))sym("ncclAllGather");
        r.group_start = (decltype(r.group_start))sym("ncclGroupStart");
        r.group_end = (decltype(r.group_end))sym("ncclGroupEnd");
        r.error_string = (decltype(r.error_string))sym("ncclGetErrorString");
    });
    return r;
}

}  // namespace

// fpm_api.cpp: the message fpm_last_error() returns (one error text for the whole ABI)
int fpm_detail_fail(int code, const std::string &msg);

namespace {

int cfail(int code, const std::string &m) { return fpm_detail_fail(code, m); }

int rccl_fail(const char *what, ncclResult_t rc)
{
    const Rccl &r = rccl();
    return cfail(FPM_EHIP, std::string(what) + ": " +
                               (r.error_string ? r.error_string(rc) : "rccl error"));
}

}  // namespace

struct fpm_comm {
    fpm_ctx *ctx = nullptr;
    int device = 0, nranks = 0, rank = 0;
    ncclComm_t comm = nullptr;
    // grow-only gather buffers of the min-merge: [nranks][s] hashes, [nranks] counts
    void *rows = nullptr, *counts = nullptr;
    size_t rows_bytes = 0, counts_bytes = 0;
};

namespace {

// The set-up's time limit: FPM_COMM_INIT_TIMEOUT_S (default 120 s).  A rank whose peers never
// join (a peer failed before its own set-up) gets an error instead of blocking for ever, so a
// caller can report it and go on; the abandoned set-up thread stays blocked until the process
// ends (an abort would wait for it).
double init_limit_s()
{
    const char *v = getenv("FPM_COMM_INIT_TIMEOUT_S");
    const double t = v ? atof(v) : 0.0;
    return t > 0.0 ? t : 120.0;
}

}  // namespace

extern "C" {

int fpm_comm_unique_id(uint8_t id[FPM_COMM_ID_BYTES])
{
    if (!id) return cfail(FPM_EINVAL, "null id");
    Rccl &r = rccl();
    if (!r.why.empty()) return cfail(FPM_ENODEV, r.why);
    ncclUniqueId u;
    if (ncclResult_t rc = r.get_unique_id(&u)) return rccl_fail("ncclGetUniqueId", rc);
    static_assert(sizeof(u) == FPM_COMM_ID_BYTES, "RCCL unique id size");
    memcpy(id, &u, sizeof(u));
    return FPM_OK;
}

int fpm_comm_create(fpm_ctx *ctx, int nranks, int rank, const uint8_t id[FPM_COMM_ID_BYTES],
                    fpm_comm **out)
{
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return cfail(FPM_EINVAL, "comm_create: bad argument");
    *out = nullptr;
    Rccl &r = rccl();
    if (!r.why.empty()) return cfail(FPM_ENODEV, r.why);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return cfail(FPM_EHIP, "hipGetDevice");
    // the communicator binds to the current device: the context's (fpm_ctx_stream's device)
    hipStream_t st = (hipStream_t)fpm_ctx_stream(ctx);
    int sdev = dev;
    if (hipStreamGetDevice(st, &sdev) == hipSuccess && sdev != dev &&
        hipSetDevice(sdev) != hipSuccess)
        return cfail(FPM_EHIP, "hipSetDevice");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    fpm_comm *c = new fpm_comm();
    c->ctx = ctx;
    c->device = sdev;
    c->nranks = nranks;
    c->rank = rank;
    {
        // bounded: the blocking set-up on a thread of its own, waited for up to the limit (a
        // non-blocking RCCL set-up still waited inside the call for the missing peers)
        struct Setup {
            std::mutex mu;
            std::condition_variable cv;
            bool done = false, abandoned = false;
            ncclResult_t rc = ncclSuccess;
            ncclComm_t comm = nullptr;
        };
        auto su = std::make_shared<Setup>();
        const int dev_ = sdev;
        std::thread([su, &r, nranks, u, rank, dev_] {
            (void)hipSetDevice(dev_);
            ncclComm_t cm = nullptr;
            const ncclResult_t rc = r.comm_init_rank(&cm, nranks, u, rank);
            std::lock_guard<std::mutex> lk(su->mu);
            su->rc = rc;
            su->comm = cm;
            su->done = true;
            // a caller that gave up left this communicator to the process
            su->cv.notify_all();
        }).detach();
        const double limit = init_limit_s();
        std::unique_lock<std::mutex> lk(su->mu);
        if (!su->cv.wait_for(lk, std::chrono::duration<double>(limit), [&] { return su->done; })) {
            su->abandoned = true;
            delete c;
            return cfail(FPM_EHIP, "ncclCommInitRank: not every rank joined within " +
                                       std::to_string((int)limit) + " s (FPM_COMM_INIT_TIMEOUT_S)");
        }
        if (su->rc != ncclSuccess) {
            delete c;
            return rccl_fail("ncclCommInitRank", su->rc);
        }
        c->comm = su->comm;
    }
    *out = c;
    return FPM_OK;
}

void fpm_comm_destroy(fpm_comm *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm) (void)rccl().comm_destroy(c->comm);
    if (c->rows) (void)hipFree(c->rows);
    if (c->counts) (void)hipFree(c->counts);
    delete c;
}

int fpm_comm_all_gather(fpm_comm *c, const void *d_send, void *d_recv, size_t bytes, void *stream)
{
    if (!c || (bytes && (!d_send || !d_recv))) return cfail(FPM_EINVAL, "all_gather: bad argument");
    if (!bytes) return FPM_OK;
    if (hipSetDevice(c->device) != hipSuccess) return cfail(FPM_EHIP, "hipSetDevice");
    hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)fpm_ctx_stream(c->ctx);
    if (ncclResult_t rc = rccl().all_gather(d_send, d_recv, bytes, ncclUint8, c->comm, st))
        return rccl_fail("ncclAllGather", rc);
    return FPM_OK;
}

int fpm_sketch_min_merge_comm(fpm_comm *c, const uint64_t *d_row, const uint32_t *d_count,
                              uint32_t s, uint64_t *d_out, uint32_t *d_out_count, void *stream)
{
    if (!c || !d_row || !d_count || !d_out || !d_out_count || s == 0)
        return cfail(FPM_EINVAL, "min_merge_comm: bad argument");
    if (hipSetDevice(c->device) != hipSuccess) return cfail(FPM_EHIP, "hipSetDevice");
    hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)fpm_ctx_stream(c->ctx);
    const size_t rb = (size_t)c->nranks * s * 8, cb = (size_t)c->nranks * 4;
    auto grow = [&](void **p, size_t *have, size_t want) -> int {
        if (*have >= want) return FPM_OK;
        // the previous gather into it may still be queued
        if (*p && (hipStreamSynchronize(st) != hipSuccess || hipFree(*p) != hipSuccess))
            return cfail(FPM_EHIP, "min_merge_comm: buffer release");
        *p = nullptr;
        *have = 0;
        if (hipMalloc(p, want) != hipSuccess) return cfail(FPM_ENOMEM, "min_merge_comm: hipMalloc");
        *have = want;
        return FPM_OK;
    };
    if (int rc = grow(&c->rows, &c->rows_bytes, rb)) return rc;
    if (int rc = grow(&c->counts, &c->counts_bytes, cb)) return rc;
    Rccl &r = rccl();
    if (ncclResult_t rc = r.group_start()) return rccl_fail("ncclGroupStart", rc);
    ncclResult_t a = r.all_gather(d_row, c->rows, (size_t)s * 8, ncclUint8, c->comm, st);
    ncclResult_t b = a ? a : r.all_gather(d_count, c->counts, 4, ncclUint8, c->comm, st);
    ncclResult_t e = r.group_end();
    if (a || b || e) return rccl_fail("ncclAllGather (min-merge)", a ? a : b ? b : e);
    // the merge on the same stream, after the gather (fpm_sketch_merge_dev: pairwise rounds)
    const int rc = fpm_sketch_merge_dev(c->ctx, (const uint64_t *)c->rows,
                                        (const uint32_t *)c->counts, (uint32_t)c->nranks, s,
                                        d_out, d_out_count, st);
    if (rc) return cfail(rc, std::string("min_merge_comm: ") + fpm_last_error());
    return FPM_OK;
}

}  // extern "C"
