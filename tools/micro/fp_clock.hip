// tools/micro/fp_clock.hip — is the one-off slow -fp text call the kernel, or
// the GPU?  A one-workgroup "ticker" kernel on its own stream samples the 100 MHz constant
// clock (s_memrealtime) and the shader clock counter (s_memtime) in a loop for ~0.6 s, logging
// every sample whose realtime step exceeds 20 us (a stall of the ticker's wave) plus one sample
// per ~1 ms (the shader/real clock ratio over time).  Meanwhile the host runs the bench's
// -fp text call (fpm_fp_text_stage + fetch into fresh malloc'd arrays + free) 40 times and
// prints each call's HIP-event kernel time with its host time.  Build on the CPU container:
//   hipcc --offload-arch=gfx950 -O2 -I../../include fp_clock.hip -L../../fp-mash_amd/lib \
//         -lfpmash -Wl,-rpath,'$ORIGIN/../../fp-mash_amd/lib' -o fp_clock
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "fpmash.h"

struct Sample { unsigned long long rt, st; };

// one wave: lane 0 samples; ends after `dur` realtime ticks (every wave reaches the exit)
__global__ void ticker(Sample *log, unsigned *n_log, unsigned cap, unsigned long long dur)
{
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long prev = t0, last_keep = t0;
    unsigned n = 0;
    for (;;) {
        const unsigned long long rt = __builtin_amdgcn_s_memrealtime();
        const unsigned long long st = __builtin_amdgcn_s_memtime();
        if (rt - t0 > dur) break;
        if ((rt - prev > 2000 || rt - last_keep > 100000) && n < cap) {   // 20 us gap / 1 ms
            log[n].rt = rt - t0;
            log[n].st = st;
            n++;
            last_keep = rt;
        }
        prev = rt;
    }
    *n_log = n;
}

static std::string cfl_text(size_t lines)
{
    std::string t;
    t.reserve(lines * 32);
    char buf[64];
    unsigned x = 12345;
    for (size_t i = 0; i < lines; i++) {
        const int nv = 1 + (int)(i % 9);
        int o = snprintf(buf, sizeof buf, "T%05zu", i / 2000);
        t.append(buf, o);
        for (int v = 0; v < nv; v++) {
            x = x * 1103515245u + 12345u;
            o = snprintf(buf, sizeof buf, " %u", (x >> 16) % 200);
            t.append(buf, o);
        }
        t.push_back('\n');
    }
    return t;
}

int main()
{
    fpm_ctx *ctx;
    if (fpm_ctx_create(0, &ctx)) { fprintf(stderr, "%s\n", fpm_last_error()); return 1; }
    const std::string text = cfl_text(1000000);
    const unsigned cap = 1 << 16;
    Sample *d_log;
    unsigned *d_n;
    hipMalloc(&d_log, cap * sizeof(Sample));
    hipMalloc(&d_n, 4);
    hipStream_t ts;
    hipStreamCreateWithFlags(&ts, hipStreamNonBlocking);
    // warm the -fp kernels and the pinned ring first
    for (int w = 0; w < 2; w++) {
        fpm_fptext *j; uint64_t n;
        fpm_fp_text_stage(ctx, text.data(), text.size(), 1000000, 42, 0, &j, &n);
        fpm_fp_text_free(j);
    }
    fpm_ctx_synchronize(ctx);
    const auto h0 = std::chrono::steady_clock::now();
    double worst_call = 0;
    hipLaunchKernelGGL(ticker, dim3(1), dim3(64), 0, ts, d_log, d_n, cap, 60000000ull);   // 0.6 s
    for (int c = 0; c < 40; c++) {
        fpm_ctx_reset_timing(ctx);
        fpm_ctx_set_timing(ctx, 1);
        const auto a = std::chrono::steady_clock::now();
        fpm_fptext *j; uint64_t n;
        if (fpm_fp_text_stage(ctx, text.data(), text.size(), 1000000, 42, 0, &j, &n)) {
            fprintf(stderr, "%s\n", fpm_last_error());
            return 1;
        }
        uint64_t *io = (uint64_t *)malloc(n * 8);
        uint32_t *il = (uint32_t *)malloc(n * 4), *nv = (uint32_t *)malloc(n * 4),
                 *h = (uint32_t *)malloc(n * 4);
        uint8_t *ni = (uint8_t *)malloc(n);
        fpm_fp_text_fetch(j, io, il, nv, h, ni);
        fpm_fp_text_free(j);
        free(io); free(il); free(nv); free(h); free(ni);
        fpm_ctx_set_timing(ctx, 0);
        const auto b = std::chrono::steady_clock::now();
        double ms; uint64_t l;
        fpm_ctx_kernel_time(ctx, FPM_K_FPTEXT, &ms, &l);
        worst_call = std::max(worst_call, ms);
        printf("call %2d: host %.3f..%.3f ms, kernels %.3f ms\n", c,
               std::chrono::duration<double, std::milli>(a - h0).count(),
               std::chrono::duration<double, std::milli>(b - h0).count(), ms);
    }
    hipStreamSynchronize(ts);
    unsigned n_log = 0;
    hipMemcpy(&n_log, d_n, 4, hipMemcpyDeviceToHost);
    std::vector<Sample> lg(n_log);
    hipMemcpy(lg.data(), d_log, n_log * sizeof(Sample), hipMemcpyDeviceToHost);
    double worst_gap = 0;
    for (unsigned i = 1; i < n_log; i++)
        worst_gap = std::max(worst_gap, (double)(lg[i].rt - lg[i - 1].rt) / 100.0);
    printf("SUMMARY worst kernel-time call %.3f ms, worst ticker gap %.1f us, pageable_direct=%s\n",
           worst_call, worst_gap, getenv("FPM_PAGEABLE_DIRECT") ? getenv("FPM_PAGEABLE_DIRECT") : "0");
    printf("ticker: %u samples (gaps > 20 us and one per ms)\n", n_log);
    for (unsigned i = 1; i < n_log; i++) {
        const double drt = (double)(lg[i].rt - lg[i - 1].rt) / 100.0;        // us
        const double dst = (double)(lg[i].st - lg[i - 1].st);
        printf("t=%9.1f us  step %8.1f us  shader ticks/us %7.1f\n", lg[i].rt / 100.0, drt,
               drt > 0 ? dst / drt : 0.0);
    }
    fpm_ctx_destroy(ctx);
    return 0;
}
