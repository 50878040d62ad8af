// tools/micro/fill_rates.hip — write rate of the dist grid's no-shared-hash fill on gfx950.
// 1e8 cells x 25 B (u32 numer, u32 denom, f64 distance, f64 p-value, u8 pass) in five arrays,
// as dist_fill_kernel writes them, against launch shapes: one workgroup per 1024 / 4096 cells,
// a grid-stride loop over CUs x 8 workgroups, non-temporal stores; and hipMemset of the same
// bytes.  Prints GB/s per variant (each alone on the chip).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct Out { uint32_t *nu, *de; double *di, *pv; uint8_t *pa; };

template <bool NT>
__device__ __forceinline__ void put4(Out o, uint64_t c, uint32_t d)
{
    const uint4 z = make_uint4(0, 0, 0, 0), dn = make_uint4(d, d, d, d);
    const double2 one = make_double2(1.0, 1.0);
    if (NT) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        typedef double v2d __attribute__((ext_vector_type(2)));
        const v4u vz = {0, 0, 0, 0}, vd = {d, d, d, d};
        const v2d v1 = {1.0, 1.0};
        __builtin_nontemporal_store(vz, (v4u *)(o.nu + c));
        __builtin_nontemporal_store(vd, (v4u *)(o.de + c));
        __builtin_nontemporal_store(v1, (v2d *)(o.di + c));
        __builtin_nontemporal_store(v1, (v2d *)(o.di + c + 2));
        __builtin_nontemporal_store(v1, (v2d *)(o.pv + c));
        __builtin_nontemporal_store(v1, (v2d *)(o.pv + c + 2));
        __builtin_nontemporal_store(0x01010101u, (uint32_t *)(o.pa + c));
    } else {
        *(uint4 *)(o.nu + c) = z;
        *(uint4 *)(o.de + c) = dn;
        *(double2 *)(o.di + c) = one;
        *(double2 *)(o.di + c + 2) = one;
        *(double2 *)(o.pv + c) = one;
        *(double2 *)(o.pv + c + 2) = one;
        *(uint32_t *)(o.pa + c) = 0x01010101u;
    }
}

// one workgroup per CELLS cells, 4 cells per lane per pass
template <int CELLS, bool NT>
__global__ __launch_bounds__(256) void fill_oneshot(Out o, uint64_t n, uint32_t d)
{
    const uint64_t base = (uint64_t)blockIdx.x * CELLS;
#pragma unroll
    for (int p = 0; p < CELLS / 1024; p++) {
        const uint64_t c = base + p * 1024 + threadIdx.x * 4;
        if (c < n) put4<NT>(o, c, d);
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void fill_stride(Out o, uint64_t n, uint32_t d)
{
    for (uint64_t c = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4; c < n;
         c += (uint64_t)gridDim.x * 1024)
        put4<NT>(o, c, d);
}

// f64 only (8 B/cell), one workgroup per 1024 cells
__global__ __launch_bounds__(256) void fill_one_array(double *di, uint64_t n)
{
    const uint64_t c = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
    if (c < n) {
        *(double2 *)(di + c) = make_double2(1.0, 1.0);
        *(double2 *)(di + c + 2) = make_double2(1.0, 1.0);
    }
}

// stand-in for the rank kernel: LDS-resident table, dependent 64-bit compare / select
// search steps (VALU + LDS bound, no HBM traffic)
__global__ __launch_bounds__(256) void compute_like_rank(uint64_t *sink, int iters)
{
    __shared__ uint64_t tab[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) tab[i] = (uint64_t)i * 0x9E3779B97F4A7C15ULL;
    __syncthreads();
    uint64_t x = (uint64_t)(blockIdx.x * 256 + threadIdx.x) * 0xC2B2AE3D27D4EB4FULL;
    uint32_t lo[4] = {0, 0, 0, 0};
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
            uint32_t len = 2048, l = 0;
#pragma unroll
            for (int st = 0; st < 4; st++) {
                const uint32_t half = len >> 1;
                const bool less = tab[(l + half + g) & 2047] < x;
                l = less ? l + half + 1 : l;
                len = less ? len - half - 1 : half;
            }
            lo[g] += l;
        }
        x = x * 6364136223846793005ULL + 1442695040888963407ULL;
    }
    if (lo[0] + lo[1] + lo[2] + lo[3] == 0xFFFFFFFFu) sink[threadIdx.x] = x;
}

int main()
{
    const uint64_t n = 100000000ULL;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    Out o;
    hipMalloc(&o.nu, n * 4);
    hipMalloc(&o.de, n * 4);
    hipMalloc(&o.di, n * 8);
    hipMalloc(&o.pv, n * 8);
    hipMalloc(&o.pa, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double bytes = 25.0 * n;
    auto run = [&](const char *name, double b, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; it++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, best, b / best / 1e6);
    };
    const uint32_t g1k = (uint32_t)((n + 1023) / 1024), g4k = (uint32_t)((n + 4095) / 4096);
    run("oneshot_1024_cells_per_wg", bytes, [&] { hipLaunchKernelGGL((fill_oneshot<1024, false>), dim3(g1k), dim3(256), 0, 0, o, n, 1000u); });
    run("oneshot_4096_cells_per_wg", bytes, [&] { hipLaunchKernelGGL((fill_oneshot<4096, false>), dim3(g4k), dim3(256), 0, 0, o, n, 1000u); });
    run("oneshot_1024_nt", bytes, [&] { hipLaunchKernelGGL((fill_oneshot<1024, true>), dim3(g1k), dim3(256), 0, 0, o, n, 1000u); });
    for (int per = 4; per <= 32; per *= 2) {
        char nm[64];
        snprintf(nm, sizeof nm, "stride_%dwg_per_cu", per);
        run(nm, bytes, [&] { hipLaunchKernelGGL((fill_stride<false>), dim3(cus * per), dim3(256), 0, 0, o, n, 1000u); });
    }
    run("stride_8wg_per_cu_nt", bytes, [&] { hipLaunchKernelGGL((fill_stride<true>), dim3(cus * 8), dim3(256), 0, 0, o, n, 1000u); });
    run("one_f64_array_oneshot", 8.0 * n, [&] { hipLaunchKernelGGL(fill_one_array, dim3(g1k), dim3(256), 0, 0, o.di, n); });
    run("hipMemset_25B_per_cell", bytes, [&] {
        hipMemsetAsync(o.nu, 0, n * 4); hipMemsetAsync(o.de, 0, n * 4); hipMemsetAsync(o.di, 0, n * 8);
        hipMemsetAsync(o.pv, 0, n * 8); hipMemsetAsync(o.pa, 0, n); });
    // ---- the fill beside a compute kernel: default streams, and CU-masked streams
    uint64_t *sink;
    hipMalloc(&sink, 4096);
    hipStream_t s_c, s_f;
    hipStreamCreateWithFlags(&s_c, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s_f, hipStreamNonBlocking);
    const int citers = 200;
    auto comp = [&](hipStream_t s) { hipLaunchKernelGGL(compute_like_rank, dim3(10000), dim3(256), 0, s, sink, citers); };
    auto fill = [&](hipStream_t s) { hipLaunchKernelGGL((fill_oneshot<1024, false>), dim3(g1k), dim3(256), 0, s, o, n, 1000u); };
    auto timed2 = [&](const char *name, hipStream_t a, hipStream_t b, bool doc, bool dof) {
        for (int w = 0; w < 2; w++) { if (doc) comp(a); if (dof) fill(b); }
        hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; it++) {
            hipEventRecord(e0, 0);
            hipStreamWaitEvent(a, e0, 0); hipStreamWaitEvent(b, e0, 0);
            if (doc) comp(a);
            if (dof) fill(b);
            hipEvent_t ea, eb; hipEventCreate(&ea); hipEventCreate(&eb);
            hipEventRecord(ea, a); hipEventRecord(eb, b);
            hipStreamWaitEvent(0, ea, 0); hipStreamWaitEvent(0, eb, 0);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
            hipEventDestroy(ea); hipEventDestroy(eb);
        }
        printf("{\"variant\": \"%s\", \"ms\": %.4f}\n", name, best);
    };
    timed2("compute_alone", s_c, s_f, true, false);
    timed2("fill_alone_stream", s_c, s_f, false, true);
    timed2("compute_and_fill_unmasked", s_c, s_f, true, true);
    for (int ncu : {32, 64, 128}) {
        for (int pat = 0; pat < 2; pat++) {
            uint32_t mf[8] = {0}, mc[8] = {0};
            int set = 0;
            for (int c = 0; c < cus && c < 256; c++) {
                bool in = pat == 0 ? (c < ncu) : (c % (cus / ncu) == 0);
                if (in) { mf[c / 32] |= 1u << (c % 32); set++; }
                else mc[c / 32] |= 1u << (c % 32);
            }
            hipStream_t sf, sc;
            if (hipExtStreamCreateWithCUMask(&sf, 8, mf) != hipSuccess ||
                hipExtStreamCreateWithCUMask(&sc, 8, mc) != hipSuccess) { printf("mask fail\n"); continue; }
            char nm[96];
            snprintf(nm, sizeof nm, "fill_alone_on_%d_cus_%s", set, pat ? "strided" : "first");
            timed2(nm, s_c, sf, false, true);
            snprintf(nm, sizeof nm, "compute_unmasked_fill_on_%d_cus_%s", set, pat ? "strided" : "first");
            timed2(nm, s_c, sf, true, true);
            snprintf(nm, sizeof nm, "compute_on_rest_fill_on_%d_cus_%s", set, pat ? "strided" : "first");
            timed2(nm, sc, sf, true, true);
            hipStreamDestroy(sf); hipStreamDestroy(sc);
        }
    }
    hipFree(sink);
    hipFree(o.nu); hipFree(o.de); hipFree(o.di); hipFree(o.pv); hipFree(o.pa);
    return 0;
}
