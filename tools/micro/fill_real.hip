// tools/micro/fill_real.hip — the library's dist_fill_kernel alone at the bench shape
// (10,000 x 10,000 cells: distance, p-value, pass = 17 B/cell), against a bare 17 B/cell
// store stream, to separate the kernel's own write rate from its slowdown beside the rank
// kernel.  Prints GB/s.
#include "../../fp-mash_amd/csrc/dist.hip"

#include <stdio.h>
#include <stdlib.h>
#include <vector>

using namespace fpm;

__global__ __launch_bounds__(256) void bare17(double *di, double *pv, uint8_t *pa, uint64_t n)
{
    const uint64_t c = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (c >= n) return;
    *(double2 *)(di + c) = make_double2(1.0, 1.0);
    *(double2 *)(di + c + 2) = make_double2(1.0, 1.0);
    *(double2 *)(pv + c) = make_double2(1.0, 1.0);
    *(double2 *)(pv + c + 2) = make_double2(1.0, 1.0);
    *(uint32_t *)(pa + c) = 0x01010101u;
}

// the fill with flat indexing: workgroup k takes cells [1024 k, 1024 k + 1024) of the whole
// grid (rows found per lane), so every wave store is line-aligned and no workgroup is partial
__global__ __launch_bounds__(256) void flat_fill(const uint32_t *__restrict__ ref_len, uint32_t n_ref,
                                                 const uint32_t *__restrict__ qry_len, uint64_t cells,
                                                 uint32_t S, PairFill fill)
{
    const uint64_t o = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (o >= cells) return;
    const uint32_t q = (uint32_t)(o / n_ref), r = (uint32_t)(o - (uint64_t)q * n_ref);
    const uint32_t lq = qry_len[q];
    const uint4 rl = *(const uint4 *)(ref_len + r);
    const uint32_t d[4] = {rl.x + lq, rl.y + lq, rl.z + lq, rl.w + lq};
    double dv[4], pv[4];
    uint32_t pa = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        dv[u] = d[u] == 0 ? 0.0 : 1.0;
        pv[u] = 1.0;
        pa |= 1u << (8 * u);
    }
    *(double2 *)(fill.dist + o) = make_double2(dv[0], dv[1]);
    *(double2 *)(fill.dist + o + 2) = make_double2(dv[2], dv[3]);
    *(double2 *)(fill.pval + o) = make_double2(pv[0], pv[1]);
    *(double2 *)(fill.pval + o + 2) = make_double2(pv[2], pv[3]);
    *(uint32_t *)(fill.pass + o) = pa;
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 10000;
    const uint64_t cells = (uint64_t)n * n;
    std::vector<uint32_t> len(n, 1000);
    uint32_t *d_len;
    double *di, *pv;
    uint8_t *pa;
    hipMalloc(&d_len, n * 4);
    hipMemcpy(d_len, len.data(), n * 4, hipMemcpyHostToDevice);
    hipMalloc(&di, cells * 8);
    hipMalloc(&pv, cells * 8);
    hipMalloc(&pa, cells);
    PairFill f;
    f.dist = di; f.pval = pv; f.pass = pa; f.max_dist = 1.0; f.max_pvalue = 1.0;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9;
        for (int it = 0; it < 5; it++) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, best, 17.0 * cells / best / 1e6);
    };
    run("dist_fill_kernel", [&] { launch_dist_fill(d_len, n, d_len, n, 1000, Counts{}, f, 0); });
    // no length loads (the prefill form: every list non-empty, constant cells)
    run("dist_fill_kernel_no_lengths", [&] { launch_dist_fill(nullptr, n, nullptr, n, 1000, Counts{}, f, 0); });
    run("flat_fill", [&] { hipLaunchKernelGGL(flat_fill, dim3((uint32_t)((cells / 4 + 255) / 256)), dim3(256), 0, 0, d_len, n, d_len, cells, 1000, f); });
    run("bare_17B_stores", [&] { hipLaunchKernelGGL(bare17, dim3((uint32_t)((cells / 4 + 255) / 256)), dim3(256), 0, 0, di, pv, pa, cells); });
    return 0;
}
