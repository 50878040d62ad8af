// tools/micro/sketch_phases.hip — where a sketch tile's time goes, C2 shape (10,000 tiles of
// 2,000 random ACGT bases, k = 21, s = 1,000, canonical).  Builds the library's tile kernel
// with FPM_SKETCH_PHASES (thread 0 stamps s_memtime at each phase boundary) and prints the
// mean cycles spent per phase, plus the kernel time.
#define FPM_SKETCH_PHASES 1
#ifndef K_ARG
#define K_ARG 21
#endif
#ifndef P_ARG
#define P_ARG 2048        // 4096: C5's long-record chunks (with a sampled bound, -DTHR_FRAC)
#endif
#ifndef THR_FRAC
#define THR_FRAC 0.0      // > 0: tiles keep hashes below this fraction of the hash range
#endif
#include "../../fp-mash_amd/csrc/sketch.hip"

#include <random>
#include <stdio.h>
#include <vector>

using namespace fpm;

int main(int argc, char **argv)
{
    const int k = 21;
    const int n = argc > 1 ? atoi(argv[1]) : (P_ARG == 2048 ? 10000 : 12000);
    const int L = P_ARG == 2048 ? 2000 : P_ARG + k - 1, s = P_ARG == 2048 ? 1000 : 10000;
    std::vector<uint8_t> seq((size_t)n * (L + 1) + 64, 0);
    std::vector<TileDesc> tiles(n);
    std::mt19937_64 rng(1);
    const char *acgt = "ACGT";
    for (int r = 0; r < n; r++) {
        for (int i = 0; i < L; i++) seq[(size_t)r * (L + 1) + i] = acgt[rng() & 3];
        tiles[r] = TileDesc{(uint64_t)r * (L + 1), (uint32_t)L, (uint32_t)r, THR_FRAC > 0 ? 1u : 0u, 0};
    }
    SketchKParams p{};
    p.k = k; p.s = s; p.seed = 42; p.use64 = 1; p.canonical = 1; p.preserve_case = 0; p.compl_acgt = 1;
    for (int c = 0; c < 256; c++) { p.alphabet[c] = 0; p.complement[c] = 'N'; }
    p.alphabet['A'] = p.alphabet['C'] = p.alphabet['G'] = p.alphabet['T'] = 1;
    p.complement['A'] = 'T'; p.complement['T'] = 'A'; p.complement['C'] = 'G'; p.complement['G'] = 'C';
    uint8_t *d_seq; TileDesc *d_t; uint64_t *d_out, *d_ph, *d_thr; uint32_t *d_cnt;
    const uint64_t thr = (uint64_t)(THR_FRAC * 18446744073709551615.0);
    hipMalloc(&d_thr, 8);
    hipMemcpy(d_thr, &thr, 8, hipMemcpyHostToDevice);
    hipMalloc(&d_seq, seq.size());
    hipMalloc(&d_t, n * sizeof(TileDesc));
    hipMalloc(&d_out, (size_t)n * s * 8);
    hipMalloc(&d_cnt, n * 4);
    hipMalloc(&d_ph, (size_t)n * 8 * 8);
    hipMemcpy(d_seq, seq.data(), seq.size(), hipMemcpyHostToDevice);
    hipMemcpy(d_t, tiles.data(), n * sizeof(TileDesc), hipMemcpyHostToDevice);
    hipMemcpyToSymbol(HIP_SYMBOL(g_phase), &d_ph, sizeof(d_ph));
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int it = 0; it < 6; it++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((sketch_tiles_kernel<P_ARG, K_ARG>), dim3(n), dim3(256), 0, 0, d_seq, d_t, p,
                           (const uint64_t *)d_thr, d_out, d_cnt, (TileDesc *)nullptr, (uint32_t *)nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (it && ms < best) best = ms;
    }
    std::vector<uint64_t> ph((size_t)n * 8);
    hipMemcpy(ph.data(), d_ph, ph.size() * 8, hipMemcpyDeviceToHost);
    const char *names[7] = {"stage", "hash", "count", "scan", "scatter", "sort", "distinct+write"};
    double sum[7] = {0}, tot = 0;
    for (int t = 0; t < n; t++) {
        for (int i = 0; i < 7; i++) sum[i] += (double)(ph[t * 8 + i + 1] - ph[t * 8 + i]);
        tot += (double)(ph[t * 8 + 7] - ph[t * 8]);
    }
    printf("{\"kernel_ms\": %.4f, \"tiles\": %d, \"mean_wg_cycles\": %.0f, \"phases\": {", best, n, tot / n);
    for (int i = 0; i < 7; i++) printf("%s\"%s\": %.0f", i ? ", " : "", names[i], sum[i] / n);
    printf("}}\n");
    return 0;
}
