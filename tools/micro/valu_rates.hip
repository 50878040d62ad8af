// tools/micro/valu_rates.hip — issue cost of the integer ops MurmurHash3 lowers to on gfx950
// (v_mul_lo_u32, v_mad_u64_u32, v_lshl_add_u64) against v_add_u32.  8 independent chains per
// lane, 256-thread blocks, 8 blocks per CU; prints ns per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed)
{
    uint32_t a[8];
    uint64_t b[8];
#pragma unroll
    for (int c = 0; c < 8; c++) { a[c] = seed + threadIdx.x + c; b[c] = a[c] * 0x9E3779B97F4A7C15ULL; }
    for (int i = 0; i < kIters; i++) {
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(a[(c + 1) & 7]));
            if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(a[(c + 1) & 7]));
            if (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(b[c]) : "v"(a[c]), "v"(a[(c + 1) & 7]) : "vcc");
            if (OP == 3) asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(b[c]));
            if (OP == 4) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(a[(c + 1) & 7]));
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += a[c] + b[c];
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

int main()
{
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus * 8;
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mad_u64_u32", "v_lshl_add_u64", "v_mul_hi_u32"};
    void (*fns[])(uint32_t *, uint32_t) = {k<0>, k<1>, k<2>, k<3>, k<4>};
    for (int op = 0; op < 5; op++) {
        hipLaunchKernelGGL(fns[op], dim3(blocks), dim3(256), 0, 0, out, 1u);   // warm
        hipEventRecord(e0);
        hipLaunchKernelGGL(fns[op], dim3(blocks), dim3(256), 0, 0, out, 2u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        // wave-instructions per SIMD: blocks*4 waves * iters*8 / (cus*4 SIMDs)
        const double wi_per_simd = (double)blocks * 4 * kIters * 8 / (cus * 4.0);
        printf("{\"op\": \"%s\", \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f, \"cycles_at_2.4GHz\": %.2f}\n",
               names[op], ms, ms * 1e6 / wi_per_simd, ms * 1e6 / wi_per_simd * 2.4);
    }
    hipFree(out);
    return 0;
}
