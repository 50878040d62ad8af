// fingerprint.hip — the -fp k-finger line hash for gfx950.
//
// Replaces the per-line getHashFingerPrint call of Sketch::initFromFingerprints
// (Sketch.cpp:131, hash.cpp:45-73): Murmur over the 8*n little-endian bytes of
// the line's u64 values; -fp forces 32-bit hashes (sketchParameterSetup.cpp:78-84).
// One lane per line; lines are short (CFL k-fingers: 1-15 values), so the
// value loads of adjacent lanes fall in the same cache lines.
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

namespace fpm {

__global__ __launch_bounds__(256) void fp_hash_kernel(const uint64_t *__restrict__ vals,
                                                     const uint64_t *__restrict__ line_off,
                                                     uint64_t n_lines, uint32_t seed,
                                                     uint32_t use64, void *__restrict__ out)
{
    uint64_t line = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (line >= n_lines) return;
    const uint64_t b = line_off[line], e = line_off[line + 1];
    const uint64_t *v = vals + b;
    uint64_t h = murmur_h1_u64s([&](uint64_t i) { return v[i]; }, e - b, seed);
    if (use64) reinterpret_cast<uint64_t *>(out)[line] = h;
    else reinterpret_cast<uint32_t *>(out)[line] = (uint32_t)h;
}

hipError_t launch_fp_hash(const uint64_t *d_vals, const uint64_t *d_line_off, uint64_t n_lines,
                          uint32_t seed, uint32_t use64, void *d_out, hipStream_t st)
{
    if (n_lines == 0) return hipSuccess;
    uint64_t blocks = (n_lines + 255) / 256;
    hipLaunchKernelGGL(fp_hash_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, d_vals, d_line_off,
                       n_lines, seed, use64, d_out);
    return hipGetLastError();
}

}  // namespace fpm
