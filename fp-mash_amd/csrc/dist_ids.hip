// dist_ids.hip — dense value ids of a sketch set (EXPERIMENT, FPM_RANK_IDS=1): every distinct
// hash of the set gets its rank among the set's distinct hashes, written at its cell, so the
// candidate compare (rank_ids_kernel) can walk u32 rows.  Built here by a library radix sort
// of (value, cell) pairs, a head-flag scan and a scatter: the measurement of what the u32 walk
// saves, before a build folded into the bucket index is worth writing.
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

#include <hipcub/hipcub.hpp>

namespace fpm {

__global__ __launch_bounds__(256) void ids_keys_kernel(const uint64_t *__restrict__ rows,
                                                      const uint32_t *__restrict__ len,
                                                      uint64_t stride, uint64_t E,
                                                      uint64_t *__restrict__ keys,
                                                      uint32_t *__restrict__ cells)
{
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const uint64_t r = e / stride, i = e - r * stride;
    keys[e] = i < len[r] ? rows[e] : ~0ULL;
    cells[e] = (uint32_t)e;
}

__global__ __launch_bounds__(256) void ids_heads_kernel(const uint64_t *__restrict__ keys,
                                                       uint64_t E, uint32_t *__restrict__ head)
{
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    head[e] = (e > 0 && keys[e] != keys[e - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void ids_scatter_kernel(const uint32_t *__restrict__ rank,
                                                         const uint32_t *__restrict__ cells,
                                                         uint64_t E, uint32_t *__restrict__ ids)
{
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    ids[cells[e]] = rank[e];
}

// scratch: keys 2 x 8E, cells 2 x 4E, head / rank 2 x 4E, + the sort's temporary storage
size_t dense_ids_scratch(uint64_t E)
{
    size_t sort_tmp = 0, scan_tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (const uint64_t *)nullptr,
                                             (uint64_t *)nullptr, (const uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (int)E);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, scan_tmp, (const uint32_t *)nullptr,
                                           (uint32_t *)nullptr, (int)E);
    return E * (16 + 8 + 8) + std::max(sort_tmp, scan_tmp) + 4096;
}

hipError_t launch_dense_ids(const uint64_t *d_rows, const uint32_t *d_len, uint64_t stride,
                            uint32_t n_rows, void *scratch, size_t scratch_bytes, uint32_t *d_ids,
                            hipStream_t st)
{
    const uint64_t E = (uint64_t)n_rows * stride;
    if (!E) return hipSuccess;
    if (E >= (1ULL << 31)) return hipErrorInvalidValue;
    char *p = static_cast<char *>(scratch);
    uint64_t *k0 = (uint64_t *)p, *k1 = k0 + E;
    uint32_t *c0 = (uint32_t *)(k1 + E), *c1 = c0 + E, *h = c1 + E, *rk = h + E;
    void *tmp = rk + E;
    size_t tmp_bytes = scratch_bytes - (size_t)((char *)tmp - p);
    const uint32_t g = (uint32_t)((E + 255) / 256);
    hipLaunchKernelGGL(ids_keys_kernel, dim3(g), dim3(256), 0, st, d_rows, d_len, stride, E, k0, c0);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, c0, c1, (int)E, 0,
                                                      64, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ids_heads_kernel, dim3(g), dim3(256), 0, st, k1, E, h);
    tmp_bytes = scratch_bytes - (size_t)((char *)tmp - p);
    e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, h, rk, (int)E, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ids_scatter_kernel, dim3(g), dim3(256), 0, st, rk, c1, E, d_ids);
    return hipGetLastError();
}

}  // namespace fpm
