// dist_index.hip — sparse all-pairs dist for gfx950: inverted index + row bitmaps.
//
// compareSketches (CommandDistance.cpp:365-430) walks <= S steps for EVERY pair.
// Observation used here: if two lists share no value, the literal walk never hits
// the equal branch, so it ends with common = 0 and denom = min(S, lenA + lenB) —
// for sorted sketches and for the unsorted -fp lists alike.  So only pairs that
// share at least one hash ("candidates") need the walk.  The candidates come from
// an inverted index over the reference lists:
//   1. insert every ref hash into an open-addressing table (key -> slot), count
//      postings per slot, exclusive-scan, scatter ref ids into posting lists;
//   2. one workgroup per query row probes its hashes and ORs the ref ids of every
//      posting into a row bitmap held in LDS (no global atomics), then writes the
//      row bitmap and appends the row's candidate pairs;
//   3. the literal walk (dist.hip) runs on the candidates only; dist_finalize
//      writes (0, min(S, la+lb)) for every other pair.
// Work is O(N*S + sum_v n_v^2 + candidates*S) instead of O(pairs*S).  When the
// posting events exceed a fraction of pairs*S (highly similar collections) the
// host falls back to walking every pair.
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

namespace fpm {

constexpr uint64_t kEmpty = ~0ULL;

__device__ __forceinline__ uint32_t slot_hash(uint64_t key, int log2t)
{
    return (uint32_t)((key * 0x9E3779B97F4A7C15ULL) >> (64 - log2t));
}

__device__ __forceinline__ uint64_t load_key(const void *lists, uint32_t hash_bytes, uint64_t idx)
{
    return hash_bytes == 8 ? reinterpret_cast<const uint64_t *>(lists)[idx]
                           : (uint64_t) reinterpret_cast<const uint32_t *>(lists)[idx];
}

// key ~0 (only possible with 8-byte hashes) lives in the extra slot T
__device__ __forceinline__ uint32_t idx_insert(uint64_t *keys, uint64_t key, int log2t)
{
    const uint32_t T = 1u << log2t;
    if (key == kEmpty) return T;
    uint32_t s = slot_hash(key, log2t);
    for (;;) {
        unsigned long long old = atomicCAS((unsigned long long *)&keys[s], (unsigned long long)kEmpty,
                                           (unsigned long long)key);
        if (old == kEmpty || old == key) return s;
        s = (s + 1) & (T - 1);
    }
}

__device__ __forceinline__ int64_t idx_find(const uint64_t *keys, uint64_t key, int log2t)
{
    const uint32_t T = 1u << log2t;
    if (key == kEmpty) return T;
    uint32_t s = slot_hash(key, log2t);
    for (;;) {
        uint64_t k = keys[s];
        if (k == key) return s;
        if (k == kEmpty) return -1;
        s = (s + 1) & (T - 1);
    }
}

__global__ __launch_bounds__(256) void idx_insert_kernel(
    const void *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t stride,
    uint32_t n_ref, uint32_t hash_bytes, uint64_t *__restrict__ keys, uint32_t *__restrict__ cnt,
    uint32_t *__restrict__ slot_of, int log2t, uint32_t *__restrict__ unsorted)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool uns = false;
    if (e < (uint64_t)n_ref * stride) {
        const uint32_t r = (uint32_t)(e / stride), i = (uint32_t)(e % stride);
        const uint32_t la = ref_len[r];
        if (i < la) {
            const uint64_t key = load_key(ref, hash_bytes, e);
            const uint32_t s = idx_insert(keys, key, log2t);
            atomicAdd(&cnt[s], 1u);
            slot_of[e] = s;
            uns = i + 1 < la && !(key < load_key(ref, hash_bytes, e + 1));
        }
    }
    if (__any(uns) && (threadIdx.x & 63) == 0) atomicOr(unsorted, 1u);
}

__global__ __launch_bounds__(256) void idx_scatter_kernel(
    const uint32_t *__restrict__ ref_len, uint64_t stride, uint32_t n_ref,
    const uint32_t *__restrict__ slot_of, uint32_t *__restrict__ cursor,
    uint32_t *__restrict__ postings)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (uint64_t)n_ref * stride) return;
    const uint32_t r = (uint32_t)(e / stride), i = (uint32_t)(e % stride);
    if (i >= ref_len[r]) return;
    const uint32_t p = atomicAdd(&cursor[slot_of[e]], 1u);
    postings[p] = r;
}

// ---- exclusive scan of u32 counts (n <= 2^31), three launches ----
constexpr int kScanBlock = 1024;   // elements per block (256 threads x 4)

__global__ __launch_bounds__(256) void scan_local_kernel(const uint32_t *__restrict__ in,
                                                        uint32_t *__restrict__ out, uint64_t n,
                                                        uint32_t *__restrict__ block_sums)
{
    __shared__ uint32_t wsum[4];
    const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
    uint32_t v[4], t = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) { v[k] = (base + k < n) ? in[base + k] : 0u; t += v[k]; }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t wpre = 0;
    for (int w = 0; w < wave; w++) wpre += wsum[w];
    uint32_t run = wpre + x - t;
#pragma unroll
    for (int k = 0; k < 4; k++) { if (base + k < n) out[base + k] = run; run += v[k]; }
    if (threadIdx.x == 255) block_sums[blockIdx.x] = wpre + x;
}

__global__ __launch_bounds__(256) void scan_sums_kernel(uint32_t *__restrict__ sums, uint32_t nb,
                                                       uint32_t *__restrict__ total)
{
    // single workgroup, sequential chunks of 256
    __shared__ uint32_t carry;
    __shared__ uint32_t wsum[4];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < nb; c0 += 256) {
        uint32_t i = c0 + threadIdx.x;
        uint32_t v = i < nb ? sums[i] : 0u;
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint32_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t wpre = 0;
        for (int w = 0; w < wave; w++) wpre += wsum[w];
        if (i < nb) sums[i] = carry + wpre + x - v;
        __syncthreads();
        if (threadIdx.x == 255) carry += wpre + x;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(256) void scan_add_kernel(uint32_t *__restrict__ out, uint64_t n,
                                                      const uint32_t *__restrict__ sums,
                                                      uint32_t *__restrict__ out2)
{
    const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + threadIdx.x * 4;
    const uint32_t add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (base + k < n) {
            uint32_t v = out[base + k] + add;
            out[base + k] = v;
            if (out2) out2[base + k] = v;
        }
}

// ---- probing ----
// Posting events = sum over query hashes of their posting-list length (= the work the
// row probe will do).  Also flags unsorted / duplicate-carrying query rows.  One
// atomic per workgroup into one of 64 spread counters (a single counter serialises).
__global__ __launch_bounds__(256) void probe_count_kernel(
    const void *__restrict__ qry, const uint32_t *__restrict__ qry_len, uint64_t stride,
    uint32_t n_qry, uint32_t hash_bytes, const uint64_t *__restrict__ keys,
    const uint32_t *__restrict__ off, int log2t, unsigned long long *__restrict__ events,
    uint32_t *__restrict__ unsorted)
{
    __shared__ unsigned long long wsum[4];
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t ev = 0;
    uint32_t uns = 0;
    if (e < (uint64_t)n_qry * stride) {
        const uint32_t q = (uint32_t)(e / stride), j = (uint32_t)(e % stride);
        const uint32_t lq = qry_len[q];
        if (j < lq) {
            const uint64_t key = load_key(qry, hash_bytes, e);
            int64_t s = idx_find(keys, key, log2t);
            if (s >= 0) ev = off[s + 1] - off[s];
            if (j + 1 < lq && !(key < load_key(qry, hash_bytes, e + 1))) uns = 1;
        }
    }
    for (int d = 32; d > 0; d >>= 1) ev += __shfl_down(ev, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = ev;
    if (__any(uns) && (threadIdx.x & 63) == 0) atomicOr(unsorted, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (t) atomicAdd(&events[1 + (blockIdx.x & 63)], t);
    }
}

__global__ void sum64_kernel(unsigned long long *events)
{
    // events[1..64] -> events[0]
    unsigned long long v = events[1 + threadIdx.x];
    for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
    if (threadIdx.x == 0) events[0] = v;
}

// One workgroup per (query row, ref chunk): LDS bitmap of the chunk's refs.
__global__ __launch_bounds__(256) void probe_rows_kernel(
    const void *__restrict__ qry, const uint32_t *__restrict__ qry_len, uint64_t stride,
    uint32_t n_qry, uint32_t n_ref, uint32_t hash_bytes, const uint64_t *__restrict__ keys,
    const uint32_t *__restrict__ off, const uint32_t *__restrict__ postings, int log2t,
    uint32_t chunk_refs, const uint32_t *__restrict__ ref_len, uint32_t S,
    uint32_t *__restrict__ numer, uint32_t *__restrict__ denom, uint64_t *__restrict__ cand,
    unsigned long long *__restrict__ n_cand, uint64_t *__restrict__ row_seg)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t rowbits[];
    __shared__ uint32_t wsum[4];
    __shared__ unsigned long long row_base;
    const uint32_t q = blockIdx.x;
    const uint32_t r0 = blockIdx.y * chunk_refs;
    const uint32_t r1 = min(n_ref, r0 + chunk_refs);
    const uint32_t nwords = (r1 - r0 + 31) / 32;
    for (uint32_t w = threadIdx.x; w < nwords; w += 256) rowbits[w] = 0;
    __syncthreads();
    const uint32_t lq = qry_len[q];
    const uint64_t rowoff = (uint64_t)q * stride;
    // every pair of the row starts as "no shared value": (0, min(S, la+lb))
    for (uint32_t r = r0 + threadIdx.x; r < r1; r += 256) {
        uint64_t o = (uint64_t)q * n_ref + r;
        uint64_t d = (uint64_t)ref_len[r] + lq;
        numer[o] = 0;
        denom[o] = d < S ? (uint32_t)d : S;
    }
    for (uint32_t j = threadIdx.x; j < lq; j += 256) {
        int64_t s = idx_find(keys, load_key(qry, hash_bytes, rowoff + j), log2t);
        if (s < 0) continue;
        for (uint32_t p = off[s], pe = off[s + 1]; p < pe; p++) {
            uint32_t r = postings[p];
            if (r >= r0 && r < r1) atomicOr(&rowbits[(r - r0) >> 5], 1u << ((r - r0) & 31));
        }
    }
    __syncthreads();
    // candidates of this row: popcount per word -> block scan -> append
    uint32_t mycnt = 0;
    for (uint32_t w = threadIdx.x; w < nwords; w += 256) mycnt += __popc(rowbits[w]);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = mycnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (int w = 0; w < 4; w++) { if (w < wave) wpre += wsum[w]; tot += wsum[w]; }
    if (threadIdx.x == 0) {
        row_base = tot ? atomicAdd(n_cand, (unsigned long long)tot) : 0ULL;
        // (offset << 24 | count) of this row's candidates; one ref chunk per row here
        if (gridDim.y == 1) row_seg[q] = (row_base << 24) | (tot & 0xFFFFFF);
    }
    __syncthreads();
    uint64_t pos = row_base + wpre + x - mycnt;
    const uint64_t pair_row = (uint64_t)q * n_ref;
    for (uint32_t w = threadIdx.x; w < nwords; w += 256) {
        uint32_t b = rowbits[w];
        const uint64_t bit0 = pair_row + r0 + (uint64_t)w * 32;
        while (b) {
            int t = __builtin_ctz(b);
            b &= b - 1;
            cand[pos++] = bit0 + t;
        }
    }
}

hipError_t launch_idx_insert(const void *d_ref, const uint32_t *d_ref_len, uint64_t stride,
                             uint32_t n_ref, uint32_t hash_bytes, uint64_t *keys, uint32_t *cnt,
                             uint32_t *slot_of, int log2t, uint32_t *unsorted, hipStream_t st)
{
    uint64_t n = (uint64_t)n_ref * stride;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(idx_insert_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, d_ref,
                       d_ref_len, stride, n_ref, hash_bytes, keys, cnt, slot_of, log2t, unsorted);
    return hipGetLastError();
}

hipError_t launch_idx_scatter(const uint32_t *d_ref_len, uint64_t stride, uint32_t n_ref,
                              const uint32_t *slot_of, uint32_t *cursor, uint32_t *postings,
                              hipStream_t st)
{
    uint64_t n = (uint64_t)n_ref * stride;
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(idx_scatter_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st,
                       d_ref_len, stride, n_ref, slot_of, cursor, postings);
    return hipGetLastError();
}

uint64_t scan_scratch_words(uint64_t n) { return (n + kScanBlock - 1) / kScanBlock + 1; }

hipError_t launch_exscan(const uint32_t *in, uint32_t *out, uint32_t *out2, uint64_t n,
                         uint32_t *scratch, uint32_t *total, hipStream_t st)
{
    if (!n) return hipSuccess;
    uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
    hipLaunchKernelGGL(scan_local_kernel, dim3(nb), dim3(256), 0, st, in, out, n, scratch);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(256), 0, st, scratch, nb, total);
    hipLaunchKernelGGL(scan_add_kernel, dim3(nb), dim3(256), 0, st, out, n, scratch, out2);
    return hipGetLastError();
}

hipError_t launch_probe_count(const void *d_qry, const uint32_t *d_qry_len, uint64_t stride,
                              uint32_t n_qry, uint32_t hash_bytes, const uint64_t *keys,
                              const uint32_t *off, int log2t, unsigned long long *events,
                              uint32_t *unsorted, hipStream_t st)
{
    uint64_t n = (uint64_t)n_qry * stride;
    if (n) hipLaunchKernelGGL(probe_count_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0,
                              st, d_qry, d_qry_len, stride, n_qry, hash_bytes, keys, off, log2t,
                              events, unsorted);
    hipLaunchKernelGGL(sum64_kernel, dim3(1), dim3(64), 0, st, events);
    return hipGetLastError();
}

hipError_t launch_probe_rows(const void *d_qry, const uint32_t *d_qry_len, uint64_t stride,
                             uint32_t n_qry, uint32_t n_ref, uint32_t hash_bytes,
                             const uint64_t *keys, const uint32_t *off, const uint32_t *postings,
                             int log2t, const uint32_t *d_ref_len, uint32_t S, uint32_t *d_numer,
                             uint32_t *d_denom, uint64_t *cand, unsigned long long *n_cand,
                             uint64_t *row_seg, hipStream_t st)
{
    if (!n_qry || !n_ref) return hipSuccess;
    const uint32_t chunk = 1u << 19;   // refs per workgroup: 64 KiB of LDS bitmap
    const uint32_t nchunks = (n_ref + chunk - 1) / chunk;
    const uint32_t cref = nchunks == 1 ? n_ref : chunk;
    const size_t lds = ((cref + 31) / 32) * 4;
    hipLaunchKernelGGL(probe_rows_kernel, dim3(n_qry, nchunks), dim3(256), lds, st, d_qry, d_qry_len,
                       stride, n_qry, n_ref, hash_bytes, keys, off, postings, log2t, cref,
                       d_ref_len, S, d_numer, d_denom, cand, n_cand, row_seg);
    return hipGetLastError();
}

}  // namespace fpm
