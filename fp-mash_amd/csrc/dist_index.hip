// dist_index.hip — sparse all-pairs dist for gfx950: bucket index + row bitmaps.
//
// compareSketches (CommandDistance.cpp:365-430) walks <= S steps for EVERY pair.
// Observation used here: if two lists share no value, the literal walk never hits
// the equal branch, so it ends with common = 0 and denom = min(S, lenA + lenB) —
// for sorted sketches and for the unsorted -fp lists alike.  So only pairs that
// share at least one hash ("candidates") need the walk.  The candidates come from
// an index over the reference lists:
//   1. bucket index: every ref hash becomes one packed u32 entry (key fingerprint << rbits
//      | ref id) in a bucket array grouped by the key's bucket (its value scaled to the
//      indexed range [0, kmax]: bottom-s sketches only use the low part of the hash range),
//      with a directory dir[b] = first entry of bucket b.  Hashes are uniform (MurmurHash3),
//      so this is a two-level counting sort with no global atomics: per-tile LDS histograms
//      of the top 10 bucket bits + one exclusive scan place every entry in its partition,
//      then one workgroup per partition counting-sorts it by the next l2 bits in LDS and
//      writes its slice of the directory;
//   2. one workgroup per query row looks up the bucket of each of its hashes; each wave
//      flattens the buckets of 64 hashes into one event range and reads it coalesced,
//      ORing the ref id of every entry whose fingerprint matches into a row bitmap in LDS
//      (no global atomics), then appends the row's candidate pairs;
//   3. the rank / literal-walk kernels (dist.hip) run on the candidates only; every other
//      pair keeps the (0, min(S, la+lb)) written in step 2.
// Work is O(N*S + sum_v n_v^2 + candidates*S) instead of O(pairs*S).  When the
// posting events exceed a fraction of pairs*S (highly similar collections) the
// host falls back to walking every pair.
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

#include <algorithm>
#include <atomic>

namespace fpm {

constexpr uint32_t kParts = 1u << kIdxL1;    // level-1 partitions (top 10 key bits)
// posting events in flight per lane in the probe (4: 0.307 ms, 12 without the 8-wave cap
// 0.339 ms, against 0.298-0.301 ms at 8)
#ifndef PROBE_KU
#define PROBE_KU 8
#endif

__device__ __forceinline__ uint64_t load_key(const void *lists, uint32_t hash_bytes, uint64_t idx)
{
    return hash_bytes == 8 ? reinterpret_cast<const uint64_t *>(lists)[idx]
                           : (uint64_t) reinterpret_cast<const uint32_t *>(lists)[idx];
}

// 32-bit hashes move to the top of the word so the bucket bits are always the top bits
__device__ __forceinline__ uint64_t norm_key(uint64_t h, uint32_t hash_bytes)
{
    return hash_bytes == 8 ? h : (h << 32);
}

// Bucket of a (normalized) key: floor(K * NB / (kmax + 1)) with kmax = the largest indexed
// key (from the rows' last entries, idx_kmax_kernel), clamped to NB - 1.  Bottom-s sketches
// only hold values up to about s / (distinct k-mers) of the hash range (C2: 0.54 * 2^64), so
// plain top bits would leave half the buckets empty and double the others (8 % more posting
// events).  mult = NB * 2^64 / (kmax + 1) is computed by every kernel from the same kmax with
// the same double ops.
__device__ __forceinline__ uint64_t idx_mult(const IdxGeom &g)
{
    const double q = ldexp(1.0, 64 + (int)g.nbits) / ((double)*g.kmax + 1.0);
    return q >= 18446744073709551615.0 ? ~0ULL : (uint64_t)q;
}
__device__ __forceinline__ uint32_t bucket_of(uint64_t K, const IdxGeom &g, uint64_t mult)
{
    const uint64_t b = __umul64hi(K, mult);
    const uint64_t top = (1ULL << g.nbits) - 1;
    return (uint32_t)(b < top ? b : top);
}
// u32 entry = fingerprint << rbits | ref id, fingerprint = the top fbits of the low half of
// K * mult (for a power-of-two range: the key bits just below the bucket bits).  A fingerprint
// collision only adds a candidate pair that shares no hash; the exact candidate kernels then
// produce the same (0, min(S, la+lb)) the probe already wrote.
__device__ __forceinline__ uint32_t key_fp(uint64_t K, const IdxGeom &g, uint64_t mult)
{
    return (uint32_t)((K * mult) >> (64 - g.fbits));
}

// Tiles of g.tile (<= kIdxTile) matrix cells, 1024 threads each (16 cells per thread, 4 loads in
// flight): 611 tiles at the bench's E = 1e7, ~10 waves per SIMD.  Row of cell e = e / stride
// by a 64-bit multiply-high with magic = floor((2^64 - 1) / stride) + 1, exact for e < 2^31
// (the error term e / 2^64 stays below the 1 / stride gap to the next integer).
constexpr int kIdxThreads = 1024;
constexpr int kIdxU = 4;

__device__ __forceinline__ uint32_t row_of(uint32_t e, uint32_t stride, uint64_t magic)
{
    return stride == 1 ? e : (uint32_t)__umul64hi((uint64_t)e, magic);
}

// ---- 0. the largest normalized key among the rows' last entries (the maximum for sorted
// rows; unsorted rows may hold larger keys, which bucket_of clamps into the last bucket).
// A few workgroups (8 rows per thread in flight); each folds its maximum into acc[0] and the
// last one to finish (acc[1] counts them) zeroes the call's counters (zero[0 .. nzero), which
// may hold kmax itself), writes kmax and resets acc for the next call: no memset launch, and
// not the 14 us of one workgroup walking 10k rows.  acc[0..1] start at zero (scratch()).
constexpr int kKmaxThreads = 256;
constexpr int kKmaxU = 8;
__global__ __launch_bounds__(kKmaxThreads) void idx_kmax_kernel(
    const void *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t stride,
    uint32_t n_ref, uint32_t hash_bytes, unsigned long long *__restrict__ kmax,
    unsigned long long *__restrict__ zero, uint32_t nzero, unsigned long long *acc,
    uint32_t *__restrict__ zero32, uint32_t nzero32, unsigned long long *__restrict__ zero_x)
{
    __shared__ unsigned long long wmax[kKmaxThreads / 64];
    __shared__ uint32_t s_last;
    uint64_t mx = 0;
    const uint32_t step = gridDim.x * kKmaxThreads;
    for (uint32_t r0 = blockIdx.x * kKmaxThreads + threadIdx.x; r0 < n_ref; r0 += kKmaxU * step) {
        uint32_t l[kKmaxU];
#pragma unroll
        for (int u = 0; u < kKmaxU; u++) {
            const uint32_t r = r0 + u * step;
            l[u] = r < n_ref ? ref_len[r] : 0u;
        }
        uint64_t k[kKmaxU];
#pragma unroll
        for (int u = 0; u < kKmaxU; u++) {
            const uint32_t r = r0 + u * step;
            k[u] = l[u] ? norm_key(load_key(ref, hash_bytes, (uint64_t)r * stride + l[u] - 1), hash_bytes) : 0;
        }
#pragma unroll
        for (int u = 0; u < kKmaxU; u++) mx = max(mx, k[u]);
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint64_t)__shfl_xor((unsigned long long)mx, d, 64));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kKmaxThreads / 64; w++) mx = max(mx, (uint64_t)wmax[w]);
        atomicMax(&acc[0], (unsigned long long)mx);
        __threadfence();
        s_last = atomicAdd(&acc[1], 1ULL) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    for (uint32_t i = threadIdx.x; i < nzero; i += kKmaxThreads) zero[i] = 0;
    for (uint32_t i = threadIdx.x; i < nzero32; i += kKmaxThreads) zero32[i] = 0;
    // one more word of the caller's (the compact output's list count: no memset launch)
    if (zero_x && threadIdx.x == 0) *zero_x = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        *kmax = atomicMax(&acc[0], 0ULL);
        acc[0] = 0;
        acc[1] = 0;
    }
}

// ---- 1a. level-1 histogram: LDS counters per partition; also flags unsorted /
// duplicate-carrying rows (the next cell's key is the next lane's, lane 63 loads it)
__global__ __launch_bounds__(kIdxThreads) void idx_part_hist_kernel(
    const void *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint32_t stride,
    uint64_t magic, uint32_t n_ref, uint32_t hash_bytes, uint32_t ntiles,
    uint32_t *__restrict__ tile_hist, uint32_t *__restrict__ unsorted, IdxGeom g)
{
    __shared__ uint32_t hist[kParts];
    const uint64_t mult = idx_mult(g);
    for (uint32_t p = threadIdx.x; p < kParts; p += kIdxThreads) hist[p] = 0;
    __syncthreads();
    const uint32_t e0 = blockIdx.x * g.tile, lane = threadIdx.x & 63;
    const uint32_t n = min(n_ref * stride, e0 + g.tile);     // this tile's cells end here
    bool uns = false;
    for (uint32_t c0 = 0; c0 < g.tile; c0 += kIdxU * kIdxThreads) {
        uint64_t key[kIdxU];
        bool v[kIdxU], nx[kIdxU];
#pragma unroll
        for (int u = 0; u < kIdxU; u++) {
            const uint32_t e = e0 + c0 + u * kIdxThreads + threadIdx.x;
            const uint32_t r = row_of(e, stride, magic), i = e - r * stride;
            const uint32_t la = e < n ? ref_len[r] : 0;
            v[u] = e < n && i < la;
            nx[u] = v[u] && i + 1 < la;                 // cell e + 1 is in the same list
            key[u] = v[u] ? load_key(ref, hash_bytes, e) : 0;
        }
#pragma unroll
        for (int u = 0; u < kIdxU; u++) {
            uint64_t nk = __shfl_down((unsigned long long)key[u], 1, 64);
            if (lane == 63 && nx[u])
                nk = load_key(ref, hash_bytes, (uint64_t)e0 + c0 + u * kIdxThreads + threadIdx.x + 1);
            uns |= nx[u] && !(key[u] < nk);
            if (v[u]) atomicAdd(&hist[bucket_of(norm_key(key[u], hash_bytes), g, mult) >> g.l2], 1u);
        }
    }
    if (__any(uns) && lane == 0) atomicOr(unsorted, 1u);
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < kParts; p += kIdxThreads)
        tile_hist[(uint64_t)p * ntiles + blockIdx.x] = hist[p];
}

// ---- 1b. level-1 scatter into partitions.  One u64 per entry: the key bits below the
// partition bits that level 2 needs (l2 sub-bucket bits, then the fbits fingerprint) over
// the ref id, i.e. (sub << 32) | final u32 entry, since fbits + rbits = 32.
__device__ __forceinline__ uint64_t pack_l1(uint64_t K, uint32_t r, const IdxGeom &g, uint64_t mult)
{
    const uint32_t sub = bucket_of(K, g, mult) & ((1u << g.l2) - 1);
    return ((uint64_t)sub << 32) | ((uint64_t)key_fp(K, g, mult) << g.rbits) | r;
}

// The tile's entries are first grouped by partition in LDS (a counting sort on the hist
// pass's per-tile counts), then written out in slot order: consecutive threads write
// consecutive tent positions of one partition's run (~16 entries), instead of every lane
// storing 8 B into a different partition.  Each staged word carries its partition in the top
// bits (free: the bucket pass reads only the sub-bucket bits and the low u32).
constexpr uint32_t kPartShift = 54;
static_assert(kIdxL1 <= 64 - kPartShift, "partition id fits the staged word");
__global__ __launch_bounds__(kIdxThreads) void idx_part_scatter_kernel(
    const void *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint32_t stride,
    uint64_t magic, uint32_t n_ref, uint32_t hash_bytes, uint32_t ntiles,
    const uint32_t *__restrict__ tile_hist, const uint32_t *__restrict__ tile_off, IdxGeom g,
    uint64_t *__restrict__ tent)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t stage[];   // kIdxTile words
    __shared__ uint32_t gbase[kParts], lbase[kParts], lcur[kParts];
    __shared__ uint32_t wsum[kIdxThreads / 64];
    const uint64_t mult = idx_mult(g);
    // per-partition: global base of this tile's run, and its local base (block exscan of the
    // tile's counts)
    static_assert(kParts == kIdxThreads, "one partition per thread");
    {
        const uint32_t p = threadIdx.x;
        gbase[p] = tile_off[(uint64_t)p * ntiles + blockIdx.x];
        const uint32_t c = tile_hist[(uint64_t)p * ntiles + blockIdx.x];
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint32_t x = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t pre = 0;
        for (int w = 0; w < wave; w++) pre += wsum[w];
        lbase[p] = pre + x - c;
        lcur[p] = pre + x - c;
    }
    __syncthreads();
    const uint32_t e0 = blockIdx.x * g.tile;
    const uint32_t n = min(n_ref * stride, e0 + g.tile);     // this tile's cells end here
    for (uint32_t c0 = 0; c0 < g.tile; c0 += kIdxU * kIdxThreads) {
        uint64_t K[kIdxU];
        uint32_t rr[kIdxU];
        bool v[kIdxU];
#pragma unroll
        for (int u = 0; u < kIdxU; u++) {
            const uint32_t e = e0 + c0 + u * kIdxThreads + threadIdx.x;
            const uint32_t r = row_of(e, stride, magic), i = e - r * stride;
            v[u] = e < n && i < ref_len[min(r, n_ref - 1)];
            rr[u] = r;
            K[u] = v[u] ? norm_key(load_key(ref, hash_bytes, e), hash_bytes) : 0;
        }
#pragma unroll
        for (int u = 0; u < kIdxU; u++)
            if (v[u]) {
                const uint32_t part = bucket_of(K[u], g, mult) >> g.l2;
                const uint32_t pos = atomicAdd(&lcur[part], 1u);
                stage[pos] = ((uint64_t)part << kPartShift) | pack_l1(K[u], rr[u], g, mult);
            }
    }
    __syncthreads();
    const uint32_t total = lbase[kParts - 1] + (lcur[kParts - 1] - lbase[kParts - 1]);
    for (uint32_t i = threadIdx.x; i < total; i += kIdxThreads) {
        const uint64_t w = stage[i];
        const uint32_t part = (uint32_t)(w >> kPartShift);
        tent[gbase[part] + (i - lbase[part])] = w;
    }
}

// ---- 1b'. one-pass level 1 (g.cap != 0): the tile counts its partitions itself (LDS
// histogram), takes its run of each partition by one global atomic on part_fill[p] (tiles of
// a partition land in completion order: the level-2 pass sorts inside the partition anyway),
// and writes the runs into the partition's slot [p * cap, (p + 1) * cap) of tent.  Hash keys
// are uniform, so cap = mean + 6 sigma + 64 holds every partition; a run past it sets
// *overflow (the caller rebuilds with the exact two-pass form).  No histogram pass over the
// keys and no scan launches.  Also flags unsorted rows (as idx_part_hist_kernel does).
__global__ __launch_bounds__(kIdxThreads) void idx_part_scatter1_kernel(
    const void *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint32_t stride,
    uint64_t magic, uint32_t n_ref, uint32_t hash_bytes, IdxGeom g,
    uint32_t *__restrict__ part_fill, uint64_t *__restrict__ tent, uint32_t *__restrict__ unsorted,
    uint32_t *__restrict__ overflow)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t stage[];   // kIdxTile words
    __shared__ uint32_t gbase[kParts], lbase[kParts], lcur[kParts];
    __shared__ uint32_t wsum[kIdxThreads / 64];
    static_assert(kParts == kIdxThreads, "one partition per thread");
    const uint64_t mult = idx_mult(g);
    lcur[threadIdx.x] = 0;
    const uint32_t e0 = blockIdx.x * g.tile, lane = threadIdx.x & 63;
    const uint32_t n = min(n_ref * stride, e0 + g.tile);     // this tile's cells end here
    const uint32_t nu = g.tile / kIdxThreads;                // cells per thread (<= kPer)
    // the tile's keys stay in registers across both passes: every load of the tile issued at
    // once (cell e0 + u * 1024 + tid: each load coalesced), the length reads beside them (a
    // key past its row's length is loaded and dropped), and lane 63 loads the next cell for the
    // sortedness test gets the next cell's key from the next wave's lane 0 through the LDS.
    // (Was 4 loads in flight per thread and the keys read again for the scatter: two dependent
    // load rounds per 4 cells.)
    constexpr int kPer = kIdxTile / kIdxThreads;
    constexpr int kW = kIdxThreads / 64;
    __shared__ uint64_t first[kPer + 1][kW];                  // lane 0's key of each (u, wave)
    uint64_t key[kPer];
    uint32_t la[kPer];
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const uint32_t e = e0 + u * kIdxThreads + threadIdx.x;
        const bool in = (uint32_t)u < nu && e < n;
        la[u] = in ? ref_len[min(row_of(e, stride, magic), n_ref - 1)] : 0u;
        key[u] = in ? load_key(ref, hash_bytes, e) : 0;
    }
    const uint32_t wave_id = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int u = 0; u < kPer; u++) first[u][wave_id] = key[u];
    }
    // the cell after the tile (the last wave's lane 63 of the last u): loaded once
    if (threadIdx.x == 0) {
        const uint32_t e = e0 + nu * kIdxThreads;
        first[nu][0] = e < n_ref * stride ? load_key(ref, hash_bytes, e) : 0;
    }
    __syncthreads();                                          // lcur cleared, first[] written
    bool uns = false;
    uint32_t vbits = 0;                                       // bit u: cell u is a list entry
    // pass 1: the tile's partition counts (and the sortedness flags)
#pragma unroll
    for (int u = 0; u < kPer; u++) {
        const uint32_t e = e0 + u * kIdxThreads + threadIdx.x;
        const uint32_t r = row_of(e, stride, magic), i = e - r * stride;
        const bool v = (uint32_t)u < nu && e < n && i < la[u];
        const bool nx = v && i + 1 < la[u];
        uint64_t nk = __shfl_down((unsigned long long)key[u], 1, 64);
        if (lane == 63) nk = wave_id + 1 < kW ? first[u][wave_id + 1] : first[u + 1][0];
        uns |= nx && !(key[u] < nk);
        if (v) {
            vbits |= 1u << u;
            atomicAdd(&lcur[bucket_of(norm_key(key[u], hash_bytes), g, mult) >> g.l2], 1u);
        }
    }
    if (__any(uns) && lane == 0) atomicOr(unsorted, 1u);
    __syncthreads();
    {
        // this tile's run of partition p: local base (block exscan), global base (one atomic)
        const uint32_t p = threadIdx.x, c = lcur[p];
        const int wave = threadIdx.x >> 6;
        uint32_t x = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(x, d, 64); if ((int)lane >= d) x += y; }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t pre = 0;
        for (int w = 0; w < wave; w++) pre += wsum[w];
        lbase[p] = pre + x - c;
        lcur[p] = pre + x - c;
        gbase[p] = c ? atomicAdd(&part_fill[p], c) : 0u;
    }
    __syncthreads();
    // pass 2: the registers' keys grouped by partition in LDS
#pragma unroll
    for (int u = 0; u < kPer; u++)
        if (vbits >> u & 1u) {
            const uint32_t e = e0 + u * kIdxThreads + threadIdx.x;
            const uint64_t K = norm_key(key[u], hash_bytes);
            const uint32_t part = bucket_of(K, g, mult) >> g.l2;
            const uint32_t pos = atomicAdd(&lcur[part], 1u);
            stage[pos] = ((uint64_t)part << kPartShift) | pack_l1(K, row_of(e, stride, magic), g, mult);
        }
    __syncthreads();
    const uint32_t total = lcur[kParts - 1];
    bool over = false;
    for (uint32_t i = threadIdx.x; i < total; i += kIdxThreads) {
        const uint64_t w = stage[i];
        const uint32_t part = (uint32_t)(w >> kPartShift);
        const uint32_t at = gbase[part] + (i - lbase[part]);    // within the partition's slot
        if (at < g.cap) tent[(uint64_t)part * g.cap + at] = w;
        else over = true;
    }
    if (__any(over) && lane == 0) atomicOr(overflow, 1u);
}

// ---- 1c. level 2: LDS counting sort of each partition by the next l2 bits.
// A partition of up to 16k entries (C2: ~9.8k of 1e7 / 1024) is read once into registers
// (16 per thread), counted, scattered into an LDS copy of its entries and written out
// coalesced.  A larger one is read twice (count, then scatter through the LDS copy).  At
// l2 > 13 (C4: 16,384 sub-buckets of ~3 entries, partitions of ~49k) the sub-bucket range is
// split over 2^lsplit workgroups on one XCD (blockIdx % 8 alike: the slice is fetched from
// HBM about once, then from that XCD's L2): each counts its part of the sub-buckets (32 KB
// of counters) and the entries below it, reads the slice again and scatters its range's
// entries through the LDS, so every entry is written coalesced.  A range past `cap` scatters
// straight to `entries` in 4-B pieces (the round-4 form for C4: tent read twice, entries
// written ~6.5x their bytes: 0.64 ms).
constexpr int kBucketThreads = 1024;
static_assert(kBucketThreads == (int)kParts, "one-pass build: one partition fill per thread");
static_assert(kParts % 8 == 0, "split partitions map to one XCD");
constexpr int kBucketPer = 16;                   // entries per thread in registers
__global__ __launch_bounds__(kBucketThreads) void idx_bucket_kernel(
    const uint64_t *__restrict__ tent_all, uint32_t ntiles,
    const uint32_t *__restrict__ tile_off, IdxGeom g, uint32_t cap, uint32_t *__restrict__ dir,
    uint32_t *__restrict__ entries_all, unsigned long long *__restrict__ sqsum,
    const uint32_t *__restrict__ part_fill, uint32_t lsplit)
{
    extern __shared__ uint32_t sh[];             // the range's counters, then cursors; then cap entries
    __shared__ uint32_t wsum[kBucketThreads / 64];
    __shared__ unsigned long long wsq[kBucketThreads / 64];
    __shared__ uint32_t s_below;
    // blockIdx = ((p >> 3) << lsplit | j) << 3 | (p & 7): workgroup j of partition p
    const uint32_t ns = 1u << lsplit;
    const uint32_t p = ((blockIdx.x >> 3) >> lsplit) * 8 + (blockIdx.x & 7);
    const uint32_t j = (blockIdx.x >> 3) & (ns - 1);
    // this partition's entries are tent[s0, s1) and go to entries[s0, s1) (exact build), or
    // (one-pass build) tent[p * g.cap, + fill) going to entries from the sum of the fills of
    // the partitions before it (one fill per thread, block-reduced)
    uint32_t s0, s1;
    const uint64_t *tent = tent_all;
    uint32_t *entries = entries_all;
    if (threadIdx.x == 0) s_below = 0;
    if (part_fill) {
        const uint32_t f = min(part_fill[threadIdx.x], g.cap);
        uint32_t below = threadIdx.x < p ? f : 0u;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) below += __shfl_xor(below, d, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = below;
        __syncthreads();
        uint32_t o = 0;
        for (int w = 0; w < kBucketThreads / 64; w++) o += wsum[w];
        __syncthreads();
        const uint32_t mine = min(part_fill[p], g.cap);
        // the buffers are addressed from s0 on: shift them so tent[s0] is the slot's first
        tent = tent_all + (uint64_t)p * g.cap - o;
        s0 = o;
        s1 = o + mine;
    } else {
        s0 = tile_off[(uint64_t)p * ntiles];
        s1 = tile_off[(uint64_t)(p + 1) * ntiles];   // [kParts * ntiles] = total
    }
    const uint32_t sbmask = (1u << g.l2) - 1;
    const uint32_t nsb = 1u << (g.l2 - lsplit), lo = j * nsb;   // sub-buckets [lo, lo + nsb)
    uint32_t *const out = sh + nsb;
    const bool in_reg = ns == 1 && s1 - s0 <= min(cap, (uint32_t)(kBucketThreads * kBucketPer));
    for (uint32_t b = threadIdx.x; b < nsb; b += kBucketThreads) sh[b] = 0;
    __syncthreads();
    uint64_t K[kBucketPer];
    if (in_reg) {
#pragma unroll
        for (int u = 0; u < kBucketPer; u++) {
            const uint32_t e = s0 + threadIdx.x + u * kBucketThreads;
            K[u] = e < s1 ? tent[e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kBucketPer; u++)
            if (s0 + threadIdx.x + u * kBucketThreads < s1)
                atomicAdd(&sh[(uint32_t)(K[u] >> 32) & sbmask], 1u);
    } else {
        // 4 independent loads in flight per thread; entries of the sub-buckets below the
        // range are only counted (they sit before it in `entries`)
        constexpr uint32_t kU = 4;
        uint32_t below = 0;
        for (uint32_t e0 = s0 + threadIdx.x; e0 < s1; e0 += kU * kBucketThreads) {
            uint64_t Kg[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t e = e0 + u * kBucketThreads;
                Kg[u] = e < s1 ? tent[e] : 0;
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++)
                if (e0 + u * kBucketThreads < s1) {
                    const uint32_t sub = (uint32_t)(Kg[u] >> 32) & sbmask, d = sub - lo;
                    if (d < nsb) atomicAdd(&sh[d], 1u);
                    else below += sub < lo ? 1u : 0u;
                }
        }
        if (lsplit) {
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) below += __shfl_xor(below, d, 64);
            if ((threadIdx.x & 63) == 0 && below) atomicAdd(&s_below, below);
        }
    }
    __syncthreads();
    // exclusive scan of the nsb counters: per-thread run of `per`, then a block scan
    const uint32_t per = (nsb + kBucketThreads - 1) / kBucketThreads;
    const uint32_t b0 = threadIdx.x * per;
    uint32_t run = 0;
    for (uint32_t b = b0; b < b0 + per && b < nsb; b++) run += sh[b];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t acc = x - run, tot = 0;
    for (int w = 0; w < kBucketThreads / 64; w++) {
        acc += w < wave ? wsum[w] : 0u;
        tot += wsum[w];
    }
    const uint32_t base = s0 + s_below;          // the range's first entry
    unsigned long long sq = 0;
    for (uint32_t b = b0; b < b0 + per && b < nsb; b++) {
        const uint32_t c = sh[b];
        sh[b] = acc;
        dir[((uint64_t)p << g.l2) + lo + b] = base + acc;
        acc += c;
        sq += (unsigned long long)c * c;
    }
    // a set probed against itself does sum_b |b|^2 posting events: no separate count pass.
    // One atomic per workgroup into one of 64 spread counters (sqsum[1..64], summed by
    // sum64_kernel): 8192 per-wave atomics on one address serialised into a ~0.1 ms tail.
    if (sqsum) {
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) sq += __shfl_down(sq, d, 64);
        if (lane == 0) wsq[wave] = sq;
    }
    if (p == kParts - 1 && j == ns - 1 && threadIdx.x == 0) dir[(uint64_t)kParts << g.l2] = s1;
    __syncthreads();
    if (sqsum && threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBucketThreads / 64; w++) t += wsq[w];
        if (t) atomicAdd(&sqsum[1 + ((p * ns + j) & 63)], t);
    }
    if (in_reg) {
#pragma unroll
        for (int u = 0; u < kBucketPer; u++)
            if (s0 + threadIdx.x + u * kBucketThreads < s1) {
                const uint32_t pos = atomicAdd(&sh[(uint32_t)(K[u] >> 32) & sbmask], 1u);
                out[pos] = (uint32_t)K[u];
            }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < s1 - s0; i += kBucketThreads) entries[s0 + i] = out[i];
        return;
    }
    // the range through LDS when it fits (tot is block-uniform), else straight to `entries`
    const bool lds = tot <= cap;
    constexpr uint32_t kU = 4;
    for (uint32_t e0 = s0 + threadIdx.x; e0 < s1; e0 += kU * kBucketThreads) {
        uint64_t Kg[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t e = e0 + u * kBucketThreads;
            Kg[u] = e < s1 ? tent[e] : 0;
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++)
            if (e0 + u * kBucketThreads < s1) {
                const uint32_t d = ((uint32_t)(Kg[u] >> 32) & sbmask) - lo;
                if (d < nsb) {
                    const uint32_t pos = atomicAdd(&sh[d], 1u);
                    if (lds) out[pos] = (uint32_t)Kg[u];
                    else entries[base + pos] = (uint32_t)Kg[u];
                }
            }
    }
    if (!lds) return;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < tot; i += kBucketThreads) entries[base + i] = out[i];
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
// Posting events = sum over query hashes of their bucket sizes (an upper bound of the
// matching entries, and the work the row probe does).  Also flags unsorted /
// duplicate-carrying query rows.  One atomic per workgroup into one of 64 spread
// counters (a single counter serialises).
// kPC consecutive hashes per thread, their key loads and then their directory reads issued
// together (one hash per thread waited out three dependent global loads in a row)
constexpr uint32_t kPC = 4;
__global__ __launch_bounds__(256) void probe_count_kernel(
    const void *__restrict__ qry, const uint32_t *__restrict__ qry_len, uint64_t stride,
    uint32_t n_qry, uint32_t hash_bytes, IdxGeom g, const uint32_t *__restrict__ dir,
    unsigned long long *__restrict__ events, uint32_t *__restrict__ unsorted)
{
    __shared__ unsigned long long wsum[4];
    const uint64_t n = (uint64_t)n_qry * stride;
    const uint64_t e0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kPC;
    uint64_t ev = 0;
    uint32_t uns = 0;
    if (e0 < n) {
        uint32_t q = (uint32_t)(e0 / stride), j = (uint32_t)(e0 - (uint64_t)q * stride);
        uint64_t key[kPC + 1];
        uint32_t jj[kPC], lq[kPC];
        bool ok[kPC + 1];
#pragma unroll
        for (uint32_t u = 0; u <= kPC; u++) {
            const uint32_t l = q < n_qry ? qry_len[q] : 0u;
            ok[u] = j < l;
            key[u] = ok[u] ? load_key(qry, hash_bytes, (uint64_t)q * stride + j) : 0;
            if (u < kPC) { jj[u] = j; lq[u] = l; }
            if (++j == stride) { j = 0; q++; }
        }
        uint32_t d0[kPC], d1[kPC];
#pragma unroll
        for (uint32_t u = 0; u < kPC; u++) {
            const uint64_t b = bucket_of(norm_key(key[u], hash_bytes), g, idx_mult(g));
            d0[u] = ok[u] ? dir[b] : 0u;
            d1[u] = ok[u] ? dir[b + 1] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kPC; u++) {
            ev += d1[u] - d0[u];
            // the next value of the same row (jj + 1 < lq: not past the row's list)
            if (ok[u] && jj[u] + 1 < lq[u] && !(key[u] < key[u + 1])) uns = 1;
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

// events[1..64] -> events[0] (unused: publish_kernel folds this sum into the read-back).
// (A last-workgroup sum inside the bucket pass measured 0.1 ms slower: its done counter is
// one address taking an atomic per workgroup.)
__global__ void sum64_kernel(unsigned long long *events)
{
    unsigned long long v = events[1 + threadIdx.x];
    for (int d = 32; d > 0; d >>= 1) v += __shfl_down(v, d, 64);
    if (threadIdx.x == 0) events[0] = v;
}

// One workgroup per (query row, ref chunk): LDS bitmap of the chunk's refs.  Each wave
// takes 64 query hashes at a time: lane l looks up the bucket [st, st + cnt) of hash l,
// a wave scan flattens the 64 buckets into one event range, and the lanes then read
// consecutive entries of that range (coalesced).  The owner hash of each event comes from
// a per-wave byte map filled by the lanes for 1024-event windows (one LDS read per event).
// 8 waves per SIMD (without the attribute: 7): the kernel waits on its
// event loads most of the time, and at 105 SGPRs the compiler's own allocation left 7
template <typename C>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8)))
void probe_rows_kernel(
    const void *__restrict__ qry, const uint32_t *__restrict__ qry_len, uint64_t stride,
    uint32_t n_qry, uint32_t q_lo, uint32_t n_ref, uint32_t hash_bytes, IdxGeom g,
    const uint32_t *__restrict__ dir, const uint32_t *__restrict__ entries,
    uint32_t chunk_refs, const uint32_t *__restrict__ ref_len, uint32_t S, uint32_t sym,
    uint32_t defaults, uint32_t vec_defaults, uint32_t self_set, C *__restrict__ numer,
    C *__restrict__ denom, uint64_t *__restrict__ cand,
    unsigned long long *__restrict__ n_cand, uint64_t *__restrict__ row_seg,
    const uint32_t *__restrict__ qry_it_len, uint32_t *__restrict__ q_unsorted,
    unsigned long long *__restrict__ events, uint64_t cap, uint32_t *__restrict__ cand_over)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t rowbits[];
    __shared__ uint32_t wsum[4];
    __shared__ unsigned long long row_base;
    // per wave: (entry base, fingerprint) of its 64 hashes, and the owner map of an event
    // window (which of the 64 hashes each event belongs to)
    constexpr uint32_t kWin = 1024;
    __shared__ uint64_t w_tab[4][64];
    __shared__ uint8_t w_own[4][kWin];
    // XCD-contiguous rows (shared buckets in L2) of rows [q_lo, q_lo + n_qry)
    const uint32_t qr = xcd_row(blockIdx.x, n_qry);
    if (qr >= n_qry) return;
    const uint32_t q = q_lo + qr;
    const uint64_t mult = idx_mult(g);
    const uint32_t r0 = blockIdx.y * chunk_refs;
    const uint32_t r1 = min(n_ref, r0 + chunk_refs);
    // symmetric self-comparison: each unordered pair {q, r} is a candidate of one of its two
    // rows: of the lower row when q + r is odd, of the higher (and the diagonal) when it is
    // even, so every row ranks about half of its partners.  (r <= q gave a row all of its lower
    // partners: a family's last rows ranked ~100 candidates and its first ~1, and the rank
    // kernel ended on the heavy rows' workgroups.)  The events mark every partner; the mask is
    // applied per bitmap word when the candidates are taken (no test per event).
    auto word_mask = [&](uint32_t w) -> uint32_t {
        if (!sym) return ~0u;
        const uint32_t rb = r0 + 32 * w;                       // bit i <-> ref rb + i
        const uint32_t odd = ((q ^ rb) & 1u) ? 0x55555555u : 0xAAAAAAAAu;   // q + r odd
        // gt: the bits of refs above q
        const uint32_t gt = q < rb ? ~0u : q - rb >= 31 ? 0u : ~((2u << (q - rb)) - 1u);
        return (odd & gt) | (~odd & ~gt);
    };
    const uint32_t nwords = (r1 - r0 + 31) / 32;
    for (uint32_t w = threadIdx.x; w < nwords; w += 256) rowbits[w] = 0;
    __syncthreads();
    // lq: the row's list length (the defaults); lit: the hashes probed, which differ from lq
    // when the probed rows are the record rows of unsorted lists (record_rows_kernel)
    const uint32_t lq = qry_len[q];
    const uint32_t lit = qry_it_len ? qry_it_len[q] : lq;
    // one set against itself: row q's own entry sits in the bucket of each of its hashes,
    // so a bucket of one entry holds only that entry.  Such buckets (the unique hashes, most
    // of a sketch) are not read; the pair (q, q) they would mark is set here.
    if (self_set && threadIdx.x == 0 && lq > 0 && q >= r0 && q < r1)
        atomicOr(&rowbits[(q - r0) >> 5], 1u << ((q - r0) & 31));
    const uint64_t rowoff = (uint64_t)q * stride;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t rmask = (uint32_t)((1ULL << g.rbits) - 1);
    // batches of 64 hashes per wave; the keys and bucket ranges of up to kB batches are
    // loaded together (their global loads overlap) before the batches are expanded
    constexpr int kB = 4;
    uint64_t ev_w = 0;      // this wave's posting events (with `events`)
    uint32_t uns = 0;       // an out-of-order or repeated value in the row (with `q_unsorted`)
    for (uint32_t jb = wave * 64; jb < lit; jb += 256 * kB) {
        uint32_t st_b[kB], cnt_b[kB], tgt_b[kB];
#pragma unroll
        for (int bi = 0; bi < kB; bi++) {
            const uint32_t j = jb + 256 * bi + lane;
            const uint64_t raw = j < lit ? load_key(qry, hash_bytes, rowoff + j) : 0;
            if (q_unsorted) {
                // the next value of the row: the next lane's, or a load for the last lane
                uint64_t nx = __shfl_down(raw, 1, 64);
                if (lane == 63 && j + 1 < lit) nx = load_key(qry, hash_bytes, rowoff + j + 1);
                if (j + 1 < lit && !(raw < nx)) uns = 1;
            }
            const uint64_t K = j < lit ? norm_key(raw, hash_bytes) : 0;
            const uint64_t b = bucket_of(K, g, mult);
            const uint32_t d0 = j < lit ? dir[b] : 0u, d1 = j < lit ? dir[b + 1] : 0u;
            st_b[bi] = d0;
            cnt_b[bi] = self_set && d1 - d0 == 1 ? 0u : d1 - d0;
            tgt_b[bi] = key_fp(K, g, mult);
        }
#pragma unroll
      for (int bi = 0; bi < kB; bi++) {
        if (jb + 256 * bi >= lit) break;                  // wave-uniform
        const uint32_t st = st_b[bi], cnt = cnt_b[bi], tgt = tgt_b[bi];
        uint32_t inc = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(inc, d, 64);
            if ((int)lane >= d) inc += y;
        }
        const uint32_t total = __builtin_amdgcn_readlane(inc, 63);
        ev_w += total;
        // same wave writes and reads these slots: LDS ops of one wave complete in order.
        // Event ev of hash m reads entries[st_m + ev - pre_m] = entries[base_m + ev] (u32
        // arithmetic wraps consistently).
        const uint32_t pre = inc - cnt;
        w_tab[wave][lane] = ((uint64_t)tgt << 32) | (uint32_t)(st - pre);
        for (uint32_t wb = 0; wb < total; wb += kWin) {
            // owner map of events [wb, wb + kWin): each lane marks its own hash's events
            // (4 per dword store inside a lane's range: 3 spilled VGPRs under the 8-wave cap,
            // 0.29 -> 0.306 ms)
            const uint32_t a0 = max(pre, wb), a1 = min(pre + cnt, wb + kWin);
            for (uint32_t e = a0; e < a1; e++) w_own[wave][e - wb] = (uint8_t)lane;
            __builtin_amdgcn_wave_barrier();
            const uint32_t wn = min(kWin, total - wb);
            // kU events per lane in flight: owner byte -> (base, fingerprint) -> entry
            constexpr int kU = PROBE_KU;
            for (uint32_t e0 = lane; e0 < wn; e0 += 64 * kU) {
                uint64_t tab[kU];
#pragma unroll
                for (int u = 0; u < kU; u++) {
                    const uint32_t e = e0 + 64 * u;
                    tab[u] = w_tab[wave][w_own[wave][e < wn ? e : 0]];
                }
                uint32_t en[kU];
#pragma unroll
                for (int u = 0; u < kU; u++) {
                    const uint32_t e = e0 + 64 * u;
                    en[u] = e < wn ? entries[(uint32_t)tab[u] + wb + e] : 0u;
                }
                // a read first: lanes of a shared bucket hit the same few words (family
                // members have adjacent ids), where an atomic per lane serialises; the bits
                // are almost always set already.  Branch-free per event (the read is done for
                // every lane, at word 0 when the event is not this row's), the rare atomics
                // after the kU events: a branch per event cost 11 scalar instructions of exec
                // mask handling each
                uint32_t wi[kU], need = 0;
#pragma unroll
                for (int u = 0; u < kU; u++) {
                    const uint32_t e = e0 + 64 * u;
                    const uint32_t r = en[u] & rmask;
                    const bool hit = e < wn && (en[u] >> g.rbits) == (uint32_t)(tab[u] >> 32) &&
                                     r >= r0 && r < r1;
                    wi[u] = hit ? r - r0 : 0u;
                    const uint32_t word = rowbits[wi[u] >> 5];
                    need |= (hit && !(word & (1u << (wi[u] & 31)))) ? (1u << u) : 0u;
                }
                if (__any(need != 0)) {
#pragma unroll
                    for (int u = 0; u < kU; u++)
                        if (need >> u & 1u) atomicOr(&rowbits[wi[u] >> 5], 1u << (wi[u] & 31));
                }
            }
            __builtin_amdgcn_wave_barrier();   // before the next window's owner map
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (q_unsorted && __any(uns) && lane == 0) atomicOr(q_unsorted, 1u);
    if (events && blockIdx.y == 0 && lane == 0 && ev_w)
        atomicAdd(&events[1 + (blockIdx.x & 63)], ev_w);
    __syncthreads();
    // candidates of this row: popcount per word -> block scan -> append
    uint32_t mycnt = 0;
    for (uint32_t w = threadIdx.x; w < nwords; w += 256) mycnt += __popc(rowbits[w] & word_mask(w));
    uint32_t x = mycnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (uint32_t w = 0; w < 4; w++) { if (w < wave) wpre += wsum[w]; tot += wsum[w]; }
    if (threadIdx.x == 0) {
        row_base = tot ? atomicAdd(n_cand, (unsigned long long)tot) : 0ULL;
        // past the candidate buffer (a call enqueued before its posting events were known,
        // fpm_api.cpp's speculated probe): nothing written, the row flagged and left empty
        const bool over = row_base + tot > cap;
        if (over) atomicOr(cand_over, 1u);
        // (offset << 24 | count) of this row's candidates; one ref chunk per row here
        if (gridDim.y == 1) row_seg[q] = (row_base << 24) | (over ? 0u : (tot & 0xFFFFFF));
        if (over) row_base = ~0ULL;
    }
    __syncthreads();
    const bool dropped = row_base == ~0ULL;
    uint64_t pos = row_base + wpre + x - mycnt;
    const uint64_t pair_row = (uint64_t)q * n_ref;
    for (uint32_t w = threadIdx.x; !dropped && w < nwords; w += 256) {
        uint32_t b = rowbits[w] & word_mask(w);
        const uint64_t bit0 = pair_row + r0 + (uint64_t)w * 32;
        while (b) {
            int t = __builtin_ctz(b);
            b &= b - 1;
            cand[pos++] = bit0 + t;
        }
    }
    // every pair of the row starts as "no shared value": (0, min(S, la+lb)) (the candidate
    // kernels, later launches, rewrite the candidates).  Last in the kernel: stores count in
    // the same in-order vmcnt as loads, so stores issued first would hold up every load the
    // event loop waits on.  16-B stores when the row chunk is 4-cell aligned.
    if (defaults) {
        if (vec_defaults) {
            for (uint32_t r = r0 + threadIdx.x * 4; r < r1; r += 1024) {
                const uint64_t o = pair_row + r;
                const uint4 rl = *(const uint4 *)(ref_len + r);
                const uint32_t d0 = rl.x + lq, d1 = rl.y + lq, d2 = rl.z + lq, d3 = rl.w + lq;
                // non-temporal: the row's defaults are not read again by this kernel (C2 probe
                // 0.381 -> 0.335 ms: the 0.4 GB of defaults no longer evict the posting lists
                // the event loop reads from L2)
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                if constexpr (sizeof(C) == 2) {
                    __builtin_nontemporal_store(u32x2{0u, 0u}, (u32x2 *)(numer + o));
                    __builtin_nontemporal_store(u32x2{min(d0, S) | (min(d1, S) << 16),
                                                      min(d2, S) | (min(d3, S) << 16)},
                                                (u32x2 *)(denom + o));
                } else {
                    __builtin_nontemporal_store(u32x4{0u, 0u, 0u, 0u}, (u32x4 *)(numer + o));
                    __builtin_nontemporal_store(u32x4{min(d0, S), min(d1, S), min(d2, S), min(d3, S)},
                                                (u32x4 *)(denom + o));
                }
            }
        } else {
            for (uint32_t r = r0 + threadIdx.x; r < r1; r += 256) {
                const uint64_t o = pair_row + r;
                const uint64_t d = (uint64_t)ref_len[r] + lq;
                numer[o] = 0;
                denom[o] = (C)(d < S ? (uint32_t)d : S);
            }
        }
    }
}

// ---- unsorted (-fp) lists: which pairs can the literal walk (CommandDistance.cpp:376-400)
// count anything for?  Let KA(i) = max(A[0..i]) and KB(j) = max(B[0..j]).  At a state (i, j)
// the walk reaches, A[i] < B[j] implies KA(i) <= KB(j): the previous maximum of A was taken
// at a state (i', j') with j' <= j, so it was <= B[j'] <= KB(j).  Likewise B[j] < A[i]
// implies KB(j) <= KA(i), and an equal step A[i] == B[j] implies KA(i) == KB(j) = v: v is
// the running maximum of both prefixes, i.e. a RECORD value (a strict increase of the running
// maximum) of both lists, among their first min(len, S) entries (the walk only reads A[i]
// with i <= steps < S).  So a pair whose lists share no record value has common = 0 and
// denom = min(S, la + lb), the values the probe writes for every pair.  The index and probe
// therefore run on each row's records (strictly increasing: sorted and distinct), and the
// pairs sharing one are walked literally on the original lists.  Random-order lists hold
// ~ln(S) + 0.58 records (C3's CFL lists: 7.5 of their first 1,000 entries), and the pairs
// sharing a record are nearly exactly those the walk counts something for (C3: 5.4 % vs
// 5.3 %), where the sorted distinct copies of every entry gave 2.9e10 posting events on C3
// (its frequent k-fingers are in nearly every list) and left the dense walk cheaper.
// One wave per row: chunks of 64 entries, the running maximum by a wave max-scan, the
// records compacted by ballot into out[row * out_stride ...] (and, with pos_out, their
// positions in the row beside them: the candidate walk starts at the shared ones).
constexpr int kRecWaves = 4;
template <typename H>
__global__ __launch_bounds__(64 * kRecWaves) void record_rows_kernel(
    const H *__restrict__ in, const uint32_t *__restrict__ in_len, uint64_t in_stride, uint32_t n,
    uint32_t S, H *__restrict__ out, uint32_t *__restrict__ pos_out, uint32_t *__restrict__ out_len,
    uint64_t out_stride, uint32_t *__restrict__ unsorted)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t row = blockIdx.x * kRecWaves + (threadIdx.x >> 6);
    if (row >= n) return;
    if (unsorted) {
        // the index build's sortedness test (every entry of the row below the next one), so
        // a caller can take the record index without building the raw one first
        const uint32_t len = in_len[row];
        const H *r = in + (uint64_t)row * in_stride;
        bool uns = false;
        for (uint32_t c0 = 0; c0 < len; c0 += 64) {
            const uint32_t i = c0 + lane;
            const H v = i < len ? r[i] : H(0);
            H nx = (H)__shfl_down((unsigned long long)v, 1, 64);
            if (lane == 63 && i + 1 < len) nx = r[i + 1];
            uns |= i + 1 < len && !(v < nx);
        }
        if (__any(uns) && lane == 0) atomicOr(unsorted, 1u);
    }
    const uint32_t m = min(min(in_len[row], S), (uint32_t)out_stride);
    const H *src = in + (uint64_t)row * in_stride;
    H *dst = out + (uint64_t)row * out_stride;
    uint32_t *pdst = pos_out ? pos_out + (uint64_t)row * out_stride : nullptr;
    H run = 0;              // the running maximum before the chunk (entry 0 always counts)
    uint32_t cnt = 0;
    for (uint32_t c0 = 0; c0 < m; c0 += 64) {
        const uint32_t i = c0 + lane;
        const H v = i < m ? src[i] : H(0);
        H pm = v;           // inclusive max-scan over the chunk
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const H y = (H)__shfl_up((unsigned long long)pm, d, 64);
            if ((int)lane >= d) pm = pm > y ? pm : y;
        }
        H before = (H)__shfl_up((unsigned long long)pm, 1, 64);
        before = lane == 0 ? run : (before > run ? before : run);
        const bool rec = i < m && (i == 0 || v > before);
        const uint64_t bm = __ballot(rec);
        const uint32_t at = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        if (rec) dst[at] = v;
        if (rec && pdst) pdst[at] = i;
        cnt += (uint32_t)__popcll(bm);
        const H top = (H)__shfl((unsigned long long)pm, 63, 64);
        run = top > run ? top : run;
    }
    if (lane == 0) out_len[row] = cnt;
}

hipError_t launch_record_rows(const void *in, const uint32_t *in_len, uint64_t in_stride,
                              uint32_t n, uint32_t hash_bytes, uint32_t S, void *out,
                              uint32_t *pos_out, uint32_t *out_len, uint64_t out_stride,
                              hipStream_t st, uint32_t *unsorted)
{
    if (!n) return hipSuccess;
    const dim3 g((n + kRecWaves - 1) / kRecWaves), b(64 * kRecWaves);
    if (hash_bytes == 8)
        hipLaunchKernelGGL(record_rows_kernel<uint64_t>, g, b, 0, st, (const uint64_t *)in, in_len,
                           in_stride, n, S, (uint64_t *)out, pos_out, out_len, out_stride,
                           unsorted);
    else
        hipLaunchKernelGGL(record_rows_kernel<uint32_t>, g, b, 0, st, (const uint32_t *)in, in_len,
                           in_stride, n, S, (uint32_t *)out, pos_out, out_len, out_stride,
                           unsorted);
    return hipGetLastError();
}

__global__ __launch_bounds__(kPubWords) void publish_kernel(const unsigned long long *__restrict__ src,
                                                          uint32_t n, unsigned long long *dst,
                                                          unsigned long long seq)
{
    // src[0] = the posting events: the sum of the 64 spread partials src[1..64] (the index
    // build's bucket pass or probe_count_kernel add into those), folded in here
    unsigned long long ev = (threadIdx.x >= 1 && threadIdx.x <= 64 && n > 64) ? src[threadIdx.x] : 0;
    for (int d = 32; d > 0; d >>= 1) ev += __shfl_xor(ev, d, 64);
    __shared__ unsigned long long wsum[kPubWords / 64];
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = ev;
    __syncthreads();
    if (threadIdx.x == 0 && n > 64) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < kPubWords / 64; w++) t += wsum[w];
        dst[0] = t;
    } else if (threadIdx.x < n) {
        dst[threadIdx.x] = src[threadIdx.x];
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(dst + kPubWords - 1, seq, __ATOMIC_RELEASE,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_publish(const unsigned long long *d_src, uint32_t n, unsigned long long *h_dst,
                          unsigned long long seq, hipStream_t st)
{
    if (n >= kPubWords) return hipErrorInvalidValue;
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(kPubWords), 0, st, d_src, n, h_dst, seq);
    return hipGetLastError();
}

// scan_sums + scan_add in one launch for up to kScanFoldBlocks blocks: each block sums the
// block totals before it itself (<= 4096 reads spread over its 256 threads)
constexpr uint32_t kScanFoldBlocks = 4096;
__global__ __launch_bounds__(256) void scan_add_fold_kernel(uint32_t *__restrict__ out, uint64_t n,
                                                           const uint32_t *__restrict__ sums,
                                                           uint32_t nb, uint32_t *__restrict__ out2,
                                                           uint32_t *__restrict__ total)
{
    __shared__ uint32_t wsum[4];
    const uint32_t b = blockIdx.x;
    uint32_t part = 0;
    for (uint32_t i = threadIdx.x; i < b; i += 256) part += sums[i];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) part += __shfl_xor(part, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = part;
    __syncthreads();
    const uint32_t add = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (total && b == nb - 1 && threadIdx.x == 0) *total = add + sums[b];
    const uint64_t base = (uint64_t)b * kScanBlock + threadIdx.x * 4;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (base + k < n) {
            const uint32_t v = out[base + k] + add;
            out[base + k] = v;
            if (out2) out2[base + k] = v;
        }
}

uint64_t scan_scratch_words(uint64_t n) { return (n + kScanBlock - 1) / kScanBlock + 1; }

hipError_t launch_exscan(const uint32_t *in, uint32_t *out, uint32_t *out2, uint64_t n,
                         uint32_t *scratch, uint32_t *total, hipStream_t st)
{
    if (!n) return hipSuccess;
    uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
    hipLaunchKernelGGL(scan_local_kernel, dim3(nb), dim3(256), 0, st, in, out, n, scratch);
    if (nb <= kScanFoldBlocks) {
        hipLaunchKernelGGL(scan_add_fold_kernel, dim3(nb), dim3(256), 0, st, out, n,
                           (const uint32_t *)scratch, nb, out2, total);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(256), 0, st, scratch, nb, total);
    hipLaunchKernelGGL(scan_add_kernel, dim3(nb), dim3(256), 0, st, out, n, scratch, out2);
    return hipGetLastError();
}

// The dynamic-LDS limit of a kernel is a per-device attribute: set it once per (kernel slot,
// device ordinal) on the device current for the launch (contexts on several GPUs in one
// process each get their own).
static hipError_t dyn_lds_attr(int slot, const void *fn, int bytes)
{
    constexpr int kMaxDev = 64;
    static std::atomic<int> done[3][kMaxDev];
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= kMaxDev) return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (done[slot][dev].load(std::memory_order_acquire)) return hipSuccess;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done[slot][dev].store(1, std::memory_order_release);
    return e;
}

uint64_t idx_tent_words(const IdxGeom &g, uint64_t E)
{
    return g.cap ? (uint64_t)kParts * g.cap : E;
}

hipError_t launch_idx_build(const void *d_ref, const uint32_t *d_ref_len, uint64_t stride,
                            uint32_t n_ref, uint32_t hash_bytes, IdxGeom g, uint32_t *tile_hist,
                            uint32_t *tile_off, uint32_t *scan_s, uint64_t *tent,
                            uint32_t *dir, uint32_t *entries, uint32_t *unsorted,
                            unsigned long long *self_events, unsigned long long *zero,
                            uint32_t nzero, unsigned long long *acc, uint32_t *part_fill,
                            uint32_t *overflow, hipStream_t st, unsigned long long *zero_x)
{
    const uint32_t ntiles = g.ntiles;
    const uint64_t magic = stride > 1 ? ~0ULL / stride + 1 : 0;   // row_of's multiplier
    const uint32_t kg = std::max<uint32_t>(1, std::min<uint32_t>(
        (n_ref + kKmaxThreads * kKmaxU - 1) / (kKmaxThreads * kKmaxU), 64));
    const bool one_pass = g.cap != 0 && part_fill && overflow;
    hipLaunchKernelGGL(idx_kmax_kernel, dim3(kg), dim3(kKmaxThreads), 0, st, d_ref, d_ref_len,
                       stride, n_ref, hash_bytes, (unsigned long long *)g.kmax, zero, nzero, acc,
                       one_pass ? part_fill : nullptr, one_pass ? kParts : 0u, zero_x);
    // level 2: the sub-bucket range split over 2^lsplit workgroups until its counters fit
    // 32 KB and a range's mean entries 24k (C4, E = 5e7: 2 per partition).  The LDS copy: 16k
    // entries (80 KB with the counters, two workgroups per CU) when the ranges' mean fits 12k
    // (C2), else all the LDS beside the counters, one workgroup per CU (C4: 2 x 32k-entry
    // ranges per partition, index 0.92 -> 0.80 ms against 4 x 16k, C4 6.31-6.52 -> 6.21-6.26
    // ms, same box, r05j)
    uint32_t lsplit = 0;
    const double part_mean = (double)n_ref * (double)stride / (double)kParts;
    while (lsplit < g.l2 && lsplit < 4 &&
           (((uint64_t)4 << (g.l2 - lsplit)) > 32768 || part_mean / (double)(1u << lsplit) > 24576.0))
        lsplit++;
    const uint64_t cnt_bytes0 = (uint64_t)4 << (g.l2 - lsplit);
    constexpr uint32_t kLdsBytes = 159 * 1024;
    const uint32_t lds_cap = part_mean / (double)(1u << lsplit) <= 12288.0
                                 ? (uint32_t)(kBucketThreads * kBucketPer)
                                 : (uint32_t)((kLdsBytes - cnt_bytes0) / 4);
    const dim3 bgrid(kParts << lsplit);
    if (hipError_t e = dyn_lds_attr(1, (const void *)idx_bucket_kernel, kLdsBytes))
        return e;
    if (one_pass) {
        if (hipError_t e = dyn_lds_attr(2, (const void *)idx_part_scatter1_kernel, kIdxTile * 8))
            return e;
        hipLaunchKernelGGL(idx_part_scatter1_kernel, dim3(ntiles), dim3(kIdxThreads),
                           (size_t)g.tile * 8, st, d_ref, d_ref_len, (uint32_t)stride, magic,
                           n_ref, hash_bytes, g, part_fill, tent, unsorted, overflow);
        hipLaunchKernelGGL(idx_bucket_kernel, bgrid, dim3(kBucketThreads),
                           (size_t)(cnt_bytes0 + (uint64_t)lds_cap * 4), st, (const uint64_t *)tent,
                           ntiles, (const uint32_t *)nullptr, g, lds_cap, dir, entries, self_events,
                           (const uint32_t *)part_fill, lsplit);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(idx_part_hist_kernel, dim3(ntiles), dim3(kIdxThreads), 0, st, d_ref,
                       d_ref_len, (uint32_t)stride, magic, n_ref, hash_bytes, ntiles, tile_hist,
                       unsorted, g);
    const uint64_t nh = (uint64_t)kParts * ntiles;
    if (hipError_t e = launch_exscan(tile_hist, tile_off, nullptr, nh, scan_s, tile_off + nh, st))
        return e;
    if (hipError_t e = dyn_lds_attr(0, (const void *)idx_part_scatter_kernel, kIdxTile * 8))
        return e;
    hipLaunchKernelGGL(idx_part_scatter_kernel, dim3(ntiles), dim3(kIdxThreads),
                       (size_t)g.tile * 8, st, d_ref, d_ref_len, (uint32_t)stride, magic, n_ref,
                       hash_bytes, ntiles, (const uint32_t *)tile_hist, (const uint32_t *)tile_off,
                       g, tent);
    // LDS copy of a partition's entries when they fit beside the counters (two workgroups per
    // CU: 80 KiB each at l2 = 12); cap 0 = every partition on the global two-pass path
    hipLaunchKernelGGL(idx_bucket_kernel, bgrid, dim3(kBucketThreads),
                       (size_t)(cnt_bytes0 + (uint64_t)lds_cap * 4), st, (const uint64_t *)tent,
                       ntiles, (const uint32_t *)tile_off, g, lds_cap, dir, entries, self_events,
                       (const uint32_t *)nullptr, lsplit);
    return hipGetLastError();
}

hipError_t launch_probe_count(const void *d_qry, const uint32_t *d_qry_len, uint64_t stride,
                              uint32_t n_qry, uint32_t hash_bytes, IdxGeom g, const uint32_t *dir,
                              unsigned long long *events, uint32_t *unsorted, hipStream_t st)
{
    uint64_t n = (uint64_t)n_qry * stride;
    const uint64_t threads = (n + kPC - 1) / kPC;
    if (n) hipLaunchKernelGGL(probe_count_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256),
                              0, st, d_qry, d_qry_len, stride, n_qry, hash_bytes, g, dir, events,
                              unsorted);
    return hipGetLastError();
}

hipError_t launch_probe_rows(const void *d_qry, const uint32_t *d_qry_len, uint64_t stride,
                             uint32_t n_qry, uint32_t n_ref, uint32_t hash_bytes, IdxGeom g,
                             const uint32_t *dir, const uint32_t *entries,
                             const uint32_t *d_ref_len, uint32_t S, bool sym, bool defaults,
                             bool self_set, Counts cnt, uint64_t *cand,
                             unsigned long long *n_cand, uint64_t *row_seg,
                             const uint32_t *d_qry_it_len, uint32_t *q_unsorted,
                             unsigned long long *events, uint64_t cap, uint32_t *cand_over,
                             hipStream_t st, uint32_t q_lo)
{
    if (!n_qry || !n_ref) return hipSuccess;
    const uint32_t chunk = 1u << 19;   // refs per workgroup: 64 KiB of LDS bitmap
    const uint32_t nchunks = (n_ref + chunk - 1) / chunk;
    const uint32_t cref = nchunks == 1 ? n_ref : chunk;
    const size_t lds = ((cref + 31) / 32) * 4;
    // vector default stores (4 cells): every row and chunk start 4-cell aligned, buffers
    // 16-B aligned
    const auto al = [](const void *p) { return ((uintptr_t)p & 15) == 0; };
    const uint32_t vec_defaults = n_ref % 4 == 0 && cref % 4 == 0 && al(d_ref_len) &&
                                  al(cnt.numer) && al(cnt.denom);
#define FPM_PROBE(C)                                                                            \
    hipLaunchKernelGGL(probe_rows_kernel<C>, dim3(xcd_grid(n_qry), nchunks), dim3(256), lds, st,  \
                       d_qry, d_qry_len, stride, n_qry, q_lo, n_ref, hash_bytes, g, dir, entries, \
                       cref,                                                                     \
                       d_ref_len, S, (uint32_t)sym, (uint32_t)defaults, vec_defaults,           \
                       (uint32_t)self_set, (C *)cnt.numer, (C *)cnt.denom, cand, n_cand, row_seg, \
                       d_qry_it_len, q_unsorted, events, cap, cand_over)
    if (cnt.c16) FPM_PROBE(uint16_t);
    else FPM_PROBE(uint32_t);
#undef FPM_PROBE
    return hipGetLastError();
}

}  // namespace fpm
