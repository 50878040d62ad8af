// sketch.hip — DNA/alphabet k-mer sketching for gfx950.
//
// Replaces the per-k-mer loop of addMinHashes (Sketch.cpp:664-735) feeding
// MinHashHeap::tryInsert (MinHashHeap.cpp:68-146) and the final
// HashSet::toHashList sort (HashSet.cpp:78-118): instead of a heap walked one
// k-mer at a time, one workgroup owns a tile of up to P k-mer starts, stages the
// tile's bytes (and their reverse complement) in LDS, hashes every window in
// parallel (keys stay in registers), counting-sorts them by their top bits into LDS,
// insertion-sorts each ~2-key bucket and keeps the first s distinct.
// Result: the s smallest distinct hashes, ascending — exactly the set the
// reference heap holds at the end of the stream.
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

namespace fpm {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// Phase timestamps of the tile kernel for tools/micro/sketch_phases.hip (which defines
// FPM_SKETCH_PHASES and points g_phase at 8 u64 per workgroup); compiled out of the library.
#ifdef FPM_SKETCH_PHASES
__device__ uint64_t *g_phase;
#define FPM_PHASE_DECL uint64_t ph_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define FPM_PHASE(i) do { if (threadIdx.x == 0) ph_[i] = __builtin_amdgcn_s_memtime(); } while (0)
#define FPM_PHASE_FLUSH do { if (threadIdx.x == 0) for (int q_ = 0; q_ < 8; q_++) g_phase[blockIdx.x * 8 + q_] = ph_[q_]; } while (0)
#else
#define FPM_PHASE_DECL do {} while (0)
#define FPM_PHASE(i) do {} while (0)
#define FPM_PHASE_FLUSH do {} while (0)
#endif

// Block-wide exclusive scan of one u32 per thread; returns the exclusive prefix
// and writes the block total to *total.  `tmp` holds kWaves+1 dwords of LDS.
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *tmp, uint32_t *total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < kWaves; w++) { uint32_t t = tmp[w]; tmp[w] = acc; acc += t; }
        tmp[kWaves] = acc;
    }
    __syncthreads();
    uint32_t ex = tmp[wave] + x - v;
    *total = tmp[kWaves];
    __syncthreads();
    return ex;
}

// Bitonic sort of P keys in LDS, ascending (fallback for tiles with crowded buckets).
template <int P>
__device__ void bitonic_sort(uint64_t *keys)
{
    const int tid = threadIdx.x;
    for (int ks = 2; ks <= P; ks <<= 1) {
        for (int j = ks >> 1; j > 0; j >>= 1) {
            for (int t = tid; t < P / 2; t += kBlock) {
                int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                int l = i + j;
                bool up = (i & ks) == 0;
                uint64_t a = keys[i], b = keys[l];
                if ((a > b) == up) { keys[i] = b; keys[l] = a; }
            }
            __syncthreads();
        }
    }
}

// K != 0: the k-mer size as a compile-time constant (the window loads, tail masks and
// Murmur's block / tail branches fold); K = 0 reads p.k.
template <int P, int K>
__global__ __launch_bounds__(kBlock) void sketch_tiles_kernel(
    const uint8_t *__restrict__ seq, const TileDesc *__restrict__ tiles, SketchKParams p,
    const uint64_t *__restrict__ thr, uint64_t *__restrict__ out, uint32_t *__restrict__ out_count)
{
    // byte images padded so that 9-dword window reads past the end stay in bounds
    constexpr int kImgWords = (P + 32 + 64) / 4;
    __shared__ uint32_t fwd_img[kImgWords];
    __shared__ uint32_t rc_img[kImgWords];
    __shared__ uint32_t badmask[(P + 32 + 64) / 32];
    __shared__ uint64_t keys[P];
    __shared__ uint8_t alpha[256];
    __shared__ uint8_t compl_tab[256];
    __shared__ uint32_t scan_tmp[kWaves + 1];
    __shared__ uint32_t bins[P / 2 + 1];
    __shared__ uint32_t big_bucket;

    FPM_PHASE_DECL;
    FPM_PHASE(0);
    const TileDesc td = tiles[blockIdx.x];
    const uint32_t n = td.n_bytes;
    const uint32_t k = K ? (uint32_t)K : p.k;
    const int tid = threadIdx.x;

    alpha[tid] = p.alphabet[tid];
    compl_tab[tid] = p.complement[tid];
    __syncthreads();

    // ---- stage bytes: uppercase (Sketch.cpp:676-682), validity bitmask, rc image
    uint8_t *fb = reinterpret_cast<uint8_t *>(fwd_img);
    uint8_t *rb = reinterpret_cast<uint8_t *>(rc_img);
    constexpr int kImgBytes = kImgWords * 4;
    constexpr int kIt = (kImgBytes + kBlock - 1) / kBlock;
    // every global byte load of the tile issued before the first use (one memory latency
    // per tile instead of one per pass)
    uint8_t cb[kIt];
#pragma unroll
    for (int it = 0; it < kIt; it++) {
        const int b = tid + it * kBlock;
        cb[it] = (uint32_t)b < n ? seq[td.byte_off + b] : (uint8_t)0;
    }
#pragma unroll
    for (int it = 0; it < kIt; it++) {
        const int b = tid + it * kBlock;
        if (b >= kImgBytes) break;
        uint8_t c = 0;
        if ((uint32_t)b < n) {
            c = cb[it];
            if (!p.preserve_case && c > 96 && c < 123) c -= 32;
        }
        fb[b] = c;
        bool bad = (uint32_t)b >= n || !alpha[c];
        unsigned long long m = __ballot(bad);
        if ((tid & 63) == 0 && b / 32 + 1 < (P + 32 + 64) / 32) {
            badmask[b / 32] = (uint32_t)m;
            badmask[b / 32 + 1] = (uint32_t)(m >> 32);
        }
        if ((uint32_t)b < n) rb[n - 1 - b] = compl_tab[c];   // reverseComplement Sketch.cpp:1252-1258
        else rb[b] = 0;
    }
    __syncthreads();
    FPM_PHASE(1);

    // ---- hash every window (one k-mer start per thread per pass)
    const uint32_t nk = n >= k ? n - k + 1 : 0;
    const int nw = (k + 3) >> 2;                           // dwords per k-mer
    const uint32_t tail_mask = (k & 3) ? ((1u << (8 * (k & 3))) - 1u) : 0xffffffffu;
    const uint32_t kmask = (k == 32) ? 0xffffffffu : ((1u << k) - 1u);
    constexpr int E = P / kBlock;                          // keys per thread (P >= 256)
    uint64_t kr[E];                                        // this thread's keys: i = tid + e*kBlock
    uint32_t vbits = 0;                                    // bit e: kr[e] is a valid k-mer hash
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int i = tid + e * kBlock;
        uint64_t key = ~0ULL;
        if ((uint32_t)i < nk) {
            // window [i, i+k) must hold alphabet bytes only (Sketch.cpp:696-713)
            uint32_t w = i >> 5, sh = i & 31;
            uint64_t bits = ((uint64_t)badmask[w] | ((uint64_t)badmask[w + 1] << 32)) >> sh;
            if (((uint32_t)bits & kmask) == 0) {
                uint32_t d[8];
#pragma unroll
                for (int m = 0; m < 8; m++)
                    d[m] = (m < nw) ? lds_u32_at(fwd_img, i + 4 * m) : 0u;
                d[nw - 1] &= tail_mask;
                if (p.canonical) {
                    // canonical = memcmp(fwd, rev) <= 0 ? fwd : rev (Sketch.cpp:719-723)
                    const uint32_t ro = n - i - k;
                    uint32_t r[8];
#pragma unroll
                    for (int m = 0; m < 8; m++)
                        r[m] = (m < nw) ? lds_u32_at(rc_img, ro + 4 * m) : 0u;
                    r[nw - 1] &= tail_mask;
                    int cmp = 0;
#pragma unroll
                    for (int m = 0; m < 8; m++) {
                        uint32_t fbe = __builtin_bswap32(d[m]), rbe = __builtin_bswap32(r[m]);
                        if (cmp == 0 && m < nw) cmp = (fbe > rbe) - (fbe < rbe);
                    }
                    if (cmp > 0) {
#pragma unroll
                        for (int m = 0; m < 8; m++) d[m] = r[m];
                    }
                }
                uint64_t wd[4];
#pragma unroll
                for (int j = 0; j < 4; j++) wd[j] = (uint64_t)d[2 * j] | ((uint64_t)d[2 * j + 1] << 32);
                uint64_t h = murmur_h1_le32(wd, (int)k, p.seed);
                key = p.use64 ? h : (h & 0xffffffffULL);   // getHash hash.cpp:30-37
                vbits |= 1u << e;
            }
        }
        kr[e] = key;
    }

    // ---- long groups: keep only hashes <= the group's bound (the s-th smallest hash of a
    // sample of the group's tiles, an upper bound of the group's own s-th smallest)
    FPM_PHASE(2);
    uint64_t hmax = p.use64 ? ~0ULL : 0xffffffffULL;
    if (td.thr_slot) {
        hmax = min(hmax, thr[td.thr_slot - 1]);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (kr[e] > hmax) vbits &= ~(1u << e);
    }

    // ---- sort: counting sort by the top log2(P/2) bits of the (uniform) hash values in
    // [0, hmax], then insertion sort inside each bucket (~2 keys per bucket).  A bucket
    // holding more than kMaxBucket keys (low-complexity input: many copies of few k-mers)
    // sends the whole tile to the bitonic sort instead.
    constexpr int NB = P / 2;
    constexpr int LB = __builtin_ctz(NB);
    constexpr uint32_t kMaxBucket = 32;
    const uint32_t hbits = hmax ? 64 - __clzll(hmax) : 1;
    const uint32_t bshift = hbits > (uint32_t)LB ? hbits - LB : 0;
    for (int b = tid; b <= NB; b += kBlock) bins[b] = 0;
    if (tid == 0) big_bucket = 0;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; e++)
        if (vbits >> e & 1) atomicAdd(&bins[(uint32_t)(kr[e] >> bshift)], 1u);
    __syncthreads();
    FPM_PHASE(3);
    // exclusive scan of the bucket counts: thread t owns buckets [t*per, t*per + per)
    constexpr int per = NB >= kBlock ? NB / kBlock : 1;
    uint32_t run = 0, bmax = 0;
#pragma unroll
    for (int u = 0; u < per; u++) {
        const int b = tid * per + u;
        const uint32_t c = b < NB ? bins[b] : 0u;
        run += c;
        bmax = max(bmax, c);
    }
    uint32_t nvalid;
    uint32_t acc = block_exscan(run, scan_tmp, &nvalid);   // also a barrier over bins[]
#pragma unroll
    for (int u = 0; u < per; u++) {
        const int b = tid * per + u;
        if (b < NB) { const uint32_t c = bins[b]; bins[b] = acc; acc += c; }
    }
    if (bmax > kMaxBucket) big_bucket = 1;
    __syncthreads();
    FPM_PHASE(4);
    // scatter: afterwards bins[b] = end of bucket b, start = bins[b - 1]; each key keeps
    // its slot for the in-bucket rank below
    uint32_t slot[E];
#pragma unroll
    for (int e = 0; e < E; e++)
        if (vbits >> e & 1) {
            slot[e] = atomicAdd(&bins[(uint32_t)(kr[e] >> bshift)], 1u);
            keys[slot[e]] = kr[e];
        }
    __syncthreads();
    FPM_PHASE(5);
    if (!big_bucket) {
        // in-bucket rank of every key (ties by slot): the bucket's ~2 keys are read with
        // independent LDS loads, then every key is written to its sorted position (an
        // insertion sort per bucket was a chain of dependent LDS round trips: 26 % of the
        // tile's time, tools/micro/sketch_phases.hip)
#pragma unroll
        for (int e = 0; e < E; e++)
            if (vbits >> e & 1) {
                const uint32_t b = (uint32_t)(kr[e] >> bshift);
                const uint32_t s0 = b ? bins[b - 1] : 0u, s1 = bins[b];
                const uint32_t mb = s1 - s0;
                uint32_t r = 0;
                // 8 speculative reads cover a bucket of <= 8 keys (Poisson(2) buckets: a
                // longer one is rare) with one LDS round trip
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    const uint32_t t = s0 + u;
                    const uint64_t y = keys[t < (uint32_t)P ? t : (uint32_t)P - 1];
                    r += (u < mb) & ((y < kr[e]) | ((y == kr[e]) & (t < slot[e])));
                }
                for (uint32_t t = s0 + 8; t < s1; t++) {
                    const uint64_t y = keys[t];
                    r += (y < kr[e]) | ((y == kr[e]) & (t < slot[e]));
                }
                slot[e] = s0 + r;
            }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < E; e++)
            if (vbits >> e & 1) keys[slot[e]] = kr[e];
        __syncthreads();
    } else {
        for (int i = tid; i < P; i += kBlock)
            if ((uint32_t)i >= nvalid) keys[i] = ~0ULL;
        __syncthreads();
        bitonic_sort<P>(keys);
    }
    FPM_PHASE(6);

    // ---- first s distinct (ties removed: the heap is a set, MinHashHeap.cpp:74)
    const int base = tid * E;
    uint32_t cnt = 0;
#pragma unroll
    for (int e = 0; e < E; e++) {
        int idx = base + e;
        if (idx < P && (uint32_t)idx < nvalid && (idx == 0 || keys[idx] != keys[idx - 1])) cnt++;
    }
    uint32_t total;
    uint32_t rank = block_exscan(cnt, scan_tmp, &total);
    uint64_t *row = out + (uint64_t)td.out_row * p.s;
#pragma unroll
    for (int e = 0; e < E; e++) {
        int idx = base + e;
        if (idx < P && (uint32_t)idx < nvalid && (idx == 0 || keys[idx] != keys[idx - 1])) {
            if (rank < p.s) row[rank] = keys[idx];
            rank++;
        }
    }
    if (tid == 0) out_count[td.out_row] = total < p.s ? total : p.s;
    FPM_PHASE(7);
    FPM_PHASE_FLUSH;
}

// Merge of two ascending distinct lists, keeping the first s distinct of the union.
// A[i] lands at i + lower_bound(B, A[i]) - #dups among A[0..i); B[j] that equals an
// A element is dropped, the others land at j + upper_bound(A, B[j]) - #dups among B[0..j).
__device__ __forceinline__ uint32_t lower_bound_u64(const uint64_t *v, uint32_t n, uint64_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (v[m] < x) lo = m + 1; else hi = m; }
    return lo;
}
__device__ __forceinline__ uint32_t upper_bound_u64(const uint64_t *v, uint32_t n, uint64_t x)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (v[m] <= x) lo = m + 1; else hi = m; }
    return lo;
}

__global__ __launch_bounds__(kBlock) void merge_kernel(const MergeDesc *__restrict__ descs, uint32_t s)
{
    __shared__ uint32_t scan_tmp[kWaves + 1];
    const MergeDesc md = descs[blockIdx.x];
    const uint32_t la = *md.alen, lb = md.b ? *md.blen : 0;
    uint32_t dups_total = 0;
    // A side
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < la; c0 += kBlock) {
        uint32_t i = c0 + threadIdx.x;
        uint64_t a = 0; uint32_t pos = 0; uint32_t dup = 0;
        if (i < la) {
            a = md.a[i];
            pos = lb ? lower_bound_u64(md.b, lb, a) : 0;
            dup = (pos < lb && md.b[pos] == a) ? 1u : 0u;
        }
        uint32_t tot;
        uint32_t ex = block_exscan(dup, scan_tmp, &tot);
        if (i < la) {
            uint32_t f = i + pos - (carry + ex);
            if (f < s) md.c[f] = a;
        }
        carry += tot;
    }
    dups_total = carry;
    // B side
    carry = 0;
    for (uint32_t c0 = 0; c0 < lb; c0 += kBlock) {
        uint32_t j = c0 + threadIdx.x;
        uint64_t b = 0; uint32_t pos = 0; uint32_t dup = 0;
        if (j < lb) {
            b = md.b[j];
            pos = upper_bound_u64(md.a, la, b);
            dup = (pos > 0 && md.a[pos - 1] == b) ? 1u : 0u;
        }
        uint32_t tot;
        uint32_t ex = block_exscan(dup, scan_tmp, &tot);
        if (j < lb && !dup) {
            uint32_t f = j + pos - (carry + ex);
            if (f < s) md.c[f] = b;
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        uint32_t u = la + lb - dups_total;
        *md.clen = u < s ? u : s;
    }
}

template <int P>
static hipError_t launch_p(const uint8_t *d_seq, const TileDesc *d_tiles, uint32_t n_tiles,
                           const SketchKParams &p, const uint64_t *d_thr, uint64_t *d_out,
                           uint32_t *d_count, hipStream_t st)
{
    if (n_tiles == 0) return hipSuccess;
    if (p.k == 21)      // Mash's default k (sketchParameterSetup, C2/C4/C5)
        hipLaunchKernelGGL((sketch_tiles_kernel<P, 21>), dim3(n_tiles), dim3(kBlock), 0, st,
                           d_seq, d_tiles, p, d_thr, d_out, d_count);
    else
        hipLaunchKernelGGL((sketch_tiles_kernel<P, 0>), dim3(n_tiles), dim3(kBlock), 0, st,
                           d_seq, d_tiles, p, d_thr, d_out, d_count);
    return hipGetLastError();
}

hipError_t launch_sketch_tiles(int cls, const uint8_t *d_seq, const TileDesc *d_tiles,
                               uint32_t n_tiles, const SketchKParams &p, const uint64_t *d_thr,
                               uint64_t *d_out, uint32_t *d_count, hipStream_t st)
{
    switch (cls) {
    case 0: return launch_p<256>(d_seq, d_tiles, n_tiles, p, d_thr, d_out, d_count, st);
    case 1: return launch_p<512>(d_seq, d_tiles, n_tiles, p, d_thr, d_out, d_count, st);
    case 2: return launch_p<1024>(d_seq, d_tiles, n_tiles, p, d_thr, d_out, d_count, st);
    case 3: return launch_p<2048>(d_seq, d_tiles, n_tiles, p, d_thr, d_out, d_count, st);
    case 4: return launch_p<4096>(d_seq, d_tiles, n_tiles, p, d_thr, d_out, d_count, st);
    case 5: return launch_p<8192>(d_seq, d_tiles, n_tiles, p, d_thr, d_out, d_count, st);
    default: return hipErrorInvalidValue;
    }
}

__global__ void sketch_threshold_kernel(const uint32_t *__restrict__ srow, uint32_t n_slots,
                                        const uint64_t *__restrict__ rows,
                                        const uint32_t *__restrict__ count, uint32_t s,
                                        uint64_t *__restrict__ thr)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots) return;
    const uint32_t r = srow[i];
    thr[i] = count[r] >= s ? rows[(uint64_t)r * s + s - 1] : ~0ULL;
}

hipError_t launch_sketch_threshold(const uint32_t *d_srow, uint32_t n_slots, const uint64_t *d_rows,
                                   const uint32_t *d_count, uint32_t s, uint64_t *d_thr,
                                   hipStream_t st)
{
    if (!n_slots) return hipSuccess;
    hipLaunchKernelGGL(sketch_threshold_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, st,
                       d_srow, n_slots, d_rows, d_count, s, d_thr);
    return hipGetLastError();
}

// The same merge with the searched list staged in LDS (every list holds <= s hashes): B for
// the A side's lower bounds, then A for the B side's upper bounds.  1024 threads, so a list
// of s = 10,000 (C5) is 10 chunks per side, each a 14-step binary search in LDS instead of
// 40 chunks of 14 dependent global loads (C5's final rounds are one merge per genome: ~125
// workgroups, so per-workgroup latency is the whole round).
constexpr int kMBlock = 1024;
constexpr int kMWaves = kMBlock / 64;

__device__ __forceinline__ uint32_t block_exscan_m(uint32_t v, uint32_t *tmp, uint32_t *total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t w = threadIdx.x < kMWaves ? tmp[threadIdx.x] : 0u;
        uint32_t sc = w;
#pragma unroll
        for (int d = 1; d < kMWaves; d <<= 1) {
            uint32_t y = __shfl_up(sc, d, 64);
            if ((int)threadIdx.x >= d) sc += y;
        }
        if (threadIdx.x < kMWaves) tmp[threadIdx.x] = sc - w;
        if (threadIdx.x == kMWaves - 1) tmp[kMWaves] = sc;
    }
    __syncthreads();
    const uint32_t ex = tmp[wave] + x - v;
    *total = tmp[kMWaves];
    __syncthreads();
    return ex;
}

__global__ __launch_bounds__(kMBlock) void merge_lds_kernel(const MergeDesc *__restrict__ descs,
                                                           uint32_t s)
{
    extern __shared__ uint64_t sl[];                 // the list being searched (<= s hashes)
    __shared__ uint32_t scan_tmp[kMWaves + 1];
    const MergeDesc md = descs[blockIdx.x];
    const uint32_t la = *md.alen, lb = md.b ? *md.blen : 0;
    for (uint32_t j = threadIdx.x; j < lb; j += kMBlock) sl[j] = md.b[j];
    __syncthreads();
    // A side: A[i] lands at i + lower_bound(B, A[i]) - #(A elements before i found in B)
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < la; c0 += kMBlock) {
        const uint32_t i = c0 + threadIdx.x;
        uint64_t a = 0;
        uint32_t pos = 0, dup = 0;
        if (i < la) {
            a = md.a[i];
            pos = lower_bound_u64(sl, lb, a);
            dup = (pos < lb && sl[pos] == a) ? 1u : 0u;
        }
        uint32_t tot;
        const uint32_t ex = block_exscan_m(dup, scan_tmp, &tot);
        if (i < la) {
            const uint32_t f = i + pos - (carry + ex);
            if (f < s) md.c[f] = a;
        }
        carry += tot;
    }
    const uint32_t dups_total = carry;
    if (lb) {
        // B side: A in LDS; B[j] equal to an A element is dropped, the others land at
        // j + upper_bound(A, B[j]) - #(B elements before j found in A)
        for (uint32_t i = threadIdx.x; i < la; i += kMBlock) sl[i] = md.a[i];
        __syncthreads();
        carry = 0;
        for (uint32_t c0 = 0; c0 < lb; c0 += kMBlock) {
            const uint32_t j = c0 + threadIdx.x;
            uint64_t b = 0;
            uint32_t pos = 0, dup = 0;
            if (j < lb) {
                b = md.b[j];
                pos = upper_bound_u64(sl, la, b);
                dup = (pos > 0 && sl[pos - 1] == b) ? 1u : 0u;
            }
            uint32_t tot;
            const uint32_t ex = block_exscan_m(dup, scan_tmp, &tot);
            if (j < lb && !dup) {
                const uint32_t f = j + pos - (carry + ex);
                if (f < s) md.c[f] = b;
            }
            carry += tot;
        }
    }
    if (threadIdx.x == 0) {
        const uint32_t u = la + lb - dups_total;
        *md.clen = u < s ? u : s;
    }
}


// Merge rounds whose lists are known to be short (the threshold-bounded tile lists of long
// groups: ~2 * 16 * s / tiles hashes each in C5's first rounds): 256 threads per merge and a
// fixed 16 KiB of LDS instead of 1,024 threads and s * 8 bytes (80 KiB at s = 10,000, two
// merges per CU), so up to 8 merges share a CU.  A list longer than kSCap is searched in global
// memory instead (same results; the host's size estimate only steers speed).
#ifndef FPM_SBLOCK
#define FPM_SBLOCK 256
#endif
#ifndef FPM_SCAP
#define FPM_SCAP 2048
#endif
constexpr int kSBlock = FPM_SBLOCK, kSWaves = kSBlock / 64;
constexpr uint32_t kSCap = FPM_SCAP;
uint32_t merge_small_cap() { return kSCap; }

__device__ __forceinline__ uint32_t block_exscan_s(uint32_t v, uint32_t *tmp, uint32_t *total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kSWaves; w++) { const uint32_t t = tmp[w]; pre += w < wave ? t : 0u; tot += t; }
    __syncthreads();
    *total = tot;
    return pre + x - v;
}

__global__ __launch_bounds__(kSBlock) void merge_small_kernel(const MergeDesc *__restrict__ descs,
                                                              uint32_t s)
{
    __shared__ uint64_t sl[kSCap];
    __shared__ uint32_t scan_tmp[kSWaves];
    const MergeDesc md = descs[blockIdx.x];
    const uint32_t la = *md.alen, lb = md.b ? *md.blen : 0;
    const bool bfit = lb <= kSCap;
    if (bfit)
        for (uint32_t j = threadIdx.x; j < lb; j += kSBlock) sl[j] = md.b[j];
    __syncthreads();
    const uint64_t *Bv = bfit ? sl : md.b;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < la; c0 += kSBlock) {
        const uint32_t i = c0 + threadIdx.x;
        uint64_t a = 0;
        uint32_t pos = 0, dup = 0;
        if (i < la) {
            a = md.a[i];
            pos = lower_bound_u64(Bv, lb, a);
            dup = (pos < lb && Bv[pos] == a) ? 1u : 0u;
        }
        uint32_t tot;
        const uint32_t ex = block_exscan_s(dup, scan_tmp, &tot);
        if (i < la) {
            const uint32_t f = i + pos - (carry + ex);
            if (f < s) md.c[f] = a;
        }
        carry += tot;
    }
    const uint32_t dups_total = carry;
    if (lb) {
        const bool afit = la <= kSCap;
        __syncthreads();                               // every search of sl is done
        if (afit)
            for (uint32_t i = threadIdx.x; i < la; i += kSBlock) sl[i] = md.a[i];
        __syncthreads();
        const uint64_t *Av = afit ? sl : md.a;
        carry = 0;
        for (uint32_t c0 = 0; c0 < lb; c0 += kSBlock) {
            const uint32_t j = c0 + threadIdx.x;
            uint64_t b = 0;
            uint32_t pos = 0, dup = 0;
            if (j < lb) {
                b = md.b[j];
                pos = upper_bound_u64(Av, la, b);
                dup = (pos > 0 && Av[pos - 1] == b) ? 1u : 0u;
            }
            uint32_t tot;
            const uint32_t ex = block_exscan_s(dup, scan_tmp, &tot);
            if (j < lb && !dup) {
                const uint32_t f = j + pos - (carry + ex);
                if (f < s) md.c[f] = b;
            }
            carry += tot;
        }
    }
    if (threadIdx.x == 0) {
        const uint32_t u = la + lb - dups_total;
        *md.clen = u < s ? u : s;
    }
}

hipError_t launch_merge(const MergeDesc *d_desc, uint32_t n, uint32_t s, bool small,
                        hipStream_t st)
{
    if (n == 0) return hipSuccess;
    if (small) {
        hipLaunchKernelGGL(merge_small_kernel, dim3(n), dim3(kSBlock), 0, st, d_desc, s);
        return hipGetLastError();
    }
    // up to 128 KiB of staged list (s <= 16,384); beyond, the global-memory searches
    constexpr size_t kMaxLds = 128 * 1024;
    const size_t lds = (size_t)s * sizeof(uint64_t);
    if (lds <= kMaxLds &&
        hipFuncSetAttribute((const void *)merge_lds_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds) == hipSuccess) {
        hipLaunchKernelGGL(merge_lds_kernel, dim3(n), dim3(kMBlock), lds, st, d_desc, s);
        return hipGetLastError();
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(merge_kernel, dim3(n), dim3(kBlock), 0, st, d_desc, s);
    return hipGetLastError();
}

}  // namespace fpm
