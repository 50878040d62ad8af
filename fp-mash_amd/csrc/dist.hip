// dist.hip — all-pairs Mash distance for gfx950.
//
// compare_grid: the shared-hash walk of compareSketches (CommandDistance.cpp:
// 365-430), one lane per (ref, query) pair, executed literally so that sorted
// DNA sketches and the unsorted, duplicate-carrying -fp lists give the
// reference's exact (numer, denom).  Output order is query-major, ref-minor
// (the order CommandDistance::run chunks and writes pairs, :224-261, :276-333).
//
// dist_finalize: distance (:404-419) and p-value (pValue :433-450 with
// gsl_cdf_binomial_Q restated as I_r(x, n-x+1), GSL cdf/beta_inc.c's continued
// fraction) in FP64, plus the -d / -v pass filter.
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

// Floating-point expressions are evaluated as written, one rounding per operation: no
// multiply-add contraction (HIP's default contracts a*b + c into one FMA).  The reference's
// distance and GSL p-value arithmetic is x86-64 double code without FMA, and contracting here
// moved results by an ulp; where the p-value is ill-conditioned (k = 3, genome-sized lengths:
// the random-match probability r within 1e-7 of 1, so -log r keeps ~7 of its 16 digits) an ulp
// of r became 1e-11 relative in the p-value (test_pvalue_asymptotic_branches_on_device).
#pragma clang fp contract(off)

#include <cstdlib>

#include <float.h>

#include <algorithm>

namespace fpm {

constexpr int kTile = 16;   // 16 x 16 pairs per 256-lane workgroup
constexpr int kWalkBlk = 4;   // steps per LDS window of the u32 / u64 dense walk

// The literal walk of compareSketches for one pair (CommandDistance.cpp:376-400),
// with the remainder rule (:402-415).
template <typename H>
__device__ __forceinline__ void walk_pair(const H *__restrict__ A, uint32_t la,
                                          const H *__restrict__ B, uint32_t lb, uint32_t S,
                                          uint32_t &numer, uint32_t &denom)
{
    uint32_t i = 0, j = 0, common = 0, d = 0;
    H a = la ? A[0] : H(0), b = lb ? B[0] : H(0);
    while (d < S && i < la && j < lb) {
        const bool lt = a < b, gt = b < a;
        if (!gt) { i++; if (i < la) a = A[i]; }
        if (!lt) { j++; if (j < lb) b = B[j]; }
        common += (!lt && !gt) ? 1u : 0u;
        d++;
    }
    if (d < S) {
        uint64_t dd = (uint64_t)d + (la - i) + (lb - j);
        d = dd > S ? S : (uint32_t)dd;
    }
    numer = common;
    denom = d;
}

template <typename H, typename C>
__global__ __launch_bounds__(256) void compare_grid_kernel(
    const H *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const H *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t n_qry, uint32_t S, C *__restrict__ numer,
    C *__restrict__ denom)
{
    const uint32_t r = blockIdx.x * kTile + (threadIdx.x & (kTile - 1));
    const uint32_t q = blockIdx.y * kTile + (threadIdx.x / kTile);
    if (r >= n_ref || q >= n_qry) return;
    uint32_t c, d;
    walk_pair(ref + (uint64_t)r * ref_stride, ref_len[r], qry + (uint64_t)q * qry_stride,
              qry_len[q], S, c, d);
    const uint64_t o = (uint64_t)q * n_ref + r;
    numer[o] = (C)c;
    denom[o] = (C)d;
}

// per lane: bit lane of m ? y : x (one v_cndmask per dword)
__device__ __forceinline__ uint32_t lane_sel(uint32_t x, uint32_t y, uint64_t m)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "s"(m));
    return r;
}
__device__ __forceinline__ uint64_t lane_sel(uint64_t x, uint64_t y, uint64_t m)
{
    return ((uint64_t)lane_sel((uint32_t)(x >> 32), (uint32_t)(y >> 32), m) << 32) |
           lane_sel((uint32_t)x, (uint32_t)y, m);
}

// The same literal walk with the tile's 16 ref + 16 query lists staged in LDS (the first
// W = min(S, stride) entries of each: a walk of <= S steps never reads past index S - 1).
// Unsorted -fp lists (C3) take this path: every step is a compare and a data-dependent
// advance, so from global memory each step waited an L2 round trip; from LDS the next
// window of BLK entries of each list is loaded per block of BLK steps (below), so one LDS
// latency covers BLK steps.
// One wave per SIMD (up to 160 KB of lists per workgroup), one pair per lane: the walk's
// dependent VALU chain is not hidden by other waves, which bounds it (C3: 5,000 x 5,000 pairs
// of 2,000 u32 in ~35 ms, against 67 ms for the global-memory walk).
template <typename H, int BLK, typename C>
__global__ __launch_bounds__(256) void compare_grid_lds_kernel(
    const H *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const H *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t n_qry, uint32_t S, uint32_t W, C *__restrict__ numer,
    C *__restrict__ denom)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    H *lds = reinterpret_cast<H *>(smem);
    __shared__ uint32_t cnt[2 * kTile];
    const uint32_t Wp = (W + BLK + 3) & ~3u;   // 16-B rows; a block's window reads past W stay in the slot
    const uint32_t r0 = blockIdx.x * kTile, q0 = blockIdx.y * kTile;
    if (threadIdx.x < 2 * kTile) {
        const uint32_t l = threadIdx.x, isq = l >= (uint32_t)kTile, row = (isq ? q0 : r0) + (l & (kTile - 1));
        uint32_t c = 0;
        if (row < (isq ? n_qry : n_ref)) c = isq ? qry_len[row] : ref_len[row];
        cnt[l] = c < W ? c : W;
    }
    __syncthreads();
    // staging: wave w copies lists w, w+4, ..., w+28 with 16-B loads, every load of the wave
    // issued before the first LDS store (one memory latency per workgroup); rows that are
    // not 16-B aligned take the element loop
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr uint32_t kV = 16 / sizeof(H);                  // entries per 16-B vector
    constexpr int kL = 2 * kTile / 4;                         // lists per wave
    const bool vec = ((ref_stride * sizeof(H)) & 15) == 0 && ((qry_stride * sizeof(H)) & 15) == 0 &&
                     (((uintptr_t)ref | (uintptr_t)qry) & 15) == 0;
    if (vec) {
        // each list: ceil(W / kV) vectors, lane t takes vectors t, t + 64, ...
        const uint32_t nvec = (W + kV - 1) / kV;
        for (uint32_t v0 = 0; v0 < nvec; v0 += 64 * 2) {
            uint4 buf[kL][2];
#pragma unroll
            for (int li = 0; li < kL; li++) {
                const uint32_t l = wave + 4 * li, isq = l >= (uint32_t)kTile;
                const uint32_t row = (isq ? q0 : r0) + (l & (kTile - 1));
                const uint32_t c = cnt[l];
                const H *src = isq ? qry + (uint64_t)row * qry_stride : ref + (uint64_t)row * ref_stride;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t vi = v0 + h * 64 + lane;
                    buf[li][h] = make_uint4(0, 0, 0, 0);
                    if ((vi + 1) * kV <= c) buf[li][h] = *(const uint4 *)(src + (uint64_t)vi * kV);
                }
            }
#pragma unroll
            for (int li = 0; li < kL; li++) {
                const uint32_t l = wave + 4 * li, isq = l >= (uint32_t)kTile;
                const uint32_t row = (isq ? q0 : r0) + (l & (kTile - 1));
                const uint32_t c = cnt[l];
                const H *src = isq ? qry + (uint64_t)row * qry_stride : ref + (uint64_t)row * ref_stride;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint32_t vi = v0 + h * 64 + lane;
                    if ((vi + 1) * kV <= c) {
                        *(uint4 *)(lds + l * Wp + vi * kV) = buf[li][h];
                    } else if (vi * kV < c) {          // the list's ragged last vector
                        for (uint32_t e = vi * kV; e < c; e++) lds[l * Wp + e] = src[e];
                    }
                }
            }
        }
    } else {
        for (uint32_t l = wave; l < 2 * kTile; l += 4) {
            const uint32_t isq = l >= (uint32_t)kTile, row = (isq ? q0 : r0) + (l & (kTile - 1));
            const H *src = isq ? qry + (uint64_t)row * qry_stride : ref + (uint64_t)row * ref_stride;
            for (uint32_t e = lane; e < cnt[l]; e += 64) lds[l * Wp + e] = src[e];
        }
    }
    __syncthreads();
    const uint32_t r = r0 + (threadIdx.x & (kTile - 1)), q = q0 + (threadIdx.x / kTile);
    if (r >= n_ref || q >= n_qry) return;
    const uint32_t la = ref_len[r], lb = qry_len[q];
    const H *A = lds + (threadIdx.x & (kTile - 1)) * Wp;
    const H *B = lds + (kTile + threadIdx.x / kTile) * Wp;
    // Blocks of BLK steps: a block reads A[i .. i+BLK) and B[j .. j+BLK) into registers with
    // independent LDS loads (one latency per block), then walks BLK steps in registers, each
    // advance shifting its window down by one (before step u at most u advances happened, so
    // the window holds the current head).  The trip count is uniform: a lane that has left
    // the walk (i = la or j = lb) only stops advancing; entries past min(len, W) are read but
    // never compared.
    uint32_t i = 0, j = 0, common = 0, d = 0;
    for (uint32_t d0 = 0; d0 < S; d0 += BLK) {
        if (!__any((i < la) & (j < lb))) break;
        H a[BLK], b[BLK];
#pragma unroll
        for (int u = 0; u < BLK; u++) {
            a[u] = A[i + u];
            b[u] = B[j + u];
        }
#pragma unroll
        for (int u = 0; u < BLK; u++) {
            const bool act = (d0 + u < S) & (i < la) & (j < lb);
            const bool lt = a[0] < b[0], gt = b[0] < a[0];
            const bool adv_a = act & !gt, adv_b = act & !lt;
            d += act ? 1u : 0u;
            i += adv_a ? 1u : 0u;
            j += adv_b ? 1u : 0u;
            // the shifts as explicit v_cndmask on the advance lane masks: written as
            // selects, the compiler re-derived every head as a compare-select chain over
            // the advance count (~4x the VALU)
            const uint64_t ma = __builtin_amdgcn_ballot_w64(adv_a), mb = __builtin_amdgcn_ballot_w64(adv_b);
#pragma unroll
            for (int v = 0; v + 1 < BLK - u; v++) {
                a[v] = lane_sel(a[v], a[v + 1], ma);
                b[v] = lane_sel(b[v], b[v + 1], mb);
            }
        }
    }
    // every active step advanced i, j or both (both exactly on an equal pair): the equal
    // pairs come from the step count instead of a per-step count
    common = i + j - d;
    if (d < S) {
        uint64_t dd = (uint64_t)d + (la - i) + (lb - j);
        d = dd > S ? S : (uint32_t)dd;
    }
    const uint64_t o = (uint64_t)q * n_ref + r;
    numer[o] = (C)common;
    denom[o] = (C)d;
}

// The literal walk restricted to its tie stretches (unsorted lists; the record filter in
// dist_index.hip).  Every equal step happens where both running maxima equal one shared record
// value v; the walk enters that stretch exactly at (pA(v), pB(v)), the records' positions:
// every earlier entry of either list has a running maximum below v, so it is taken before
// the other list's v (KA(i) < KB(j) implies A[i] < B[j] at a reached state), and the walk
// cannot pass v in one list while the other is short of it.  Entering takes
// pA + pB - (equal steps so far) steps.  The stretch ends when either list reaches its next
// record (a value above v: no equal step until the next shared record).  So the shared
// records are merged in increasing order and only their stretches are walked literally;
// denom = min(S, la + lb - common), the reference's steps + remainders (:402-415).
template <typename H>
__device__ __forceinline__ void walk_pair_rec(const H *__restrict__ A, uint32_t la,
                                              const H *__restrict__ B, uint32_t lb, uint32_t S,
                                              const H *__restrict__ RA, const uint32_t *__restrict__ PA,
                                              uint32_t na, const H *__restrict__ RB,
                                              const uint32_t *__restrict__ PB, uint32_t nb,
                                              uint32_t &numer, uint32_t &denom)
{
    uint32_t common = 0, x = 0, y = 0;
    H ra = na ? RA[0] : H(0), rb = nb ? RB[0] : H(0);
    while (x < na && y < nb) {
        if (ra < rb) { if (++x < na) ra = RA[x]; continue; }
        if (rb < ra) { if (++y < nb) rb = RB[y]; continue; }
        uint32_t i = PA[x], j = PB[y];
        uint32_t n = i + j - common;
        if (n >= S) break;
        // (the last stretch ends at min(len, S): no step reads past entry S - 1)
        const uint32_t ea = x + 1 < na ? PA[x + 1] : min(la, S);
        const uint32_t eb = y + 1 < nb ? PB[y + 1] : min(lb, S);
        // (branch-free steps reloading both heads every step: 1.47 -> 1.59 ms on C3)
        H a = A[i], b = B[j];
        while (i < ea && j < eb && n < S) {
            const bool lt = a < b, gt = b < a;
            if (!gt) { i++; if (i < ea) a = A[i]; }
            if (!lt) { j++; if (j < eb) b = B[j]; }
            common += (!lt && !gt) ? 1u : 0u;
            n++;
        }
        if (++x < na) ra = RA[x];
        if (++y < nb) rb = RB[y];
    }
    numer = common;
    const uint64_t dd = (uint64_t)la + lb - common;
    denom = dd > S ? S : (uint32_t)dd;
}

// Walk only the candidate pairs found by the inverted index (dist_index.hip).
template <typename H, typename C>
__global__ __launch_bounds__(256) void walk_cand_kernel(
    const uint64_t *__restrict__ cand, const unsigned long long *__restrict__ n_cand,
    const H *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const H *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t S, RecRows rr, RecRows rq, C *__restrict__ numer,
    C *__restrict__ denom)
{
    const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= *n_cand) return;
    const uint64_t o = cand[idx];
    const uint32_t q = (uint32_t)(o / n_ref), r = (uint32_t)(o % n_ref);
    uint32_t c, d;
    const H *A = ref + (uint64_t)r * ref_stride, *B = qry + (uint64_t)q * qry_stride;
    if (A == B && ref_len[r] == qry_len[q]) {
        // a list against itself (the diagonal of a set against itself): every step is an
        // equal pair, so the walk's S steps (the longest in its wave) come out as
        // common = min(l, S), denom = min(S, 2 l - common).  C3: 3.0 -> 2.25 ms; loading the
        // stretches 4 entries at a time instead measured no change (3.04 vs 2.9-3.0 ms, r04e)
        const uint32_t l = ref_len[r];
        c = l < S ? l : S;
        const uint64_t dd = 2ull * l - c;
        d = dd > S ? S : (uint32_t)dd;
    } else if (rr.val)
        walk_pair_rec(ref + (uint64_t)r * ref_stride, ref_len[r], qry + (uint64_t)q * qry_stride,
                      qry_len[q], S, (const H *)rr.val + (uint64_t)r * rr.stride,
                      rr.pos + (uint64_t)r * rr.stride, rr.len[r],
                      (const H *)rq.val + (uint64_t)q * rq.stride, rq.pos + (uint64_t)q * rq.stride,
                      rq.len[q], c, d);
    else
        walk_pair(ref + (uint64_t)r * ref_stride, ref_len[r], qry + (uint64_t)q * qry_stride,
                  qry_len[q], S, c, d);
    numer[o] = (C)c;
    denom[o] = (C)d;
}

// Sorted, distinct lists (every sketch the k-mer path produces): the walk of
// compareSketches (CommandDistance.cpp:365-398) is a merge of two sets and visits the
// union elements in ascending order, so with U(c) = the union rank of value c
//   numer = #{shared c : U(c) < S},   denom = min(S, |A| + |B| - #shared).
// For A[i] = c with j = #{B < c} and k = #{shared values below c}: U(c) = i + j - k.
//
// Rank kernel, one workgroup per query row B, one wave per candidate ref row A:
//  * B is staged once in LDS with a bucket directory over its value range (bucket = value
//    >> shift, ~8 buckets per B element for CAP 1024): Bkt[b] = #{B < b << shift}, u16.
//  * lane l takes A[64t + l] (coalesced 512-byte buffer loads, prefetched one candidate
//    ahead into registers).  j = #{B < a} and the equality test come from NP independent
//    LDS reads Bs[lo .. lo + NP) at lo = Bkt[a >> shift]: NP = the row's largest bucket
//    (2-4 for hash values), so every element of a's bucket is read; positions past the
//    bucket hold larger values (later buckets, or the ~0 sentinels past the end), so
//    j = lo + #{reads < a} and eq = any(read == a) need no bucket-end test.  No dependent
//    search chain: one directory read, then NP reads in flight together.  Rows with a
//    bucket past kRankProbeMax (or a ~0 value, which equals the sentinel) take a bounded
//    binary search inside the bucket instead.
//  * k is a running ballot count: popc of this chunk's shared lanes below l + earlier chunks.
//  * when max(|A|, |B|) >= S, denom is S whatever #shared is, and no A element after the
//    first one whose union rank reaches S can count: the wave stops there (about half of A
//    for unrelated pairs).
constexpr int kRankWaves = 4;        // waves per query row (2 and 8 measured slower)
constexpr int kRankProbeMax = 8;     // sentinels past the end of B = the widest unrolled probe
constexpr uint32_t kRankLogB = 12;   // log2 buckets for CAP 1024 (CAP 2048: one more)
                                     // (11: 4 KB less LDS, 8 workgroups per CU instead of 7,
                                     // but larger buckets: 0.346 -> 0.383 ms; 13: 0.345 ->
                                     // 0.365 ms, same box, r04.  A CAP = 1000 instance,
                                     // 20.3 KB of LDS: 8 workgroups per CU at 12 bits, rank
                                     // 0.347 either way, same box, r04)

// One chunk of 64 A elements against B (one per lane): j = #{B < a} and the lanes whose a
// is in B (a wave mask).
// NP > 0 (the fast path): B's values have distinct 32-bit keys K32 = the top 32 bits of the
// row's value window (v >> max(bits - 32, 0)), which order them exactly, and the bucket of
// a value is the top kLogB bits of its key.  The NP reads K32[lo .. lo + NP) at lo =
// Bkt[bucket(a)] cover a's whole bucket (NP >= the row's largest bucket); later positions
// hold larger keys (next buckets, or the 0xFFFFFFFF sentinels past the end), so
// p = lo + #{keys < key(a)} is the first position whose value is not below a on the key,
// and one 64-bit read of Bs[p] settles the rest: j = p + (Bs[p] < a), eq = (Bs[p] == a).
// A value past the last B value's bucket `top` clamps to bucket top + 1 (lo = lb, the
// sentinels): j = lb.
// NP = 0 (any row): 64-bit reads over the row's largest bucket (maxn), every position
// clamped to the sentinel and tested against lb.
// HI (rows whose bucket shift is >= 32: values of >= 32 + log2(buckets) bits, every 64-bit
// hash sketch; a k = 21 bottom-s row holds values up to ~2^63): the key is a's high dword and
// the bucket a 32-bit shift of it clamped to the directory's end (filled with lb up to
// kBuckets), instead of two 64-bit shifts, a 64-bit compare and a select per value.  The high
// dwords of a row with fewer than 64 bits are still distinct in practice (a row where two
// are not takes the NP = 0 loop).
template <int NP, bool HI = false>
__device__ __forceinline__ uint64_t rank_chunk(const uint64_t *Bs, const uint32_t *K32,
                                               const uint16_t *Bkt, uint32_t shift,
                                               uint32_t kshift, uint32_t top, uint32_t lb,
                                               uint32_t maxn, uint32_t kb, uint64_t a, uint32_t &j)
{
    bool over;
    uint32_t lo;
    if constexpr (HI) {
        // the directory past top holds lb (the sentinels) up to Bkt[kBuckets]
        over = false;
        lo = Bkt[min((uint32_t)(a >> 32) >> (shift - 32), kb)];
    } else {
        const uint64_t t = a >> shift;
        over = t > (uint64_t)top;
        lo = Bkt[over ? top + 1 : (uint32_t)t];
    }
    if constexpr (NP > 0) {
        const uint32_t ka = HI ? (uint32_t)(a >> 32) : (uint32_t)(a >> kshift);
        uint32_t p = lo;
#pragma unroll
        for (int q = 0; q < NP; q++) p += K32[lo + q] < ka ? 1u : 0u;
        const uint64_t v = Bs[p];
        j = p + (v < a ? 1u : 0u);
        if constexpr (HI) return __builtin_amdgcn_ballot_w64(v == a);
        return __builtin_amdgcn_ballot_w64(v == a) & ~__builtin_amdgcn_ballot_w64(over);
    } else {
        uint32_t jj = lo;
        uint64_t eqm = 0;
        for (uint32_t q = 0; q < maxn; q++) {
            const uint32_t p = min(lo + q, lb);
            const uint64_t v = Bs[p];
            jj += ((v < a) & (p < lb)) ? 1u : 0u;
            eqm |= __builtin_amdgcn_ballot_w64((v == a) & (p < lb));
        }
        j = jj;
        return eqm;
    }
}

template <int CAP, typename C>
__global__ __launch_bounds__(64 * kRankWaves) void rank_rows_kernel(
    const uint64_t *__restrict__ cand, const uint64_t *__restrict__ row_seg, uint32_t n_qry,
    uint32_t q_lo, const uint64_t *__restrict__ ref, const uint32_t *__restrict__ ref_len,
    uint64_t ref_stride, uint32_t n_ref, const uint64_t *__restrict__ qry,
    const uint32_t *__restrict__ qry_len, uint64_t qry_stride, uint32_t S, uint32_t sym,
    C *__restrict__ numer, C *__restrict__ denom, uint32_t *__restrict__ cnum,
    uint32_t *__restrict__ cden)
{
    constexpr uint32_t kLogBuckets = (CAP <= 1024) ? kRankLogB : kRankLogB + 1;
    constexpr uint32_t kBuckets = 1u << kLogBuckets;
    // fixed-size LDS arrays: their compile-time offsets fold into the ds_read instructions.
    // (Sizing them by the launch instead — 20.3 KB at s = 1000, 8 workgroups per CU — put a
    // runtime base add on every probe read: the kernel ran 0.645 -> 0.70 ms beside the fill
    // at 6, 7 or 8 workgroups per CU alike, same-box A/B r03o.)
    // one block with the keys first: the NP key reads K32[lo + q] are ds_read2_b32 pairs
    // whose 8-bit dword offsets then hold q (the allocator put K32 after Bs and Bkt, at
    // 16 KB: one address add per key read)
    __shared__ struct {
        uint32_t k[CAP + kRankProbeMax];
        uint64_t v[CAP + kRankProbeMax];
    } sKB;
    uint32_t *const K32 = sKB.k;
    uint64_t *const Bs = sKB.v;
    __shared__ uint16_t Bkt[kBuckets + 1];             // Bkt[b] = #{B < b << shift}
    __shared__ uint32_t s_maxn, s_keydup, s_unsorted;
    // rows [q_lo, q_lo + n_qry) of the grid (a part of the rows, whose probe ran before)
    const uint32_t qr = xcd_row(blockIdx.x, n_qry);
    if (qr >= n_qry) return;
    const uint32_t q = q_lo + qr;
    const uint64_t seg = row_seg[q];
    const uint32_t n = (uint32_t)(seg & 0xFFFFFF);
    if (n == 0) return;
    const uint64_t base = seg >> 24;
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lb = qry_len[q];
    const uint64_t *B = qry + (uint64_t)q * qry_stride;
    if (threadIdx.x == 0) { s_maxn = 0; s_keydup = 0; s_unsorted = 0; }
    {
        // stage B: every load of the row issued before the first LDS store (4 in flight per
        // thread: CAP / 256 with CAP 1024; a serial load-store loop paid the global latency
        // once per value)
        constexpr int kStage = (CAP + 64 * kRankWaves - 1) / (64 * kRankWaves);
        uint64_t v[kStage];
#pragma unroll
        for (int u = 0; u < kStage; u++) {
            const uint32_t t = threadIdx.x + u * 64 * kRankWaves;
            v[u] = t < lb ? B[t] : 0;
        }
#pragma unroll
        for (int u = 0; u < kStage; u++) {
            const uint32_t t = threadIdx.x + u * 64 * kRankWaves;
            if (t < lb) Bs[t] = v[u];
        }
    }
    // sentinels past the end: no A value is below them
    if (threadIdx.x < kRankProbeMax) {
        Bs[lb + threadIdx.x] = ~0ULL;
        K32[lb + threadIdx.x] = 0xFFFFFFFFu;
    }
    __syncthreads();
    const uint64_t bmax = lb ? Bs[lb - 1] : 0;
    const uint32_t bits = bmax ? 64 - __clzll(bmax) : 0;
    const uint32_t shift = bits > kLogBuckets ? bits - kLogBuckets : 0;
    // HI rows (shift >= 32): the keys are the values' high dwords
    const uint32_t kshift = shift >= 32 ? 32 : bits > 32 ? bits - 32 : 0;
    // top = the last B value's bucket; the directory stops at Bkt[top + 1] = lb (filling
    // every bucket up to kBuckets cost one thread up to kBuckets / 2 serial stores)
    const uint32_t top = (uint32_t)(bmax >> shift);
    // keys (distinct and below the sentinel for the fast path, else the row takes NP = 0)
    // and the bucket directory: bucket b = values [b << shift, (b + 1) << shift) = B
    // positions [Bkt[b], Bkt[b + 1]).  Element j owns the buckets after its predecessor's
    // bucket up to its own, so each thread fills one gap.
    uint32_t dup = 0, uns = 0;
    for (uint32_t j = threadIdx.x; j <= lb; j += blockDim.x) {
        const uint64_t v = j < lb ? Bs[j] : 0, vp = j > 0 ? Bs[j - 1] : 0;
        if (j < lb) {
            const uint32_t k = (uint32_t)(v >> kshift);
            K32[j] = k;
            dup |= (j > 0 && (uint32_t)(vp >> kshift) == k) | (k == 0xFFFFFFFFu);
            uns |= j > 0 && !(vp < v);
        }
        const uint32_t bj = j < lb ? (uint32_t)(v >> shift) : top + 1;
        const uint32_t bp = j > 0 ? (uint32_t)(vp >> shift) + 1 : 0;
        for (uint32_t b = bp; b <= bj; b++) Bkt[b] = (uint16_t)j;
    }
    // the directory past top + 1 (HI rows read it unclamped; top >= 2^(kLogBuckets - 1))
    for (uint32_t b = top + 2 + threadIdx.x; b <= kBuckets; b += blockDim.x) Bkt[b] = (uint16_t)lb;
    if (dup) s_keydup = 1;
    if (uns) s_unsorted = 1;
    __syncthreads();
    // a row that is not strictly ascending (a rank kernel enqueued before the probe's
    // sortedness flag was read, fpm_api.cpp; its results are then dropped): nothing to rank,
    // and its directory would not bound the bucket loop below
    if (s_unsorted) return;
    // the largest bucket: element j is the (j - Bkt[bucket(j)] + 1)-th of its bucket
    uint32_t mx = 0;
    for (uint32_t j = threadIdx.x; j < lb; j += blockDim.x)
        mx = max(mx, j + 1 - (uint32_t)Bkt[(uint32_t)(Bs[j] >> shift)]);
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
    if (lane == 0 && mx) atomicMax(&s_maxn, mx);
    __syncthreads();
    const uint32_t maxn = s_maxn;
    // probe width (row-uniform): unrolled reads for buckets of up to 2 / 3 / 4 / 8 values;
    // 0 = the clamped loop (a crowded bucket, or keys that do not order the row)
    // (two keys per value with a rare one-key-at-a-time continuation past them measured
    // slower: 0.346 -> 0.372 ms, the wave-wide test of the continuation costs more than the
    // second ds_read2 it saves)
    const uint32_t np = s_keydup ? 0u
                      : maxn <= 2 ? 2u : maxn <= 3 ? 3u : maxn <= 4 ? 4u
                      : maxn <= (uint32_t)kRankProbeMax ? (uint32_t)kRankProbeMax : 0u;

    const uint32_t ld = ref_stride < (uint64_t)CAP ? (uint32_t)ref_stride : (uint32_t)CAP;
    const uint64_t pair_row = (uint64_t)q * n_ref;
    // A rows are read in chunks of 128 values, two 8-B loads per lane (lane l holds A[i0 + l]
    // and A[i0 + 64 + l]: neighbouring lanes then probe neighbouring directory words and keys
    // of B, about half the LDS bank conflicts of one 16-B load of A[i0 + 2l], A[i0 + 2l + 1]
    // per lane: rank kernel 0.415 -> 0.405 ms, C2 step 1.051 -> 1.042 ms, same box, r04c), in
    // groups of kGroup chunks through a bounds-checked buffer descriptor (reads past ld
    // return 0).
    // Three register groups: `cur` (being ranked), `nxt` (this candidate's next group,
    // issued before `cur` is ranked) and `pf` (the next candidate's first group, issued when
    // a candidate starts); the groups after an early exit are never loaded.
    constexpr int kGroup = 1;      // chunks per load group (2 and 4 measured slower)
    constexpr uint32_t kChunk = 128;
    struct Row { __amdgpu_buffer_rsrc_t rsrc; uint32_t la; uint64_t o; };
    auto open_row = [&](uint64_t o) -> Row {
        const uint32_t rr = __builtin_amdgcn_readfirstlane((uint32_t)(o - pair_row));
        const uintptr_t Ar = (uintptr_t)(ref + (uint64_t)rr * ref_stride);
        const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)Ar);
        const uint32_t phi = __builtin_amdgcn_readfirstlane((uint32_t)(Ar >> 32));
        Row R;
        R.rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)(((uintptr_t)phi << 32) | plo), 0,
                                                   (int)__builtin_amdgcn_readfirstlane(ld * 8u),
                                                   0x00020000);
        R.la = ref_len[rr];
        R.o = o;
        return R;
    };
    struct Pair { uint64_t e0, e1; };
    auto load_group = [&](const Row &R, uint32_t gi, Pair (&dst)[kGroup]) {
#pragma unroll
        for (int u = 0; u < kGroup; u++) {
            const uint32_t t = gi * kGroup + u;
            const auto v0 = __builtin_amdgcn_raw_buffer_load_b64(R.rsrc, (t * kChunk + lane) * 8u, 0, 0);
            const auto v1 = __builtin_amdgcn_raw_buffer_load_b64(R.rsrc, (t * kChunk + 64 + lane) * 8u,
                                                                 0, 0);
            dst[u].e0 = ((uint64_t)v0[1] << 32) | v0[0];
            dst[u].e1 = ((uint64_t)v1[1] << 32) | v1[0];
        }
    };
    auto cand_at = [&](uint32_t cc) -> uint64_t {
        return cand[base + __builtin_amdgcn_readfirstlane(cc)];
    };
    // one chunk (kGroup = 1): shared-hash count below the union rank S (cnt), shared values
    // so far (shared_below); returns the union rank of the chunk's largest value (full chunks)
    // vm0 / vm1: the lanes whose e0 / e1 are values of the row (all of them but in a row's
    // last chunk, whose masks the candidate loop computes once)
    // Union ranks increase with the value, so a full chunk whose largest value (lane 63's e1)
    // ranks below S counts every shared value it holds: that rank comes from one lane's j and
    // scalar popcounts, and the per-lane ranks (mbcnt, the u < S ballots) are only computed for
    // the chunk that crosses S and for the row's last chunk.
    auto rank_group = [&](auto probe, uint32_t g0, bool last, uint64_t vm0, uint64_t vm1,
                          const Pair (&cur)[kGroup], uint32_t &shared_below,
                          uint32_t &cnt) -> uint32_t {
        uint32_t j0, j1;
        const uint64_t m0 = probe(cur[0].e0, j0);
        const uint64_t m1 = probe(cur[0].e1, j1);
        const uint32_t i0 = g0 * kChunk;
        const uint64_t a0 = m0 & vm0, a1 = m1 & vm1;
        const uint32_t p0 = (uint32_t)__popcll(a0), p1 = (uint32_t)__popcll(a1);
        uint32_t u_last = 0;
        if (!last) {
            const uint32_t jl = (uint32_t)__builtin_amdgcn_readlane((int)j1, 63);
            u_last = i0 + (kChunk - 1) + jl -
                     (shared_below + p0 + (uint32_t)__popcll(a1 & 0x7FFFFFFFFFFFFFFFULL));
        }
        if (!last && u_last < S) {
            cnt += p0 + p1;
        } else {
            const uint32_t b0 = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(a0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)a0, 0u));
            const uint32_t b1 = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(a1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)a1, 0u));
            const uint32_t k0 = shared_below + b0;
            const uint32_t k1 = shared_below + p0 + b1;
            const uint32_t u0 = i0 + lane + j0 - k0, u1 = i0 + 64 + lane + j1 - k1;
            cnt += __popcll(a0 & __builtin_amdgcn_ballot_w64(u0 < S)) +
                   __popcll(a1 & __builtin_amdgcn_ballot_w64(u1 < S));
        }
        shared_below += p0 + p1;
        return u_last;
    };
    auto run = [&](auto probe, bool fast) {
        Pair cur[kGroup], nxt[kGroup], pf[kGroup];
        Row Rc{};
        if (wave < n) { Rc = open_row(cand_at(wave)); load_group(Rc, 0, pf); }
        for (uint32_t c = wave; c < n; c += kRankWaves) {
            const Row R = Rc;
#pragma unroll
            for (int u = 0; u < kGroup; u++) cur[u] = pf[u];
            if (c + kRankWaves < n) { Rc = open_row(cand_at(c + kRankWaves)); load_group(Rc, 0, pf); }
            const uint32_t la = R.la;
            const uint64_t o = R.o;
            const bool need_all = la < S && lb < S;       // denom depends on #shared
            const uint32_t nch = (la + kChunk - 1) / kChunk;
            const uint32_t ngr = (nch + kGroup - 1) / kGroup;
            static_assert(kGroup == 1, "the last-chunk masks assume one chunk per group");
            // values past la (row padding) count nothing: in the last chunk (lane l holds
            // A[i0 + l], A[i0 + 64 + l]) the lanes below r0 / r1 hold row values.  Computed once
            // per candidate, selected per chunk (computed in the chunk loop they cost ~20 scalar
            // instructions per chunk: the compiler turns a branch around them into selects)
            const int rl = (int)la - (int)(nch - 1) * (int)kChunk;          // 1 .. 128
            const int r0 = min(rl, 64), r1 = rl - 64;
            const uint64_t vl0 = r0 >= 64 ? ~0ULL : r0 > 0 ? (1ULL << r0) - 1 : 0ULL;
            const uint64_t vl1 = r1 >= 64 ? ~0ULL : r1 > 0 ? (1ULL << r1) - 1 : 0ULL;
            uint32_t shared_below = 0, cnt = 0;
            // the early exit: after a chunk whose last value's union rank reaches S no later
            // value can count (need_all: the denom needs every shared value, no exit)
            const uint32_t s_exit = need_all ? 0xFFFFFFFFu : S;
            // the full chunks, then the row's last chunk with its masks (peeled: the loop
            // carries no per-chunk mask selects).  (Chunks loaded two ahead instead of one:
            // 0.345 -> 0.375 ms.)
            bool exited = false;
            uint32_t gi = 0;
            for (; gi + 1 < ngr; gi++) {
                load_group(R, gi + 1, nxt);
                const uint32_t u_last = rank_group(probe, gi * kGroup, false, ~0ULL, ~0ULL, cur,
                                                   shared_below, cnt);
                if (u_last >= s_exit) { exited = true; break; }
#pragma unroll
                for (int u = 0; u < kGroup; u++) cur[u] = nxt[u];
            }
            if (!exited && ngr) {
                // fast-path rows: B holds no ~0 value (its key would equal the sentinel's), and
                // an A value ~0 (only ever A's last) would match the sentinel: not shared
                const uint64_t x0 = fast ? __builtin_amdgcn_ballot_w64(cur[0].e0 == ~0ULL) : 0;
                const uint64_t x1 = fast ? __builtin_amdgcn_ballot_w64(cur[0].e1 == ~0ULL) : 0;
                rank_group(probe, gi * kGroup, true, vl0 & ~x0, vl1 & ~x1, cur, shared_below, cnt);
            }
            if (lane == 0) {
                const uint64_t un = (uint64_t)la + lb - shared_below;
                const uint32_t dn = need_all ? (un < S ? (uint32_t)un : S) : S;
                if (cnum) {      // compact: the candidate finalize scatters (and mirrors)
                    cnum[base + c] = cnt;
                    cden[base + c] = dn;
                    continue;
                }
                numer[o] = (C)cnt;
                denom[o] = (C)dn;
                const uint32_t r = (uint32_t)(o - pair_row);
                if (sym && r != q) {                      // mirror cell (r, q)
                    const uint64_t o2 = (uint64_t)r * n_ref + q;
                    numer[o2] = (C)cnt;
                    denom[o2] = (C)dn;
                }
            }
        }
    };
    const uint16_t *bk_ = Bkt;
    const uint64_t *bs_ = Bs;
    const uint32_t *k_ = K32;
#define FPM_RANK_NP(NP_, HI_) \
    run([&](uint64_t a, uint32_t &j) { \
        return rank_chunk<NP_, HI_>(bs_, k_, bk_, shift, kshift, top, lb, maxn, kBuckets, a, j); }, NP_ > 0)
    const bool hi = shift >= 32;    // bits >= 32 + kLogBuckets (then kshift = 32)
    switch (np) {
    case 2: if (hi) FPM_RANK_NP(2, true); else FPM_RANK_NP(2, false); break;
    case 3: if (hi) FPM_RANK_NP(3, true); else FPM_RANK_NP(3, false); break;
    case 4: if (hi) FPM_RANK_NP(4, true); else FPM_RANK_NP(4, false); break;
    case kRankProbeMax: FPM_RANK_NP(kRankProbeMax, false); break;
    default: FPM_RANK_NP(0, false); break;
    }
#undef FPM_RANK_NP
}

template <typename C>
static hipError_t merge_rows_c(const uint64_t *d_cand, const uint64_t *row_seg, uint32_t n_qry,
                               const uint64_t *d_ref, const uint32_t *d_ref_len,
                               uint64_t ref_stride, uint32_t n_ref, const uint64_t *d_qry,
                               const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t S,
                               bool sym, C *d_numer, C *d_denom, uint32_t *d_cnum,
                               uint32_t *d_cden, hipStream_t st, uint32_t q_lo)
{
    const dim3 g(xcd_grid(n_qry)), b(64 * kRankWaves);
    const uint64_t cap = std::max(ref_stride, qry_stride);
    if (cap <= 1024)
        hipLaunchKernelGGL((rank_rows_kernel<1024, C>), g, b, 0, st, d_cand, row_seg, n_qry, q_lo,
                           d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len, qry_stride, S,
                           (uint32_t)sym, d_numer, d_denom, d_cnum, d_cden);
    else if (cap <= 2048)
        hipLaunchKernelGGL((rank_rows_kernel<2048, C>), g, b, 0, st, d_cand, row_seg, n_qry, q_lo,
                           d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len, qry_stride, S,
                           (uint32_t)sym, d_numer, d_denom, d_cnum, d_cden);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_merge_rows(const uint64_t *d_cand, const uint64_t *row_seg, uint32_t n_qry,
                             const uint64_t *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                             uint32_t n_ref, const uint64_t *d_qry, const uint32_t *d_qry_len,
                             uint64_t qry_stride, uint32_t S, bool sym, Counts cnt,
                             uint32_t *d_cnum, uint32_t *d_cden, hipStream_t st, uint32_t q_lo)
{
    if (!n_qry) return hipSuccess;
    if (cnt.c16)
        return merge_rows_c(d_cand, row_seg, n_qry, d_ref, d_ref_len, ref_stride, n_ref, d_qry,
                            d_qry_len, qry_stride, S, sym, (uint16_t *)cnt.numer,
                            (uint16_t *)cnt.denom, d_cnum, d_cden, st, q_lo);
    return merge_rows_c(d_cand, row_seg, n_qry, d_ref, d_ref_len, ref_stride, n_ref, d_qry,
                        d_qry_len, qry_stride, S, sym, (uint32_t *)cnt.numer,
                        (uint32_t *)cnt.denom, d_cnum, d_cden, st, q_lo);
}

// ---- FP64 p-value (same algorithm as the oracle restatement)

__device__ double lngs_large(double x)
{
    double x2 = 1.0 / (x * x);
    double s = (1.0 / 12.0) - x2 * ((1.0 / 360.0) - x2 * ((1.0 / 1260.0) - x2 * ((1.0 / 1680.0)
               - x2 * ((1.0 / 1188.0) - x2 * ((691.0 / 360360.0) - x2 * (1.0 / 156.0))))));
    return s / x;
}

__device__ double lngammastar(double x)
{
    if (x >= 10.0) return lngs_large(x);
    double n = ceil(10.0 - x), y = x + n, prod = 1.0;
    for (double t = x; t < y - 0.5; t += 1.0) prod *= t;
    double lg = lngs_large(y) + (y - 0.5) * log(y) - y - log(prod);
    return lg - ((x - 0.5) * log(x) - x);
}

__device__ double lnbeta(double a, double b)
{
    double s = a + b;
    double t = -(a - 0.5) * log1p(b / a) - (b - 0.5) * log1p(a / b) - 0.5 * log(s);
    return lngammastar(a) + lngammastar(b) - lngammastar(s) + 0.91893853320467274178 + t;
}

__device__ double beta_cf(double a, double b, double x, double epsabs)
{
    const double cutoff = 2.0 * DBL_MIN;
    unsigned it = 0;
    double num = 1.0, den = 1.0 - (a + b) * x / (a + 1.0);
    if (fabs(den) < cutoff) den = __builtin_nan("");
    den = 1.0 / den;
    double cf = den;
    while (it < 512) {
        const int k = (int)it + 1;
        double coeff = k * (b - k) * x / (((a - 1.0) + 2 * k) * (a + 2 * k));
        den = 1.0 + coeff * den;
        num = 1.0 + coeff / num;
        if (fabs(den) < cutoff) den = __builtin_nan("");
        if (fabs(num) < cutoff) num = __builtin_nan("");
        den = 1.0 / den;
        double delta = den * num;
        cf *= delta;
        coeff = -(a + k) * (a + b + k) * x / ((a + 2 * k) * (a + 2 * k + 1.0));
        den = 1.0 + coeff * den;
        num = 1.0 + coeff / num;
        if (fabs(den) < cutoff) den = __builtin_nan("");
        if (fabs(num) < cutoff) num = __builtin_nan("");
        den = 1.0 / den;
        delta = den * num;
        cf *= delta;
        if (fabs(delta - 1.0) < 2.0 * DBL_EPSILON) break;
        if (cf * fabs(delta - 1.0) < epsabs) break;
        ++it;
    }
    if (it >= 512) return __builtin_nan("");
    return cf;
}

// Regularized incomplete gamma for the asymptotic branches below (shape < 10: the series
// under a + 1, Legendre's continued fraction above), as the oracle restates
// gsl_sf_gamma_inc_P / _Q there (only union sizes above 1e5 reach it; inlined: an out-of-line
// call gave the finalize kernels a 16 B/lane stack frame, i.e. scratch)
__device__ double lngamma_pos(double x)
{
    return lngammastar(x) + (x - 0.5) * log(x) - x + 0.91893853320467274178;
}

__device__ __forceinline__ double gamma_inc_PQ(double a, double x, bool upper)
{
    if (x <= 0.0) return upper ? 1.0 : 0.0;
    if (x < a + 1.0) {
        double sum = 1.0, term = 1.0;
        for (int n = 1; n < 100000; n++) {
            term *= x / (a + n);
            sum += term;
            if (term < sum * DBL_EPSILON) break;
        }
        const double P = exp(a * log(x) - x - lngamma_pos(a + 1.0)) * sum;
        return upper ? 1.0 - P : P;
    }
    const double tiny = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
    for (int i = 1; i < 100000; i++) {
        const double an = -(double)i * ((double)i - a);
        b += 2.0;
        d = an * d + b;
        if (fabs(d) < tiny) d = tiny;
        c = b + an / c;
        if (fabs(c) < tiny) c = tiny;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < DBL_EPSILON) break;
    }
    const double Q = exp(a * log(x) - x - lngamma_pos(a)) * h;
    return upper ? Q : 1.0 - Q;
}

// gsl_cdf_beta_P = beta_inc_AXPY(1, 0, ...): the asymptotic regimes of A&S 26.5.17 (union
// sizes above 1e5), then the general continued fraction
__device__ double beta_P(double x, double a, double b)
{
    if (x == 0.0) return 0.0;
    if (x == 1.0) return 1.0;
    if (a > 1e5 && b < 10 && x > a / (a + b))
        return gamma_inc_PQ(b, -(a + (b - 1.0) / 2.0) * log(x), true);
    if (b > 1e5 && a < 10 && x < b / (a + b))
        return gamma_inc_PQ(a, -(b + (a - 1.0) / 2.0) * log1p(-x), false);
    double pre = exp(-lnbeta(a, b) + a * log(x) + b * log1p(-x));
    if (x < (a + 1.0) / (a + b + 2.0)) return pre * beta_cf(a, b, x, 0.0) / a;
    double epsabs = DBL_EPSILON / fabs(pre / b);
    return 1.0 - pre * beta_cf(b, a, 1.0 - x, epsabs) / b;
}

__device__ double pvalue_dev(uint32_t x, uint64_t len_ref, uint64_t len_qry, double kmer_space,
                             uint32_t n)
{
    if (x == 0) return 1.0;
    double px = 1.0 / (1.0 + kmer_space / (double)len_ref);
    double py = 1.0 / (1.0 + kmer_space / (double)len_qry);
    double r = px * py / (px + py - px * py);
    uint32_t k = x - 1;
    if (k >= n) return 0.0;
    return beta_P(r, (double)k + 1.0, (double)n - (double)k);
}

// distance (CommandDistance.cpp:404-419), p-value and the -d / -v filters, one pair per
// thread (a candidate's p-value continued fraction stays on its own lane)
template <typename C>
__global__ __launch_bounds__(256) void dist_finalize_kernel(
    const C *__restrict__ numer, const C *__restrict__ denom,
    const uint64_t *__restrict__ ref_length, const uint64_t *__restrict__ qry_length,
    uint32_t n_ref, uint64_t n_pairs, uint32_t kmer_size, double kmer_space, double max_dist,
    double max_pvalue, double *__restrict__ dist, double *__restrict__ pval,
    uint8_t *__restrict__ pass)
{
    const uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_pairs) return;
    const uint32_t c = numer[o], d = denom[o];
    const uint32_t r = (uint32_t)(o % n_ref), q = (uint32_t)(o / n_ref);
    double dv;
    if (c == d) dv = 0.0;
    else if (c == 0) dv = 1.0;
    else {
        double jac = (double)c / (double)d;
        dv = -log(2.0 * jac / (1.0 + jac)) / (double)kmer_size;
        if (dv > 1.0) dv = 1.0;
    }
    bool ok = !(max_dist >= 0 && dv > max_dist);
    double pv = 0.0;
    if (ok) {
        pv = pvalue_dev(c, ref_length[r], qry_length[q], kmer_space, d);
        ok = !(max_pvalue >= 0 && pv > max_pvalue);
    }
    dist[o] = dv;
    pval[o] = pv;
    if (pass) pass[o] = ok ? 1 : 0;
}

// Every cell's no-shared-hash values (PairFill): a pure write stream, 25 B per cell, one
// workgroup per 1024 cells of one query row (row = blockIdx.x / blocks-per-row, uniform).
// VEC (n_ref % 4 == 0, so a row starts 4-cell aligned): each lane writes 4 consecutive
// cells with 16-B stores (1 KiB per wave store; the pass bytes as one dword).
constexpr uint32_t kFillCells = 1024;
template <bool VEC, typename C>
__global__ __launch_bounds__(256) void dist_fill_kernel(
    const uint32_t *__restrict__ ref_len, uint32_t n_ref, const uint32_t *__restrict__ qry_len,
    uint32_t nrb, uint32_t ntask, uint32_t S, C *__restrict__ numer,
    C *__restrict__ denom, PairFill fill)
{
    const bool keep1 = !(fill.max_dist >= 0 && 1.0 > fill.max_dist);   // distance 0 always kept
    const bool pkeep = !(fill.max_pvalue >= 0 && 1.0 > fill.max_pvalue);
    for (uint32_t t = blockIdx.x; t < ntask; t += gridDim.x) {
    const uint32_t q = t / nrb, rb = t - q * nrb;
    const uint32_t lq = qry_len[q];
    const uint64_t row = (uint64_t)q * n_ref;
    if (VEC) {
        const uint32_t r = rb * kFillCells + threadIdx.x * 4;
        if (r >= n_ref) continue;
        const uint64_t o = row + r;
        const uint4 rl = *(const uint4 *)(ref_len + r);
        const uint32_t d[4] = {rl.x + lq, rl.y + lq, rl.z + lq, rl.w + lq};  // <= 2 stride
        uint32_t dn[4], pa = 0;
        double dv[4], pv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const bool ok = d[u] == 0 || keep1;
            dn[u] = d[u] < S ? d[u] : S;
            dv[u] = d[u] == 0 ? 0.0 : 1.0;
            pv[u] = ok ? 1.0 : 0.0;
            pa |= (ok && pkeep ? 1u : 0u) << (8 * u);
        }
        // plain stores: non-temporal ones (nt) let the candidate compare beside run 15%
        // faster but slowed this stream by 20% (step 1.99 -> 2.14 ms); 16-B write-through
        // (sc1) buffer stores slowed it 1.9x (0.9 -> 1.67 ms beside the compare)
        if (numer) {
            store_counts4(numer + o, 0, 0, 0, 0);
            store_counts4(denom + o, dn[0], dn[1], dn[2], dn[3]);
        }
        if (fill.dist) {     // (null: the counts only, the compact output)
            *(double2 *)(fill.dist + o) = make_double2(dv[0], dv[1]);
            *(double2 *)(fill.dist + o + 2) = make_double2(dv[2], dv[3]);
            *(double2 *)(fill.pval + o) = make_double2(pv[0], pv[1]);
            *(double2 *)(fill.pval + o + 2) = make_double2(pv[2], pv[3]);
            if (fill.pass) *(uint32_t *)(fill.pass + o) = pa;
        }
        continue;
    }
#pragma unroll
    for (uint32_t u = 0; u < kFillCells / 256; u++) {
        const uint32_t r = rb * kFillCells + u * 256 + threadIdx.x;
        if (r >= n_ref) break;
        const uint64_t o = row + r;
        const uint32_t d = ref_len[r] + lq;   // both <= stride, no overflow
        const bool ok = d == 0 || keep1;
        if (numer) {
            numer[o] = 0;
            denom[o] = (C)(d < S ? d : S);
        }
        if (!fill.dist) continue;
        fill.dist[o] = d == 0 ? 0.0 : 1.0;
        fill.pval[o] = ok ? 1.0 : 0.0;
        if (fill.pass) fill.pass[o] = ok && pkeep ? 1 : 0;
    }
    }
}

// The fill over the flattened grid (n_ref % 4 == 0): workgroup k takes cells [1024 k,
// 1024 k + 1024) of the q-range, 4 per lane (never across a row: rows are 4-cell aligned),
// the row of each lane from a double reciprocal and one integer correction.  Row-aligned
// workgroups put every wave store off the 64-B line grid whenever n_ref is not a multiple of
// 1024, and left a partial workgroup per row: 4.8 -> 6.5 TB/s at n_ref = 10,000, 4.1 -> 5.8 at
// 21,876, 5.6 -> 6.6 at 50,000 (tools/micro/fill_real.hip, one MI355X).
// (A counts-only form with 8 cells and one 16-B store per array per lane, half the lanes: the
// fill took as long and the rank kernel beside it 2.95 -> 3.4 ms, C4 6.67 -> 6.89 ms, same
// box, r04.)
template <typename C>
__global__ __launch_bounds__(256) void dist_fill_flat_kernel(
    const uint32_t *__restrict__ ref_len, uint32_t n_ref, const uint32_t *__restrict__ qry_len,
    uint64_t cells, double inv_n, uint32_t S, C *__restrict__ numer, C *__restrict__ denom,
    PairFill fill)
{
    const bool keep1 = !(fill.max_dist >= 0 && 1.0 > fill.max_dist);   // distance 0 always kept
    const bool pkeep = !(fill.max_pvalue >= 0 && 1.0 > fill.max_pvalue);
    // one pass per thread (a grid-stride loop measured slower)
    const uint64_t o = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (o >= cells) return;
    uint32_t q = (uint32_t)((double)o * inv_n);
    int64_t rr = (int64_t)(o - (uint64_t)q * n_ref);
    if (rr < 0) { q--; rr += n_ref; }
    else if (rr >= (int64_t)n_ref) { q++; rr -= n_ref; }
    const uint32_t r = (uint32_t)rr;
    const uint32_t lq = qry_len[q];
    const uint4 rl = *(const uint4 *)(ref_len + r);
    const uint32_t d[4] = {rl.x + lq, rl.y + lq, rl.z + lq, rl.w + lq};  // <= 2 stride
    uint32_t dn[4], pa = 0;
    double dv[4], pv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const bool ok = d[u] == 0 || keep1;
        dn[u] = d[u] < S ? d[u] : S;
        dv[u] = d[u] == 0 ? 0.0 : 1.0;
        pv[u] = ok ? 1.0 : 0.0;
        pa |= (ok && pkeep ? 1u : 0u) << (8 * u);
    }
    if (numer) {
        store_counts4(numer + o, 0, 0, 0, 0);
        store_counts4(denom + o, dn[0], dn[1], dn[2], dn[3]);
    }
    if (fill.dist) {         // (null: the counts only, the compact output)
        *(double2 *)(fill.dist + o) = make_double2(dv[0], dv[1]);
        *(double2 *)(fill.dist + o + 2) = make_double2(dv[2], dv[3]);
        *(double2 *)(fill.pval + o) = make_double2(pv[0], pv[1]);
        *(double2 *)(fill.pval + o + 2) = make_double2(pv[2], pv[3]);
        if (fill.pass) *(uint32_t *)(fill.pass + o) = pa;
    }
}

hipError_t launch_dist_fill(const uint32_t *d_ref_len, uint32_t n_ref, const uint32_t *d_qry_len,
                            uint32_t n_qry, uint32_t S, Counts cnt, const PairFill &fill,
                            hipStream_t st, bool flat)
{
    void *d_numer = cnt.numer, *d_denom = cnt.denom;
    if (!n_ref || !n_qry) return hipSuccess;
    const uint32_t nrb = (n_ref + kFillCells - 1) / kFillCells;
    const uint64_t blocks = (uint64_t)nrb * n_qry;
    if (blocks >= (1ULL << 31)) return hipErrorInvalidValue;
    // 16-B stores need 16-B aligned rows of every output (the pass row as 4-B aligned)
    const auto al = [](const void *p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
    // (null outputs are aligned)
    const bool vec = n_ref % 4 == 0 && al(d_ref_len, 16) && al(d_numer, 16) &&
                     al(d_denom, 16) && al(fill.dist, 16) && al(fill.pval, 16) &&
                     al(fill.pass, 4);
    // the full grid: short workgroups hand their slots back to the candidate compare running
    // beside (a capped grid-stride fill of 256-4096 workgroups held them and measured slower)
    const uint32_t grid = (uint32_t)blocks;
    const uint64_t cells = (uint64_t)n_ref * n_qry;
    if (flat && vec && cells < (1ULL << 50)) {
        const uint64_t fb = (cells / 4 + 255) / 256;
        if (fb >= (1ULL << 31)) return hipErrorInvalidValue;
        const double inv_n = 1.0 / (double)n_ref;
#define FPM_FLAT(C_)                                                                               \
    hipLaunchKernelGGL((dist_fill_flat_kernel<C_>), dim3((uint32_t)fb), dim3(256), 0, st,          \
                       d_ref_len, n_ref, d_qry_len, cells, inv_n, S, (C_ *)d_numer, (C_ *)d_denom, \
                       fill)
        if (cnt.c16) FPM_FLAT(uint16_t);
        else FPM_FLAT(uint32_t);
#undef FPM_FLAT
        return hipGetLastError();
    }
#define FPM_FILL(V, C)                                                                         \
    hipLaunchKernelGGL((dist_fill_kernel<V, C>), dim3(grid), dim3(256), 0, st, d_ref_len, n_ref, \
                       d_qry_len, nrb, (uint32_t)blocks, S, (C *)d_numer, (C *)d_denom, fill)
    if (cnt.c16) {
        if (vec) FPM_FILL(true, uint16_t);
        else FPM_FILL(false, uint16_t);
    } else {
        if (vec) FPM_FILL(true, uint32_t);
        else FPM_FILL(false, uint32_t);
    }
#undef FPM_FILL
    return hipGetLastError();
}

// A compact grid's counts before its sketches exist (fpm_dist_list_prefill): numer 0 and
// denom S in every cell, i.e. min(S, la + lb) (CommandDistance.cpp:416-418 at common = 0) for
// every pair whose lists hold at least S hashes together.  VEC: 8 cells per lane, one 16-B
// store per array (both arrays 16-B aligned).
template <bool VEC>
__global__ __launch_bounds__(256) void dist_counts_const_kernel(uint16_t *__restrict__ numer,
                                                                uint16_t *__restrict__ denom,
                                                                uint64_t cells, uint32_t S)
{
    const uint64_t o = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (o >= cells) return;
    if (VEC && o + 8 <= cells) {
        const uint32_t d = S | (S << 16);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store((u32x4){0u, 0u, 0u, 0u}, (u32x4 *)(numer + o));
        __builtin_nontemporal_store((u32x4){d, d, d, d}, (u32x4 *)(denom + o));
        return;
    }
    for (uint64_t c = o; c < cells && c < o + 8; c++) {
        numer[c] = 0;
        denom[c] = (uint16_t)S;
    }
}

hipError_t launch_dist_counts_const(uint16_t *numer, uint16_t *denom, uint64_t cells, uint32_t S,
                                    hipStream_t st)
{
    if (!cells) return hipSuccess;
    const uint64_t blocks = (cells + 8 * 256 - 1) / (8 * 256);
    if (blocks >= (1ULL << 31)) return hipErrorInvalidValue;
    const bool vec = (((uintptr_t)numer | (uintptr_t)denom) & 15) == 0;
    if (vec)
        hipLaunchKernelGGL(dist_counts_const_kernel<true>, dim3((uint32_t)blocks), dim3(256), 0, st,
                           numer, denom, cells, S);
    else
        hipLaunchKernelGGL(dist_counts_const_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0,
                           st, numer, denom, cells, S);
    return hipGetLastError();
}

// After a prefill, the pairs whose lists hold fewer than S hashes together: denom = la + lb.
// One workgroup per 64 query rows; a row with lq >= S has none (la + lq >= S for every ref),
// so with full sketches every workgroup stops after one length read per row.
__global__ __launch_bounds__(256) void dist_counts_fixup_kernel(
    const uint32_t *__restrict__ ref_len, uint32_t n_ref, const uint32_t *__restrict__ qry_len,
    uint32_t n_qry, uint32_t S, uint16_t *__restrict__ denom)
{
    __shared__ uint64_t s_rows;
    const uint32_t q0 = blockIdx.x * 64;
    if (threadIdx.x < 64) {                      // wave 0: the rows that need a sweep
        const uint32_t q = q0 + threadIdx.x;
        const uint64_t m = __builtin_amdgcn_ballot_w64(q < n_qry && qry_len[q] < S);
        if (threadIdx.x == 0) s_rows = m;
    }
    __syncthreads();
    for (uint64_t m = s_rows; m; m &= m - 1) {
        const uint32_t q = q0 + (uint32_t)__builtin_ctzll(m);
        const uint32_t lq = qry_len[q];
        uint16_t *const row = denom + (uint64_t)q * n_ref;
        for (uint32_t r = threadIdx.x; r < n_ref; r += 256) {
            const uint32_t d = ref_len[r] + lq;
            if (d < S) row[r] = (uint16_t)d;
        }
    }
}

hipError_t launch_dist_counts_fixup(const uint32_t *d_ref_len, uint32_t n_ref,
                                    const uint32_t *d_qry_len, uint32_t n_qry, uint32_t S,
                                    uint16_t *denom, hipStream_t st)
{
    if (!n_ref || !n_qry) return hipSuccess;
    hipLaunchKernelGGL(dist_counts_fixup_kernel, dim3((n_qry + 63) / 64), dim3(256), 0, st,
                       d_ref_len, n_ref, d_qry_len, n_qry, S, denom);
    return hipGetLastError();
}

// The same per-pair arithmetic as dist_finalize_kernel, for the candidate cells of the
// sparse path only (the probe wrote every other cell's final values).  Grid-stride over the
// device-side candidate count; with `sym` each candidate (q, r) (one of the pair's two cells,
// probe_rows_kernel) also finalizes its mirror (r, q), whose numer / denom the rank kernel
// wrote.
__device__ __forceinline__ void finalize_cell(uint64_t o, uint32_t c, uint32_t d, uint64_t len_ref,
                                              uint64_t len_qry, uint32_t kmer_size,
                                              double kmer_space, double max_dist,
                                              double max_pvalue, double *dist, double *pval,
                                              uint8_t *pass)
{
    double dv;
    if (c == d) dv = 0.0;
    else if (c == 0) dv = 1.0;
    else {
        double jac = (double)c / (double)d;
        dv = -log(2.0 * jac / (1.0 + jac)) / (double)kmer_size;
        if (dv > 1.0) dv = 1.0;
    }
    bool ok = !(max_dist >= 0 && dv > max_dist);
    double pv = 0.0;
    if (ok) {
        pv = pvalue_dev(c, len_ref, len_qry, kmer_space, d);
        ok = !(max_pvalue >= 0 && pv > max_pvalue);
    }
    dist[o] = dv;
    pval[o] = pv;
    if (pass) pass[o] = ok ? 1 : 0;
}

template <typename C>
__global__ __launch_bounds__(256) void dist_cand_finalize_kernel(
    const uint64_t *__restrict__ cand, const unsigned long long *__restrict__ n_cand,
    uint32_t sym, const uint32_t *__restrict__ cnum, const uint32_t *__restrict__ cden,
    C *__restrict__ numer, C *__restrict__ denom,
    const uint64_t *__restrict__ ref_length, const uint64_t *__restrict__ qry_length,
    uint32_t n_ref, uint32_t kmer_size, double kmer_space, double max_dist, double max_pvalue,
    double *__restrict__ dist, double *__restrict__ pval, uint8_t *__restrict__ pass,
    MirrorOut mir)
{
    const uint64_t n = *n_cand;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t o = cand[c];
        const uint32_t q = (uint32_t)(o / n_ref), r = (uint32_t)(o - (uint64_t)q * n_ref);
        uint32_t nm, dn;
        if (cnum) {          // compact results: scatter numer / denom too
            nm = cnum[c];
            dn = cden[c];
            numer[o] = (C)nm;
            denom[o] = (C)dn;
        } else {
            nm = numer[o];
            dn = denom[o];
        }
        finalize_cell(o, nm, dn, ref_length[r], qry_length[q], kmer_size, kmer_space, max_dist,
                      max_pvalue, dist, pval, pass);
        if (sym && r != q) {   // cell (r, q): query r against ref q
            const uint64_t o2 = (uint64_t)r * n_ref + q;
            if (cnum) {
                numer[o2] = (C)nm;
                denom[o2] = (C)dn;
            }
            finalize_cell(o2, nm, dn, ref_length[q], qry_length[r], kmer_size, kmer_space,
                          max_dist, max_pvalue, dist, pval, pass);
        }
        if (mir.dist) {        // transposed grid: ref r as the query, query q as the ref
            const uint64_t o2 = (uint64_t)r * mir.n_qry + q;
            ((C *)mir.cnt.numer)[o2] = (C)nm;
            ((C *)mir.cnt.denom)[o2] = (C)dn;
            finalize_cell(o2, nm, dn, qry_length[q], ref_length[r], kmer_size, kmer_space,
                          max_dist, max_pvalue, mir.dist, mir.pval, mir.pass);
        }
    }
}

hipError_t launch_dist_cand_finalize(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                     uint64_t cap, bool sym, const uint32_t *d_cnum,
                                     const uint32_t *d_cden, Counts cnt,
                                     const uint64_t *d_ref_length,
                                     const uint64_t *d_qry_length, uint32_t n_ref,
                                     uint32_t kmer_size, double kmer_space, double max_dist,
                                     double max_pvalue, double *d_dist, double *d_pvalue,
                                     uint8_t *d_pass, const MirrorOut &mir, hipStream_t st)
{
    if (!cap) return hipSuccess;
    if (mir.dist && (!mir.cnt.numer || !mir.cnt.denom || mir.cnt.c16 != cnt.c16 || !d_cnum))
        return hipErrorInvalidValue;
    const uint64_t blocks = std::min<uint64_t>((cap + 255) / 256, 4096);
#define FPM_CFIN(C)                                                                          \
    hipLaunchKernelGGL(dist_cand_finalize_kernel<C>, dim3((uint32_t)blocks), dim3(256), 0, st,  \
                       d_cand, d_n_cand, (uint32_t)sym, d_cnum, d_cden, (C *)cnt.numer,        \
                       (C *)cnt.denom, d_ref_length, d_qry_length, n_ref, kmer_size,           \
                       kmer_space, max_dist, max_pvalue, d_dist, d_pvalue, d_pass, mir)
    if (cnt.c16) FPM_CFIN(uint16_t);
    else FPM_CFIN(uint32_t);
#undef FPM_CFIN
    return hipGetLastError();
}

// ---- Compact output: dense numer / denom cells plus a list of the
// cells that share hashes (numer > 0) with their distance / p-value / pass.  Every other cell
// has closed-form values (CommandDistance.cpp:404-419, 433-450 at common = 0), so nothing is
// written for it beyond its counts.

// distance, p-value and -d / -v pass of one cell (finalize_cell's arithmetic, by value)
__device__ __forceinline__ void cell_values(uint32_t c, uint32_t d, uint64_t len_ref,
                                            uint64_t len_qry, uint32_t kmer_size,
                                            double kmer_space, double max_dist, double max_pvalue,
                                            double &dv, double &pv, bool &ok)
{
    if (c == d) dv = 0.0;
    else if (c == 0) dv = 1.0;
    else {
        double jac = (double)c / (double)d;
        dv = -log(2.0 * jac / (1.0 + jac)) / (double)kmer_size;
        if (dv > 1.0) dv = 1.0;
    }
    ok = !(max_dist >= 0 && dv > max_dist);
    pv = 0.0;
    if (ok) {
        pv = pvalue_dev(c, len_ref, len_qry, kmer_space, d);
        ok = !(max_pvalue >= 0 && pv > max_pvalue);
    }
}

// Distance and p-value of n independent cells from their counts and genome lengths (the
// optional batch call of SURVEY §8(b): the values the compact output leaves out, for the cells
// a caller asks for), no filters.
template <typename C>
__global__ __launch_bounds__(256) void pvalue_batch_kernel(const C *__restrict__ numer,
                                                           const C *__restrict__ denom,
                                                           const uint64_t *__restrict__ len_ref,
                                                           const uint64_t *__restrict__ len_qry,
                                                           uint64_t n, uint32_t kmer_size,
                                                           double kmer_space,
                                                           double *__restrict__ dist,
                                                           double *__restrict__ pvalue)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double dv, pv;
    bool ok;
    cell_values(numer[i], denom[i], len_ref[i], len_qry[i], kmer_size, kmer_space, -1.0, -1.0,
                dv, pv, ok);
    if (dist) dist[i] = dv;
    if (pvalue) pvalue[i] = pv;
}

hipError_t launch_pvalue_batch(const void *numer, const void *denom, uint32_t count_bytes,
                               const uint64_t *len_ref, const uint64_t *len_qry, uint64_t n,
                               uint32_t kmer_size, double kmer_space, double *dist,
                               double *pvalue, hipStream_t st)
{
    if (!n) return hipSuccess;
    const dim3 g((uint32_t)((n + 255) / 256));
    if (count_bytes == 2)
        hipLaunchKernelGGL(pvalue_batch_kernel<uint16_t>, g, dim3(256), 0, st,
                           (const uint16_t *)numer, (const uint16_t *)denom, len_ref, len_qry, n,
                           kmer_size, kmer_space, dist, pvalue);
    else
        hipLaunchKernelGGL(pvalue_batch_kernel<uint32_t>, g, dim3(256), 0, st,
                           (const uint32_t *)numer, (const uint32_t *)denom, len_ref, len_qry, n,
                           kmer_size, kmer_space, dist, pvalue);
    return hipGetLastError();
}

// Block-wide slot reservation: thread t needs k_t entries; returns its first slot.  One
// global atomic per workgroup (a per-wave atomic on the one counter serialised: the C2
// candidate list took 0.21 ms for 1e6 cells).  Every thread of the block calls it.
constexpr int kListThreads = 256;
__device__ __forceinline__ uint64_t block_reserve(unsigned long long *count, uint32_t k,
                                                  uint32_t *wsum, unsigned long long *base)
{
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = k;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < kListThreads / 64; w++) {
            const uint32_t t = wsum[w];
            wsum[w] = run;
            run += t;
        }
        *base = run ? atomicAdd(count, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    const uint64_t r = *base + wsum[wave] + x - k;
    __syncthreads();                         // wsum / base are reused by the next call
    return r;
}

__device__ __forceinline__ void list_put(const CellList &L, uint64_t i, uint32_t q, uint32_t r,
                                         double dv, double pv, bool ok)
{
    if (i >= L.cap) return;                  // counted, not written: the caller re-runs larger
    L.qry[i] = q;
    L.ref[i] = r;
    L.dist[i] = dv;
    L.pval[i] = pv;
    if (L.pass) L.pass[i] = ok ? 1 : 0;
}

// The candidate cells of the sparse path in compact form: scatter each candidate's
// (numer, denom) to its cell (and, with `sym`, to its mirror (r, q); with a transposed grid,
// to that grid's cell), then list the cells whose numer > 0.  cnum == nullptr: the walk kernel
// wrote the counts in place; they are read from the grid.
template <typename C>
__global__ __launch_bounds__(kListThreads) void dist_cand_list_kernel(
    const uint64_t *__restrict__ cand, const unsigned long long *__restrict__ n_cand,
    uint32_t sym, const uint32_t *__restrict__ cnum, const uint32_t *__restrict__ cden,
    C *__restrict__ numer, C *__restrict__ denom, const uint64_t *__restrict__ ref_length,
    const uint64_t *__restrict__ qry_length, uint32_t n_ref, uint32_t kmer_size,
    double kmer_space, double max_dist, double max_pvalue, CellList L, Counts mcnt,
    uint32_t m_nqry, CellList ML)
{
    __shared__ uint32_t wsum[kListThreads / 64];
    __shared__ unsigned long long base;
    const uint64_t n = *n_cand;
    for (uint64_t c0 = (uint64_t)blockIdx.x * kListThreads; c0 < n;
         c0 += (uint64_t)gridDim.x * kListThreads) {
        const uint64_t c = c0 + threadIdx.x;
        uint32_t nm = 0, dn = 0, q = 0, r = 0;
        bool mirror_cell = false;
        if (c < n) {
            const uint64_t o = cand[c];
            q = (uint32_t)(o / n_ref);
            r = (uint32_t)(o - (uint64_t)q * n_ref);
            if (cnum) {
                nm = cnum[c];
                dn = cden[c];
                numer[o] = (C)nm;
                denom[o] = (C)dn;
            } else {
                nm = numer[o];
                dn = denom[o];
            }
            mirror_cell = sym && r != q;
            if (mirror_cell) {
                const uint64_t o2 = (uint64_t)r * n_ref + q;
                numer[o2] = (C)nm;
                denom[o2] = (C)dn;
            }
            if (mcnt.numer) {
                const uint64_t o2 = (uint64_t)r * m_nqry + q;
                ((C *)mcnt.numer)[o2] = (C)nm;
                ((C *)mcnt.denom)[o2] = (C)dn;
            }
        }
        double dv = 1.0, pv = 1.0;
        bool ok = false;
        if (nm > 0)
            cell_values(nm, dn, ref_length[r], qry_length[q], kmer_size, kmer_space, max_dist,
                        max_pvalue, dv, pv, ok);
        // sorted distinct lists: the pair seen from the other side has the same counts, and
        // distance and p-value are symmetric in the two lengths (pValue's r is)
        const uint32_t k = nm > 0 ? (mirror_cell ? 2u : 1u) : 0u;
        const uint64_t at = block_reserve(L.count, k, wsum, &base);
        if (k) list_put(L, at, q, r, dv, pv, ok);
        if (k == 2) list_put(L, at + 1, r, q, dv, pv, ok);
        if (mcnt.numer) {
            const uint64_t am = block_reserve(ML.count, nm > 0 ? 1u : 0u, wsum, &base);
            if (nm > 0) list_put(ML, am, r, q, dv, pv, ok);
        }
    }
}

// The dense path in compact form: every cell's counts are in the grid; list those with
// numer > 0 (4 cells per lane).
template <typename C>
__global__ __launch_bounds__(kListThreads) void dist_grid_list_kernel(
    const C *__restrict__ numer, const C *__restrict__ denom, uint32_t n_ref, uint64_t n_pairs,
    const uint64_t *__restrict__ ref_length, const uint64_t *__restrict__ qry_length,
    uint32_t kmer_size, double kmer_space, double max_dist, double max_pvalue, CellList L)
{
    __shared__ uint32_t wsum[kListThreads / 64];
    __shared__ unsigned long long base;
    for (uint64_t b0 = (uint64_t)blockIdx.x * kListThreads * 4; b0 < n_pairs;
         b0 += (uint64_t)gridDim.x * kListThreads * 4) {
        const uint64_t o0 = b0 + threadIdx.x * 4;
        uint32_t c[4], k = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            c[u] = o0 + u < n_pairs ? (uint32_t)numer[o0 + u] : 0u;
            k += c[u] > 0 ? 1u : 0u;
        }
        uint64_t at = block_reserve(L.count, k, wsum, &base);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (c[u] == 0) continue;
            const uint64_t o = o0 + u;
            const uint32_t q = (uint32_t)(o / n_ref), r = (uint32_t)(o - (uint64_t)q * n_ref);
            double dv, pv;
            bool ok;
            cell_values(c[u], denom[o], ref_length[r], qry_length[q], kmer_size, kmer_space,
                        max_dist, max_pvalue, dv, pv, ok);
            list_put(L, at++, q, r, dv, pv, ok);
        }
    }
}

hipError_t launch_dist_cand_list(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                 uint64_t cap, bool sym, const uint32_t *d_cnum,
                                 const uint32_t *d_cden, Counts cnt, const uint64_t *d_ref_length,
                                 const uint64_t *d_qry_length, uint32_t n_ref, uint32_t kmer_size,
                                 double kmer_space, double max_dist, double max_pvalue,
                                 const CellList &list, Counts mcnt, uint32_t m_nqry,
                                 const CellList &mlist, hipStream_t st)
{
    if (!cap) return hipSuccess;
    if (mcnt.numer && (!mcnt.denom || mcnt.c16 != cnt.c16 || !d_cnum || !mlist.count))
        return hipErrorInvalidValue;
    const uint64_t blocks = std::min<uint64_t>((cap + kListThreads - 1) / kListThreads, 4096);
#define FPM_CLIST(C)                                                                          \
    hipLaunchKernelGGL(dist_cand_list_kernel<C>, dim3((uint32_t)blocks), dim3(kListThreads), 0, st, \
                       d_cand, d_n_cand, (uint32_t)sym, d_cnum, d_cden, (C *)cnt.numer,        \
                       (C *)cnt.denom, d_ref_length, d_qry_length, n_ref, kmer_size,           \
                       kmer_space, max_dist, max_pvalue, list, mcnt, m_nqry, mlist)
    if (cnt.c16) FPM_CLIST(uint16_t);
    else FPM_CLIST(uint32_t);
#undef FPM_CLIST
    return hipGetLastError();
}

hipError_t launch_dist_grid_list(Counts cnt, uint32_t n_ref, uint32_t n_qry,
                                 const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                                 uint32_t kmer_size, double kmer_space, double max_dist,
                                 double max_pvalue, const CellList &list, hipStream_t st)
{
    const uint64_t n = (uint64_t)n_ref * n_qry;
    if (!n) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((n / 4 + kListThreads - 1) / kListThreads + 1, 1u << 16);
#define FPM_GLIST(C)                                                                          \
    hipLaunchKernelGGL(dist_grid_list_kernel<C>, dim3((uint32_t)blocks), dim3(kListThreads), 0, st, \
                       (const C *)cnt.numer, (const C *)cnt.denom, n_ref, n, d_ref_length,     \
                       d_qry_length, kmer_size, kmer_space, max_dist, max_pvalue, list)
    if (cnt.c16) FPM_GLIST(uint16_t);
    else FPM_GLIST(uint32_t);
#undef FPM_GLIST
    return hipGetLastError();
}

// triangle -fp's compareFingerprints (CommandTriangle.cpp:255-302): positional compare of
// two lists over min(len) entries.  The fork reads the hash64 half of a u32 union whose
// upper bits are uninitialised (:279); here u32 values are zero-extended, so a match is
// an equal value at the same position.  distance = 1 - m/min(len) (NaN for an empty
// list, as the reference), p-value = gsl_cdf_chisq_Q(m, 1) = erfc(sqrt(m/2)), pass =
// distance <= max_dist && p <= max_pvalue.  One lane per pair, query-major output.
template <typename H>
__global__ __launch_bounds__(256) void positional_grid_kernel(
    const H *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const H *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t n_qry, double max_dist, double max_pvalue,
    uint32_t *__restrict__ numer, uint32_t *__restrict__ denom, double *__restrict__ dist,
    double *__restrict__ pval, uint8_t *__restrict__ pass)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x, q = blockIdx.y;
    if (r >= n_ref) return;
    const H *a = ref + (uint64_t)r * ref_stride, *b = qry + (uint64_t)q * qry_stride;
    const uint32_t m = min(ref_len[r], qry_len[q]);
    uint32_t matches = 0;
    for (uint32_t i = 0; i < m; i++) matches += a[i] == b[i];
    const double dv = 1.0 - (double)matches / (double)m;
    const double pv = erfc(sqrt((double)matches / 2.0));
    const uint64_t o = (uint64_t)q * n_ref + r;
    numer[o] = matches;
    denom[o] = m;
    dist[o] = dv;
    pval[o] = pv;
    pass[o] = (dv <= max_dist && pv <= max_pvalue) ? 1 : 0;
}

hipError_t launch_positional_grid(const void *d_ref, const uint32_t *d_ref_len,
                                  uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                  const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                                  uint32_t hash_bytes, double max_dist, double max_pvalue,
                                  uint32_t *d_numer, uint32_t *d_denom, double *d_dist,
                                  double *d_pvalue, uint8_t *d_pass, hipStream_t st)
{
    if (!n_ref || !n_qry) return hipSuccess;
    const dim3 g((n_ref + 255) / 256, n_qry);
    if (n_qry > 65535) return hipErrorInvalidValue;
    if (hash_bytes == 8)
        hipLaunchKernelGGL(positional_grid_kernel<uint64_t>, g, dim3(256), 0, st,
                           (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint64_t *)d_qry, d_qry_len, qry_stride, n_qry, max_dist,
                           max_pvalue, d_numer, d_denom, d_dist, d_pvalue, d_pass);
    else
        hipLaunchKernelGGL(positional_grid_kernel<uint32_t>, g, dim3(256), 0, st,
                           (const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint32_t *)d_qry, d_qry_len, qry_stride, n_qry, max_dist,
                           max_pvalue, d_numer, d_denom, d_dist, d_pvalue, d_pass);
    return hipGetLastError();
}

template <typename C>
static hipError_t compare_grid_c(const void *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                                 uint32_t n_ref, const void *d_qry, const uint32_t *d_qry_len,
                                 uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes,
                                 uint32_t sketch_size, C *d_numer, C *d_denom, hipStream_t st)
{
    if (n_ref == 0 || n_qry == 0) return hipSuccess;
    dim3 grid((n_ref + kTile - 1) / kTile, (n_qry + kTile - 1) / kTile);
    // LDS-staged walk when the tile's 32 lists of W = min(S, stride) entries fit
    {
        constexpr size_t kMaxLds = 156 * 1024;
        const uint64_t W = std::min<uint64_t>({(uint64_t)sketch_size, std::max(ref_stride, qry_stride)});
        constexpr int kBlk = kWalkBlk;
        const size_t lds = (size_t)2 * kTile * ((W + kBlk + 3) & ~3ull) * hash_bytes;
        if (W > 0 && lds <= kMaxLds && (hash_bytes == 4 || hash_bytes == 8)) {
            const void *fn = hash_bytes == 8 ? (const void *)compare_grid_lds_kernel<uint64_t, kBlk, C>
                                             : (const void *)compare_grid_lds_kernel<uint32_t, kBlk, C>;
            if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds) ==
                hipSuccess) {
                if (hash_bytes == 8)
                    hipLaunchKernelGGL((compare_grid_lds_kernel<uint64_t, kBlk, C>), grid, dim3(256), lds, st,
                                       (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                                       (const uint64_t *)d_qry, d_qry_len, qry_stride, n_qry,
                                       sketch_size, (uint32_t)W, d_numer, d_denom);
                else
                    hipLaunchKernelGGL((compare_grid_lds_kernel<uint32_t, kBlk, C>), grid, dim3(256), lds, st,
                                       (const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                                       (const uint32_t *)d_qry, d_qry_len, qry_stride, n_qry,
                                       sketch_size, (uint32_t)W, d_numer, d_denom);
                return hipGetLastError();
            }
            (void)hipGetLastError();
        }
    }
    if (hash_bytes == 8)
        hipLaunchKernelGGL((compare_grid_kernel<uint64_t, C>), grid, dim3(256), 0, st,
                           (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint64_t *)d_qry, d_qry_len, qry_stride, n_qry, sketch_size,
                           d_numer, d_denom);
    else if (hash_bytes == 4)
        hipLaunchKernelGGL((compare_grid_kernel<uint32_t, C>), grid, dim3(256), 0, st,
                           (const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint32_t *)d_qry, d_qry_len, qry_stride, n_qry, sketch_size,
                           d_numer, d_denom);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_compare_grid(const void *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                               uint32_t n_ref, const void *d_qry, const uint32_t *d_qry_len,
                               uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes,
                               uint32_t sketch_size, Counts cnt, hipStream_t st)
{
    if (cnt.c16)
        return compare_grid_c(d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len, qry_stride,
                              n_qry, hash_bytes, sketch_size, (uint16_t *)cnt.numer,
                              (uint16_t *)cnt.denom, st);
    return compare_grid_c(d_ref, d_ref_len, ref_stride, n_ref, d_qry, d_qry_len, qry_stride, n_qry,
                          hash_bytes, sketch_size, (uint32_t *)cnt.numer, (uint32_t *)cnt.denom,
                          st);
}

// ---- Dense walk of u32 lists on 16-bit rank images (the -fp shape: C3).
// The walk only compares values (<, ==, >).  For a block of 32 query lists with U = the
// sorted distinct union of their first W entries, f(x) = 2 * #{u in U : u < x} + [x in U]
// preserves every comparison between a value x of ANY list and a value b of the block
// (f(b) = 2 rank(b) + 1; x < b => f(x) <= 2 rank(b) < f(b); x == b => equal;
// x > b => f(x) >= 2 rank(b) + 2), and |U| <= 32 W <= 32736 keeps f below 2^16.
// Half-width images double the lists an LDS tile holds: 32 x 32 pairs per workgroup
// (64 lists of W u16) instead of 16 x 16 (32 lists of W u32), i.e. 4 waves per SIMD
// instead of one, which hides the walk's dependent compare/select chain.
// qblock_union_kernel (once per query block): U and the block's u16 images.
// compare_grid_img_kernel (per tile): U staged in LDS, the 32 ref lists' values mapped by
// a fixed-step lower bound, then both images in LDS and the literal walk of 1,024 pairs.
constexpr int kImgTile = 32;
constexpr int kImgBlk3 = 3;   // walk steps per LDS window (4, merged into unaligned ds_read_b64: 27 vs 15 ms on C3)
constexpr uint32_t kImgMaxW = 1023;          // 2 * 32 * W + 1 < 2^16
constexpr uint32_t kImgNP = 32768;           // pow2 >= 32 * kImgMaxW
constexpr uint32_t kInfA = 0xFFFF, kInfB = 0xFFFE;
// U of a query block is followed by a directory over its values' top 12 bits (dir[v >> 20] =
// lower bound of v's bucket, 4097 entries): ~8 values per bucket, so a lower bound is one
// directory read + a few in-bucket steps instead of 15 steps over the whole U
constexpr uint32_t kDirBits = 12, kDir = 1u << kDirBits;
constexpr uint32_t kImgBlk = kImgNP + kDir + 4;   // u32 per query block in ublk (16-B multiple)   // padded-walk sentinels (> 2 * 32736 + 1)

// x + (bit lane of m): one v_addc with the mask as carry-in
__device__ __forceinline__ uint32_t add_mask(uint32_t x, uint64_t m)
{
    uint32_t r;
    uint64_t c;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(c) : "v"(x), "s"(m));
    return r;
}

__global__ __launch_bounds__(1024) void qblock_union_kernel(
    const uint32_t *__restrict__ qry, const uint32_t *__restrict__ qry_len, uint64_t qry_stride,
    uint32_t n_qry, uint32_t W, uint32_t Wimg, uint32_t *__restrict__ ublk,
    uint32_t *__restrict__ usize, uint16_t *__restrict__ bimg)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t key[];   // kImgNP + kDir + 1
    __shared__ uint32_t wsum[16];
    const uint32_t b = blockIdx.x, q0 = b * kImgTile, t = threadIdx.x;
    const uint32_t nv = kImgTile * W;
    for (uint32_t x = t; x < kImgNP; x += 1024) {
        uint32_t v = 0xFFFFFFFFu;
        if (x < nv) {
            const uint32_t l = x / W, e = x - l * W, row = q0 + l;
            if (row < n_qry && e < min(qry_len[row], W)) v = qry[(uint64_t)row * qry_stride + e];
        }
        key[x] = v;
    }
    uint32_t n_valid = 0;
    for (uint32_t l = 0; l < (uint32_t)kImgTile; l++)
        if (q0 + l < n_qry) n_valid += min(qry_len[q0 + l], W);
    __syncthreads();
    for (uint32_t k = 2; k <= kImgNP; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < kImgNP; i += 1024) {
                const uint32_t x = i ^ j;
                if (x > i) {
                    const uint32_t a = key[i], c = key[x];
                    if ((a > c) == ((i & k) == 0)) { key[i] = c; key[x] = a; }
                }
            }
            __syncthreads();
        }
    // distinct values among the n_valid smallest (pads sort last; a real 0xFFFFFFFF is
    // kept because only positions < n_valid are read)
    constexpr int PT = kImgNP / 1024;
    uint32_t v[PT], f = 0, cnt = 0;
#pragma unroll
    for (int u = 0; u < PT; u++) {
        const uint32_t i = t * PT + u;
        v[u] = key[i];
        const bool first = i < n_valid && (i == 0 || key[i - 1] != v[u]);
        f |= (first ? 1u : 0u) << u;
        cnt += first ? 1u : 0u;
    }
    const uint32_t lane = t & 63, wave = t >> 6;
    uint32_t x = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { const uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t pos = x - cnt, tot = 0;
    for (uint32_t w = 0; w < 16; w++) { if (w < wave) pos += wsum[w]; tot += wsum[w]; }
#pragma unroll
    for (int u = 0; u < PT; u++)
        if (f >> u & 1u) { key[pos] = v[u]; ublk[(uint64_t)b * kImgBlk + pos] = v[u]; pos++; }
    __syncthreads();
    uint32_t P = 1;
    while (P <= tot) P <<= 1;
    // directory: dir[k] = #{U < k << 20}, dir[kDir] = |U|; and the largest bucket
    uint32_t *dir = key + kImgNP;
    __shared__ uint32_t maxb;
    if (t == 0) maxb = 0;
    for (uint32_t k = t; k <= kDir; k += 1024) {
        uint32_t lo = 0;
        if (k < kDir) {
            const uint32_t a = k << (32 - kDirBits);
            for (uint32_t st = P >> 1; st >= 1; st >>= 1)
                if (lo + st <= tot && key[lo + st - 1] < a) lo += st;
        } else {
            lo = tot;
        }
        dir[k] = lo;
        ublk[(uint64_t)b * kImgBlk + kImgNP + k] = lo;
    }
    __syncthreads();
    for (uint32_t k = t; k < kDir; k += 1024) atomicMax(&maxb, dir[k + 1] - dir[k]);
    __syncthreads();
    if (t == 0) { usize[2 * b] = tot; usize[2 * b + 1] = maxb; }
    for (uint32_t y = t; y < nv; y += 1024) {
        const uint32_t l = y / W, e = y - l * W, row = q0 + l;
        if (row >= n_qry) continue;
        uint32_t img = 0;
        if (e < min(qry_len[row], W)) {
            const uint32_t a = qry[(uint64_t)row * qry_stride + e];
            uint32_t lo = 0;
            for (uint32_t st = P >> 1; st >= 1; st >>= 1)
                if (lo + st <= tot && key[lo + st - 1] < a) lo += st;
            img = 2 * lo + 1;                       // a is in U
        }
        bimg[(uint64_t)row * Wimg + e] = (uint16_t)img;
    }
}

// LDS image row in u16: an odd number of dwords, so the 32 ref rows that lanes 0-31 (and
// 32-63) of a wave read at similar offsets fall in 32 different banks of ds_read_u16's
// (a/4) mod 32 banking (an even stride such as 504 dwords put them in 4 banks)
__host__ __device__ __forceinline__ uint32_t img_row_u16(uint32_t W, uint32_t blk)
{
    return 2 * (((W + blk + 1) / 2) | 1u);
}


template <int BLK, typename C>
__global__ __launch_bounds__(1024) void compare_grid_img_kernel(
    const uint32_t *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const uint32_t *__restrict__ qry_len, uint32_t n_qry,
    const uint32_t *__restrict__ ublk, const uint32_t *__restrict__ usize,
    const uint16_t *__restrict__ bimg, uint32_t Wimg, uint32_t S, uint32_t W,
    uint32_t nrb, C *__restrict__ numer, C *__restrict__ denom)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
    uint16_t *img = reinterpret_cast<uint16_t *>(lds32);
    constexpr int kPer = (kImgTile * kImgMaxW + 1023) / 1024;   // ref values per thread (<= 32)
    const uint32_t Wp = img_row_u16(W, BLK);
    // XCD-aware tiles: workgroup b runs on XCD b % 8, and XCD x owns ref blocks [x per,
    // (x + 1) per), per = nrb / 8, which it sweeps for one query block after another: its ref
    // rows (~2.4 MB at C3's 5,000 x 1,000 u32) stay in the XCD's 4 MB L2 for every query
    // block, and a query block's union and images are fetched once per XCD (row-major tiles
    // re-read every ref block from the fabric once per query block).  The nrb % 8 ref blocks
    // left over are dealt tile by tile round the XCDs, so every XCD gets the same number of
    // tiles (whole leftover blocks per XCD left 3 XCDs idle at the end: +1.7 %).
    uint32_t rb, qb;
    {
        const uint32_t nqb = (n_qry + kImgTile - 1) / kImgTile;
        const uint32_t x = blockIdx.x % kXcds, k = blockIdx.x / kXcds;
        const uint32_t per = nrb / kXcds, rem = nrb - per * kXcds;
        if (k < per * nqb) {
            qb = k / per;
            rb = x * per + (k - qb * per);
        } else {
            const uint32_t e = x + kXcds * (k - per * nqb);
            if (!rem || e >= rem * nqb) return;
            qb = e / rem;
            rb = per * kXcds + (e - qb * rem);
        }
    }
    const uint32_t t = threadIdx.x, r0 = rb * kImgTile, q0 = qb * kImgTile;
    const uint32_t us = usize[2 * qb], maxb = usize[2 * qb + 1];
    const uint32_t nv = kImgTile * W;
    uint32_t *dirL = lds32 + kImgNP;
    {   // U: every thread's 16-B loads in flight before its LDS stores
        constexpr int kUV = kImgNP / 4096;
        const uint32_t *src = ublk + (uint64_t)qb * kImgBlk;
        for (uint32_t k = t; k <= kDir; k += 1024) dirL[k] = src[kImgNP + k];
        uint4 buf[kUV];
#pragma unroll
        for (int v = 0; v < kUV; v++) {
            const uint32_t x = t * 4 + 4096u * v;
            buf[v] = x + 4 <= us ? *(const uint4 *)(src + x) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int v = 0; v < kUV; v++) {
            const uint32_t x = t * 4 + 4096u * v;
            if (x + 4 <= us) *(uint4 *)(lds32 + x) = buf[v];
            else if (x < us) for (uint32_t y = x; y < us; y++) lds32[y] = src[y];
        }
    }
    __syncthreads();
    uint32_t P = 1;
    while (P <= maxb) P <<= 1;
    // the 32 ref lists' first W values: entry t + 1024 k.  Groups of 8, the next group's
    // global loads issued before the current group's lower bounds in U (branch-free, every
    // step's 8 LDS reads in flight); results packed two u16 per register
    auto load_group = [&](int k0, uint32_t *val, uint32_t &okg) {
        okg = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t y = t + 1024u * (k0 + u);
            const uint32_t l = y / W, e = y - l * W, row = r0 + l;
            const bool ok = y < nv && row < n_ref && e < min(ref_len[min(row, n_ref - 1)], W);
            val[u] = ok ? ref[(uint64_t)row * ref_stride + e] : 0u;
            okg |= (ok ? 1u : 0u) << u;
        }
    };
    uint32_t res[kPer / 2];
    uint32_t cur[8], nxt[8], okc, okn = 0;
    load_group(0, cur, okc);
#pragma unroll
    for (int k0 = 0; k0 < kPer; k0 += 8) {
        if (k0 + 8 < kPer) load_group(k0 + 8, nxt, okn);
        uint32_t lo[8], hi[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint32_t bk = cur[u] >> (32 - kDirBits);
            lo[u] = dirL[bk];
            hi[u] = dirL[bk + 1];
        }
        for (uint32_t st = P >> 1; st >= 1; st >>= 1) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t x = lo[u] + st - 1;
                v[u] = lds32[x < hi[u] ? x : 0u];
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                lo[u] += ((lo[u] + st <= hi[u]) & (v[u] < cur[u])) ? st : 0u;
        }
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            uint32_t mm[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t e = lds32[lo[u + h] < us ? lo[u + h] : 0u];
                mm[h] = (okc >> (u + h) & 1u)
                            ? 2 * lo[u + h] + (((lo[u + h] < us) & (e == cur[u + h])) ? 1u : 0u)
                            : kInfA;
            }
            res[(k0 + u) / 2] = mm[0] | (mm[1] << 16);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) cur[u] = nxt[u];
        okc = okn;
    }
    __syncthreads();
    // images: ref lists 0..31, query lists 32..63, rows of Wp u16
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t y = t + 1024u * k;
        if (y < nv) {
            const uint32_t l = y / W, e = y - l * W;
            img[e * kImgTile + l] =
                (uint16_t)(res[k / 2] >> (16 * (k & 1)));
        }
    }
    for (uint32_t y = t; y < nv; y += 1024) {
        const uint32_t l = y / W, e = y - l * W, row = q0 + l;
        img[(kImgTile + l) * Wp + e] =
            row < n_qry && e < min(qry_len[row], W) ? bimg[(uint64_t)row * Wimg + e] : (uint16_t)kInfB;
    }
    {   // the rows' tails [W, Wp): sentinels
        const uint32_t tw = Wp - W;
        for (uint32_t y = t; y < 2 * kImgTile * tw; y += 1024) {
            const uint32_t l = y / tw;
            if (l < (uint32_t)kImgTile)
                img[(W + (y - l * tw)) * kImgTile + l] = (uint16_t)kInfA;
            else
                img[l * Wp + W + (y - l * tw)] = (uint16_t)(l < (uint32_t)kImgTile ? kInfA : kInfB);
        }
    }
    __syncthreads();
    const uint32_t lane = t & 63;
    const uint32_t r = r0 + (t & (kImgTile - 1)), q = q0 + t / kImgTile;
    if (r >= n_ref || q >= n_qry) return;
    const uint32_t la = ref_len[r], lb = qry_len[q];
    // ref images interleaved: position e of ref l at e * 32 + l, so the 32 ref rows that lanes
    // read at their own walk positions fall into distinct LDS banks unless two positions of
    // one 2-row pair collide (a row-major layout spreads them at random: ~3.7 conflict cycles
    // per read in PMC)
    const uint16_t *A = img + (t & (kImgTile - 1));
    constexpr uint32_t kAs = kImgTile;   // A element stride
    const uint16_t *B = img + (kImgTile + t / kImgTile) * Wp;
    (void)lane;
    // Padded walk: past its first min(len, W) entries each image row holds a sentinel,
    // kInfA (ref) > kInfB (query) > every image value, so the walk needs no end-of-list
    // tests: it runs S steps (S <= W here), an exhausted list is never advanced again
    // while the other one is real, the sentinels never compare equal, and with
    // i* = min(i, la), j* = min(j, lb) the reference's denom (steps + remainders, capped
    // at S: CommandDistance.cpp:376-415) is min(S, i* + j* - common).  Per step: two
    // compares into lane masks, three masked increments, the window shifts.
    uint32_t i = 0, j = 0, common = 0, steps = 0;
    // both lists of a pair are exhausted after at least max(la, lb) steps (each step advances
    // each index by at most one): when that is >= S on every lane the walk runs S steps and
    // the per-block test below never fires (the C3 rows: W = S entries each)
    const bool full = !__any(max(la, lb) < S);
    for (uint32_t d0 = 0; d0 < S; d0 += BLK) {
        if (!full && !__any((i < la) | (j < lb))) break;
        uint32_t a[BLK], b[BLK];
#pragma unroll
        for (int u = 0; u < BLK; u++) {
            a[u] = A[(i + u) * kAs];
            b[u] = B[j + u];
        }
#pragma unroll
        for (int u = 0; u < BLK; u++) {
            if (d0 + u >= S) break;                    // uniform
            // every step advances i, j or both (both exactly on an equal pair), so after n
            // steps i + j = n + common: no per-step count of the equal pairs
            const uint64_t ma = __builtin_amdgcn_ballot_w64(a[0] <= b[0]);
            const uint64_t mb = __builtin_amdgcn_ballot_w64(b[0] <= a[0]);
            steps++;
            i = add_mask(i, ma);
            j = add_mask(j, mb);
#pragma unroll
            for (int v = 0; v + 1 < BLK - u; v++) {
                a[v] = lane_sel(a[v], a[v + 1], ma);
                b[v] = lane_sel(b[v], b[v + 1], mb);
            }
        }
    }
    common = i + j - steps;
    const uint32_t is = min(i, la), js = min(j, lb);
    const uint32_t d = min(S, is + js - common);
    const uint64_t o = (uint64_t)q * n_ref + r;
    numer[o] = (C)common;
    denom[o] = (C)d;
}

bool compare_grid_img_ok(uint32_t hash_bytes, uint32_t sketch_size, uint64_t ref_stride,
                         uint64_t qry_stride)
{
    const uint64_t W = std::min<uint64_t>(sketch_size, std::max(ref_stride, qry_stride));
    // the padded walk runs S steps inside rows of W + BLK entries: S <= W
    return hash_bytes == 4 && W >= 64 && W <= kImgMaxW && sketch_size <= W;
}

void compare_grid_img_scratch(uint32_t n_qry, uint32_t sketch_size, uint64_t ref_stride,
                              uint64_t qry_stride, size_t *ublk_bytes, size_t *bimg_bytes)
{
    const uint64_t W = std::min<uint64_t>(sketch_size, std::max(ref_stride, qry_stride));
    const uint64_t nqb = (n_qry + kImgTile - 1) / kImgTile;
    const uint64_t Wimg = (W + 7) & ~7ull;
    *ublk_bytes = nqb * kImgBlk * 4 + nqb * 8 + 64;
    *bimg_bytes = (uint64_t)n_qry * Wimg * 2 + 64;
}

template <typename C>
static hipError_t compare_grid_img_c(const uint32_t *ref, const uint32_t *ref_len,
                                     uint64_t ref_stride, uint32_t n_ref, const uint32_t *qry,
                                     const uint32_t *qry_len, uint64_t qry_stride, uint32_t n_qry,
                                     uint32_t S, void *ublk_p, void *bimg_p, C *numer, C *denom,
                                     hipStream_t st)
{
    constexpr int kBlk = kImgBlk3;
    const uint32_t W = (uint32_t)std::min<uint64_t>(S, std::max(ref_stride, qry_stride));
    const uint32_t nqb = (n_qry + kImgTile - 1) / kImgTile, nrb = (n_ref + kImgTile - 1) / kImgTile;
    const uint32_t Wimg = (W + 7) & ~7u, Wp = img_row_u16(W, kBlk);
    uint32_t *ublk = (uint32_t *)ublk_p, *usize = ublk + (size_t)nqb * kImgBlk;
    uint16_t *bimg = (uint16_t *)bimg_p;
    const size_t lds_u = (size_t)(kImgNP + kDir + 1) * 4;
    const size_t lds_t = std::max<size_t>((size_t)(kImgNP + kDir + 1) * 4, (size_t)2 * kImgTile * Wp * 2);
    if (hipError_t e = hipFuncSetAttribute((const void *)qblock_union_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_u))
        return e;
    const void *fn = (const void *)compare_grid_img_kernel<kBlk, C>;
    if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_t))
        return e;
    hipLaunchKernelGGL(qblock_union_kernel, dim3(nqb), dim3(1024), lds_u, st, qry, qry_len,
                       qry_stride, n_qry, W, Wimg, ublk, usize, bimg);
    // a 1-D grid: kXcds x (the XCD's own ref blocks x query blocks + its share of the leftover
    // tiles) (the kernel's tile map)
    const uint32_t per = nrb / kXcds, rem = nrb - per * kXcds;
    const uint32_t grid = kXcds * (per * nqb + (rem * nqb + kXcds - 1) / kXcds);
    hipLaunchKernelGGL((compare_grid_img_kernel<kBlk, C>), dim3(grid, 1), dim3(1024),
                       lds_t, st, ref, ref_len, ref_stride, n_ref, qry_len, n_qry,
                       (const uint32_t *)ublk, (const uint32_t *)usize, (const uint16_t *)bimg,
                       Wimg, S, W, nrb, numer, denom);
    return hipGetLastError();
}

hipError_t launch_compare_grid_img(const void *d_ref, const uint32_t *d_ref_len,
                                   uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                   const uint32_t *d_qry_len, uint64_t qry_stride, uint32_t n_qry,
                                   uint32_t sketch_size, void *ublk, void *bimg, Counts cnt,
                                   hipStream_t st)
{
    if (n_ref == 0 || n_qry == 0) return hipSuccess;
    if (cnt.c16)
        return compare_grid_img_c((const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                                  (const uint32_t *)d_qry, d_qry_len, qry_stride, n_qry,
                                  sketch_size, ublk, bimg, (uint16_t *)cnt.numer,
                                  (uint16_t *)cnt.denom, st);
    return compare_grid_img_c((const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                              (const uint32_t *)d_qry, d_qry_len, qry_stride, n_qry, sketch_size,
                              ublk, bimg, (uint32_t *)cnt.numer, (uint32_t *)cnt.denom, st);
}

template <typename C>
static hipError_t walk_candidates_c(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                    uint64_t cap, const void *d_ref, const uint32_t *d_ref_len,
                                    uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                    const uint32_t *d_qry_len, uint64_t qry_stride,
                                    uint32_t hash_bytes, uint32_t S, RecRows rr, RecRows rq,
                                    C *d_numer, C *d_denom, hipStream_t st)
{
    dim3 grid((uint32_t)((cap + 255) / 256));
    if (hash_bytes == 8)
        hipLaunchKernelGGL((walk_cand_kernel<uint64_t, C>), grid, dim3(256), 0, st, d_cand, d_n_cand,
                           (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint64_t *)d_qry, d_qry_len, qry_stride, S, rr, rq, d_numer,
                           d_denom);
    else
        hipLaunchKernelGGL((walk_cand_kernel<uint32_t, C>), grid, dim3(256), 0, st, d_cand, d_n_cand,
                           (const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint32_t *)d_qry, d_qry_len, qry_stride, S, rr, rq, d_numer,
                           d_denom);
    return hipGetLastError();
}

hipError_t launch_walk_candidates(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                  uint64_t cap, const void *d_ref, const uint32_t *d_ref_len,
                                  uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                  const uint32_t *d_qry_len, uint64_t qry_stride,
                                  uint32_t hash_bytes, uint32_t S, Counts cnt, RecRows rec_ref,
                                  RecRows rec_qry, hipStream_t st)
{
    if (!cap) return hipSuccess;
    if (!rec_ref.val || !rec_qry.val) rec_ref = rec_qry = RecRows{};   // both sides or neither
    if (cnt.c16)
        return walk_candidates_c(d_cand, d_n_cand, cap, d_ref, d_ref_len, ref_stride, n_ref, d_qry,
                                 d_qry_len, qry_stride, hash_bytes, S, rec_ref, rec_qry,
                                 (uint16_t *)cnt.numer, (uint16_t *)cnt.denom, st);
    return walk_candidates_c(d_cand, d_n_cand, cap, d_ref, d_ref_len, ref_stride, n_ref, d_qry,
                             d_qry_len, qry_stride, hash_bytes, S, rec_ref, rec_qry,
                             (uint32_t *)cnt.numer, (uint32_t *)cnt.denom, st);
}

hipError_t launch_dist_finalize(Counts cnt, const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                                uint32_t n_ref, uint32_t n_qry, uint32_t kmer_size,
                                double kmer_space, double max_dist, double max_pvalue,
                                double *d_dist, double *d_pvalue, uint8_t *d_pass,
                                hipStream_t st)
{
    uint64_t n = (uint64_t)n_ref * n_qry;
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 255) / 256;
#define FPM_DFIN(C)                                                                          \
    hipLaunchKernelGGL(dist_finalize_kernel<C>, dim3((uint32_t)blocks), dim3(256), 0, st,       \
                       (const C *)cnt.numer, (const C *)cnt.denom, d_ref_length, d_qry_length, \
                       n_ref, n, kmer_size, kmer_space, max_dist, max_pvalue, d_dist, d_pvalue, \
                       d_pass)
    if (cnt.c16) FPM_DFIN(uint16_t);
    else FPM_DFIN(uint32_t);
#undef FPM_DFIN
    return hipGetLastError();
}

}  // namespace fpm
