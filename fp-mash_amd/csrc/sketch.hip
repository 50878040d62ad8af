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
constexpr int kSkWpe = 7;   // waves per SIMD asked of the tile kernel for P <= 2048
constexpr int kSkWpeThr = 8;   // and of the survivors-only instance (17.9 KB of LDS: 8 tiles per CU)
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

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The first s distinct values of the ascending keys[0, nv) to row[0, s): slot i = e * 256 + tid
// (round e, lane-consecutive), kept iff it starts a run of equal keys; its rank = the kept
// count of the (round, wave) pairs before it + its lane prefix in the wave's ballot.  Stores
// of consecutive lanes land at consecutive ranks.  `wcnt` holds E * 4 + 1 dwords of LDS;
// *total = the distinct count (all of keys[0, nv), not capped at s).
template <int P>
__device__ __forceinline__ void write_distinct(const uint64_t *keys, uint32_t nv, uint64_t *row,
                                               uint32_t s, uint32_t *wcnt, uint32_t *total, int tid)
{
    constexpr int E = P / kBlock;
    constexpr int NW = E * kWaves;
    constexpr int PL = (NW + 63) / 64;                     // pairs per lane of the scan
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * kBlock + tid);
        const bool f = i < nv && (i == 0 || keys[i] != keys[i - 1]);
        const uint64_t m = __ballot(f);
        if (lane == 0) wcnt[e * kWaves + wave] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (tid < 64) {
        uint32_t v[PL], sum = 0;
#pragma unroll
        for (int q = 0; q < PL; q++) {
            const int i = tid * PL + q;
            v[q] = i < NW ? wcnt[i] : 0u;
            sum += v[q];
        }
        uint32_t x = sum;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        uint32_t ex = x - sum;
#pragma unroll
        for (int q = 0; q < PL; q++) {
            const int i = tid * PL + q;
            if (i < NW) wcnt[i] = ex;
            ex += v[q];
        }
        if (tid == 63) wcnt[NW] = x;
    }
    __syncthreads();
    *total = wcnt[NW];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const uint32_t i = (uint32_t)(e * kBlock + tid);
        const uint64_t key = i < nv ? keys[i] : 0ULL;
        const bool f = i < nv && (i == 0 || key != keys[i - 1]);
        const uint64_t m = __ballot(f);
        const uint32_t rank = wcnt[e * kWaves + wave] + lane_prefix(m);
        if (f && rank < s) row[rank] = key;
    }
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

// SWAR helpers on 4 ASCII bytes
__device__ __forceinline__ uint32_t upper4(uint32_t x)
{
    // bytes in 'a'..'z' (0x61..0x7a) lose 0x20 (Sketch.cpp:676-682); per byte: x >= 0x61 and
    // x <= 0x7a, computed without carries between bytes
    const uint32_t hi = x & 0x80808080u, lo = x & 0x7f7f7f7fu;
    const uint32_t ge = (lo + 0x1f1f1f1fu) & ~hi;              // bit 7: lo >= 0x61
    const uint32_t le = ~(lo + 0x05050505u) & ~hi;             // bit 7: lo <= 0x7a
    const uint32_t m = (ge & le & 0x80808080u) >> 2;           // 0x20 in the lowercase bytes
    return x - m;
}

// complement of A/C/G/T (Sketch.cpp:1223-1250: A<->T, C<->G).  Other bytes never take part in
// a canonical comparison (their windows are invalid), so their image value is irrelevant.
__device__ __forceinline__ uint32_t compl4(uint32_t x)
{
    // C 0x43 / G 0x47 have bit 1 set: xor 0x04; A 0x41 / T 0x54 clear: xor 0x15
    const uint32_t b1 = (x >> 1) & 0x01010101u;
    return x ^ (b1 * 0x04u + (b1 ^ 0x01010101u) * 0x15u);
}

// LDS layout of one staged tile (the sketch and the multiplicity kernels)
template <int P>
struct TileImg {
    static constexpr int E = P / kBlock;                   // windows per thread (P >= 256)
    static constexpr int kRcPad = ((E + 15) / 16) * 16;    // R positions of the last thread's
                                                           // invalid windows stay >= 0
    static constexpr int kFBytes = ((P + 31 + 15 + 96 + 31) / 32) * 32;   // even # of 16-B chunks
    static constexpr int kRBytes = ((kRcPad + P + 31 + 15 + 96 + 15) / 16) * 16;
    static constexpr int kMaskWords = kFBytes / 32 + 2;
    static constexpr int kBytes = kFBytes + kRBytes + 4 * kMaskWords + 512;   // + alpha, compl
};

// Byte images in LDS (one 16-B global load per 16 bytes, b128 LDS stores):
//   F[y]     = tile byte y - a0 (uppercased), a0 = byte_off & 15 (F starts on the 16-B
//              aligned global address below the tile)
//   R[z]     = reverse complement: tile byte x (x < n) lands at R[rc0 + n - 1 - x], with rc0
//              chosen so that F's 16-B chunks land on R's 16-B chunks reversed
//   bad bit y = F[y] is outside the tile or not in the alphabet
// `img` holds TileImg<P>::kBytes; its alphabet / complement tables (the last 512 bytes) are
// filled and made visible by the caller.
template <int P>
__device__ __forceinline__ void tile_stage(const uint8_t *__restrict__ seq, const TileDesc &td,
                                           const SketchKParams &p, uint32_t *img, int tid)
{
    using I = TileImg<P>;
    uint32_t *const fwd_img = img;
    uint32_t *const rc_img = fwd_img + I::kFBytes / 4;
    uint32_t *const badmask = rc_img + I::kRBytes / 4;
    const uint8_t *const alpha = reinterpret_cast<const uint8_t *>(badmask + I::kMaskWords);
    const uint8_t *const compl_tab = alpha + 256;
    const uint32_t n = td.n_bytes;
    const uint32_t a0 = (uint32_t)(td.byte_off & 15);
    const uint8_t *g0 = seq + (td.byte_off - a0);
    const uint32_t nimg = a0 + n;                          // F bytes holding tile data
    const uint32_t rc0 = I::kRcPad + ((16u - (nimg & 15u)) & 15u);
    constexpr int kChunks = I::kFBytes / 16;
    for (int ch = tid; ch < kChunks; ch += kBlock) {
        const uint32_t y0 = (uint32_t)ch * 16;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (y0 < nimg) v = *reinterpret_cast<const uint4 *>(g0 + y0);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t bad = 0;                                  // bit m: F[y0 + m] invalid
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (!p.preserve_case) w[q] = upper4(w[q]);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t y = y0 + 4 * q + b;
                const bool ok = y >= a0 && y < nimg && alpha[(w[q] >> (8 * b)) & 0xffu];
                bad |= (ok ? 0u : 1u) << (4 * q + b);
            }
        }
        *reinterpret_cast<uint4 *>(&fwd_img[y0 / 4]) = make_uint4(w[0], w[1], w[2], w[3]);
        if (p.canonical && y0 < nimg) {
            // F[y0 .. y0 + 16) = tile bytes x = y0 - a0 + m -> R[rc0 + n - 1 - x], i.e. the 16-B
            // chunk at zc = rc0 + nimg - 16 - y0 (16-aligned), byte order reversed
            const uint32_t zc = rc0 + nimg - 16 - y0;
            uint32_t c[4];
            if (p.compl_acgt) {
#pragma unroll
                for (int q = 0; q < 4; q++) c[q] = compl4(w[q]);
            } else {
                // alphabets beyond ACGT: the reference's complement table, byte by byte
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    uint32_t x = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        x |= (uint32_t)compl_tab[(w[q] >> (8 * b)) & 0xffu] << (8 * b);
                    c[q] = x;
                }
            }
            *reinterpret_cast<uint4 *>(&rc_img[zc / 4]) =
                make_uint4(__builtin_bswap32(c[3]), __builtin_bswap32(c[2]),
                           __builtin_bswap32(c[1]), __builtin_bswap32(c[0]));
        }
        // two chunks per badmask word: the odd chunk's bits go to the high half
        const uint32_t hi = __shfl_down(bad, 1, 64);
        if ((ch & 1) == 0) badmask[ch / 2] = bad | (hi << 16);
    }
    if (tid < 2) badmask[I::kMaskWords - 2 + tid] = 0xffffffffu;
}

// K != 0: the k-mer size as a compile-time constant (the window loads, tail masks and
// Murmur's block / tail branches fold); K = 0 reads p.k.
// Thread t hashes the E consecutive windows i = tE .. tE + E - 1 of the staged tile: their
// bytes are one run of F (and of R, backwards), loaded as ~E/4 + 9 dwords once and cut per
// window by v_alignbyte with compile-time shifts.  Returns bit e set when kr[e] is the hash
// of a valid k-mer (kr[e] = ~0 otherwise).
// Each valid window's key goes to sink(e, key) (the caller's register array, or the
// thresholded kernel's survivor slots).
template <int P, int K, typename Sink>
__device__ __forceinline__ uint32_t tile_hash(const TileDesc &td, const SketchKParams &p,
                                              const uint32_t *img, int tid, Sink &&sink)
{
    using I = TileImg<P>;
    constexpr int E = I::E;
    const uint32_t *const fwd_img = img;
    const uint32_t *const rc_img = fwd_img + I::kFBytes / 4;
    const uint32_t *const badmask = rc_img + I::kRBytes / 4;
    const uint32_t n = td.n_bytes;
    const uint32_t k = K ? (uint32_t)K : p.k;
    const uint32_t a0 = (uint32_t)(td.byte_off & 15);
    const uint32_t nimg = a0 + n;
    const uint32_t rc0 = I::kRcPad + ((16u - (nimg & 15u)) & 15u);
    const uint32_t nk = n >= k ? n - k + 1 : 0;
    const int nw = (k + 3) >> 2;                           // dwords per k-mer
    const uint32_t tail_mask = (k & 3) ? ((1u << (8 * (k & 3))) - 1u) : 0xffffffffu;
    const uint32_t kmask = (k == 32) ? 0xffffffffu : ((1u << k) - 1u);
    constexpr int KW = K ? (K + 3) / 4 : 8;                // dwords per window (max)
    constexpr int W = (E + 3) / 4 + KW + 1;                // dwords covering the E windows
    uint32_t vbits = 0;                                    // bit e: window e is a valid k-mer
    // the seed through an opaque move: otherwise the compiler, short of SGPRs in the unrolled
    // window loop, reloads it from the kernel arguments once per window (an s_load and an
    // s_waitcnt lgkmcnt(0) per hash)
    uint32_t seed;
    asm volatile("s_mov_b32 %0, %1" : "=s"(seed) : "s"(p.seed));
    const uint32_t i0 = (uint32_t)tid * E;
    if (i0 < nk) {
        // validity of the E windows from one 64-bit read of the bit image
        const uint32_t yb = a0 + i0;
        uint32_t okbits = 0;
        {
            // bits [yb, yb + 64) of the bit image (E + k - 1 <= 63 of them are used)
            const uint32_t wq = yb >> 5, sh = yb & 31;
            uint64_t bits = ((uint64_t)badmask[wq] | ((uint64_t)badmask[wq + 1] << 32)) >> sh;
            if (sh) bits |= (uint64_t)badmask[wq + 2] << (64 - sh);
#pragma unroll
            for (int e = 0; e < E; e++) {
                // window e's k bits start at bit e of `bits` (E + k <= 64 for E <= 32)
                const bool ok = i0 + e < nk && (((uint32_t)(bits >> e) & kmask) == 0);
                okbits |= (ok ? 1u : 0u) << e;
            }
        }
        if (okbits) {
            // forward run: S[m] = the dwords of F from byte yb
            uint32_t S[W];
            {
                const uint32_t q0 = yb >> 2, sh0 = yb & 3;
                uint32_t D[W + 1];
#pragma unroll
                for (int m = 0; m <= W; m++) D[m] = fwd_img[q0 + m];
#pragma unroll
                for (int m = 0; m < W; m++) S[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], sh0);
            }
            // reverse-complement run: window e's rc bytes start at R[rc0 + n - (i0 + e) - k]
            // = R[zb + (E - 1 - e)], zb the start for e = E - 1
            uint32_t SR[W];
            if (p.canonical) {
                const uint32_t zb = rc0 + n - i0 - k - (E - 1);
                const uint32_t qr = zb >> 2, shr = zb & 3;
                uint32_t D[W + 1];
#pragma unroll
                for (int m = 0; m <= W; m++) D[m] = rc_img[qr + m];
#pragma unroll
                for (int m = 0; m < W; m++) SR[m] = __builtin_amdgcn_alignbyte(D[m + 1], D[m], shr);
            }
#pragma unroll
            for (int e = 0; e < E; e++) {
                if (!(okbits >> e & 1)) continue;
                uint32_t d[8];
#pragma unroll
                for (int m = 0; m < 8; m++)
                    d[m] = (m < nw) ? __builtin_amdgcn_alignbyte(S[(e >> 2) + m + 1], S[(e >> 2) + m],
                                                                 e & 3)
                                    : 0u;
                d[nw - 1] &= tail_mask;
                if (p.canonical) {
                    // canonical = memcmp(fwd, rev) <= 0 ? fwd : rev (Sketch.cpp:719-723)
                    const int f = E - 1 - e;   // unrolled: a constant
                    uint32_t r[8];
#pragma unroll
                    for (int m = 0; m < 8; m++)
                        r[m] = (m < nw) ? __builtin_amdgcn_alignbyte(SR[(f >> 2) + m + 1],
                                                                     SR[(f >> 2) + m], f & 3)
                                        : 0u;
                    r[nw - 1] &= tail_mask;
                    // memcmp order = the big-endian order of the bytes: 64-bit big-endian words
                    // (dwords past nw are 0 in both), compared most significant first with
                    // lane masks (3 64-bit compares for k = 21 instead of a per-dword chain)
                    constexpr int NQ = K ? ((K + 3) / 4 + 1) / 2 : 4;
                    bool gt = false, eq = true;
#pragma unroll
                    for (int q = 0; q < NQ; q++) {
                        const uint64_t fq = ((uint64_t)__builtin_bswap32(d[2 * q]) << 32) |
                                            __builtin_bswap32(d[2 * q + 1]);
                        const uint64_t rq = ((uint64_t)__builtin_bswap32(r[2 * q]) << 32) |
                                            __builtin_bswap32(r[2 * q + 1]);
                        gt = gt || (eq && fq > rq);
                        eq = eq && fq == rq;
                    }
                    const int cmp = gt ? 1 : 0;
                    if (cmp > 0) {
#pragma unroll
                        for (int m = 0; m < 8; m++) d[m] = r[m];
                    }
                }
                uint64_t wd[4];
#pragma unroll
                for (int j = 0; j < 4; j++) wd[j] = (uint64_t)d[2 * j] | ((uint64_t)d[2 * j + 1] << 32);
                const uint64_t h = murmur_h1_le32(wd, (int)k, seed);
                sink(e, p.use64 ? h : (h & 0xffffffffULL));   // getHash hash.cpp:30-37
            }
            vbits = okbits;
        }
    }
    return vbits;
}

// THR (tiles of long groups, every one with a bound: C5's genomes): the windows' keys above the
// group's bound are dropped as they are hashed, the others go to kSurv LDS slots of their
// thread and, past those, to a block-shared overflow area (an LDS atomic), so no thread holds
// E keys in registers (VGPRs 128 -> 68: 7 waves per SIMD instead of 4) and the sort runs on at
// most kBlock * kSurv + kSurvShared = 1024 keys (a bound keeps ~3 % of a tile's 4,096: ~0.5
// per thread).  A tile whose survivors do not fit appends itself to `redo` and writes
// nothing; the caller runs those tiles again through the plain kernel.  (4 slots per thread
// and no shared area sent 2.7 % of C5's tiles to the redo pass.)
constexpr int kSurv = 2;
constexpr int kSurvShared = 512;
static_assert(kBlock * kSurv + kSurvShared == (int)kThrTileKeys, "fpm_api.cpp sizes thr4 by it");
// One tile: the body of sketch_tiles_kernel (one workgroup per tile) and of
// sketch_redo_kernel (the tiles a THR pass listed, taken in turn by a fixed grid).
template <int P, int K, bool THR>
__device__ __forceinline__ void sketch_tile(
    const uint8_t *__restrict__ seq, const TileDesc td, SketchKParams p,
    const uint64_t *__restrict__ thr, uint64_t *__restrict__ out, uint32_t *__restrict__ out_count,
    TileDesc *__restrict__ redo, uint32_t *__restrict__ redo_n)
{
    using I = TileImg<P>;
    constexpr int E = I::E;
    constexpr int PS = THR ? kBlock * kSurv + kSurvShared : P;   // keys the sort holds at most
    constexpr int ES = PS / kBlock;                         // their slots per thread
    // the staging images live inside keys[] (dead before the first key is scattered): 20 KB
    // of LDS per P = 2048 tile instead of 25.7 KB, 7 tiles per CU instead of 6
    constexpr int KW = THR ? (PS > (I::kBytes + 7) / 8 ? PS : (I::kBytes + 7) / 8) : P;
    __shared__ __attribute__((aligned(16))) uint64_t keys[KW];
    static_assert(I::kBytes <= 8 * KW, "staging fits in keys");
    // THR: the sort's bucket counters (bins) reuse the survivor slots, dead once their keys
    // are copied into keys[]: 17.7 KB of LDS per tile instead of 21.9 KB (9 tiles per CU fit,
    // 8 by waves)
    constexpr int kBins = P >= 4096 ? P / 4 : P / 2;
    static_assert(!THR || kBins <= 2 * (kBlock * kSurv + kSurvShared), "bins fit the slots");
    __shared__ uint64_t surv[THR ? kBlock * kSurv + kSurvShared : 1];   // shared area last
    __shared__ uint32_t s_over, s_shared;
    uint32_t *const img = reinterpret_cast<uint32_t *>(keys);
    uint8_t *const alpha = reinterpret_cast<uint8_t *>(img + (I::kFBytes + I::kRBytes) / 4 +
                                                       I::kMaskWords);
    uint8_t *const compl_tab = alpha + 256;
    __shared__ uint32_t scan_tmp[kWaves + 1];
    __shared__ uint32_t wcnt[ES * kWaves + 1];
    __shared__ uint32_t bins_own[THR ? 1 : kBins];
    uint32_t *const bins = THR ? reinterpret_cast<uint32_t *>(surv) : bins_own;
    __shared__ uint32_t big_bucket, s_cut;

    FPM_PHASE_DECL;
    FPM_PHASE(0);
    const int tid = threadIdx.x;

    alpha[tid] = p.alphabet[tid];
    compl_tab[tid] = p.complement[tid];
    if (THR && tid == 0) { s_over = 0; s_shared = 0; }
    __syncthreads();

    // ---- stage the tile: uppercase, validity bits, reverse complement
    tile_stage<P>(seq, td, p, img, tid);
    __syncthreads();
    FPM_PHASE(1);

    uint64_t kr[ES];                                       // key of window tE + e (THR: of
    uint32_t vbits;                                        // sort slot e * kBlock + tid)
    uint64_t hmax = p.use64 ? ~0ULL : 0xffffffffULL;
    if constexpr (THR) {
        // ---- hash, keeping the keys <= the group's bound in this thread's survivor slots
        hmax = min(hmax, thr[td.thr_slot - 1]);
        uint32_t ns = 0;
        tile_hash<P, K>(td, p, img, tid, [&](int, uint64_t h) {
            if (h <= hmax) {
                if (ns < (uint32_t)kSurv) {
                    surv[tid * kSurv + ns] = h;
                    ns++;
                } else {
                    const uint32_t j = atomicAdd(&s_shared, 1u);
                    if (j < (uint32_t)kSurvShared) surv[kBlock * kSurv + j] = h;
                    else s_over = 1;
                }
            }
        });
        uint32_t total;
        uint32_t at = block_exscan(ns, scan_tmp, &total);      // (barriers: s_over settled)
        if (s_over) {                                          // block-uniform
            if (tid == 0) redo[atomicAdd(redo_n, 1u)] = td;
            return;
        }
        // keys[] aliases the staging images: every window read is done (the scan's barriers);
        // the shared area's keys follow the threads' own
        for (uint32_t i = 0; i < ns; i++) keys[at + i] = surv[tid * kSurv + i];
        const uint32_t nsh = s_shared;
        for (uint32_t i = tid; i < nsh; i += kBlock) keys[total + i] = surv[kBlock * kSurv + i];
        total += nsh;
        __syncthreads();
        if (total <= 64) {
            // (block-uniform) a tight bound leaves a C5 tile ~15 survivors: one wave ranks them
            // against each other (a loop of `total` broadcasts), drops repeats and writes the row,
            // instead of the bucket table, its scans and barriers below
            if (tid < 64) {
                const uint64_t v = tid < total ? keys[tid] : 0;
                const uint32_t vlo = (uint32_t)v, vhi = (uint32_t)(v >> 32);
                // the first copy of each value, then the distinct values below each key
                bool first = tid < total;
#pragma unroll 1
                for (uint32_t j = 0; j < total; j++) {
                    const uint64_t y = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)vhi, (int)j) << 32) |
                                       (uint32_t)__builtin_amdgcn_readlane((int)vlo, (int)j);
                    first = first && !(j < tid && y == v);
                }
                const uint64_t fm = __builtin_amdgcn_ballot_w64(first);
                uint32_t rank = 0;
#pragma unroll 1
                for (uint32_t j = 0; j < total; j++) {
                    const uint64_t y = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)vhi, (int)j) << 32) |
                                       (uint32_t)__builtin_amdgcn_readlane((int)vlo, (int)j);
                    rank += ((fm >> j) & 1) && y < v ? 1u : 0u;
                }
                if (first && rank < p.s) out[(uint64_t)td.out_row * p.s + rank] = v;
                if (tid == 0) {
                    const uint32_t nd = (uint32_t)__popcll(fm);
                    out_count[td.out_row] = nd < p.s ? nd : p.s;
                }
            }
            return;
        }
        vbits = 0;
#pragma unroll
        for (int e = 0; e < ES; e++) {
            const uint32_t j = (uint32_t)tid + (uint32_t)e * kBlock;
            kr[e] = ~0ULL;
            if (j < total) { kr[e] = keys[j]; vbits |= 1u << e; }
        }
        __syncthreads();
    } else {
#pragma unroll
    for (int e = 0; e < E; e++) kr[e] = ~0ULL;
    // ---- hash this thread's E consecutive windows
    vbits = tile_hash<P, K>(td, p, img, tid, [&](int e, uint64_t h) { kr[e] = h; });

    // ---- long groups: keep only hashes <= the group's bound (the s-th smallest hash of a
    // sample of the group's tiles, an upper bound of the group's own s-th smallest)
    FPM_PHASE(2);
    if (td.thr_slot) {
        hmax = min(hmax, thr[td.thr_slot - 1]);
#pragma unroll
        for (int e = 0; e < E; e++)
            if (kr[e] > hmax) vbits &= ~(1u << e);
        // the bound keeps a few percent of the keys (C5: ~130 of 4,096): compact them to the
        // first slots of the threads (key j -> thread j % 256, slot j / 256), so the sort
        // phases below run one slot instead of E mostly-empty ones (a slot runs for the whole
        // wave as soon as one lane holds a key)
        if (E > 1) {
            uint32_t total;
            uint32_t at = block_exscan((uint32_t)__popc(vbits), scan_tmp, &total);
            if (total <= (uint32_t)(kBlock * (E / 2))) {   // block-uniform
                // keys[] aliases the staging images: every window read is done (the scan's
                // barriers) before the first write
#pragma unroll
                for (int e = 0; e < E; e++)
                    if (vbits >> e & 1) keys[at++] = kr[e];
                __syncthreads();
                vbits = 0;
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const uint32_t j = (uint32_t)tid + (uint32_t)e * kBlock;
                    if (j < total) { kr[e] = keys[j]; vbits |= 1u << e; }
                }
                __syncthreads();
            }
        }
    }
    }

    // ---- sort: counting sort by the top log2(P/2) bits of the (uniform) hash values in
    // [0, hmax], then insertion sort inside each bucket (~2 keys per bucket).  A bucket
    // holding more than kMaxBucket keys (low-complexity input: many copies of few k-mers)
    // sends the whole tile to the bitonic sort instead.
    // ~2 keys per bucket; 4 for the long-record tiles (P >= 4096: C5's chunks keep only the
    // keys below their group's sampled bound, so their buckets are sparse anyway, and the
    // smaller table lets 4 tiles share a CU)
    constexpr int NB = P >= 4096 ? P / 4 : P / 2;
    constexpr int LB = __builtin_ctz(NB);
    constexpr uint32_t kMaxBucket = 32;
    const uint32_t hbits = hmax ? 64 - __clzll(hmax) : 1;
    const uint32_t bshift = hbits > (uint32_t)LB ? hbits - LB : 0;
    for (int b = tid; b < NB; b += kBlock) bins[b] = 0;
    if (tid == 0) { big_bucket = 0; s_cut = NB; }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < ES; e++)
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
    // the bucket holding sorted position s - 1: every key in a later bucket is larger than
    // the s smallest keys (duplicates included), so those buckets are left out of the sort
    // unless duplicates leave fewer than s distinct values below them (then a second pass
    // places them too)
#pragma unroll
    for (int u = 0; u < per; u++) {
        const int b = tid * per + u;
        if (b < NB) {
            const uint32_t c = bins[b];
            bins[b] = acc;
            if (acc < p.s && acc + c >= p.s) s_cut = (uint32_t)b + 1;
            acc += c;
        }
    }
    if (bmax > kMaxBucket) big_bucket = 1;
    __syncthreads();
    const uint32_t cut = big_bucket ? (uint32_t)NB : s_cut;
    const uint32_t nkept = cut < (uint32_t)NB ? bins[cut] : nvalid;   // before the scatter
    FPM_PHASE(4);
    uint32_t lo_b = 0, hi_b = cut, nv = nkept;
    for (int pass = 0; pass < 2; pass++) {
        // an opaque copy of the shift per pass: otherwise the compiler hoists every key's
        // bucket addresses (2 x E VGPRs) out of this loop and spills (72-VGPR budget at P = 2048)
        uint32_t bsh = bshift;
        asm volatile("" : "+v"(bsh));
        // scatter the keys of buckets [lo_b, hi_b): afterwards bins[b] = end of bucket b,
        // start = bins[b - 1]; each key keeps its slot for the in-bucket rank below
        uint32_t act = 0;
#pragma unroll
        for (int e = 0; e < ES; e++) {
            const uint32_t bk = (uint32_t)(kr[e] >> bsh);
            act |= ((vbits >> e & 1) && bk >= lo_b && bk < hi_b) ? (1u << e) : 0u;
        }
        uint32_t slot[ES];
#pragma unroll
        for (int e = 0; e < ES; e++)
            if (act >> e & 1) {
                slot[e] = atomicAdd(&bins[(uint32_t)(kr[e] >> bsh)], 1u);
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
            for (int e = 0; e < ES; e++)
                if (act >> e & 1) {
                    const uint32_t b = (uint32_t)(kr[e] >> bsh);
                    const uint32_t s0 = b ? bins[b - 1] : 0u, s1 = bins[b];
                    const uint32_t mb = s1 - s0;
                    uint32_t r = 0;
                    // 8 speculative reads cover a bucket of <= 8 keys (Poisson(2) buckets: a
                    // longer one is rare) with one LDS round trip
#pragma unroll
                    for (uint32_t u = 0; u < 8; u++) {
                        const uint32_t t = s0 + u;
                        const uint64_t y = keys[t < (uint32_t)PS ? t : (uint32_t)PS - 1];
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
            for (int e = 0; e < ES; e++)
                if (act >> e & 1) keys[slot[e]] = kr[e];
            __syncthreads();
        } else {
            for (int i = tid; i < PS; i += kBlock)
                if ((uint32_t)i >= nvalid) keys[i] = ~0ULL;
            __syncthreads();
            bitonic_sort<PS>(keys);
        }
        FPM_PHASE(6);

        // ---- first s distinct of keys[0, nv) (ties removed: the heap is a set,
        // MinHashHeap.cpp:74).  Lane-consecutive slots (slot e * 256 + tid), so the row is
        // written by consecutive lanes at consecutive ranks (coalesced); a slot's rank is
        // the distinct count of the (round, wave) pairs before it + its lane prefix.
        uint32_t total;
        write_distinct<PS>(keys, nv, out + (uint64_t)td.out_row * p.s, p.s, wcnt, &total, tid);
        // block-uniform: done unless duplicates left fewer than s distinct in the kept buckets
        if (total >= p.s || hi_b >= (uint32_t)NB) {
            if (tid == 0) out_count[td.out_row] = total < p.s ? total : p.s;
            break;
        }
        lo_b = hi_b;
        hi_b = NB;
        nv = nvalid;
    }
    FPM_PHASE(7);
    FPM_PHASE_FLUSH;
}

template <int P, int K, bool THR = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(THR ? (K ? kSkWpeThr : 6) : P <= 2048 ? kSkWpe : P == 4096 ? 4 : 1))) void sketch_tiles_kernel(
    const uint8_t *__restrict__ seq, const TileDesc *__restrict__ tiles, SketchKParams p,
    const uint64_t *__restrict__ thr, uint64_t *__restrict__ out, uint32_t *__restrict__ out_count,
    TileDesc *__restrict__ redo, uint32_t *__restrict__ redo_n)
{
    sketch_tile<P, K, THR>(seq, tiles[blockIdx.x], p, thr, out, out_count, redo, redo_n);
}

// The tiles a THR pass could not keep (redo[0 .. *redo_n)), through the plain kernel's body:
// a fixed grid takes them in turn, so the count stays on the device (no host read between
// the two launches: fpm_sketch_run stays asynchronous on its stream).
template <int K>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void sketch_redo_kernel(
    const uint8_t *__restrict__ seq, const TileDesc *__restrict__ redo,
    const uint32_t *__restrict__ redo_n, SketchKParams p, const uint64_t *__restrict__ thr,
    uint64_t *__restrict__ out, uint32_t *__restrict__ out_count)
{
    const uint32_t n = *redo_n;
    for (uint32_t t = blockIdx.x; t < n; t += gridDim.x) {
        sketch_tile<4096, K, false>(seq, redo[t], p, thr, out, out_count, nullptr, nullptr);
        __syncthreads();                       // the next tile reuses the LDS
    }
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
                           d_seq, d_tiles, p, d_thr, d_out, d_count, nullptr, nullptr);
    else
        hipLaunchKernelGGL((sketch_tiles_kernel<P, 0>), dim3(n_tiles), dim3(kBlock), 0, st,
                           d_seq, d_tiles, p, d_thr, d_out, d_count, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_sketch_tiles_thr(const uint8_t *d_seq, const TileDesc *d_tiles, uint32_t n_tiles,
                                   const SketchKParams &p, const uint64_t *d_thr, uint64_t *d_out,
                                   uint32_t *d_count, TileDesc *d_redo, uint32_t *d_redo_n,
                                   hipStream_t st)
{
    if (n_tiles == 0) return hipSuccess;
    if (p.k == 21)
        hipLaunchKernelGGL((sketch_tiles_kernel<4096, 21, true>), dim3(n_tiles), dim3(kBlock), 0,
                           st, d_seq, d_tiles, p, d_thr, d_out, d_count, d_redo, d_redo_n);
    else
        hipLaunchKernelGGL((sketch_tiles_kernel<4096, 0, true>), dim3(n_tiles), dim3(kBlock), 0,
                           st, d_seq, d_tiles, p, d_thr, d_out, d_count, d_redo, d_redo_n);
    return hipGetLastError();
}

hipError_t launch_sketch_redo(const uint8_t *d_seq, const TileDesc *d_redo, const uint32_t *d_redo_n,
                              uint32_t max_tiles, const SketchKParams &p, const uint64_t *d_thr,
                              uint64_t *d_out, uint32_t *d_count, hipStream_t st)
{
    if (max_tiles == 0) return hipSuccess;
    // about one resident workgroup per slot of the chip (4 per CU at 128 VGPRs): most exit at
    // once (C5: no tile overflows), and a low-complexity input's many redo tiles are taken in
    // turn
    const uint32_t grid = std::min<uint32_t>(max_tiles, 1024);
    if (p.k == 21)
        hipLaunchKernelGGL((sketch_redo_kernel<21>), dim3(grid), dim3(kBlock), 0, st, d_seq, d_redo,
                           d_redo_n, p, d_thr, d_out, d_count);
    else
        hipLaunchKernelGGL((sketch_redo_kernel<0>), dim3(grid), dim3(kBlock), 0, st, d_seq, d_redo,
                           d_redo_n, p, d_thr, d_out, d_count);
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

// ---- -M multiplicities: the counts MinHashHeap keeps beside its hashes (MinHashHeap.cpp:68-146,
// multiplicityMinimum 1; written with -M, Sketch.cpp:584-596).  A hash of the final sketch is
// never evicted once inserted (an evicted hash has s smaller ones that stay), so its count is
// every occurrence from its first one on -- except the final maximum M of a full sketch: once
// the heap holds exactly the final set (position T_top = the last first-occurrence among
// the final hashes) M is the heap's top and tryInsert rejects it (`hash < top` fails, :73).
//   pass 0: each window hashing into its group's sketch adds 1 to its count (not M of a full
//           sketch) and takes the min of its position into first[]
//   pass 1: windows hashing to M of a full sketch at positions <= T_top add 1 to M's count
// Position = the window's byte offset in the staged buffer (a group's records are laid out in
// stream order).  Tiles carry their group in TileDesc::pad.
__device__ __forceinline__ uint32_t lower_bound_row(const uint64_t *__restrict__ v, uint32_t n,
                                                    uint64_t x)
{
    uint32_t lo = 0;
    while (n) {
        const uint32_t h = n >> 1;
        if (v[lo + h] < x) { lo += h + 1; n -= h + 1; }
        else n = h;
    }
    return lo;
}

template <int P>
__global__ __launch_bounds__(kBlock) void sketch_mult_kernel(
    const uint8_t *__restrict__ seq, const TileDesc *__restrict__ tiles, SketchKParams p,
    const uint64_t *__restrict__ rows, const uint32_t *__restrict__ count, int pass,
    uint32_t *__restrict__ mult, unsigned long long *__restrict__ first,
    const uint64_t *__restrict__ ttop)
{
    using I = TileImg<P>;
    constexpr int E = I::E;
    __shared__ __attribute__((aligned(16))) uint32_t img[I::kBytes / 4];
    uint8_t *const alpha = reinterpret_cast<uint8_t *>(img + (I::kFBytes + I::kRBytes) / 4 +
                                                       I::kMaskWords);
    uint8_t *const compl_tab = alpha + 256;
    const TileDesc td = tiles[blockIdx.x];
    const uint32_t g = td.pad;
    const uint32_t ng = count[g];
    const bool full = ng >= p.s;
    // block-uniform exits
    if (ng == 0) return;
    if (pass == 1 && (!full || td.byte_off > ttop[g])) return;
    const int tid = threadIdx.x;
    alpha[tid] = p.alphabet[tid];
    compl_tab[tid] = p.complement[tid];
    __syncthreads();
    tile_stage<P>(seq, td, p, img, tid);
    __syncthreads();
    uint64_t kr[E];
#pragma unroll
    for (int e = 0; e < E; e++) kr[e] = ~0ULL;
    const uint32_t vbits = tile_hash<P, 0>(td, p, img, tid, [&](int e, uint64_t h) { kr[e] = h; });
    const uint64_t *row = rows + (uint64_t)g * p.s;
    const uint64_t hmax = row[ng - 1];
    uint32_t *mrow = mult + (uint64_t)g * p.s;
#pragma unroll
    for (int e = 0; e < E; e++) {
        if (!(vbits >> e & 1) || kr[e] > hmax) continue;
        const uint64_t pos = td.byte_off + (uint64_t)tid * E + e;
        if (pass == 0) {
            const uint32_t i = lower_bound_row(row, ng, kr[e]);
            if (row[i] != kr[e]) continue;
            if (!(full && i == ng - 1)) atomicAdd(&mrow[i], 1u);
            atomicMin(&first[(uint64_t)g * p.s + i], (unsigned long long)pos);
        } else if (kr[e] == hmax && pos <= ttop[g]) {
            atomicAdd(&mrow[ng - 1], 1u);
        }
    }
}

// T_top of each full group: the largest first-occurrence position among its hashes
__global__ __launch_bounds__(kBlock) void mult_ttop_kernel(const uint32_t *__restrict__ count,
                                                         uint32_t n_groups, uint32_t s,
                                                         const unsigned long long *__restrict__ first,
                                                         uint64_t *__restrict__ ttop)
{
    __shared__ unsigned long long red[kWaves];
    const uint32_t g = blockIdx.x;
    if (g >= n_groups) return;
    const uint32_t ng = count[g];
    unsigned long long m = 0;
    for (uint32_t i = threadIdx.x; i < ng; i += kBlock) m = max(m, first[(uint64_t)g * s + i]);
    for (int o = 32; o; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kWaves; w++) m = max(m, red[w]);
        ttop[g] = m;
    }
}

hipError_t launch_sketch_mult(int cls, int pass, const uint8_t *d_seq, const TileDesc *d_tiles,
                              uint32_t n_tiles, const SketchKParams &p, const uint64_t *d_rows,
                              const uint32_t *d_count, uint32_t *d_mult,
                              unsigned long long *d_first, const uint64_t *d_ttop, hipStream_t st)
{
    if (n_tiles == 0) return hipSuccess;
#define FPM_MULT_CASE(c, P)                                                                    \
    case c:                                                                                    \
        hipLaunchKernelGGL((sketch_mult_kernel<P>), dim3(n_tiles), dim3(kBlock), 0, st, d_seq,  \
                           d_tiles, p, d_rows, d_count, pass, d_mult, d_first, d_ttop);         \
        break;
    switch (cls) {
        FPM_MULT_CASE(0, 256)
        FPM_MULT_CASE(1, 512)
        FPM_MULT_CASE(2, 1024)
        FPM_MULT_CASE(3, 2048)
        FPM_MULT_CASE(4, 4096)
        FPM_MULT_CASE(5, 8192)
    default: return hipErrorInvalidValue;
    }
#undef FPM_MULT_CASE
    return hipGetLastError();
}

hipError_t launch_mult_ttop(const uint32_t *d_count, uint32_t n_groups, uint32_t s,
                            const unsigned long long *d_first, uint64_t *d_ttop, hipStream_t st)
{
    if (n_groups == 0) return hipSuccess;
    hipLaunchKernelGGL(mult_ttop_kernel, dim3(n_groups), dim3(kBlock), 0, st, d_count, n_groups,
                       s, d_first, d_ttop);
    return hipGetLastError();
}

// thr_safe[i] = the s-th smallest of sample row srow[i] when it holds s hashes (a subset's
// order statistic: >= the group's own s-th smallest), else no bound.  thr[i] = the tighter
// kt[i]-th smallest (kt: null = the safe bound): the sample holds ~f of the group's windows,
// so ~kt / f of the group's distinct hashes lie below it, and kt = f s + 8 sqrt(f s) + 32
// leaves the group >= s of them unless its values repeat across its tiles; a group left with
// fewer than s is found after its selection (sketch_short_kernel) and redone with thr_safe.
__global__ void sketch_threshold_kernel(const uint32_t *__restrict__ srow, uint32_t n_slots,
                                        const uint64_t *__restrict__ rows,
                                        const uint32_t *__restrict__ count, uint32_t s,
                                        const uint32_t *__restrict__ kt,
                                        uint64_t *__restrict__ thr, uint64_t *__restrict__ thr_safe)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots) return;
    const uint32_t r = srow[i];
    const bool full = count[r] >= s;
    const uint64_t safe = full ? rows[(uint64_t)r * s + s - 1] : ~0ULL;
    if (thr_safe) thr_safe[i] = safe;
    thr[i] = full && kt ? rows[(uint64_t)r * s + min(kt[i], s) - 1] : safe;
}

hipError_t launch_sketch_threshold(const uint32_t *d_srow, uint32_t n_slots, const uint64_t *d_rows,
                                   const uint32_t *d_count, uint32_t s, const uint32_t *d_kt,
                                   uint64_t *d_thr, uint64_t *d_thr_safe, hipStream_t st)
{
    if (!n_slots) return hipSuccess;
    hipLaunchKernelGGL(sketch_threshold_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, st,
                       d_srow, n_slots, d_rows, d_count, s, d_kt, d_thr, d_thr_safe);
    return hipGetLastError();
}

// The sampled groups whose tight bound left fewer than s distinct hashes (their values repeat
// across tiles): listed in short_slots[0 .. *n_short) (zeroed by the caller), and with `raise`
// their bound raised to the safe one for the redo of their tiles and selection (a listing
// without it has no effect but the list, so it may run before the counts are known final).
// Under the safe bound (the sample's s-th smallest, < ~0 when the sample holds s values) a
// group always keeps >= s, so a count below s means the tight bound.
__global__ void sketch_short_kernel(const uint32_t *__restrict__ slot_group, uint32_t n_slots,
                                    const uint32_t *__restrict__ count, uint32_t s,
                                    uint64_t *__restrict__ thr,
                                    const uint64_t *__restrict__ thr_safe,
                                    uint32_t *__restrict__ n_short, uint32_t *__restrict__ short_slots,
                                    uint32_t raise)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots) return;
    if (count[slot_group[i]] < s && thr[i] < thr_safe[i]) {
        short_slots[atomicAdd(n_short, 1u)] = i;
        if (raise) thr[i] = thr_safe[i];
    }
}

// The samples whose a-priori bound (sbound[i], fpm_sketch_stage) left fewer than s hashes
// (values repeated across the sample's tiles): listed, and their bound lifted for the redo.
__global__ void sketch_sample_short_kernel(const uint32_t *__restrict__ srow, uint32_t n_slots,
                                           const uint32_t *__restrict__ count, uint32_t s,
                                           uint64_t *__restrict__ sbound,
                                           uint32_t *__restrict__ n_short,
                                           uint32_t *__restrict__ short_slots, uint32_t raise)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_slots) return;
    if (count[srow[i]] < s && sbound[i] != ~0ULL) {
        short_slots[atomicAdd(n_short, 1u)] = i;
        if (raise) sbound[i] = ~0ULL;
    }
}

hipError_t launch_sketch_sample_short(const uint32_t *d_srow, uint32_t n_slots,
                                      const uint32_t *d_count, uint32_t s, uint64_t *d_sbound,
                                      uint32_t *d_n_short, uint32_t *d_short_slots, bool raise,
                                      hipStream_t st)
{
    if (!n_slots) return hipSuccess;
    hipLaunchKernelGGL(sketch_sample_short_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, st,
                       d_srow, n_slots, d_count, s, d_sbound, d_n_short, d_short_slots,
                       (uint32_t)raise);
    return hipGetLastError();
}

hipError_t launch_sketch_short(const uint32_t *d_slot_group, uint32_t n_slots,
                               const uint32_t *d_count, uint32_t s, uint64_t *d_thr,
                               const uint64_t *d_thr_safe, uint32_t *d_n_short,
                               uint32_t *d_short_slots, bool raise, hipStream_t st)
{
    if (!n_slots) return hipSuccess;
    hipLaunchKernelGGL(sketch_short_kernel, dim3((n_slots + 255) / 256), dim3(256), 0, st,
                       d_slot_group, n_slots, d_count, s, d_thr, d_thr_safe, d_n_short,
                       d_short_slots, (uint32_t)raise);
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
constexpr int kSBlock = 256, kSWaves = kSBlock / 64;
constexpr uint32_t kSCap = 2048;
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

// merges whose lists did not fit kSCap (searched in global memory): the host's length
// estimate mis-routed them (results are the same, only slower); read by fpm_merge_small_spills
__device__ unsigned long long g_merge_small_spill;

__global__ __launch_bounds__(kSBlock) void merge_small_kernel(const MergeDesc *__restrict__ descs,
                                                              uint32_t s)
{
    __shared__ uint64_t sl[kSCap];
    __shared__ uint32_t scan_tmp[kSWaves];
    const MergeDesc md = descs[blockIdx.x];
    const uint32_t la = *md.alen, lb = md.b ? *md.blen : 0;
    const bool bfit = lb <= kSCap;
    if (threadIdx.x == 0 && (!bfit || (lb && la > kSCap))) atomicAdd(&g_merge_small_spill, 1ULL);
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

// ---- one sketch from the bounded tile lists of a long group (C5 genomes), in one workgroup.
// After the sample bound, a genome's ~1,200 tile lists hold ~16 s keys in all (each list
// ascending and distinct, lists may share values: repeats across chunks).  Instead of ~11
// rounds of pairwise merges, the group's workgroup selects directly:
//   1. a 4096-bucket histogram over [0, bound] of every kept key -> the bucket b1 holding
//      sorted position T - 1 (T = s plus slack for values repeated across lists)
//   2. the keys below R = (b1 + 1) buckets (m ~ T of them) are counting-sorted in LDS by a
//      second 4096-bucket histogram over [0, R), ranked inside their buckets, deduplicated
//   3. >= s distinct (or every key taken): the first s distinct are the sketch.  Fewer (more
//      repeats than the slack): T grows by the shortfall and 1-2 run again.
// A group whose keys below the cut exceed kSelCap fails (flag set); the host then merges
// that group's lists pairwise instead (fpm_sketch_run).
constexpr int kSelThreads = 1024;
constexpr uint32_t kSelCap = 15360;                      // keys staged in LDS (120 KiB)
constexpr int kSelPer = (kSelCap + kSelThreads - 1) / kSelThreads;   // 15 per thread
uint32_t group_select_cap() { return kSelCap; }

__device__ __forceinline__ uint32_t bits_of(uint64_t x) { return x ? 64 - __clzll(x) : 0; }

__global__ __launch_bounds__(kSelThreads) void group_select_kernel(
    const SelDesc *__restrict__ descs, const uint32_t *__restrict__ row_ids,
    const uint64_t *__restrict__ rows, uint32_t *__restrict__ count, uint32_t s,
    const uint64_t *__restrict__ thr, uint32_t *__restrict__ failed)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t K[];   // kSelCap keys
    __shared__ uint32_t h[4096];
    __shared__ uint32_t wsum[kSelThreads / 64 + 1];
    __shared__ uint32_t sh_b1;
    const SelDesc d = descs[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr uint32_t kWaves = kSelThreads / 64;
    const uint64_t hmax = d.slot == 0xFFFFFFFFu ? ~0ULL : thr[d.slot];   // no bound: a sample
    const uint32_t sh1 = bits_of(hmax) > 12 ? bits_of(hmax) - 12 : 0;
    // block sum / exclusive scan of one u32 per thread
    auto block_scan = [&](uint32_t v, uint32_t &tot) -> uint32_t {
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if ((int)lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t pre = 0, t = 0;
        for (uint32_t w = 0; w < kWaves; w++) { const uint32_t y = wsum[w]; pre += w < wave ? y : 0u; t += y; }
        __syncthreads();
        tot = t;
        return pre + x - v;
    };
    // The rows' mean length picks how the waves walk them: a wave per row, lanes over its keys
    // (the sample's rows: thousands of keys each), or, for short rows (a tight bound leaves a
    // C5 tile ~11 keys), a lane per row, 64 rows per wave in flight (a wave per row waited
    // out three dependent loads per ~11 keys: the selection took 1.9 ms of C5's step)
    uint32_t n_keys = 0;
    for (uint32_t ri = tid; ri < d.n_rows; ri += kSelThreads) n_keys += count[row_ids[d.row_begin + ri]];
    {
        uint32_t tot;
        (void)block_scan(n_keys, tot);
        n_keys = tot;
    }
    const bool lane_rows = n_keys < 32u * d.n_rows;
    // every kept key of the group with key < lim (lim = 0: all), handed to f(key)
    auto for_keys = [&](uint64_t lim, auto f) {
        if (lane_rows) {
            for (uint32_t r0 = wave * 64; r0 < d.n_rows; r0 += kWaves * 64) {
                const uint32_t ri = r0 + lane;
                uint32_t c = 0;
                const uint64_t *base = rows;
                if (ri < d.n_rows) {
                    const uint32_t row = row_ids[d.row_begin + ri];
                    c = count[row];
                    base = rows + (uint64_t)row * s;
                }
                uint32_t cmax = c;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, (uint32_t)__shfl_xor(cmax, o, 64));
                for (uint32_t i = 0; i < cmax; i++) {
                    if (i < c) {
                        const uint64_t key = base[i];
                        if (lim && key >= lim) c = i;      // lists are ascending: this row is done
                        else f(key);
                    }
                }
            }
            return;
        }
        for (uint32_t ri = wave; ri < d.n_rows; ri += kWaves) {
            const uint32_t row = row_ids[d.row_begin + ri];
            const uint32_t c = count[row];
            const uint64_t *base = rows + (uint64_t)row * s;
            for (uint32_t i = lane; i < c; i += 64) {
                const uint64_t key = base[i];
                if (lim && key >= lim) break;              // lists are ascending
                f(key);
            }
        }
    };
    uint32_t T = s + s / 8 + 64;
    for (;;) {
        // ---- 1. level-1 histogram over [0, hmax]: the cut R
        for (uint32_t b = tid; b < 4096; b += kSelThreads) h[b] = 0;
        __syncthreads();
        uint32_t mine = 0;
        for_keys(0, [&](uint64_t key) { atomicAdd(&h[(uint32_t)(key >> sh1)], 1u); mine++; });
        __syncthreads();
        uint32_t total;
        (void)block_scan(mine, total);
        uint64_t R = 0;                                     // 0: every key
        uint32_t m = total;
        if (total > kSelCap || total > T) {
            // bucket holding position T - 1: thread t scans buckets [4t, 4t + 4)
            uint32_t c4[4], run = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) { c4[u] = h[tid * 4 + u]; run += c4[u]; }
            uint32_t tot;
            uint32_t acc = block_scan(run, tot);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (acc < T && acc + c4[u] >= T) { sh_b1 = tid * 4 + u; }
                acc += c4[u];
            }
            __syncthreads();
            const uint32_t b1 = sh_b1;
            // (b1 + 1) << sh1 wraps to 0 only for the last bucket of a full 64-bit range: all keys
            R = (uint64_t)(b1 + 1) << sh1;
            // keys below R
            uint32_t below = 0;
            for (uint32_t b = tid; b <= b1; b += kSelThreads) below += h[b];
            uint32_t mb;
            (void)block_scan(below, mb);
            m = R ? mb : total;
        }
        if (m > kSelCap) {
            if (tid == 0) atomicOr(failed, 1u);
            return;
        }
        // ---- 2. counting sort of the m keys below R in LDS (4096 buckets over [0, R))
        const uint32_t sh2 = R ? (bits_of(R - 1) > 12 ? bits_of(R - 1) - 12 : 0) : sh1;
        __syncthreads();
        for (uint32_t b = tid; b < 4096; b += kSelThreads) h[b] = 0;
        __syncthreads();
        for_keys(R, [&](uint64_t key) { atomicAdd(&h[(uint32_t)(key >> sh2)], 1u); });
        __syncthreads();
        {
            uint32_t c4[4], run = 0;
#pragma unroll
            for (int u = 0; u < 4; u++) { c4[u] = h[tid * 4 + u]; run += c4[u]; }
            uint32_t tot;
            uint32_t acc = block_scan(run, tot);
#pragma unroll
            for (int u = 0; u < 4; u++) { h[tid * 4 + u] = acc; acc += c4[u]; }
        }
        __syncthreads();
        for_keys(R, [&](uint64_t key) { K[atomicAdd(&h[(uint32_t)(key >> sh2)], 1u)] = key; });
        __syncthreads();
        // h[b] = end of bucket b; rank inside the bucket (ties by position)
        uint64_t kk[kSelPer];
        uint32_t np[kSelPer];
#pragma unroll
        for (int u = 0; u < kSelPer; u++) {
            const uint32_t p = tid + (uint32_t)u * kSelThreads;
            if (p >= m) continue;
            const uint64_t key = K[p];
            const uint32_t b = (uint32_t)(key >> sh2);
            const uint32_t s0 = b ? h[b - 1] : 0u, s1 = h[b];
            uint32_t r = 0;
            for (uint32_t t = s0; t < s1; t++) {
                const uint64_t y = K[t];
                r += (y < key) | ((y == key) & (t < p));
            }
            kk[u] = key;
            np[u] = s0 + r;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kSelPer; u++)
            if (tid + (uint32_t)u * kSelThreads < m) K[np[u]] = kk[u];
        __syncthreads();
        // ---- 3. distinct values, the first s of them out
        uint32_t dc = 0;
        const uint32_t p0 = tid * kSelPer;
#pragma unroll
        for (int u = 0; u < kSelPer; u++) {
            const uint32_t p = p0 + u;
            dc += (p < m && (p == 0 || K[p] != K[p - 1])) ? 1u : 0u;
        }
        uint32_t dist;
        uint32_t rank = block_scan(dc, dist);
        if (dist >= s || R == 0) {
            uint64_t *out = const_cast<uint64_t *>(rows) + (uint64_t)d.out_row * s;
#pragma unroll
            for (int u = 0; u < kSelPer; u++) {
                const uint32_t p = p0 + u;
                if (p < m && (p == 0 || K[p] != K[p - 1])) {
                    if (rank < s) out[rank] = K[p];
                    rank++;
                }
            }
            if (tid == 0) count[d.out_row] = dist < s ? dist : s;
            return;
        }
        // more repeats than the slack: widen the cut by the shortfall
        T += 2 * (s - dist) + 64;
        __syncthreads();
    }
}

hipError_t launch_group_select(const SelDesc *d_desc, uint32_t n, const uint32_t *d_row_ids,
                               uint64_t *d_rows, uint32_t *d_count, uint32_t s,
                               const uint64_t *d_thr, uint32_t *d_failed, hipStream_t st)
{
    if (!n) return hipSuccess;
    const size_t lds = (size_t)kSelCap * 8;
    hipError_t e = hipFuncSetAttribute((const void *)group_select_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(group_select_kernel, dim3(n), dim3(kSelThreads), lds, st, d_desc, d_row_ids,
                       d_rows, d_count, s, d_thr, d_failed);
    return hipGetLastError();
}

hipError_t merge_small_spills(uint64_t *count)
{
    unsigned long long v = 0;
    hipError_t e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_merge_small_spill), sizeof(v));
    if (e != hipSuccess) return e;
    const unsigned long long z = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_merge_small_spill), &z, sizeof(z));
    *count = v;
    return e;
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
