// fingerprint.hip — the -fp k-finger text parse and line hash for gfx950.
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

// ---- CFL k-finger text → per-line (ID, value count, hash), the parse of
// Sketch::initFromFingerprints (Sketch.cpp:82-101: getline, `iss >> id`, `while (iss >> v)`)
// and its getHashFingerPrint call (:131), with the values streamed into Murmur instead of
// being stored.  Lines: split on '\n'; a last line without '\n' counts (getline).

constexpr int kTextChunk = 4096;   // text bytes per workgroup (256 threads x 16)

__device__ __forceinline__ bool fp_is_space(uint8_t c)
{
    return c == ' ' || (c >= '\t' && c <= '\r');   // isspace in the "C" locale
}

// newline flags of one 16-B text block (one uint4 load per thread; bytes at or past len are
// masked: the text buffer has 16 bytes of padding): bit 8 i + 7 of word i set where byte is '\n'
// (exact zero-byte test of w ^ 0x0A0A0A0A, no carries between bytes)
__device__ __forceinline__ uint4 nl_flags16(const uint8_t *__restrict__ text, uint64_t b0,
                                            uint64_t len)
{
    const uint4 w = *reinterpret_cast<const uint4 *>(text + b0);
    uint32_t m[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t x = m[i] ^ 0x0A0A0A0Au;
        uint32_t f = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
        const int64_t valid = (int64_t)len - (int64_t)(b0 + 4 * i);   // bytes of word i in range
        if (valid < 4) f &= valid <= 0 ? 0u : (1u << (8 * valid)) - 1;
        m[i] = f;
    }
    return make_uint4(m[0], m[1], m[2], m[3]);
}

__global__ __launch_bounds__(256) void nl_count_kernel(const uint8_t *__restrict__ text,
                                                      uint64_t len, uint32_t *__restrict__ cnt)
{
    __shared__ uint32_t wsum[4];
    const uint64_t b0 = (uint64_t)blockIdx.x * kTextChunk + threadIdx.x * 16;
    uint32_t c = 0;
    if (b0 < len) {
        const uint4 f = nl_flags16(text, b0, len);
        c = __popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w);
    }
    for (int d = 32; d > 0; d >>= 1) c += __shfl_down(c, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// line_start[k + 1] = 1 + position of the k-th '\n' (line_start[0] = 0, set by the host)
__global__ __launch_bounds__(256) void nl_scatter_kernel(const uint8_t *__restrict__ text,
                                                        uint64_t len,
                                                        const uint32_t *__restrict__ blk_off,
                                                        uint64_t *__restrict__ line_start)
{
    __shared__ uint32_t wsum[4];
    const uint64_t b0 = (uint64_t)blockIdx.x * kTextChunk + threadIdx.x * 16;
    uint4 f = make_uint4(0, 0, 0, 0);
    if (b0 < len) f = nl_flags16(text, b0, len);
    const uint32_t c = __popc(f.x) + __popc(f.y) + __popc(f.z) + __popc(f.w);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t k = blk_off[blockIdx.x] + x - c;
    for (int w = 0; w < wave; w++) k += wsum[w];
    const uint32_t m[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int i = 0; i < 4; i++)
        for (uint32_t b = m[i]; b; b &= b - 1)
            line_start[++k] = b0 + 4 * i + (__builtin_ctz(b) >> 3) + 1;
}

// One lane per line, the wave's text span staged in LDS: the 64 lines of a wave (and the line
// before them, for the new-ID test) are contiguous in the text, so the wave copies that span
// with 16-B loads and every lane parses its line from LDS, reading each byte once (the
// former global byte loads ran at 0.3 TB/s).  A span over kFpSpan bytes reads global memory.
constexpr uint32_t kFpSpan = 4096;

// bytes of a staged span through a one-word cache: the parse walks forward, so 3 of 4 reads
// come from the register
struct SpanBytes {
    const uint32_t *w;
    uint64_t base;                   // 16-B aligned text position of w[0]
    uint32_t ci, cw;
    __device__ __forceinline__ uint8_t operator()(uint64_t q)
    {
        const uint32_t o = (uint32_t)(q - base), wi = o >> 2;
        if (wi != ci) { ci = wi; cw = w[wi]; }
        return (uint8_t)(cw >> (8 * (o & 3)));
    }
};

template <typename Get>
__device__ __forceinline__ void fp_id_bounds(Get &get, uint64_t b, uint64_t e, uint64_t &ib,
                                             uint64_t &ie)
{
    uint64_t p = b;
    while (p < e && fp_is_space(get(p))) p++;
    ib = p;
    while (p < e && !fp_is_space(get(p))) p++;
    ie = p;
}

template <typename Get>
__device__ __forceinline__ void fp_parse_line(Get get, uint64_t li, uint64_t b, uint64_t e,
                                              uint64_t prev_b, uint32_t seed, uint32_t use64,
                                              uint64_t *__restrict__ id_off,
                                              uint32_t *__restrict__ id_len,
                                              uint32_t *__restrict__ n_vals,
                                              void *__restrict__ hash,
                                              uint8_t *__restrict__ new_id)
{
    uint64_t ib, ie;
    fp_id_bounds(get, b, e, ib, ie);
    uint64_t p = ie;
    // `while (iss >> v)`: optional sign, digits; a non-digit or an overflow ends the line.
    // c = the byte at p, 0 past the line end (0 is no space, sign or digit, as a NUL byte)
    uint64_t h1 = seed, h2 = seed, pend = 0, nv = 0;
    if (ie > ib) {
        uint8_t c = p < e ? get(p) : 0;
        for (;;) {
            while (fp_is_space(c)) { p++; c = p < e ? get(p) : 0; }
            bool neg = false;
            if (c == '+' || c == '-') { neg = c == '-'; p++; c = p < e ? get(p) : 0; }
            if (c < '0' || c > '9') break;
            uint64_t v = 0;
            bool ovf = false;
            while (c >= '0' && c <= '9') {
                const uint64_t d = (uint64_t)(c - '0');
                if (v > (~0ULL - d) / 10) ovf = true;
                v = v * 10 + d;
                p++;
                c = p < e ? get(p) : 0;
            }
            if (ovf) break;
            if (neg) v = 0 - v;
            if (nv & 1) mur_block(h1, h2, pend, v);          // value pairs are Murmur blocks
            else pend = v;
            nv++;
        }
    }
    if (nv & 1) {                                            // odd last value: the k1 tail
        uint64_t k1 = pend;
        k1 = mul_opaque(k1, kC1); k1 = rotl64(k1, 31); k1 *= kC2; h1 ^= k1;
    }
    const uint64_t h = mur_final(h1, h2, (uint64_t)(int64_t)(int)(nv * 8));
    id_off[li] = ib;
    id_len[li] = (uint32_t)(ie - ib);
    n_vals[li] = (uint32_t)nv;
    if (use64) reinterpret_cast<uint64_t *>(hash)[li] = h;
    else reinterpret_cast<uint32_t *>(hash)[li] = (uint32_t)h;
    // a new Reference starts where the ID differs from the previous line's (:104-129);
    // line 0 is compared with the previous file's last ID by the host (2 = unknown)
    uint8_t nid = 2;
    if (li > 0) {
        uint64_t pb, pe;
        Get gp = get;                                        // its own word cache
        fp_id_bounds(gp, prev_b, b - 1, pb, pe);
        nid = 0;
        if (pe - pb != ie - ib) nid = 1;
        else
            for (uint64_t t = 0; t < ie - ib; t++)
                if (gp(pb + t) != get(ib + t)) { nid = 1; break; }
    }
    new_id[li] = nid;
}

__global__ __launch_bounds__(256) void fp_line_kernel(
    const uint8_t *__restrict__ text, uint64_t len, const uint64_t *__restrict__ line_start,
    uint64_t n_nl, uint64_t n_lines, uint32_t seed, uint32_t use64,
    uint64_t *__restrict__ id_off, uint32_t *__restrict__ id_len, uint32_t *__restrict__ n_vals,
    void *__restrict__ hash, uint8_t *__restrict__ new_id)
{
    __shared__ __attribute__((aligned(16))) uint8_t span[4][kFpSpan];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t l0 = (uint64_t)blockIdx.x * 256 + wave * 64;
    // the wave's span: from the 16-B block holding the previous line's start to the end of
    // its last line (the text buffer has 16 bytes of padding past len)
    uint64_t s0 = 0, s1 = 0;
    if (l0 < n_lines) {
        s0 = line_start[l0 > 0 ? l0 - 1 : 0] & ~15ULL;
        const uint64_t ll = min(l0 + 63, n_lines - 1);
        s1 = ll < n_nl ? line_start[ll + 1] : len;
    }
    const bool staged = l0 < n_lines && s1 - s0 <= kFpSpan;
    if (staged)
        for (uint64_t off = lane * 16; s0 + off < s1; off += 64 * 16)
            *reinterpret_cast<uint4 *>(&span[wave][off]) =
                *reinterpret_cast<const uint4 *>(text + s0 + off);
    __syncthreads();
    const uint64_t li = l0 + lane;
    if (li >= n_lines) return;
    const uint64_t b = line_start[li], e = li < n_nl ? line_start[li + 1] - 1 : len;
    const uint64_t prev_b = li > 0 ? line_start[li - 1] : 0;
    if (staged) {
        fp_parse_line(SpanBytes{reinterpret_cast<const uint32_t *>(span[wave]), s0, ~0u, 0u}, li,
                      b, e, prev_b, seed, use64, id_off, id_len, n_vals, hash, new_id);
    } else {
        fp_parse_line([&](uint64_t q) { return text[q]; }, li, b, e, prev_b, seed, use64,
                      id_off, id_len, n_vals, hash, new_id);
    }
}

uint32_t text_blocks(uint64_t len) { return (uint32_t)((len + kTextChunk - 1) / kTextChunk); }

hipError_t launch_fp_nl_count(const uint8_t *d_text, uint64_t len, uint32_t *blk_cnt,
                              uint32_t *blk_off, uint32_t *scan_s, hipStream_t st)
{
    const uint32_t nb = text_blocks(len);
    if (!nb) return hipSuccess;
    hipLaunchKernelGGL(nl_count_kernel, dim3(nb), dim3(256), 0, st, d_text, len, blk_cnt);
    return launch_exscan(blk_cnt, blk_off, nullptr, nb, scan_s, blk_off + nb, st);
}

hipError_t launch_fp_nl_scatter(const uint8_t *d_text, uint64_t len, const uint32_t *blk_off,
                                uint64_t *d_line_start, hipStream_t st)
{
    const uint32_t nb = text_blocks(len);
    if (!nb) return hipSuccess;
    hipLaunchKernelGGL(nl_scatter_kernel, dim3(nb), dim3(256), 0, st, d_text, len, blk_off,
                       d_line_start);
    return hipGetLastError();
}

hipError_t launch_fp_lines(const uint8_t *d_text, uint64_t len, const uint64_t *d_line_start,
                           uint64_t n_nl, uint64_t n_lines, uint32_t seed, uint32_t use64,
                           uint64_t *id_off, uint32_t *id_len, uint32_t *n_vals, void *hash,
                           uint8_t *new_id, hipStream_t st)
{
    if (!n_lines) return hipSuccess;
    hipLaunchKernelGGL(fp_line_kernel, dim3((uint32_t)((n_lines + 255) / 256)), dim3(256), 0, st,
                       d_text, len, d_line_start, n_nl, n_lines, seed, use64, id_off, id_len,
                       n_vals, hash, new_id);
    return hipGetLastError();
}

// ---- the References of one parsed file (Sketch::initFromFingerprints' grouping, Sketch.cpp:
// 104-145): a new Reference starts at line 0 (checked against the previous file's last ID by
// the host) and wherever the ID differs from the previous line's (new_id == 1); its length is
// the first line's value count (set at creation, :117) plus every line's count (:134, the first
// line's again).  Heads are compacted in line order (per-block counts, an exclusive scan, an
// ordered scatter), then one wave per Reference sums its lines' counts.  The host then fetches
// ~ a few KB per file instead of every line's ID bounds and counts (21 B per line).
constexpr uint32_t kHeadLines = 1024;   // lines per workgroup (256 threads x 4)

__device__ __forceinline__ uint32_t fp_is_head(const uint8_t *__restrict__ new_id, uint64_t li,
                                               uint64_t n)
{
    return li < n && (li == 0 || new_id[li] == 1) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void fp_head_count_kernel(const uint8_t *__restrict__ new_id,
                                                           uint64_t n, uint32_t *__restrict__ cnt)
{
    __shared__ uint32_t wsum[4];
    const uint64_t l0 = (uint64_t)blockIdx.x * kHeadLines + threadIdx.x * 4;
    uint32_t c = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) c += fp_is_head(new_id, l0 + u, n);
    for (int d = 32; d > 0; d >>= 1) c += __shfl_down(c, d, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void fp_head_scatter_kernel(const uint8_t *__restrict__ new_id,
                                                             uint64_t n,
                                                             const uint32_t *__restrict__ blk_off,
                                                             uint64_t *__restrict__ first)
{
    __shared__ uint32_t wsum[4];
    const uint64_t l0 = (uint64_t)blockIdx.x * kHeadLines + threadIdx.x * 4;
    uint32_t h[4], c = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) { h[u] = fp_is_head(new_id, l0 + u, n); c += h[u]; }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { uint32_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t k = blk_off[blockIdx.x] + x - c;
    for (int w = 0; w < wave; w++) k += wsum[w];
#pragma unroll
    for (int u = 0; u < 4; u++)
        if (h[u]) first[k++] = l0 + u;
}

// one wave per Reference r: lines [first[r], first[r + 1]) (the last one to n)
__global__ __launch_bounds__(256) void fp_ref_len_kernel(
    const uint64_t *__restrict__ first, uint64_t n_refs, uint64_t n,
    const uint32_t *__restrict__ n_vals, const uint64_t *__restrict__ id_off,
    const uint32_t *__restrict__ id_len, uint64_t *__restrict__ length,
    uint64_t *__restrict__ ref_id_off, uint32_t *__restrict__ ref_id_len)
{
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (r >= n_refs) return;
    const uint64_t a = first[r], b = r + 1 < n_refs ? first[r + 1] : n;
    uint64_t sum = 0;
    for (uint64_t l = a + lane; l < b; l += 64) sum += n_vals[l];
    for (int d = 32; d > 0; d >>= 1) sum += __shfl_down(sum, d, 64);
    if (lane == 0) {
        length[r] = sum + n_vals[a];
        ref_id_off[r] = id_off[a];
        ref_id_len[r] = id_len[a];
    }
}

uint32_t fp_head_blocks(uint64_t n_lines) { return (uint32_t)((n_lines + kHeadLines - 1) / kHeadLines); }

hipError_t launch_fp_heads(const uint8_t *d_new_id, uint64_t n_lines, uint32_t *blk_cnt,
                           uint32_t *blk_off, uint32_t *scan_s, hipStream_t st)
{
    const uint32_t nb = fp_head_blocks(n_lines);
    if (!nb) return hipSuccess;
    hipLaunchKernelGGL(fp_head_count_kernel, dim3(nb), dim3(256), 0, st, d_new_id, n_lines, blk_cnt);
    return launch_exscan(blk_cnt, blk_off, nullptr, nb, scan_s, blk_off + nb, st);
}

hipError_t launch_fp_refs(const uint8_t *d_new_id, uint64_t n_lines, const uint32_t *blk_off,
                          uint64_t n_refs, const uint32_t *d_n_vals, const uint64_t *d_id_off,
                          const uint32_t *d_id_len, uint64_t *d_first, uint64_t *d_length,
                          uint64_t *d_ref_id_off, uint32_t *d_ref_id_len, hipStream_t st)
{
    const uint32_t nb = fp_head_blocks(n_lines);
    if (!nb || !n_refs) return hipSuccess;
    hipLaunchKernelGGL(fp_head_scatter_kernel, dim3(nb), dim3(256), 0, st, d_new_id, n_lines,
                       blk_off, d_first);
    hipLaunchKernelGGL(fp_ref_len_kernel, dim3((uint32_t)((n_refs + 3) / 4)), dim3(256), 0, st,
                       d_first, n_refs, n_lines, d_n_vals, d_id_off, d_id_len, d_length,
                       d_ref_id_off, d_ref_id_len);
    return hipGetLastError();
}

}  // namespace fpm
