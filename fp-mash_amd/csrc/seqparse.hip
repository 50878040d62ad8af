// seqparse.hip — FASTA record parsing on the device.
//
// Replaces the main-thread kseq loop that feeds sketching (kseq_read, kseq.h:170-208, as
// called by sketchFile / sketchFileBySequence, Sketch.cpp:478-522, 1299-1488): the file
// image is parsed where the sequences are needed, and the records come out already packed
// in the layout the tile kernel reads (each record's sequence bytes followed by one 0x00).
//
// kseq_read as a 3-state machine over the bytes of one file:
//   S0  no header seen yet (the "jump to the next header line" loop)
//   S1  in sequence text (the current line holds no header marker)
//   S2  in a header line (the current line holds a '>' / '@' that started a record)
// A '>' or '@' outside S2 starts a record (S0 / S1 -> S2); a '\n' ends a header line
// (S2 -> S1: the name / comment reads stop at the first '\n'); in S1 every isgraph byte is
// sequence.  A '+' in S1 would start FASTQ quality parsing (kseq.h:196-206): that is
// flagged and the caller parses the file on the host instead.
// Because the machine has three states, the effect of any byte range is a map
// {S0,S1,S2} -> {S0,S1,S2} plus, per input state, the records started and sequence bytes
// kept: such summaries compose associatively, so a whole file is parsed with two passes of
// block scans and one chunk-level scan (no sequential dependence between workgroups).
//
// Text layout (set up by the caller, fpm_api.cpp): each file starts on a kSpChunk boundary
// (its first chunk resets the state to S0), the gap after it and the tail of the buffer are
// '\n' bytes (so every header line ends with a '\n' inside the buffer).
#include "fpm_device.hpp"
#include "fpm_kernels.hpp"

namespace fpm {

constexpr int kSpBlock = 256;
constexpr int kSpBytes = 16;                              // bytes per thread (one 16-B load)
static_assert(kSpBlock * kSpBytes == (int)kSpChunk, "chunk = one workgroup's bytes");
constexpr int kSpScanThreads = 1024;

// summary of a byte range: out state and counts for each input state
struct Xf {
    uint32_t st;          // bits 2s..2s+1: the out state for input state s
    uint32_t plus;        // bit s: a '+' in sequence text for input state s
    uint32_t starts[3];   // records started
    uint32_t kept[3];     // sequence bytes kept
};

__device__ __forceinline__ uint32_t sel3(const uint32_t *a, uint32_t m)
{
    return m == 0 ? a[0] : (m == 1 ? a[1] : a[2]);
}

// f then g
__device__ __forceinline__ Xf compose(const Xf &f, const Xf &g)
{
    Xf r;
    r.st = 0;
    r.plus = 0;
#pragma unroll
    for (int s = 0; s < 3; s++) {
        const uint32_t m = (f.st >> (2 * s)) & 3u;
        r.st |= ((g.st >> (2 * m)) & 3u) << (2 * s);
        r.plus |= (((f.plus >> s) | (g.plus >> m)) & 1u) << s;
        r.starts[s] = f.starts[s] + sel3(g.starts, m);
        r.kept[s] = f.kept[s] + sel3(g.kept, m);
    }
    return r;
}

__device__ __forceinline__ Xf identity_xf()
{
    Xf r;
    r.st = 0 | (1u << 2) | (2u << 4);
    r.plus = 0;
#pragma unroll
    for (int s = 0; s < 3; s++) { r.starts[s] = 0; r.kept[s] = 0; }
    return r;
}

// byte classes
__device__ __forceinline__ bool is_marker(uint32_t c) { return c == '>' || c == '@'; }
__device__ __forceinline__ bool is_seq(uint32_t c)
{
    // isgraph ("C" locale) minus the bytes that end a sequence (kseq.h:187)
    return c >= 0x21 && c <= 0x7e && c != '>' && c != '@' && c != '+';
}

// the summary of one thread's 16 bytes
__device__ __forceinline__ Xf thread_xf(const uint8_t *b)
{
    uint32_t st[3] = {0, 1, 2}, n[3] = {0, 0, 0}, kc[3] = {0, 0, 0}, pl = 0;
#pragma unroll
    for (int i = 0; i < kSpBytes; i++) {
        const uint32_t c = b[i];
        const bool nl = c == '\n', mk = is_marker(c), sq = is_seq(c), ps = c == '+';
#pragma unroll
        for (int s = 0; s < 3; s++) {
            const uint32_t x = st[s];
            n[s] += (mk && x != 2) ? 1u : 0u;
            kc[s] += (sq && x == 1) ? 1u : 0u;
            pl |= (ps && x == 1) ? (1u << s) : 0u;
            st[s] = mk ? 2u : ((nl && x == 2) ? 1u : x);
        }
    }
    Xf r;
    r.st = st[0] | (st[1] << 2) | (st[2] << 4);
    r.plus = pl;
#pragma unroll
    for (int s = 0; s < 3; s++) { r.starts[s] = n[s]; r.kept[s] = kc[s]; }
    return r;
}

// inclusive block scan of Xf in LDS (Hillis-Steele, in order: element t = x_0 o ... o x_t)
template <int N>
__device__ Xf block_scan_xf(Xf x, Xf *buf)
{
    const int t = threadIdx.x;
    buf[t] = x;
    __syncthreads();
    for (int d = 1; d < N; d <<= 1) {
        Xf y = x;
        if (t >= d) y = compose(buf[t - d], x);
        __syncthreads();
        buf[t] = y;
        x = y;
        __syncthreads();
    }
    return x;
}

__device__ __forceinline__ void load16(const uint8_t *text, uint64_t off, uint8_t (&b)[kSpBytes])
{
    const uint4 v = *reinterpret_cast<const uint4 *>(text + off);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < kSpBytes; i++) b[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

// pass 1: the summary of every chunk (a chunk that starts a file resets to S0 first)
__global__ __launch_bounds__(kSpBlock) void seq_chunk_summary_kernel(
    const uint8_t *__restrict__ text, const uint8_t *__restrict__ reset, Xf *__restrict__ out)
{
    __shared__ Xf buf[kSpBlock];
    uint8_t b[kSpBytes];
    load16(text, (uint64_t)blockIdx.x * kSpChunk + threadIdx.x * kSpBytes, b);
    const Xf r = block_scan_xf<kSpBlock>(thread_xf(b), buf);
    if (threadIdx.x == kSpBlock - 1) {
        Xf o = r;
        if (reset[blockIdx.x]) {
            // every input state behaves as S0
            const uint32_t s0 = o.st & 3u;
            o.st = s0 | (s0 << 2) | (s0 << 4);
            o.plus = (o.plus & 1u) ? 7u : 0u;
            o.starts[1] = o.starts[2] = o.starts[0];
            o.kept[1] = o.kept[2] = o.kept[0];
        }
        out[blockIdx.x] = o;
    }
}

// pass 2 (one workgroup): state, records and kept bytes before each chunk, from S0
struct ChunkIn { uint64_t starts, kept; uint32_t st, pad; };
struct XfL { uint32_t st, plus; uint64_t starts[3], kept[3]; };

__device__ __forceinline__ uint64_t sel3l(const uint64_t *a, uint32_t m)
{
    return m == 0 ? a[0] : (m == 1 ? a[1] : a[2]);
}

__device__ __forceinline__ XfL composel(const XfL &f, const XfL &g)
{
    XfL r;
    r.st = 0;
    r.plus = 0;
#pragma unroll
    for (int s = 0; s < 3; s++) {
        const uint32_t m = (f.st >> (2 * s)) & 3u;
        r.st |= ((g.st >> (2 * m)) & 3u) << (2 * s);
        r.plus |= (((f.plus >> s) | (g.plus >> m)) & 1u) << s;
        r.starts[s] = f.starts[s] + sel3l(g.starts, m);
        r.kept[s] = f.kept[s] + sel3l(g.kept, m);
    }
    return r;
}

__device__ __forceinline__ XfL widen(const Xf &x)
{
    XfL r;
    r.st = x.st;
    r.plus = x.plus;
#pragma unroll
    for (int s = 0; s < 3; s++) { r.starts[s] = x.starts[s]; r.kept[s] = x.kept[s]; }
    return r;
}

__global__ __launch_bounds__(kSpScanThreads) void seq_chunk_scan_kernel(
    const Xf *__restrict__ xf, const uint8_t *__restrict__ reset, uint32_t n_chunks,
    ChunkIn *__restrict__ cin, uint64_t *__restrict__ totals)
{
    __shared__ XfL buf[kSpScanThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n_chunks + kSpScanThreads - 1) / kSpScanThreads;
    const uint32_t c0 = min(t * per, n_chunks), c1 = min(c0 + per, n_chunks);
    XfL mine;
    {
        Xf id = identity_xf();
        mine = widen(id);
    }
    for (uint32_t c = c0; c < c1; c++) mine = composel(mine, widen(xf[c]));
    // inclusive scan, then shift to exclusive
    buf[t] = mine;
    __syncthreads();
    XfL x = mine;
    for (int d = 1; d < kSpScanThreads; d <<= 1) {
        XfL y = x;
        if ((int)t >= d) y = composel(buf[t - d], x);
        __syncthreads();
        buf[t] = y;
        x = y;
        __syncthreads();
    }
    XfL pre;
    if (t == 0) pre = widen(identity_xf());
    else pre = buf[t - 1];
    // apply the prefix to S0
    uint32_t st = pre.st & 3u;
    uint64_t ns = pre.starts[0], nk = pre.kept[0];
    uint32_t plus = pre.plus & 1u;
    for (uint32_t c = c0; c < c1; c++) {
        const Xf f = xf[c];
        const uint32_t s = st;
        ChunkIn ci;
        ci.starts = ns;
        ci.kept = nk;
        ci.st = reset[c] ? 0u : s;
        ci.pad = 0;
        cin[c] = ci;
        ns += sel3(f.starts, s);
        nk += sel3(f.kept, s);
        plus |= (f.plus >> s) & 1u;
        st = (f.st >> (2 * s)) & 3u;
    }
    if (t == kSpScanThreads - 1) {
        // the last thread's range ends at n_chunks (empty ranges carry the prefix through)
        totals[0] = ns;
        totals[1] = nk;
        totals[2] = plus;
    }
}

// pass 3: per byte; record table + packed sequence bytes
__global__ __launch_bounds__(kSpBlock) void seq_chunk_emit_kernel(
    const uint8_t *__restrict__ text, const ChunkIn *__restrict__ cin,
    uint64_t *__restrict__ hdr_pos, uint64_t *__restrict__ hdr_end, uint64_t *__restrict__ kept_at,
    uint8_t *__restrict__ out)
{
    __shared__ Xf buf[kSpBlock];
    uint8_t b[kSpBytes];
    const uint64_t base = (uint64_t)blockIdx.x * kSpChunk + threadIdx.x * kSpBytes;
    load16(text, base, b);
    const Xf mine = thread_xf(b);
    const Xf inc = block_scan_xf<kSpBlock>(mine, buf);
    const ChunkIn ci = cin[blockIdx.x];
    // this thread's input state and counts: the chunk's state through the exclusive prefix
    uint32_t st = ci.st;
    uint64_t ns = ci.starts, nk = ci.kept;
    if (threadIdx.x > 0) {
        const Xf pre = buf[threadIdx.x - 1];
        ns += sel3(pre.starts, st);
        nk += sel3(pre.kept, st);
        st = (pre.st >> (2 * st)) & 3u;
    }
    (void)inc;
#pragma unroll
    for (int i = 0; i < kSpBytes; i++) {
        const uint32_t c = b[i];
        if (c == '\n') {
            if (st == 2) { hdr_end[ns - 1] = base + i; st = 1; }
        } else if (is_marker(c)) {
            if (st != 2) { hdr_pos[ns] = base + i; kept_at[ns] = nk; ns++; st = 2; }
        } else if (st == 1 && is_seq(c)) {
            out[nk + ns - 1] = (uint8_t)c;   // record ns - 1, after its predecessors' separators
            nk++;
        }
    }
}

// pass 4: per record: packed offset and length, and its 0x00 separator
__global__ void seq_records_kernel(const uint64_t *__restrict__ kept_at, uint64_t n_rec,
                                   uint64_t total_kept, uint64_t *__restrict__ seq_off,
                                   uint64_t *__restrict__ seq_len, uint8_t *__restrict__ out)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    const uint64_t a = kept_at[r], e = r + 1 < n_rec ? kept_at[r + 1] : total_kept;
    seq_off[r] = a + r;
    seq_len[r] = e - a;
    out[e + r] = 0;
}

hipError_t launch_seq_scan(const uint8_t *d_text, const uint8_t *d_reset, uint32_t n_chunks,
                           void *d_xf, void *d_cin, uint64_t *d_totals, hipStream_t st)
{
    if (!n_chunks) return hipSuccess;
    hipLaunchKernelGGL(seq_chunk_summary_kernel, dim3(n_chunks), dim3(kSpBlock), 0, st, d_text,
                       d_reset, (Xf *)d_xf);
    hipLaunchKernelGGL(seq_chunk_scan_kernel, dim3(1), dim3(kSpScanThreads), 0, st,
                       (const Xf *)d_xf, d_reset, n_chunks, (ChunkIn *)d_cin, d_totals);
    return hipGetLastError();
}

hipError_t launch_seq_emit(const uint8_t *d_text, uint32_t n_chunks, const void *d_cin,
                           uint64_t n_rec, uint64_t total_kept, uint64_t *d_hdr_pos,
                           uint64_t *d_hdr_end, uint64_t *d_kept_at, uint64_t *d_seq_off,
                           uint64_t *d_seq_len, uint8_t *d_out, hipStream_t st)
{
    if (!n_chunks) return hipSuccess;
    hipLaunchKernelGGL(seq_chunk_emit_kernel, dim3(n_chunks), dim3(kSpBlock), 0, st, d_text,
                       (const ChunkIn *)d_cin, d_hdr_pos, d_hdr_end, d_kept_at, d_out);
    if (n_rec)
        hipLaunchKernelGGL(seq_records_kernel, dim3((uint32_t)((n_rec + 255) / 256)), dim3(256), 0,
                           st, d_kept_at, n_rec, total_kept, d_seq_off, d_seq_len, d_out);
    return hipGetLastError();
}

size_t seq_xf_bytes() { return sizeof(Xf); }
size_t seq_cin_bytes() { return sizeof(ChunkIn); }

}  // namespace fpm
