// seqparse.hip — FASTA record parsing on the device.
//
// Replaces the main-thread kseq loop that feeds sketching (kseq_read, kseq.h:170-208, as
// called by sketchFile / sketchFileBySequence, Sketch.cpp:478-522, 1299-1488): the file
// image is parsed where the sequences are needed, and the records come out already packed
// in the layout the tile kernel reads (each record's sequence bytes followed by one 0x00).
//
// kseq_read as a 4-state machine over the bytes of one file:
//   S0  no header seen yet (the "jump to the next header line" loop)
//   S1  in sequence text (the current line holds no header marker)
//   S2  in a header line (the current line holds a '>' / '@' that started a record)
//   S3  the stream has ended (absorbing until the next file)
// A '>' or '@' outside S2 starts a record (S0 / S1 -> S2); a '\n' ends a header line
// (S2 -> S1: the name / comment reads stop at the first '\n'); in S1 every isgraph byte is
// sequence.  A '+' in S1 starts FASTQ quality parsing (kseq.h:196-206): that is flagged and
// the 4-line FASTQ path below (or the caller's host walk) takes the file instead.
// Byte 0xff: kstream's buffer is `char *` and ks_getc returns (int)buf[i], so on x86 (signed
// char) a 0xff byte reads as -1, kseq's end of file.  In the skip loop (S0) kseq_read returns
// -1 there and the caller stops reading the file (S3); in the sequence loop (S1) the record
// ends while last_char still holds its marker, so the next kseq_read reads a header from the
// byte after it: 0xff acts as a marker (S1 -> S2, a record starts).  The name and comment
// reads (ks_getuntil) scan the buffer directly: 0xff is an ordinary header byte in S2.
// Because the machine has four states, the effect of any byte range is a map
// {S0..S3} -> {S0..S3} plus, per input state, the records started and sequence bytes
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
constexpr int kSpStates = 4;
constexpr uint32_t kSpDead = 3;
struct Xf {
    uint32_t st;          // bits 2s..2s+1: the out state for input state s
    uint32_t plus;        // bit s: a '+' in sequence text for input state s
    uint32_t starts[kSpStates];   // records started
    uint32_t kept[kSpStates];     // sequence bytes kept
};

__device__ __forceinline__ uint32_t sel3(const uint32_t *a, uint32_t m)
{
    return m == 0 ? a[0] : (m == 1 ? a[1] : (m == 2 ? a[2] : a[3]));
}

// f then g
__device__ __forceinline__ Xf compose(const Xf &f, const Xf &g)
{
    Xf r;
    r.st = 0;
    r.plus = 0;
#pragma unroll
    for (int s = 0; s < kSpStates; s++) {
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
    r.st = 0 | (1u << 2) | (2u << 4) | (3u << 6);
    r.plus = 0;
#pragma unroll
    for (int s = 0; s < kSpStates; s++) { r.starts[s] = 0; r.kept[s] = 0; }
    return r;
}

// byte classes
__device__ __forceinline__ bool is_marker(uint32_t c) { return c == '>' || c == '@'; }
__device__ __forceinline__ bool is_seq(uint32_t c)
{
    // isgraph ("C" locale) minus the bytes that end a sequence (kseq.h:187)
    return c >= 0x21 && c <= 0x7e && c != '>' && c != '@' && c != '+';
}

// one byte's transition: state x -> returned state; *start: a record starts here
__device__ __forceinline__ uint32_t step_byte(uint32_t x, uint32_t c, bool *start)
{
    const bool mk = is_marker(c), eof = c == 0xffu;
    *start = (mk && (x == 0 || x == 1)) || (eof && x == 1);
    if (x == kSpDead || (eof && x == 0)) return kSpDead;
    if (mk || (eof && x == 1)) return 2u;
    return (c == '\n' && x == 2) ? 1u : x;
}

// the summary of one thread's 16 bytes
__device__ __forceinline__ Xf thread_xf(const uint8_t *b)
{
    uint32_t st[kSpStates] = {0, 1, 2, 3}, n[kSpStates] = {0, 0, 0, 0},
             kc[kSpStates] = {0, 0, 0, 0}, pl = 0;
#pragma unroll
    for (int i = 0; i < kSpBytes; i++) {
        const uint32_t c = b[i];
        const bool sq = is_seq(c), ps = c == '+';
#pragma unroll
        for (int s = 0; s < kSpStates; s++) {
            const uint32_t x = st[s];
            bool start;
            st[s] = step_byte(x, c, &start);
            n[s] += start ? 1u : 0u;
            kc[s] += (sq && x == 1) ? 1u : 0u;
            pl |= (ps && x == 1) ? (1u << s) : 0u;
        }
    }
    Xf r;
    r.st = st[0] | (st[1] << 2) | (st[2] << 4) | (st[3] << 6);
    r.plus = pl;
#pragma unroll
    for (int s = 0; s < kSpStates; s++) { r.starts[s] = n[s]; r.kept[s] = kc[s]; }
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
            o.st = s0 | (s0 << 2) | (s0 << 4) | (s0 << 6);
            o.plus = (o.plus & 1u) ? 15u : 0u;
            o.starts[1] = o.starts[2] = o.starts[3] = o.starts[0];
            o.kept[1] = o.kept[2] = o.kept[3] = o.kept[0];
        }
        out[blockIdx.x] = o;
    }
}

// pass 2 (one workgroup): state, records and kept bytes before each chunk, from S0
struct ChunkIn { uint64_t starts, kept; uint32_t st, pad; };
struct XfL { uint32_t st, plus; uint64_t starts[kSpStates], kept[kSpStates]; };

__device__ __forceinline__ uint64_t sel3l(const uint64_t *a, uint32_t m)
{
    return m == 0 ? a[0] : (m == 1 ? a[1] : (m == 2 ? a[2] : a[3]));
}

__device__ __forceinline__ XfL composel(const XfL &f, const XfL &g)
{
    XfL r;
    r.st = 0;
    r.plus = 0;
#pragma unroll
    for (int s = 0; s < kSpStates; s++) {
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
    for (int s = 0; s < kSpStates; s++) { r.starts[s] = x.starts[s]; r.kept[s] = x.kept[s]; }
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
        if (st == 1 && is_seq(c)) {
            out[nk + ns - 1] = (uint8_t)c;   // record ns - 1, after its predecessors' separators
            nk++;
        }
        if (c == '\n' && st == 2) hdr_end[ns - 1] = base + i;
        bool start;
        st = step_byte(st, c, &start);
        if (start) { hdr_pos[ns] = base + i; kept_at[ns] = nk; ns++; }
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

// ---- FASTQ (a '+' in sequence text) --------------------------------------------------
// kseq's quality branch (kseq.h:194-206) reads, after the '+' line, quality bytes until it
// holds as many in 33..127 as the sequence has bases, consumes one more byte, and then skips
// to the next '>' / '@' (last_char = 0).  That count makes the machine above non-finite, so
// FASTQ takes the layout every sequencer writes: 4 lines per record (header, sequence, '+',
// quality), parsed by line index over the newline index of the text (fingerprint.hip's
// nl_count / nl_scatter).  Each record is VERIFIED to be read the same way by kseq_read:
//   * the header line starts with '>' / '@' (for a file's first record: the file's first byte,
//     kseq skips nothing before it) and ends with a '\n' inside the file;
//   * the sequence line holds no '>', '@' or '+' (the sequence loop runs to the next line's
//     '+'), and its isgraph bytes are the bases;
//   * the third line starts with '+' and its '\n' is inside the file (kseq returns -2 at EOF);
//   * the quality line holds the base count of bytes in 33..127, and after the byte consumed
//     behind the last of them no '>' / '@' follows on that line (the skip to the next header
//     would start a record there);
//   * lines after a file's last record hold no '>' / '@';
//   * no 0xff byte (kseq's getc reads it as end of file, see above) in the sequence line, the
//     '+' line, the quality bytes kseq reads, or after them on the quality line.
// Any record that fails sets *fail and the caller parses the files on the host instead.

// per file: its first line (the line starting at seg_off) and its line count (lines starting
// before seg_off + seg_len), by binary search of the sorted line starts
__global__ void fq_files_kernel(const uint64_t *__restrict__ line_start, uint64_t n_starts,
                                const uint64_t *__restrict__ seg, uint32_t n_seg,
                                uint64_t *__restrict__ file_lines)
{
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_seg) return;
    auto lower = [&](uint64_t x) {   // first line starting at or after byte x
        uint64_t lo = 0, hi = n_starts;
        while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (line_start[m] < x) lo = m + 1; else hi = m;
        }
        return lo;
    };
    const uint64_t a = lower(seg[2 * f]), b = lower(seg[2 * f] + seg[2 * f + 1]);
    file_lines[2 * f] = a;
    file_lines[2 * f + 1] = b - a;
}

__device__ __forceinline__ bool fq_marker(uint32_t c) { return c == '>' || c == '@'; }

// one thread per record: verify, then header position / end and base count
__global__ void fq_records_kernel(const uint8_t *__restrict__ text,
                                  const uint64_t *__restrict__ line_start,
                                  const uint64_t *__restrict__ seg,
                                  const uint64_t *__restrict__ file_lines,
                                  const uint64_t *__restrict__ rec_base, uint32_t n_seg,
                                  uint64_t n_rec, uint64_t *__restrict__ hdr_pos,
                                  uint64_t *__restrict__ hdr_end, uint64_t *__restrict__ seq_len,
                                  uint32_t *__restrict__ fail)
{
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rec) return;
    uint32_t lo = 0, hi = n_seg;                  // the file: last rec_base[f] <= r
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (rec_base[m] <= r) lo = m; else hi = m;
    }
    const uint32_t f = lo;
    const uint64_t fend = seg[2 * f] + seg[2 * f + 1];
    const uint64_t L = file_lines[2 * f] + 4 * (r - rec_base[f]);
    const uint64_t h0 = line_start[L], h1 = line_start[L + 1] - 1;      // '\n' positions
    const uint64_t s0 = h1 + 1, s1 = line_start[L + 2] - 1;
    const uint64_t p0 = s1 + 1, p1 = line_start[L + 3] - 1;
    const uint64_t q0 = p1 + 1, q1 = line_start[L + 4] - 1;
    bool ok = fq_marker(text[h0]) && h1 < fend && text[p0] == '+' && p1 < fend;
    uint64_t kept = 0;
    for (uint64_t i = s0; ok && i < s1; i++) {
        const uint32_t c = text[i];
        if (fq_marker(c) || c == '+' || c == 0xffu) ok = false;
        kept += (c >= 0x21 && c <= 0x7e) ? 1u : 0u;
    }
    for (uint64_t i = p0 + 1; ok && i < p1; i++)
        if (text[i] == 0xffu) ok = false;
    // quality: the kept-th byte in 33..127, the byte after it is consumed, then no marker
    uint64_t v = 0, i = q0;
    if (ok && kept) {
        for (; i < q1; i++) {
            const uint32_t c = text[i];
            if (c == 0xffu) { ok = false; break; }
            if (c >= 33 && c <= 127 && ++v == kept) break;
        }
        ok = ok && v == kept;
        i++;                                     // the consumed byte after the last one
    }
    for (uint64_t x = i + 1; ok && x < q1; x++)
        if (fq_marker(text[x]) || text[x] == 0xffu) ok = false;
    if (!ok) {
        atomicOr(fail, 1u);
        return;
    }
    hdr_pos[r] = h0;
    hdr_end[r] = h1;
    seq_len[r] = kept;
}

// lines after a file's last record: no marker (kseq_read would start a record there)
__global__ void fq_tail_kernel(const uint8_t *__restrict__ text,
                               const uint64_t *__restrict__ line_start,
                               const uint64_t *__restrict__ seg,
                               const uint64_t *__restrict__ file_lines, uint32_t n_seg,
                               uint32_t *__restrict__ fail)
{
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= n_seg) return;
    const uint64_t n = file_lines[2 * f + 1];
    const uint64_t a = line_start[file_lines[2 * f] + n / 4 * 4];
    const uint64_t e = seg[2 * f] + seg[2 * f + 1];
    for (uint64_t x = a; x < e; x++)
        if (fq_marker(text[x])) { atomicOr(fail, 1u); return; }
}

// exclusive scan of u64 counts, 1024 per workgroup; block totals to sums[]
__global__ __launch_bounds__(256) void scan64_local_kernel(const uint64_t *__restrict__ in,
                                                          uint64_t *__restrict__ out, uint64_t n,
                                                          uint64_t *__restrict__ sums)
{
    __shared__ uint64_t wsum[4];
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
    uint64_t v[4], t = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) { v[k] = base + k < n ? in[base + k] : 0; t += v[k]; }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t x = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) { const uint64_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint64_t run = x - t;
    for (int w = 0; w < wave; w++) run += wsum[w];
#pragma unroll
    for (int k = 0; k < 4; k++) { if (base + k < n) out[base + k] = run; run += v[k]; }
    if (threadIdx.x == 255) sums[blockIdx.x] = run;
}

// one workgroup: the block totals -> exclusive prefixes (sequential chunks of 256), total
__global__ __launch_bounds__(256) void scan64_sums_kernel(uint64_t *__restrict__ sums, uint32_t nb,
                                                         uint64_t *__restrict__ total)
{
    __shared__ uint64_t wsum[4];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t c0 = 0; c0 < nb; c0 += 256) {
        const uint32_t i = c0 + threadIdx.x;
        const uint64_t v = i < nb ? sums[i] : 0;
        uint64_t x = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) { const uint64_t y = __shfl_up(x, d, 64); if (lane >= d) x += y; }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint64_t pre = carry + x - v;
        for (int w = 0; w < wave; w++) pre += wsum[w];
        if (i < nb) sums[i] = pre;
        __syncthreads();
        if (threadIdx.x == 255) carry = pre + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void scan64_add_kernel(uint64_t *__restrict__ out, uint64_t n,
                                                        const uint64_t *__restrict__ sums)
{
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
    const uint64_t add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (base + k < n) out[base + k] += add;
}

// one wave per record: the sequence line's isgraph bytes to the packed layout (record r at
// kept_at[r] + r, then its 0x00); a line of only bases (no '\r', no spaces: the common case)
// is copied by the 64 lanes, any other line compacted by a lane-order ballot scan
__global__ __launch_bounds__(256) void fq_emit_kernel(const uint8_t *__restrict__ text,
                                                      const uint64_t *__restrict__ hdr_end,
                                                      const uint64_t *__restrict__ kept_at,
                                                      const uint64_t *__restrict__ seq_len,
                                                      uint64_t n_rec, uint64_t *__restrict__ seq_off,
                                                      uint8_t *__restrict__ out)
{
    const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (r >= n_rec) return;
    const uint64_t s0 = hdr_end[r] + 1, len = seq_len[r], dst = kept_at[r] + r;
    uint64_t w = 0;                              // bytes written so far
    for (uint64_t i0 = s0; w < len; i0 += 64) {
        const uint32_t c = text[i0 + lane];
        const bool g = c >= 0x21 && c <= 0x7e;
        const uint64_t m = __ballot(g);
        const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (g && w + pre < len) out[dst + w + pre] = (uint8_t)c;
        w += (uint64_t)__popcll(m);
    }
    if (lane == 0) {
        out[dst + len] = 0;
        seq_off[r] = dst;
    }
}

hipError_t launch_fq_files(const uint64_t *d_line_start, uint64_t n_starts, const uint64_t *d_seg,
                           uint32_t n_seg, uint64_t *d_file_lines, hipStream_t st)
{
    if (!n_seg) return hipSuccess;
    hipLaunchKernelGGL(fq_files_kernel, dim3((n_seg + 255) / 256), dim3(256), 0, st, d_line_start,
                       n_starts, d_seg, n_seg, d_file_lines);
    return hipGetLastError();
}

hipError_t launch_fq_records(const uint8_t *d_text, const uint64_t *d_line_start,
                             const uint64_t *d_seg, const uint64_t *d_file_lines,
                             const uint64_t *d_rec_base, uint32_t n_seg, uint64_t n_rec,
                             uint64_t *d_rec, uint64_t *d_scan, uint64_t *d_total, uint32_t *d_fail,
                             uint8_t *d_out, hipStream_t st)
{
    // d_rec = hdr_pos | hdr_end | kept_at | seq_off | seq_len (n_rec each)
    uint64_t *pos = d_rec, *end = d_rec + n_rec, *kat = d_rec + 2 * n_rec,
             *off = d_rec + 3 * n_rec, *len = d_rec + 4 * n_rec;
    if (n_seg)
        hipLaunchKernelGGL(fq_tail_kernel, dim3((n_seg + 255) / 256), dim3(256), 0, st, d_text,
                           d_line_start, d_seg, d_file_lines, n_seg, d_fail);
    if (!n_rec) return hipGetLastError();
    hipLaunchKernelGGL(fq_records_kernel, dim3((uint32_t)((n_rec + 255) / 256)), dim3(256), 0, st,
                       d_text, d_line_start, d_seg, d_file_lines, d_rec_base, n_seg, n_rec, pos,
                       end, len, d_fail);
    const uint32_t nb = (uint32_t)((n_rec + 1023) / 1024);
    hipLaunchKernelGGL(scan64_local_kernel, dim3(nb), dim3(256), 0, st, (const uint64_t *)len, kat,
                       n_rec, d_scan);
    hipLaunchKernelGGL(scan64_sums_kernel, dim3(1), dim3(256), 0, st, d_scan, nb, d_total);
    hipLaunchKernelGGL(scan64_add_kernel, dim3(nb), dim3(256), 0, st, kat, n_rec,
                       (const uint64_t *)d_scan);
    (void)off;
    (void)d_out;
    return hipGetLastError();
}

hipError_t launch_fq_emit(const uint8_t *d_text, uint64_t n_rec, uint64_t *d_rec, uint8_t *d_out,
                          hipStream_t st)
{
    if (!n_rec) return hipSuccess;
    const uint64_t threads = n_rec * 64;
    if ((threads + 255) / 256 >= (1ULL << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fq_emit_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, st,
                       d_text, (const uint64_t *)(d_rec + n_rec), (const uint64_t *)(d_rec + 2 * n_rec),
                       (const uint64_t *)(d_rec + 4 * n_rec), n_rec, d_rec + 3 * n_rec, d_out);
    return hipGetLastError();
}

size_t seq_xf_bytes() { return sizeof(Xf); }
size_t seq_cin_bytes() { return sizeof(ChunkIn); }

}  // namespace fpm
