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

#include <float.h>

#include <algorithm>

namespace fpm {

constexpr int kTile = 16;   // 16 x 16 pairs per 256-lane workgroup

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

template <typename H>
__global__ __launch_bounds__(256) void compare_grid_kernel(
    const H *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const H *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t n_qry, uint32_t S, uint32_t *__restrict__ numer,
    uint32_t *__restrict__ denom)
{
    const uint32_t r = blockIdx.x * kTile + (threadIdx.x & (kTile - 1));
    const uint32_t q = blockIdx.y * kTile + (threadIdx.x / kTile);
    if (r >= n_ref || q >= n_qry) return;
    uint32_t c, d;
    walk_pair(ref + (uint64_t)r * ref_stride, ref_len[r], qry + (uint64_t)q * qry_stride,
              qry_len[q], S, c, d);
    const uint64_t o = (uint64_t)q * n_ref + r;
    numer[o] = c;
    denom[o] = d;
}

// Walk only the candidate pairs found by the inverted index (dist_index.hip).
template <typename H>
__global__ __launch_bounds__(256) void walk_cand_kernel(
    const uint64_t *__restrict__ cand, const unsigned long long *__restrict__ n_cand,
    const H *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const H *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t S, uint32_t *__restrict__ numer, uint32_t *__restrict__ denom)
{
    const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= *n_cand) return;
    const uint64_t o = cand[idx];
    const uint32_t q = (uint32_t)(o / n_ref), r = (uint32_t)(o % n_ref);
    uint32_t c, d;
    walk_pair(ref + (uint64_t)r * ref_stride, ref_len[r], qry + (uint64_t)q * qry_stride,
              qry_len[q], S, c, d);
    numer[o] = c;
    denom[o] = d;
}

// Sorted, distinct lists (every sketch the k-mer path produces): the walk of
// compareSketches is a merge of two sets, so with the shared values c_0 < c_1 < ...
// at (i_k, j_k) in (A, B): walk step of c_k = union rank = i_k + j_k - k, hence
//   numer = #{k : i_k + j_k - k < S},  denom = min(S, |A| + |B| - #shared).
// One workgroup per query row (B staged in LDS once), one wave per candidate ref
// (A staged in the wave's LDS slice with coalesced loads); lane l owns A's chunk
// [l*CH, (l+1)*CH): one binary search into B, then a linear co-walk.
constexpr int kMergeWaves = 8;

template <int CH>
__global__ __launch_bounds__(512) void merge_rows_kernel(
    const uint64_t *__restrict__ cand, const uint64_t *__restrict__ row_seg,
    const uint64_t *__restrict__ ref, const uint32_t *__restrict__ ref_len, uint64_t ref_stride,
    uint32_t n_ref, const uint64_t *__restrict__ qry, const uint32_t *__restrict__ qry_len,
    uint64_t qry_stride, uint32_t S, uint32_t *__restrict__ numer, uint32_t *__restrict__ denom)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t Bs[];
    const uint32_t q = blockIdx.x;
    const uint64_t seg = row_seg[q];
    const uint32_t n = (uint32_t)(seg & 0xFFFFFF);
    if (n == 0) return;
    const uint64_t base = seg >> 24;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t lb = qry_len[q];
    const uint64_t *B = qry + (uint64_t)q * qry_stride;
    // B[m] lives at m + m/16: lanes co-walk B ~16 elements apart, and an unpadded
    // 128-byte lane stride would put 16 lanes of a half-wave on one bank pair
    auto P = [](uint32_t m) { return m + (m >> 4); };
    for (uint32_t t = threadIdx.x; t < lb; t += blockDim.x) Bs[P(t)] = B[t];
    __syncthreads();
    constexpr uint32_t kInvalid = 0xFFFFFFFFu;
    uint64_t o_next = wave < n ? cand[base + wave] : 0;
    for (uint32_t c = wave; c < n; c += kMergeWaves) {
        const uint64_t o = o_next;
        const uint32_t r = (uint32_t)(o % n_ref);
        const uint32_t la = ref_len[r];
        if (c + kMergeWaves < n) o_next = cand[base + c + kMergeWaves];
        const uint64_t *A = ref + (uint64_t)r * ref_stride;
        // lane owns A[i0, i0+CH): batched 16-byte loads into registers
        const uint32_t i0 = lane * CH;
        uint64_t a[CH];
        if (i0 + CH <= la && (((uintptr_t)(A + i0)) & 15) == 0) {
            const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(A + i0);
#pragma unroll
            for (int t = 0; t < CH / 2; t++) { ulonglong2 v = p[t]; a[2 * t] = v.x; a[2 * t + 1] = v.y; }
        } else {
#pragma unroll
            for (int t = 0; t < CH; t++) a[t] = (i0 + t < la) ? A[i0 + t] : ~0ULL;
        }
        // co-walk my chunk against B: position of each shared value
        uint32_t sum_ij[CH];
        uint32_t dups = 0;
        uint32_t j = 0;
        if (i0 < la) {
            const uint64_t x = a[0];
            uint32_t lo = 0, hi = lb;
            while (lo < hi) { uint32_t m = (lo + hi) >> 1; if (Bs[P(m)] < x) lo = m + 1; else hi = m; }
            j = lo;
        }
#pragma unroll
        for (int t = 0; t < CH; t++) {
            sum_ij[t] = kInvalid;
            if (i0 + t < la) {
                const uint64_t x = a[t];
                while (j < lb && Bs[P(j)] < x) j++;
                if (j < lb && Bs[P(j)] == x) { sum_ij[t] = i0 + t + j; dups++; j++; }
            }
        }
        // k of my first shared value = shared values owned by lower lanes
        uint32_t incl = dups;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(incl, d, 64);
            if ((int)lane >= d) incl += y;
        }
        uint32_t k = incl - dups;
        const uint32_t total = __shfl(incl, 63, 64);
        uint32_t cnt = 0;
#pragma unroll
        for (int t = 0; t < CH; t++) {
            if (sum_ij[t] != kInvalid) {
                if (sum_ij[t] - k < S) cnt++;
                k++;
            }
        }
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) cnt += __shfl_down(cnt, d, 64);
        if (lane == 0) {
            const uint64_t u = (uint64_t)la + lb - total;
            numer[o] = cnt;
            denom[o] = u < S ? (uint32_t)u : S;
        }
    }
}

hipError_t launch_merge_rows(const uint64_t *d_cand, const uint64_t *row_seg, uint32_t n_qry,
                             const uint64_t *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                             uint32_t n_ref, const uint64_t *d_qry, const uint32_t *d_qry_len,
                             uint64_t qry_stride, uint32_t S, uint32_t *d_numer,
                             uint32_t *d_denom, hipStream_t st)
{
    if (!n_qry) return hipSuccess;
    const size_t lds = (size_t)(qry_stride + qry_stride / 16 + 1) * 8;
    const dim3 g(n_qry), b(64 * kMergeWaves);
    if (ref_stride <= 64 * 16)
        hipLaunchKernelGGL(merge_rows_kernel<16>, g, b, lds, st, d_cand, row_seg, d_ref, d_ref_len,
                           ref_stride, n_ref, d_qry, d_qry_len, qry_stride, S, d_numer, d_denom);
    else if (ref_stride <= 64 * 32)
        hipLaunchKernelGGL(merge_rows_kernel<32>, g, b, lds, st, d_cand, row_seg, d_ref, d_ref_len,
                           ref_stride, n_ref, d_qry, d_qry_len, qry_stride, S, d_numer, d_denom);
    else if (ref_stride <= 64 * 48)
        hipLaunchKernelGGL(merge_rows_kernel<48>, g, b, lds, st, d_cand, row_seg, d_ref, d_ref_len,
                           ref_stride, n_ref, d_qry, d_qry_len, qry_stride, S, d_numer, d_denom);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
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

__device__ double beta_P(double x, double a, double b)
{
    if (x == 0.0) return 0.0;
    if (x == 1.0) return 1.0;
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

__global__ __launch_bounds__(256) void dist_finalize_kernel(
    const uint32_t *__restrict__ numer, const uint32_t *__restrict__ denom,
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

hipError_t launch_compare_grid(const void *d_ref, const uint32_t *d_ref_len, uint64_t ref_stride,
                               uint32_t n_ref, const void *d_qry, const uint32_t *d_qry_len,
                               uint64_t qry_stride, uint32_t n_qry, uint32_t hash_bytes,
                               uint32_t sketch_size, uint32_t *d_numer, uint32_t *d_denom,
                               hipStream_t st)
{
    if (n_ref == 0 || n_qry == 0) return hipSuccess;
    dim3 grid((n_ref + kTile - 1) / kTile, (n_qry + kTile - 1) / kTile);
    if (hash_bytes == 8)
        hipLaunchKernelGGL(compare_grid_kernel<uint64_t>, grid, dim3(256), 0, st,
                           (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint64_t *)d_qry, d_qry_len, qry_stride, n_qry, sketch_size,
                           d_numer, d_denom);
    else if (hash_bytes == 4)
        hipLaunchKernelGGL(compare_grid_kernel<uint32_t>, grid, dim3(256), 0, st,
                           (const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint32_t *)d_qry, d_qry_len, qry_stride, n_qry, sketch_size,
                           d_numer, d_denom);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_walk_candidates(const uint64_t *d_cand, const unsigned long long *d_n_cand,
                                  uint64_t cap, const void *d_ref, const uint32_t *d_ref_len,
                                  uint64_t ref_stride, uint32_t n_ref, const void *d_qry,
                                  const uint32_t *d_qry_len, uint64_t qry_stride,
                                  uint32_t hash_bytes, uint32_t S, uint32_t *d_numer,
                                  uint32_t *d_denom, hipStream_t st)
{
    if (!cap) return hipSuccess;
    dim3 grid((uint32_t)((cap + 255) / 256));
    if (hash_bytes == 8)
        hipLaunchKernelGGL(walk_cand_kernel<uint64_t>, grid, dim3(256), 0, st, d_cand, d_n_cand,
                           (const uint64_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint64_t *)d_qry, d_qry_len, qry_stride, S, d_numer, d_denom);
    else
        hipLaunchKernelGGL(walk_cand_kernel<uint32_t>, grid, dim3(256), 0, st, d_cand, d_n_cand,
                           (const uint32_t *)d_ref, d_ref_len, ref_stride, n_ref,
                           (const uint32_t *)d_qry, d_qry_len, qry_stride, S, d_numer, d_denom);
    return hipGetLastError();
}

hipError_t launch_dist_finalize(const uint32_t *d_numer, const uint32_t *d_denom,
                                const uint64_t *d_ref_length, const uint64_t *d_qry_length,
                                uint32_t n_ref, uint32_t n_qry, uint32_t kmer_size,
                                double kmer_space, double max_dist, double max_pvalue,
                                double *d_dist, double *d_pvalue, uint8_t *d_pass,
                                hipStream_t st)
{
    uint64_t n = (uint64_t)n_ref * n_qry;
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(dist_finalize_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, d_numer,
                       d_denom, d_ref_length, d_qry_length, n_ref, n, kmer_size, kmer_space,
                       max_dist, max_pvalue, d_dist, d_pvalue, d_pass);
    return hipGetLastError();
}

}  // namespace fpm
