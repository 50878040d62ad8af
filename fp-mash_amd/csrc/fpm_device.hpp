// fpm_device.hpp — device-side building blocks shared by the gfx950 kernels.
//
// MurmurHash3_x64_128 (replaces MurmurHash3.cpp:255-331 as used by getHash,
// hash.cpp:12-40): on CDNA4 there is no 64x64 multiply, so every constant
// multiply lowers to v_mul_lo_u32/v_mul_hi_u32/v_mad_u64_u32 — the k-mer sketch
// is integer-VALU bound, not HBM bound.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpm {

constexpr uint64_t kC1 = 0x87c37b91114253d5ULL;
constexpr uint64_t kC2 = 0x4cf5ad432745937fULL;

// rotate by a constant as two v_alignbit_b32 (LLVM otherwise emits a 64-bit shift, a 32-bit
// shift and an or for some of them)
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r)
{
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (r == 32) return ((uint64_t)lo << 32) | hi;
    if (r < 32) {
        const uint32_t s = 32 - r;                       // lo' = lo << r | hi >> s
        return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, s) << 32) |
               __builtin_amdgcn_alignbit(lo, hi, s);
    }
    const uint32_t s = 64 - r;                           // rotr by s < 32
    return ((uint64_t)__builtin_amdgcn_alignbit(lo, hi, s) << 32) |
           __builtin_amdgcn_alignbit(hi, lo, s);
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

// (h * 5 as a shift-add instead of the two v_mad_u64_u32 it lowers to: 4 fewer quarter-rate
// multiplies per window, yet C5 31.3 -> 31.6 ms in r04 and 19.75 -> 19.75 ms in r06, same box;
// the rotated products below did count: profiles/r06/murmur_rot_ab.txt)
// x * c, opaque to the optimiser: a rotate of the product then shifts the product (two
// v_alignbit) instead of multiplying x again by the constant shifted (LLVM folds (x * c) << r
// into x * (c << r): two more quarter-rate multiplies per rotated product)
__device__ __forceinline__ uint64_t mul_opaque(uint64_t x, uint64_t c)
{
    uint64_t p = x * c;
    asm volatile("" : "+v"(p));
    return p;
}

__device__ __forceinline__ void mur_block(uint64_t &h1, uint64_t &h2, uint64_t k1, uint64_t k2)
{
    k1 = mul_opaque(k1, kC1); k1 = rotl64(k1, 31); k1 *= kC2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 = mul_opaque(k2, kC2); k2 = rotl64(k2, 33); k2 *= kC1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
}

__device__ __forceinline__ uint64_t mur_final(uint64_t h1, uint64_t h2, uint64_t len)
{
    h1 ^= len; h2 ^= len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    return h1 + h2;   // h1 of the 128-bit result (the only half getHash reads)
}

// Murmur over `len` (<= 32) bytes held little-endian in w[0..3]; bytes past len are 0.
// `len` is wave-uniform (the k-mer size), so the branches do not diverge.
__device__ __forceinline__ uint64_t murmur_h1_le32(const uint64_t w[4], int len, uint32_t seed)
{
    uint64_t h1 = seed, h2 = seed;
    int nb = len >> 4;
    if (nb >= 1) mur_block(h1, h2, w[0], w[1]);
    if (nb >= 2) mur_block(h1, h2, w[2], w[3]);
    int rem = len & 15;
    if (rem) {
        uint64_t k1 = (nb == 0) ? w[0] : w[2];
        uint64_t k2 = (nb == 0) ? w[1] : w[3];
        if (rem > 8) { k2 = mul_opaque(k2, kC2); k2 = rotl64(k2, 33); k2 *= kC1; h2 ^= k2; }
        k1 = mul_opaque(k1, kC1); k1 = rotl64(k1, 31); k1 *= kC2; h1 ^= k1;
    }
    return mur_final(h1, h2, (uint64_t)len);
}

// Murmur over n little-endian u64 values (getHashFingerPrint hash.cpp:45-73,
// length = 8*n bytes): blocks are value pairs, an odd last value is the k1 tail.
template <typename LoadFn>
__device__ __forceinline__ uint64_t murmur_h1_u64s(LoadFn load, uint64_t n, uint32_t seed)
{
    uint64_t h1 = seed, h2 = seed;
    uint64_t i = 0;
    for (; i + 2 <= n; i += 2) mur_block(h1, h2, load(i), load(i + 1));
    if (i < n) {
        uint64_t k1 = load(i);
        k1 = mul_opaque(k1, kC1); k1 = rotl64(k1, 31); k1 *= kC2; h1 ^= k1;
    }
    return mur_final(h1, h2, (uint64_t)(int64_t)(int)(n * 8));
}

// 4 bytes starting at an arbitrary byte offset of an LDS byte image (read as dwords).
__device__ __forceinline__ uint32_t lds_u32_at(const uint32_t *img, uint32_t byte_off)
{
    uint32_t q = byte_off >> 2, r = byte_off & 3;
    return __builtin_amdgcn_alignbyte(img[q + 1], img[q], r);
}

// Four consecutive numer / denom cells: one 16-B store (u32 cells, 16-B aligned) or one 8-B
// store (u16 cells, 8-B aligned).
__device__ __forceinline__ void store_counts4(uint32_t *p, uint32_t a, uint32_t b, uint32_t c,
                                              uint32_t d)
{
    *(uint4 *)p = make_uint4(a, b, c, d);
}
__device__ __forceinline__ void store_counts4(uint16_t *p, uint32_t a, uint32_t b, uint32_t c,
                                              uint32_t d)
{
    *(uint2 *)p = make_uint2(a | (b << 16), c | (d << 16));
}

// Row-major launches over query rows: workgroups are dealt round-robin over the 8 XCDs, so
// block b runs on XCD b % 8. Map the blocks of one XCD to a CONTIGUOUS range of rows, so the
// rows resident on an XCD at once are neighbours (same family / similar sketches) and the
// ref rows and postings they share stay in that XCD's 4 MiB L2. Launch xcd_grid(n) blocks;
// a block whose row is >= n returns.
constexpr uint32_t kXcds = 8;
__host__ __device__ __forceinline__ uint32_t xcd_grid(uint32_t n_rows)
{
    return (n_rows + kXcds - 1) / kXcds * kXcds;
}
__device__ __forceinline__ uint32_t xcd_row(uint32_t block, uint32_t n_rows)
{
    const uint32_t per = (n_rows + kXcds - 1) / kXcds;
    return (block % kXcds) * per + block / kXcds;
}

}  // namespace fpm
