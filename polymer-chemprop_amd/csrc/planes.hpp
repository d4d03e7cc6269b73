// planes.hpp — exact three-way bf16 split of fp32 values ("bf16x3 planes") and the plane-tile
// layout shared by the producers (gathers, weight packer, graph upload) and the split GEMMs.
//
// x = h + m + l with h = rne_bf16(x), m = rne_bf16(x - h), l = rne_bf16(x - h - m): both residual
// subtractions are exact in fp32 and each piece carries 8 significant bits, so the planes hold x to
// the last fp32 bit (barring bf16 underflow of l below 2^-126).
//
// Plane-tile layout of an fp32 matrix [Rp][Kp] (Rp % 64 == 0, Kp % 32 == 0): blocks of 64 rows x 32
// columns; block (rb, kc) at byte (rb * (Kp / 32) + kc) * X6_BLOCK holds plane p (h, m, l), row r,
// columns 8u .. 8u+7 (16 bytes) at p * X6_PLANE + 64 r + 16 u.  A GEMM K-chunk of 64 rows is then one
// contiguous 12 KB block: LDS-DMA copies it 1 KB per wave-instruction (gemm_x6.hpp).
#pragma once
#include "common.hpp"

namespace wd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
// native vector (not HIP's uint4 class: arrays of that in register-staging structs went to scratch)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int X6_BN = 64;                  // GEMM column tile
constexpr int X6_PLANE = 64 * 64;          // bytes of one plane of a 64-row x 32-column block
constexpr int X6_BLOCK = 3 * X6_PLANE;     // one plane-tile block (12 KB)

__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2v));  // v_cvt_pk_bf16_f32 (RNE)
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// (a, b) -> three packed bf16 pairs with a = h + m + l (element 0 in the low half)
__device__ __forceinline__ void split_pair(float a, float b, uint32_t &h, uint32_t &m, uint32_t &l) {
    h = cvt_pk_bf16(a, b);
    const float a1 = a - bf_lo(h), b1 = b - bf_hi(h);
    m = cvt_pk_bf16(a1, b1);
    const float a2 = a1 - bf_lo(m), b2 = b1 - bf_hi(m);
    l = cvt_pk_bf16(a2, b2);
}

// byte offset of 16-byte unit u of row r in a plane image with BK-wide rows (2 BK bytes per row)
template <int BK>
__device__ __forceinline__ int x6_off(int r, int u) {
    if constexpr (BK == 32) return r * 64 + 16 * (u ^ ((r >> 1) & 3));
    else return r * 128 + 16 * (u ^ (r & 7));
}
__device__ __forceinline__ int x6_slot(int r, int u) { return x6_off<32>(r, u); }

// Byte offset of (row r, column k), plane 0, in a plane-tile matrix with BR-row blocks (BR = 64: the
// natural-row layout; BR = 128: the molecule-blocked bond layout): block (r / BR, k / 32)
// of 3 x BR x 64 bytes, plane stride BR * 64.
template <int BR = 64>
__device__ __forceinline__ size_t x6_tile_off(int r, int k, int kp) {
    return ((size_t)(r / BR) * (kp >> 5) + (k >> 5)) * (3 * BR * 64) + (r % BR) * 64 + 2 * (k & 31);
}

// 16- and 8-byte global stores of produced activations, write-through (sc1: measured 1 us faster per
// fused layer than default-policy stores, which leave the lines dirty for the kernel-end write-back).
// Emitted as relaxed agent-scope 8-byte atomic stores (global_store_dwordx2 ... sc1), which the
// compiler tracks in its vmcnt accounting (inline-asm stores are invisible to it and broke later
// waits).  WD_WT (experiments): 0 = default policy, 1 = sc1, 3 = nt.
#ifndef WD_WT
#define WD_WT 1
#endif
constexpr int WD_WT_POL = WD_WT == 1 ? 16 : WD_WT == 3 ? 2 : 0;  // buffer-store aux bits: sc1 = 16, nt = 2
__device__ __forceinline__ void gst8(void *p, const uint2 &v) {
    if constexpr (WD_WT == 1) {
        const unsigned long long w = (unsigned long long)v.x | ((unsigned long long)v.y << 32);
        __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (WD_WT == 3) {
        __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t *>(p));
        __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t *>(p) + 1);
    } else {
        *reinterpret_cast<uint2 *>(p) = v;
    }
}
__device__ __forceinline__ void gst16(void *p, const u32x4 &v) {
    if constexpr (WD_WT == 1) {
        gst8(p, make_uint2(v.x, v.y));
        gst8(reinterpret_cast<uint8_t *>(p) + 8, make_uint2(v.z, v.w));
    } else if constexpr (WD_WT == 3) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    } else {
        *reinterpret_cast<u32x4 *>(p) = v;
    }
}

// write values lo, hi = columns k..k+7 (k % 8 == 0) of row r into a plane-tile matrix
template <int BR = 64>
__device__ __forceinline__ void x6_store8(uint8_t *base, int kp, int r, int k, const float4 &lo, const float4 &hi) {
    uint32_t h[4], m[4], l[4];
    split_pair(lo.x, lo.y, h[0], m[0], l[0]);
    split_pair(lo.z, lo.w, h[1], m[1], l[1]);
    split_pair(hi.x, hi.y, h[2], m[2], l[2]);
    split_pair(hi.z, hi.w, h[3], m[3], l[3]);
    uint8_t *d = base + x6_tile_off<BR>(r, k, kp);
    gst16(d, u32x4{h[0], h[1], h[2], h[3]});
    gst16(d + BR * 64, u32x4{m[0], m[1], m[2], m[3]});
    gst16(d + 2 * BR * 64, u32x4{l[0], l[1], l[2], l[3]});
}

// The same for a row of ONE row block whose base is wave-uniform (a workgroup's own block): three
// 16-byte buffer stores with the sc1 (write-through) policy, offsets relative to the block base
template <int BR>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t x6_block_rsrc(uint8_t *base, int kp, int blk) {
    uint8_t *b = base + (size_t)blk * (kp >> 5) * (3 * BR * 64);
    return __builtin_amdgcn_make_buffer_rsrc(b, 0, (kp >> 5) * (3 * BR * 64), 0x00020000);
}
template <int BR>
__device__ __forceinline__ void x6_store8_blk(__amdgpu_buffer_rsrc_t rs, int r, int k, const float4 &lo,
                                              const float4 &hi) {
    uint32_t h[4], m[4], l[4];
    split_pair(lo.x, lo.y, h[0], m[0], l[0]);
    split_pair(lo.z, lo.w, h[1], m[1], l[1]);
    split_pair(hi.x, hi.y, h[2], m[2], l[2]);
    split_pair(hi.z, hi.w, h[3], m[3], l[3]);
    const int o = (k >> 5) * (3 * BR * 64) + r * 64 + 2 * (k & 31);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{h[0], h[1], h[2], h[3]}, rs, o, 0, WD_WT_POL);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{m[0], m[1], m[2], m[3]}, rs, o + BR * 64, 0, WD_WT_POL);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{l[0], l[1], l[2], l[3]}, rs, o + 2 * BR * 64, 0, WD_WT_POL);
}

// columns k..k+3 (k % 4 == 0): three 8-byte pieces
template <int BR = 64>
__device__ __forceinline__ void x6_store4(uint8_t *base, int kp, int r, int k, const float4 &v) {
    uint32_t h[2], m[2], l[2];
    split_pair(v.x, v.y, h[0], m[0], l[0]);
    split_pair(v.z, v.w, h[1], m[1], l[1]);
    uint8_t *d = base + x6_tile_off<BR>(r, k, kp);
    gst8(d, make_uint2(h[0], h[1]));
    gst8(d + BR * 64, make_uint2(m[0], m[1]));
    gst8(d + 2 * BR * 64, make_uint2(l[0], l[1]));
}

// fp32 [rows][ld] (first kp columns) -> plane tiles [out_rows][kp] with BR-row blocks; one thread per 8
// values.
// row_map == null: row r -> r (out_rows == rows); else row r -> row_map[r] (skipped when < 0) and every
// output row that no source row maps to must be zero-filled by the caller.
template <int BR = 64>
__global__ __launch_bounds__(256) void split_tiles_kernel(const float *__restrict__ src, int ld, int rows, int kp,
                                                          uint8_t *__restrict__ dst,
                                                          const int32_t *__restrict__ row_map = nullptr) {
    const int q8 = kp >> 3;
    const size_t total = (size_t)rows * q8;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / q8), k = (int)(t % q8) * 8;
        const int ro = row_map ? row_map[r] : r;
        if (ro < 0) continue;
        const float *s = src + (size_t)r * ld + k;
        x6_store8<BR>(dst, kp, ro, k, ld4(s), ld4(s + 4));
    }
}

// Several dense splits in one launch (blockIdx.y = job; BR 64 or 80 per job): the weight packing of
// a training forward splits five small matrices, and five launches cost more than the work.
struct SplitJob { const float *src; uint8_t *dst; int ld, rows, kp, br; };
struct SplitJobs { SplitJob j[6]; int n; };

__global__ __launch_bounds__(256) void split_tiles_batch_kernel(SplitJobs J) {
    const SplitJob S = J.j[blockIdx.y];
    const int q8 = S.kp >> 3;
    const size_t total = (size_t)S.rows * q8;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / q8), k = (int)(t % q8) * 8;
        const float *s = S.src + (size_t)r * S.ld + k;
        if (S.br == 80) x6_store8<80>(S.dst, S.kp, r, k, ld4(s), ld4(s + 4));
        else x6_store8<64>(S.dst, S.kp, r, k, ld4(s), ld4(s + 4));
    }
}

// ---------------------------------------------------------------------------------------------
// fp16 hi / lo pairs ("h2"): the message-passing layer's GEMM operands (fused_mp.hpp).
//
// With a power-of-two scale s that puts max |x| s in [2^14, 2^15) (the max over the rows one GEMM tile
// multiplies), x s = hi + lo + r with hi = rne_f16(x s), lo = rne_f16(x s - hi) and |r| <= 2^-22 |x s|
// (values far below the max go subnormal in lo and keep an absolute error <= 2^-25 of the scaled unit,
// 2^-39 of the max).  A
// product is hi_a hi_b + hi_a lo_b + lo_a hi_b (each exact in fp32, accumulated in fp32 by
// v_mfma_f32_16x16x32_f16); the dropped lo_a lo_b is <= 2^-22 |ab|.  Three MFMAs per fp32 product
// instead of the planes' six, 4 bytes per value instead of 6; the whole encoder stays at the error of
// an fp32 GEMM against fp64 (tools/split_precision_sim.py: 1.2-2.9e-7 normwise, fp32 1.1-2.6e-7).
//
// The scale comes from the maximum of the rows one GEMM tile multiplies.  Producers publish partial
// maxima as plain u32 words (absolute-value bits), one per producing workgroup, into slot arrays that
// each forward overwrites completely: the embed and the message layers one word per (molecule block,
// column tile), so the consumer of a block reads that block's few words (a per-block scale: the A tile
// of a fused layer workgroup is one block); the weight packer one word per workgroup, folded into one
// word by split_h2_kernel.  No atomics, no reset, deterministic.
// ---------------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t absbits(float x) { return __float_as_uint(x) & 0x7fffffffu; }
// the scale s and its inverse for max |x| (its bits m): s = 2^(141 - e) with e the biased exponent of m
// (max |x| s in [2^14, 2^15)), both normal floats (clamped for all-zero / subnormal / non-finite maxima)
__device__ __forceinline__ int h2_sexp(uint32_t m) {
    const int se = 268 - (int)(m >> 23);
    return se < 1 ? 1 : (se > 253 ? 253 : se);
}
__device__ __forceinline__ float h2_scale(uint32_t m) { return __uint_as_float((uint32_t)h2_sexp(m) << 23); }
__device__ __forceinline__ float h2_inv_scale(uint32_t m) { return __uint_as_float((uint32_t)(254 - h2_sexp(m)) << 23); }
// Max of n words at a workgroup-uniform address, in two steps so that the load can be issued early
// and waited for late: lane_word (lane i loads word i: one load, all words in flight at once; a loop of
// dependent loads cost one memory latency per word; n > 64 -- hidden sizes past 2560 -- folds words
// i, i + 64, ... into lane i), then wave_max_u32 (every lane of the wave active): DPP max within each
// 16-lane row, then the four rows' maxima read into scalars.
__device__ __forceinline__ uint32_t lane_word(const uint32_t *w, int n) {
    const int l = threadIdx.x & 63;
    uint32_t m = l < n ? w[l] : 0u;
    for (int i = l + 64; i < n; i += 64) m = max(m, w[i]);
    return m;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t m) {
    m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x124, 0xF, 0xF, false));  // row_ror:4
    m = max(m, (uint32_t)__builtin_amdgcn_mov_dpp((int)m, 0x128, 0xF, 0xF, false));  // row_ror:8
    const uint32_t a = __builtin_amdgcn_readlane(m, 0), b = __builtin_amdgcn_readlane(m, 16);
    const uint32_t c = __builtin_amdgcn_readlane(m, 32), d = __builtin_amdgcn_readlane(m, 48);
    return max(max(a, b), max(c, d));
}
__device__ __forceinline__ uint32_t max_words(const uint32_t *w, int n) { return wave_max_u32(lane_word(w, n)); }
// (a, b) scaled by s -> packed fp16 hi pair and lo pair (element 0 in the low half)
__device__ __forceinline__ void split_h2(float a, float b, float s, uint32_t &hi, uint32_t &lo) {
    const f16x2v h = __builtin_convertvector((f32x2v){a * s, b * s}, f16x2v);  // v_cvt_pk_f16_f32 (RNE)
    const float ra = fmaf(a, s, -(float)h[0]), rb = fmaf(b, s, -(float)h[1]);  // exact residuals
    hi = __builtin_bit_cast(uint32_t, h);
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){ra, rb}, f16x2v));
}
// the same with a scale per element (per-column scales of gemm_tn_x6_kernel<H2>)
__device__ __forceinline__ void split_h2(float a, float b, float sa, float sb, uint32_t &hi, uint32_t &lo) {
    const f16x2v h = __builtin_convertvector((f32x2v){a * sa, b * sb}, f16x2v);
    const float ra = fmaf(a, sa, -(float)h[0]), rb = fmaf(b, sb, -(float)h[1]);
    hi = __builtin_bit_cast(uint32_t, h);
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){ra, rb}, f16x2v));
}

// workgroup max of a u32 -> one plain store by thread 0 (red: >= blockDim.x / 64 words of LDS; every
// thread of the workgroup must call it)
__device__ __forceinline__ void publish_max(uint32_t m, uint32_t *slot, uint32_t *red) {
    m = wave_max_u32(m);
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) red[wave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < nw; ++w) m = red[w] > m ? red[w] : m;
        *slot = m;
    }
}

// the same, returning the workgroup max to every thread (a producer that scales its own output by it:
// the pair-writing epilogues); one barrier
__device__ __forceinline__ uint32_t publish_max_all(uint32_t m, uint32_t *slot, uint32_t *red) {
    m = wave_max_u32(m);
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) red[wave] = m;
    __syncthreads();
    for (int w = 0; w < nw; ++w) m = red[w] > m ? red[w] : m;
    if (threadIdx.x == 0) *slot = m;
    return m;
}

// 8 values (columns k .. k + 7 of one row, k % 8 == 0) scaled by s -> their fp16 hi and lo units of a
// pair tile (planes: hi at +0, lo at +plane bytes) by two 16-byte buffer stores, default (write-back) policy
__device__ __forceinline__ void h2_store8(__amdgpu_buffer_rsrc_t rs, int off, int plane, const float4 &a,
                                          const float4 &b, float s) {
    uint32_t h[4], l[4];
    split_h2(a.x, a.y, s, h[0], l[0]);
    split_h2(a.z, a.w, s, h[1], l[1]);
    split_h2(b.x, b.y, s, h[2], l[2]);
    split_h2(b.z, b.w, s, h[3], l[3]);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{h[0], h[1], h[2], h[3]}, rs, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{l[0], l[1], l[2], l[3]}, rs, off + plane, 0, 0);
}
// byte offset of (row r, column k) of a molecule block's pair tiles (BR rows, kp columns): chunk k / 32 of
// 2 x BR x 64 bytes, row r % BR at 64 r, column k % 32 at 2 (k % 32) (the plane-tile layout with two planes)
template <int BR>
__device__ __forceinline__ int h2_blk_off(int r, int k) { return (k >> 5) * (2 * BR * 64) + r * 64 + 2 * (k & 31); }

// fp32 [rows][ld] (first kp columns) -> h2 plane tiles with BR-row blocks: block (r / BR, k / 32) of 2 x
// BR x 64 bytes (hi plane, then lo), row r % BR, columns k % 32 at 64 (r % BR) + 2 (k % 32) -- the bf16
// plane-tile layout with two planes.  Scaled by the max of the nw words of `words` (pack_kernel's
// per-workgroup maxima, or adam_kernel's), which workgroup 0 also folds into *fold for the consumers.
__global__ __launch_bounds__(256) void split_h2_kernel(const float *__restrict__ src, int ld, int rows, int kp, int br,
                                                       uint8_t *__restrict__ dst, const uint32_t *words, int nw,
                                                       uint32_t *fold) {
    const uint32_t m = max_words(words, nw);
    const float s = h2_scale(m);
    if (blockIdx.x == 0 && threadIdx.x == 0) *fold = m;
    const int q8 = kp >> 3;
    const size_t total = (size_t)rows * q8;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / q8), k = (int)(t % q8) * 8;
        const float4 lo4 = ld4(src + (size_t)r * ld + k), hi4 = ld4(src + (size_t)r * ld + k + 4);
        uint32_t h[4], l[4];
        split_h2(lo4.x, lo4.y, s, h[0], l[0]);
        split_h2(lo4.z, lo4.w, s, h[1], l[1]);
        split_h2(hi4.x, hi4.y, s, h[2], l[2]);
        split_h2(hi4.z, hi4.w, s, h[3], l[3]);
        uint8_t *d = dst + ((size_t)(r / br) * (kp >> 5) + (k >> 5)) * (2 * br * 64) + (r % br) * 64 + 2 * (k & 31);
        *reinterpret_cast<u32x4 *>(d) = u32x4{h[0], h[1], h[2], h[3]};
        *reinterpret_cast<u32x4 *>(d + br * 64) = u32x4{l[0], l[1], l[2], l[3]};
    }
}

}  // namespace wd
