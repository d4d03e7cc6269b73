// gemm_gather.hpp — fp32 MFMA GEMM whose operand tiles come from "segmented row sources".
//
// One kernel template carries every dense contraction of the wD-MPNN encoder (mpn.py:92-143) and
// of its backward pass:
//
//   NT (forward layers):  C[m][n] = sum_k A(m,k) * W[n][k]        A = gathered / concatenated rows
//   NN (data gradients):  C[m][n] = sum_k dZ[m][k] * W[k][n]
//   TN (weight gradients): C[n][j] = sum_m dZ[m][n] * X(m,j)      split over m into slabs
//
// An operand is a Src: up to three column segments laid side by side in a padded column space
// (each segment starts at a multiple of 4).  A segment is
//   DENSE   : element (r, c) = src[r*ld + c]
//   GATHER  : element (r, c) = sum_{e=ptr[r]}^{ptr[r+1]-1} coef[e] * src[idx[e]*ld + c]
//             (the weighted in-edge sum of mpn.py:112-120 / 126-131 fused into the tile load)
//   ONES    : 1 in column 0 (appends the bias column to a weight-gradient GEMM)
// so the gathered message matrix X of mpn.py:119-120 and the concatenation of mpn.py:132 are never
// materialised in HBM: they are built tile by tile in LDS right before the MFMAs.
//
// MFMA: v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 64 FLOP/clk/SIMD).  Workgroup = WM x WN waves,
// each wave owns a (BM/WM) x (BN/WN) block of 32x32 accumulator tiles.  K is consumed in chunks of
// BK=32 staged through LDS with a one-chunk register prefetch.  Lane l of a wave supplies, at MFMA
// step s (0..15 per chunk), k = 16*(l>>5) + s: a row-major LDS tile is then read with four
// conflict-free ds_read_b128 per chunk (row stride 36 floats, checked by brute force), a k-major tile
// with one ds_read_b32 per step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wd {

typedef float floatx16 __attribute__((ext_vector_type(16)));

enum SegKind : int { SEG_DENSE = 0, SEG_GATHER = 1, SEG_ONES = 2 };

struct Seg {
    const float *src;
    const int32_t *ptr;
    const int32_t *idx;
    const float *coef;
    int ld;
    int K;      // real width
    int kp0;    // first padded column (multiple of 4)
    int kind;
    int vec;    // 1: rows 16-byte aligned and ld % 4 == 0 -> float4 loads
};

struct Src {
    Seg s[3];
    int nseg;
    int rows;      // valid rows
    int cols_p;    // padded width (multiple of 4)
};

enum Act : int { ACT_RELU = 0, ACT_LEAKY = 1, ACT_PRELU = 2, ACT_TANH = 3, ACT_SELU = 4, ACT_ELU = 5,
                 ACT_IDENTITY = 6 };

constexpr float SELU_ALPHA = 1.6732632423543772848170429916717f;
constexpr float SELU_SCALE = 1.0507009873554804934193349852946f;

__device__ __forceinline__ float act_fwd(int act, float z, float slope) {
    switch (act) {
    case ACT_RELU: return z < 0.f ? 0.f : z;
    case ACT_LEAKY: return z > 0.f ? z : 0.1f * z;
    case ACT_PRELU: return z > 0.f ? z : slope * z;
    case ACT_TANH: return tanhf(z);
    case ACT_SELU: return z > 0.f ? SELU_SCALE * z : SELU_SCALE * (SELU_ALPHA * expm1f(z));
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    default: return z;
    }
}

// d act / d z expressed with z (pre-activation).
__device__ __forceinline__ float act_grad(int act, float z, float slope) {
    switch (act) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_LEAKY: return z > 0.f ? 1.f : 0.1f;
    case ACT_PRELU: return z > 0.f ? 1.f : slope;
    case ACT_TANH: { float t = tanhf(z); return 1.f - t * t; }
    case ACT_SELU: return z > 0.f ? SELU_SCALE : SELU_SCALE * SELU_ALPHA * expf(z);
    case ACT_ELU: return z > 0.f ? 1.f : expf(z);
    default: return 1.f;
    }
}

// Counter-based dropout mask: keep with probability 1-p, scale 1/(1-p).  Re-derived in backward
// from (seed, layer, row, col), so no mask is stored.
__device__ __forceinline__ float dropout_scale(uint64_t seed, uint32_t layer, uint32_t row, uint32_t col,
                                               float p) {
    uint64_t x = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(layer + 1));
    x ^= ((uint64_t)row << 32) | col;
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    float u = (float)(uint32_t)(x >> 40) * (1.0f / 16777216.0f);
    return u >= p ? 1.0f / (1.0f - p) : 0.0f;
}

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 load4(const float *p, int n_valid, bool vec) {
    if (vec && n_valid >= 4) return *reinterpret_cast<const float4 *>(p);
    float4 v = f4zero();
    if (n_valid > 0) v.x = p[0];
    if (n_valid > 1) v.y = p[1];
    if (n_valid > 2) v.z = p[2];
    if (n_valid > 3) v.w = p[3];
    return v;
}

__device__ __forceinline__ void fma4(float4 &acc, float c, const float4 &v) {
    acc.x = fmaf(c, v.x, acc.x);
    acc.y = fmaf(c, v.y, acc.y);
    acc.z = fmaf(c, v.z, acc.z);
    acc.w = fmaf(c, v.w, acc.w);
}

// Value of padded columns [cp, cp+4) of row r of a segment.
__device__ __forceinline__ float4 seg_load4(const Seg &g, int r, int kk) {
    int nv = g.K - kk;
    if (nv <= 0) return f4zero();
    const bool vec = g.vec != 0;
    if (g.kind == SEG_DENSE) return load4(g.src + (size_t)r * g.ld + kk, nv, vec);
    if (g.kind == SEG_ONES) return kk == 0 ? make_float4(1.f, 0.f, 0.f, 0.f) : f4zero();
    float4 acc = f4zero();
    const int e0 = g.ptr[r], e1 = g.ptr[r + 1];
    for (int e = e0; e < e1; ++e) {
        const int j = g.idx[e];
        const float c = g.coef ? g.coef[e] : 1.0f;
        fma4(acc, c, load4(g.src + (size_t)j * g.ld + kk, nv, vec));
    }
    return acc;
}

__device__ __forceinline__ float4 src_load4(const Src &S, int r, int cp, int rlim, int clim) {
    if (r >= rlim || cp >= clim) return f4zero();
    if (S.nseg == 1) return seg_load4(S.s[0], r, cp - S.s[0].kp0);
    if (S.nseg == 2 || cp < S.s[2].kp0) {
        if (cp >= S.s[1].kp0) return seg_load4(S.s[1], r, cp - S.s[1].kp0);
        return seg_load4(S.s[0], r, cp);
    }
    return seg_load4(S.s[2], r, cp - S.s[2].kp0);
}

// ---------------------------------------------------------------------------------------------
// GEMM kernel
// ---------------------------------------------------------------------------------------------
enum EpiKind : int { EPI_ACT = 0, EPI_STORE = 1 };

struct Epi {
    int kind;
    const float *bias;     // [N] or null
    const float *resid;    // [M][ld_resid] or null (mpn.py:123 `input + message`)
    int ld_resid;
    float *Z;              // pre-activation out or null
    int ld_z;
    float *Y;              // output
    int ld_y;
    long long slab_stride; // EPI_STORE: Y += blockIdx.y * slab_stride
    int accumulate;        // EPI_STORE: Y += C
    int act;
    const float *slope;    // PReLU slope (device)
    float p_drop;
    uint64_t seed;
    uint32_t layer;
};

struct GemmParams {
    Src A, B;        // A tile: rows = i (or k if A_KMAJ); B tile: rows = j (or k if B_KMAJ)
    int M, N;        // output rows (i) / cols (j)
    int K;           // reduction extent (padded cols for NT, rows for TN)
    int k_per_split; // multiple of 32
    int tiles_n;
    Epi epi;
};

constexpr int BK = 32;

template <int BM, int BN, int WM, int WN, bool A_KMAJ, bool B_KMAJ>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(GemmParams P) {
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM / 32;
    constexpr int TN = BN / WN / 32;
    static_assert(TM >= 1 && TN >= 1, "wave tile must be a multiple of 32");
    // LDS tile geometry: row-major [rows=i][BK+4]; k-major [rows=k(BK)][cols+4]
    constexpr int A_ROWS = A_KMAJ ? BK : BM, A_COLS = A_KMAJ ? BM : BK, A_LD = A_COLS + 4;
    constexpr int B_ROWS = B_KMAJ ? BK : BN, B_COLS = B_KMAJ ? BN : BK, B_LD = B_COLS + 4;
    constexpr int A_V4 = A_ROWS * A_COLS / 4, B_V4 = B_ROWS * B_COLS / 4;
    constexpr int PA = (A_V4 + NT - 1) / NT, PB = (B_V4 + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) float lds[A_ROWS * A_LD + B_ROWS * B_LD];
    float *As = lds;
    float *Bs = lds + A_ROWS * A_LD;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int wi = wave / WN, wj = wave % WN;
    const int h = lane >> 5, l32 = lane & 31;

    const int tile = blockIdx.x;
    const int mt = tile / P.tiles_n, nt = tile % P.tiles_n;
    const int m0 = mt * BM, n0 = nt * BN;
    const int kbeg = blockIdx.y * P.k_per_split;
    const int kend = min(P.K, kbeg + P.k_per_split);

    floatx16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

    float4 ra[PA], rb[PB];
    auto load_chunk = [&](int k0) {
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int q = tid + p * NT;
            float4 v = f4zero();
            if (q < A_V4) {
                const int r = q / (A_COLS / 4), c = (q % (A_COLS / 4)) * 4;
                if (A_KMAJ) v = src_load4(P.A, k0 + r, m0 + c, kend, P.A.cols_p);
                else        v = src_load4(P.A, m0 + r, k0 + c, P.A.rows, kend);
            }
            ra[p] = v;
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int q = tid + p * NT;
            float4 v = f4zero();
            if (q < B_V4) {
                const int r = q / (B_COLS / 4), c = (q % (B_COLS / 4)) * 4;
                if (B_KMAJ) v = src_load4(P.B, k0 + r, n0 + c, kend, P.B.cols_p);
                else        v = src_load4(P.B, n0 + r, k0 + c, P.B.rows, kend);
            }
            rb[p] = v;
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int q = tid + p * NT;
            if (q < A_V4) {
                const int r = q / (A_COLS / 4), c = (q % (A_COLS / 4)) * 4;
                *reinterpret_cast<float4 *>(As + r * A_LD + c) = ra[p];
            }
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int q = tid + p * NT;
            if (q < B_V4) {
                const int r = q / (B_COLS / 4), c = (q % (B_COLS / 4)) * 4;
                *reinterpret_cast<float4 *>(Bs + r * B_LD + c) = rb[p];
            }
        }
    };

    const int nchunks = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    if (nchunks > 0) load_chunk(kbeg);
    for (int kc = 0; kc < nchunks; ++kc) {
        __syncthreads();
        store_chunk();
        __syncthreads();
        if (kc + 1 < nchunks) load_chunk(kbeg + (kc + 1) * BK);

        float af[TM][16], bf[TN][16];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
            const int i = wi * (BM / WM) + a * 32 + l32;
            if (A_KMAJ) {
#pragma unroll
                for (int s = 0; s < 16; ++s) af[a][s] = As[(16 * h + s) * A_LD + i];
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    float4 v = *reinterpret_cast<const float4 *>(As + i * A_LD + 16 * h + 4 * q);
                    af[a][4 * q] = v.x; af[a][4 * q + 1] = v.y; af[a][4 * q + 2] = v.z; af[a][4 * q + 3] = v.w;
                }
            }
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int j = wj * (BN / WN) + b * 32 + l32;
            if (B_KMAJ) {
#pragma unroll
                for (int s = 0; s < 16; ++s) bf[b][s] = Bs[(16 * h + s) * B_LD + j];
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    float4 v = *reinterpret_cast<const float4 *>(Bs + j * B_LD + 16 * h + 4 * q);
                    bf[b][4 * q] = v.x; bf[b][4 * q + 1] = v.y; bf[b][4 * q + 2] = v.z; bf[b][4 * q + 3] = v.w;
                }
            }
        }
#pragma unroll
        for (int s = 0; s < 16; ++s)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
    }

    // ---------------------------- epilogue ----------------------------
    const Epi &E = P.epi;
    const float slope = (E.kind == EPI_ACT && E.act == ACT_PRELU) ? E.slope[0] : 0.f;
    float *Y = E.Y + (E.kind == EPI_STORE ? (size_t)blockIdx.y * E.slab_stride : 0);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int j = n0 + wj * (BN / WN) + b * 32 + l32;
            if (j >= P.N) continue;
            const float bias = E.bias ? E.bias[j] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = m0 + wi * (BM / WM) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (i >= P.M) continue;
                float v = acc[a][b][r];
                if (E.kind == EPI_ACT) {
                    float z = v + bias;
                    if (E.resid) z += E.resid[(size_t)i * E.ld_resid + j];
                    if (E.Z) E.Z[(size_t)i * E.ld_z + j] = z;
                    float y = act_fwd(E.act, z, slope);
                    if (E.p_drop > 0.f) y *= dropout_scale(E.seed, E.layer, i, j, E.p_drop);
                    Y[(size_t)i * E.ld_y + j] = y;
                } else {
                    float *dst = Y + (size_t)i * E.ld_y + j;
                    *dst = E.accumulate ? *dst + v : v;
                }
            }
        }
}

}  // namespace wd
