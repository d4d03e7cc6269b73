// common.hpp — device helpers shared by the wD-MPNN kernels (activations, dropout hash, vector I/O).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace wd {

typedef float floatx16 __attribute__((ext_vector_type(16)));

enum Act : int { ACT_RELU = 0, ACT_LEAKY = 1, ACT_PRELU = 2, ACT_TANH = 3, ACT_SELU = 4, ACT_ELU = 5,
                 ACT_IDENTITY = 6 };

constexpr float SELU_ALPHA = 1.6732632423543772848170429916717f;
constexpr float SELU_SCALE = 1.0507009873554804934193349852946f;

// nn_utils.py:70-99 activations (ReLU, LeakyReLU(0.1), PReLU, tanh, SELU, ELU); act(0) == 0 for all,
// which keeps zero-padded columns zero through every layer.
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

// f(std::integral_constant<int, act>): one dispatch per kernel phase, so that the executed path holds one
// activation's code (act_fwd(ACT, ...) folds to it) instead of a switch per element -- per-element
// switches interleave every activation's code with the executed one and the epilogues ran out of the
// instruction cache (measured: 8 us per layer launch of straight-line epilogue work)
template <typename F>
__device__ __forceinline__ void with_act(int act, F &&f) {
    switch (act) {
    case ACT_RELU: f(std::integral_constant<int, ACT_RELU>{}); break;
    case ACT_LEAKY: f(std::integral_constant<int, ACT_LEAKY>{}); break;
    case ACT_PRELU: f(std::integral_constant<int, ACT_PRELU>{}); break;
    case ACT_TANH: f(std::integral_constant<int, ACT_TANH>{}); break;
    case ACT_SELU: f(std::integral_constant<int, ACT_SELU>{}); break;
    case ACT_ELU: f(std::integral_constant<int, ACT_ELU>{}); break;
    default: f(std::integral_constant<int, ACT_IDENTITY>{}); break;
    }
}
// the same on the host (kernels instantiated per activation)
template <typename F>
inline void host_with_act(int act, F &&f) {
    switch (act) {
    case ACT_RELU: f(std::integral_constant<int, ACT_RELU>{}); break;
    case ACT_LEAKY: f(std::integral_constant<int, ACT_LEAKY>{}); break;
    case ACT_PRELU: f(std::integral_constant<int, ACT_PRELU>{}); break;
    case ACT_TANH: f(std::integral_constant<int, ACT_TANH>{}); break;
    case ACT_SELU: f(std::integral_constant<int, ACT_SELU>{}); break;
    case ACT_ELU: f(std::integral_constant<int, ACT_ELU>{}); break;
    default: f(std::integral_constant<int, ACT_IDENTITY>{}); break;
    }
}

// d act / d z from the pre-activation z (torch's conventions at z == 0: ReLU 0, LeakyReLU/PReLU slope).
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

// Counter-based dropout: keep with probability 1-p, scale 1/(1-p).  Re-derived in backward from
// (seed, layer, row, col), so no mask is stored.
__device__ __forceinline__ float dropout_scale(uint64_t seed, uint32_t layer, uint32_t row, uint32_t col, float p) {
    uint64_t x = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(layer + 1));
    x ^= ((uint64_t)row << 32) | col;
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    const float u = (float)(uint32_t)(x >> 40) * (1.0f / 16777216.0f);
    return u >= p ? 1.0f / (1.0f - p) : 0.0f;
}

// WD_STAMPS (experiment builds only): per-workgroup phase timestamps of the fused layer kernel, from the
// chip-wide 100 MHz clock (s_memrealtime), written by one lane with a vector store; read back with
// wdmpnn_debug_stamps (tools/stamps_layer.py)
#ifndef WD_STAMPS
#define WD_STAMPS 0
#endif
#if WD_STAMPS
constexpr int WD_STAMP_SLOTS = 16, WD_STAMP_WG = 8192;
__device__ uint64_t g_wd_stamps[WD_STAMP_WG * WD_STAMP_SLOTS];
__device__ __forceinline__ void wd_stamp(int slot) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < WD_STAMP_WG)
        __hip_atomic_store(&g_wd_stamps[blockIdx.x * WD_STAMP_SLOTS + slot], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// per-chunk loop stamps (shader clock, s_memtime): [WG][chunk < 16][slot < 8], one lane of the calling wave
constexpr int WD_LSTAMP_WG = 512;
__device__ uint64_t g_wd_lstamps[WD_LSTAMP_WG * 16 * 8];
// the embed's phases (tools/stamps_embed.py): [WG][8], after the loop stamps in wdmpnn_debug_stamps' buffer
__device__ uint64_t g_wd_estamps[WD_STAMP_WG * 8];
__device__ __forceinline__ void wd_estamp(int slot) {
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < WD_STAMP_WG)
        __hip_atomic_store(&g_wd_estamps[blockIdx.x * 8 + slot], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wd_lstamp(int chunk, int slot) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0 && blockIdx.x < WD_LSTAMP_WG && chunk < 16)
        __hip_atomic_store(&g_wd_lstamps[(blockIdx.x * 16 + chunk) * 8 + slot], t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#else
__device__ __forceinline__ void wd_stamp(int) {}
__device__ __forceinline__ void wd_estamp(int) {}
__device__ __forceinline__ void wd_lstamp(int, int) {}
#endif

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ void fma4(float4 &acc, float c, const float4 &v) {
    acc.x = fmaf(c, v.x, acc.x);
    acc.y = fmaf(c, v.y, acc.y);
    acc.z = fmaf(c, v.z, acc.z);
    acc.w = fmaf(c, v.w, acc.w);
}

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, const float4 &v) { *reinterpret_cast<float4 *>(p) = v; }

// Bijective XCD-aware block -> tile map (cdna_hip_programming.md §5.5 T1): blocks b and b+8 share an
// XCD under round-robin dispatch, so give each XCD a contiguous range of tiles; tiles of one row
// block (same A rows, different column blocks) then share that XCD's L2.  Speed only, never
// correctness.
__device__ __forceinline__ int xcd_tile(int b, int ntiles) {
    const int base = ntiles >> 3, rem = ntiles & 7;
    const int x = b & 7, local = b >> 3;
    return x * base + (x < rem ? x : rem) + local;
}

// Several independent batches in one launch (wdmpnn_forward_many, the stream feed's graph builds): per batch its parameter struct and
// its first tile in the grid; a workgroup finds its batch by a short uniform scan (the structs stay in
// the kernel-argument segment: scalar loads).  One batch: n = 1, launched through the NJ = 1 form (the
// kernel arguments of eight slots are 0.9-2.2 KB, and a launch's host cost grows with its argument bytes:
// 2.5-4.3 us at 2.5 KB against 0.9-2.4 us at 64 B, tools/launch_cost.hip).
constexpr int WD_MULTI = 8;
template <typename T, int NJ = WD_MULTI> struct Multi {
    T p[NJ];
    int t0[NJ + 1];  // tile ranges: batch j owns grid tiles [t0[j], t0[j + 1])
    int n;
};
template <typename T, int NJ>
__device__ __forceinline__ const T &multi_pick(const Multi<T, NJ> &M, int g, int &tile) {
    int j = 0;
    while (j + 1 < M.n && g >= M.t0[j + 1]) ++j;
    tile = g - M.t0[j];
    return M.p[j];
}

}  // namespace wd
