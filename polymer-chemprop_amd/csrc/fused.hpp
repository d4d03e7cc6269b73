// fused.hpp — gather-fused row-panel GEMM: C[16-row panel][all N] = epi( A(panel) · Bᵀ ), where the
// A operand is built in LDS by the workgroup itself from up to two K segments, each either
//   dense     rows of a padded matrix (f_bonds / f_atoms: mpn.py:92-93, 132's concat), or
//   gathered  X_r = Σ_{e ∈ csr(r)} coef_e · src[idx_e]  (the index_select_ND + weighted sum +
//             reverse-message subtraction of mpn.py:110-120 / 126-131, as one CSR list per row).
//
// Why this shape: at the benchmark size a separate gather kernel plus a GEMM costs
// two launches with ~6-7 µs of fixed latency each, and the GEMM re-reads the gathered X from HBM.
// Here one workgroup owns 16 rows x ALL N columns (N = Hk ≤ 512, one wave per 64 columns), so
//   * each gathered row is built exactly once (no redundancy across N tiles),
//   * the A panel (16 x K floats, ≤ 76 KB) stays in LDS for the whole K loop: no barrier in the loop,
//   * B (the packed weight, ≤ 4 MB, L2-resident and shared by every workgroup) is streamed straight
//     into registers, one 32-wide K chunk ahead,
//   * the epilogue (bias + residual + activation + dropout) goes through LDS for float4 stores.
// MFMA: v_mfma_f32_16x16x4_f32 (exact fp32), wave = 16 rows x 64 cols = 4 independent accumulators;
// lane (i = l&15, g = l>>4) supplies k = 8g + s at step s of a 32-chunk (two b128 reads per operand).
// Accumulation order per gathered element is the CSR order, identical to gather8_kernel.
#pragma once
#include "gemm.hpp"

namespace wd {

constexpr int FP_ROWS = 16;
constexpr int GU = 2;       // gathered outputs per thread per round (4 spills at 256 VGPRs)

struct FSeg {
    const float *src; int ld;      // dense: A rows; gathered: source rows
    int K;                         // segment width in A (multiple of 32)
    const int32_t *ptr;            // null = dense segment
    const int32_t *idx; const float *coef; const int32_t *sym_rev;
    float *xout; int ld_xout;      // optional copy of the built segment (training: X_t / A for dW)
};

struct FusedP {
    FSeg seg[2]; int nseg;
    int rows;                      // CSR rows (gathered rows >= rows are zero)
    const float *b; int ldb;       // fragment-order packed weight (N x ldb floats), ldb == K0 + K1
    int M, N;                      // rows / cols written
    Epi epi;
};

__device__ __forceinline__ float4 f4avg(float4 v, float4 u) {
    v.x = (v.x + u.x) / 2.0f; v.y = (v.y + u.y) / 2.0f; v.z = (v.z + u.z) / 2.0f; v.w = (v.w + u.w) / 2.0f;
    return v;
}

// Build rows [m0, m0+16) of one segment into LDS columns [c0, c0 + K).
__device__ __forceinline__ void build_segment(const FSeg &S, int rows, int m0, float *lds, int lda, int c0) {
    const int nq = S.K >> 2, total = FP_ROWS * nq, NT = blockDim.x;
    if (!S.ptr) {
        for (int v = threadIdx.x; v < total; v += NT) {
            const int r = v / nq, c = (v % nq) * 4;
            const float4 x = ld4(S.src + (size_t)(m0 + r) * S.ld + c);
            st4(lds + r * lda + c0 + c, x);
            if (S.xout) st4(S.xout + (size_t)(m0 + r) * S.ld_xout + c, x);
        }
        return;
    }
    // gathered: GU outputs per thread per round; the first four CSR entries of each are fetched
    // together (predicated, pad row 0 as the dummy source) so one round is three dependent hops.
    for (int v0 = threadIdx.x; v0 < total; v0 += GU * NT) {
        int r[GU], c[GU], e0[GU], e1[GU];
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            const int v = v0 + u * NT;
            const bool in = v < total;
            r[u] = in ? v / nq : 0;
            c[u] = in ? (v % nq) * 4 : 0;
            const int row = m0 + r[u];
            const bool live = in && row < rows;
            e0[u] = live ? S.ptr[row] : 0;
            e1[u] = live ? S.ptr[row + 1] : 0;
        }
        int j[GU][4]; float w[GU][4];
#pragma unroll
        for (int u = 0; u < GU; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool ok = e0[u] + k < e1[u];
                j[u][k] = ok ? S.idx[e0[u] + k] : 0;
                w[u][k] = ok ? (S.coef ? S.coef[e0[u] + k] : 1.0f) : 0.0f;
            }
        float4 x[GU][4];
#pragma unroll
        for (int u = 0; u < GU; ++u)
#pragma unroll
            for (int k = 0; k < 4; ++k) x[u][k] = ld4(S.src + (size_t)j[u][k] * S.ld + c[u]);
        if (S.sym_rev) {
#pragma unroll
            for (int u = 0; u < GU; ++u)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    x[u][k] = f4avg(x[u][k], ld4(S.src + (size_t)S.sym_rev[j[u][k]] * S.ld + c[u]));
        }
#pragma unroll
        for (int u = 0; u < GU; ++u) {
            if (v0 + u * NT >= total) continue;
            float4 acc = f4zero();
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (e0[u] + k < e1[u]) fma4(acc, w[u][k], x[u][k]);
            for (int e = e0[u] + 4; e < e1[u]; ++e) {  // rows with more than four entries
                const int jj = S.idx[e];
                const float ww = S.coef ? S.coef[e] : 1.0f;
                float4 y = ld4(S.src + (size_t)jj * S.ld + c[u]);
                if (S.sym_rev) y = f4avg(y, ld4(S.src + (size_t)S.sym_rev[jj] * S.ld + c[u]));
                fma4(acc, ww, y);
            }
            st4(lds + r[u] * lda + c0 + c[u], acc);
            if (S.xout) st4(S.xout + (size_t)(m0 + r[u]) * S.ld_xout + c[u], acc);
        }
    }
}

// blockDim = N (multiple of 64, ≤ 512: 256 VGPRs per lane): wave w owns columns [64w, 64w + 64).  grid = Mp / 16.
// Dynamic LDS: 16 x (max(K, N) + 4) floats.
__global__ __launch_bounds__(512, 4) void gemm_fused_kernel(FusedP P) {
    extern __shared__ __attribute__((aligned(16))) float flds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, i16 = lane & 15;
    const int m0 = xcd_tile(blockIdx.x, gridDim.x) * FP_ROWS;
    const int K0 = P.seg[0].K, K = K0 + (P.nseg > 1 ? P.seg[1].K : 0);
    const int lda = K + 4;
    const Epi &E = P.epi;

    // B stream: lane needs W[64*wave + 16*b + i16][kc*32 + 8g .. +8] for its four 16-col tiles; the
    // weight is packed in fragment order (pack_kernel `frag`), so each (tile, half) of a chunk is one
    // contiguous 1 KB wave load.
    const int nchunks = K / BK;
    const float *bw = P.b + (size_t)wave * nchunks * 2048 + lane * 4;
    struct BReg { float4 v[4][2]; };
    auto load_b = [&](BReg &R, int kc) {
        const float *src = bw + (size_t)min(kc, nchunks - 1) * 2048;
#pragma unroll
        for (int b = 0; b < 4; ++b) { R.v[b][0] = ld4(src + (2 * b) * 256); R.v[b][1] = ld4(src + (2 * b + 1) * 256); }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the MFMAs it overlaps
    };
    BReg R0, R1;
    load_b(R0, 0);  // in flight across phase 1

    // phase 1: the A panel
    build_segment(P.seg[0], P.rows, m0, flds, lda, 0);
    if (P.nseg > 1) build_segment(P.seg[1], P.rows, m0, flds, lda, K0);
    __syncthreads();

    // phase 2: K loop, A from LDS, B from registers (prefetch distance 2 chunks)
    floatx4 acc[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[b] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float *arow = flds + i16 * lda + 8 * g;
    auto compute = [&](const BReg &R, int kc) {
        const float4 a0 = ld4(arow + kc * BK), a1 = ld4(arow + kc * BK + 4);
        const float af[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const float4 &h = R.v[b][s >> 2];
                const float bf = (s & 3) == 0 ? h.x : (s & 3) == 1 ? h.y : (s & 3) == 2 ? h.z : h.w;
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[s], bf, acc[b], 0, 0, 0);
            }
    };
    // prefetch distance 1 chunk: two register sets keep the kernel at <= 128 VGPRs (4 waves per
    // SIMD, 3 five-wave workgroups per CU; at 2 waves per SIMD only one fits and the grid runs in
    // rounds -- measured: SQ_WAVE_CYCLES per wave = 0.39 x kernel cycles)
    int kc = 0;
    for (; kc + 1 < nchunks; kc += 2) {
        load_b(R1, kc + 1); compute(R0, kc);
        load_b(R0, kc + 2); compute(R1, kc + 1);
    }
    if (kc < nchunks) compute(R0, kc);

    // epilogue operands (issued after the K loop: registers) -- thread -> float4 column q of rows
    // rg + 4p, p = 0..3
    const int C4 = P.N >> 2, q = tid % C4, rg = tid / C4;
    float4 bias = f4zero(), resid[4];
    if (E.kind == EPI_ACT && E.bias && 4 * q < P.N) bias = ld4(E.bias + 4 * q);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int i = m0 + rg + 4 * p;
        resid[p] = (E.kind == EPI_ACT && E.resid && i < P.M) ? ld4(E.resid + (size_t)i * E.ld + 4 * q) : f4zero();
    }

    // epilogue through LDS (row stride N + 4)
    __syncthreads();
    const int ldc = P.N + 4;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) flds[(4 * g + r) * ldc + 64 * wave + 16 * b + i16] = acc[b][r];
    __syncthreads();
    const float slope = (E.kind == EPI_ACT && E.act == ACT_PRELU) ? E.slope[0] : 0.f;
    const int j = 4 * q;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int rl = rg + 4 * p, i = m0 + rl;
        if (i >= P.M || rg >= 4) continue;
        const float4 v = ld4(flds + rl * ldc + j);
        const size_t o = (size_t)i * E.ld + j;
        if (E.kind == EPI_ACT) {
            const float vv[4] = {v.x, v.y, v.z, v.w};
            const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
            const float rr[4] = {resid[p].x, resid[p].y, resid[p].z, resid[p].w};
            float z[4], y[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                z[t] = vv[t] + bb[t] + rr[t];
                y[t] = act_fwd(E.act, z[t], slope);
                if (E.p_drop > 0.f) y[t] *= dropout_scale(E.seed, E.layer, i, j + t, E.p_drop);
            }
            if (E.Z) st4(E.Z + o, make_float4(z[0], z[1], z[2], z[3]));
            st4(E.Y + o, make_float4(y[0], y[1], y[2], y[3]));
        } else {
            float4 r = v;
            if (E.accumulate) {
                const float4 y0 = ld4(E.Y + o);
                r.x += y0.x; r.y += y0.y; r.z += y0.z; r.w += y0.w;
            }
            st4(E.Y + o, r);
        }
    }
}

}  // namespace wd
