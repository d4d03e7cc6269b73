// gemm_x6.hpp — fp32 GEMMs on the bf16 matrix cores by exact three-way operand splitting ("bf16x6").
//
// Both operands are split into bf16x3 planes (planes.hpp: x = h + m + l exactly).  A product a·b is
// the sum of nine plane products, each exact in fp32 (8 x 8 significant bits), accumulated in fp32 by
// v_mfma_f32_16x16x32_bf16.  Six are kept:
//     hh, hm, mh, hl, lh, mm
// the three dropped ones (ml, lm, ll) are below 2^-25 |a·b| together -- under half an fp32 ulp of
// the product -- so the GEMM keeps fp32 accuracy (tools/x6_precision.py and the GPU parity tests
// measure it against fp64 and against the f32-MFMA path).  Six bf16 MFMAs of K = 32 take 6 x 16 = 96
// cycles where the f32 MFMA needs 8 x 32 = 256: 2.67x the fp32 matrix rate of MI355X.
//
// C[Mp][Np] = epi([A0 | A1] · Bᵀ), tile BM x 64, waves of 32x32 (2x2 16x16x32 accumulators), K in
// 32-wide chunks.  LDS image of one plane: 64 B per row, 16-byte unit u of row r at
// 64 r + 16 (u ^ ((r >> 1) & 3)) (conflict-free fragment reads, brute-force checked against the
// ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS).
//   gemm_x6g_kernel  operands arrive as plane tiles (written by their producers: the gathers, the
//                    weight packer, the graph upload); staging is LDS-DMA (global_load_lds_dwordx4),
//                    no staging registers, no arithmetic.  The forward's default.
//   gemm_x6_kernel   fp32 operands split in registers while staging (fallback for operands that
//                    have no plane copy: atom-message mode, descriptors).
#pragma once
#include "gemm.hpp"
#include "planes.hpp"

namespace wd {

struct X6Params {
    const float *a0; int lda0; int ka0;   // A segment 0 [Mp][lda0], K extent ka0 (multiple of BK)
    const float *a1; int lda1; int ka1;   // A segment 1 (ka1 = 0: absent)
    const float *bf; int ldb;             // B fp32 [Np][ldb]
    int M, N;                             // rows / cols written
    int tiles_m, tiles_n;
    Epi epi;
};

// BM x 64 tile, 4 BM threads = (BM/32) x 2 waves of 32x32 (2x2 16x16x32 accumulators).  BK = 32 or 64
// wide K chunks, two LDS stages, two register sets (prefetch distance 2).  Operand rows are loaded as
// whole 128-byte lines (BK/4 consecutive lanes per row chunk: 8 lanes x 16 B at BK = 32) and each
// float4 is split into three 8-byte plane pieces (ds_write_b64).
template <int BM, int BK>
__global__ __launch_bounds__(4 * BM) void gemm_x6_kernel(X6Params P) {
    constexpr int NT = 4 * BM, BN = X6_BN;
    constexpr int ROWB = 2 * BK;                            // bytes per plane row
    constexpr int APL = BM * ROWB, BPL = BN * ROWB;         // plane bytes
    constexpr int STAGE = 3 * APL + 3 * BPL;
    constexpr int QR = BK / 4;                              // float4 per row chunk
    constexpr int AQ = BM * QR / NT, BQ = BN * QR / NT;     // float4 per thread per chunk
    static_assert((BN * QR) % NT == 0 && BQ >= 1, "B staging split");
    static_assert((BM * QR) % NT == 0, "A staging split");
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave >> 1, wj = wave & 1, g = lane >> 4, i16 = lane & 15;
    const int tile = xcd_tile(blockIdx.x, P.tiles_m * P.tiles_n);
    const int mt = tile / P.tiles_n, nt = tile % P.tiles_n;
    const int m0 = mt * BM, n0 = nt * BN;
    const int K = P.ka0 + P.ka1, nchunks = K / BK;
    EpiPrefetch<BM, BN, NT> ep;
    ep.load(P.epi, m0, n0, P.M, P.N);

    // staging: float4 q = tid + NT j of a chunk -> row q / QR, column quad q % QR
    const int qr = tid / QR, qc = tid % QR;
    constexpr int RSTEP = NT / QR;  // rows between a thread's successive quads
    const float *arow0 = P.a0 + (size_t)(m0 + qr) * P.lda0 + 4 * qc;
    const float *arow1 = P.ka1 ? P.a1 + (size_t)(m0 + qr) * P.lda1 + 4 * qc - P.ka0 : nullptr;
    const float *brow = P.bf + (size_t)(n0 + qr) * P.ldb + 4 * qc;
    int dst[AQ > BQ ? AQ : BQ];  // plane offset of quad j (same pattern for A and B rows)
#pragma unroll
    for (int j = 0; j < (AQ > BQ ? AQ : BQ); ++j) dst[j] = x6_off<BK>(qr + j * RSTEP, qc >> 1) + 8 * (qc & 1);

    struct Regs { float4 a[AQ], b[BQ]; };
    auto load_chunk = [&](Regs &R, int kc) {
        const int k0 = kc * BK;
        const float *src = (k0 < P.ka0 ? arow0 : arow1) + k0;
        const int lda = k0 < P.ka0 ? P.lda0 : P.lda1;
#pragma unroll
        for (int j = 0; j < AQ; ++j) R.a[j] = ld4(src + (size_t)j * RSTEP * lda);
#pragma unroll
        for (int j = 0; j < BQ; ++j) R.b[j] = ld4(brow + (size_t)j * RSTEP * P.ldb + k0);
    };
    auto put = [&](uint8_t *base, int plane_bytes, int off, const float4 &v) {
        uint32_t h0, m0_, l0, h1, m1, l1;
        split_pair(v.x, v.y, h0, m0_, l0);
        split_pair(v.z, v.w, h1, m1, l1);
        *reinterpret_cast<uint2 *>(base + off) = make_uint2(h0, h1);
        *reinterpret_cast<uint2 *>(base + plane_bytes + off) = make_uint2(m0_, m1);
        *reinterpret_cast<uint2 *>(base + 2 * plane_bytes + off) = make_uint2(l0, l1);
    };
    auto store_chunk = [&](const Regs &R, uint8_t *st) {
#pragma unroll
        for (int j = 0; j < AQ; ++j) put(st, APL, dst[j], R.a[j]);
#pragma unroll
        for (int j = 0; j < BQ; ++j) put(st + 3 * APL, BPL, dst[j], R.b[j]);
    };

    floatx4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](const uint8_t *st) {
#pragma unroll
        for (int s = 0; s < BK / 32; ++s) {
            bf16x8 af[2][3], bfr[2][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int a = 0; a < 2; ++a)
                    af[a][p] = *reinterpret_cast<const bf16x8 *>(st + p * APL + x6_off<BK>(wi * 32 + a * 16 + i16, 4 * s + g));
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    bfr[b][p] = *reinterpret_cast<const bf16x8 *>(st + 3 * APL + p * BPL +
                                                                  x6_off<BK>(wj * 32 + b * 16 + i16, 4 * s + g));
            }
            // plane products hh, hm, mh, hl, lh, mm
            constexpr int PA[6] = {0, 0, 1, 0, 2, 1}, PB[6] = {0, 1, 0, 2, 0, 1};
#pragma unroll
            for (int t = 0; t < 6; ++t)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][PA[t]], bfr[b][PB[t]], acc[a][b], 0, 0, 0);
        }
    };

    Regs R0, R1;
    load_chunk(R0, 0);
    load_chunk(R1, min(1, nchunks - 1));
    store_chunk(R0, lds);
    __syncthreads();
    auto step = [&](int kc, Regs &Rnext, Regs &Rfree) {
        load_chunk(Rfree, min(kc + 2, nchunks - 1));
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this chunk's MFMAs
        compute(lds + (kc & 1) * STAGE);
        if (kc + 1 < nchunks) store_chunk(Rnext, lds + ((kc + 1) & 1) * STAGE);
        __syncthreads();
    };
    int kc = 0;
    for (; kc + 1 < nchunks; kc += 2) {
        step(kc, R1, R0);
        step(kc + 1, R0, R1);
    }
    if (kc < nchunks) step(kc, R1, R0);

    // epilogue: C tile through LDS (row stride 68 floats), coalesced float4 with the fused
    // bias / residual / activation / dropout (gemm.hpp epilogue_v4)
    float *cl = reinterpret_cast<float *>(lds);
    constexpr int LDC = BN + 4;
    static_assert(BM * LDC * 4 <= 2 * STAGE, "C tile must fit in the staging LDS");
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) cl[(wi * 32 + a * 16 + 4 * g + r) * LDC + wj * 32 + b * 16 + i16] = acc[a][b][r];
    __syncthreads();
    epilogue_v4<BM, BN, NT>(P.epi, cl, LDC, m0, n0, P.M, P.N, ep);
}

struct X6PParams {
    const uint8_t *a0; int kp0; int ka0;  // A segment 0: plane tiles of a [Mp][kp0] matrix, K extent ka0
    const uint8_t *a1; int kp1; int ka1;  // A segment 1 (ka1 = 0: absent)
    const uint8_t *b; int kpb;            // B plane tiles [Np][kpb], kpb == ka0 + ka1
    int M, N;
    int tiles_m, tiles_n;
    Epi epi;
};

// ---------------------------------------------------------------------------------------------
// gemm_x6g_kernel: both operands pre-split (plane tiles), staged by LDS-DMA (global_load_lds_dwordx4,
// cdna_hip_programming.md §5 "Async global->LDS copy"): no staging registers, S LDS stages, S-1 chunks
// in flight behind counted vmcnt waits and raw s_barrier (a __syncthreads would drain the DMA queue).
// Each wave-instruction fills 1 KB of LDS lane-linearly; the bank swizzle is applied on the per-lane
// global source address (rows stay 64 B, unit s of row r reads source unit s ^ ((r >> 1) & 3)).
// Per 32-wide chunk: A 12 KB + B 12 KB = 24 pieces of 1 KB, 6 per wave (BM = 64).
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void *g, uint8_t *lds_wave_base) {
    __builtin_amdgcn_global_load_lds(g, (lds_void_t *)lds_wave_base, 16, 0, 0);
}

template <int S>
__global__ __launch_bounds__(256) void gemm_x6g_kernel(X6PParams P) {
    constexpr int BM = 64, BN = X6_BN, NT = 256;
    constexpr int APL = BM * 64, STAGE = 3 * APL + 3 * X6_PLANE;  // 24 KB
    __shared__ __attribute__((aligned(16))) uint8_t lds[S * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave >> 1, wj = wave & 1, g = lane >> 4, i16 = lane & 15;
    const int tile = xcd_tile(blockIdx.x, P.tiles_m * P.tiles_n);
    const int mt = tile / P.tiles_n, nt = tile % P.tiles_n;
    const int m0 = mt * BM, n0 = nt * BN;
    const int K = P.ka0 + P.ka1, nchunks = K >> 5;
    EpiPrefetch<BM, BN, NT> ep;
    ep.load(P.epi, m0, n0, P.M, P.N);

    // this wave's 6 pieces of a stage: j = 0..2 -> A piece 3 wave + j, j = 3..5 -> B piece 3 wave + j - 3;
    // piece c, lane l -> image unit q = 64 c + l = (plane q / 256, row (q / 4) % 64, slot q % 4)
    int src[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const int q = 64 * (3 * wave + (j % 3)) + lane, p = q >> 8, r = (q >> 2) & 63, sl = q & 3;
        src[j] = p * X6_PLANE + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
    }
    const uint8_t *bbase = P.b + (size_t)nt * (P.kpb >> 5) * X6_BLOCK;
    auto issue = [&](int kc, int stage) {
        const int k0 = kc << 5;
        const bool s1 = k0 >= P.ka0;
        const uint8_t *abase = s1 ? P.a1 : P.a0;
        const int kp = s1 ? P.kp1 : P.kp0, kk = s1 ? k0 - P.ka0 : k0;
        const uint8_t *ablk = abase + ((size_t)(m0 >> 6) * (kp >> 5) + (kk >> 5)) * X6_BLOCK;
        const uint8_t *bblk = bbase + (size_t)kc * X6_BLOCK;
        uint8_t *st = lds + stage * STAGE;
#pragma unroll
        for (int j = 0; j < 3; ++j) glds16(ablk + src[j], st + 1024 * (3 * wave + j));
#pragma unroll
        for (int j = 0; j < 3; ++j) glds16(bblk + src[3 + j], st + 3 * APL + 1024 * (3 * wave + j));
    };

    floatx4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    int ao[2], bo[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) ao[a] = x6_slot(wi * 32 + a * 16 + i16, g);
#pragma unroll
    for (int b = 0; b < 2; ++b) bo[b] = 3 * APL + x6_slot(wj * 32 + b * 16 + i16, g);
    auto compute = [&](const uint8_t *st) {
        bf16x8 af[2][3], bfr[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int a = 0; a < 2; ++a) af[a][p] = *reinterpret_cast<const bf16x8 *>(st + p * APL + ao[a]);
#pragma unroll
            for (int b = 0; b < 2; ++b) bfr[b][p] = *reinterpret_cast<const bf16x8 *>(st + p * X6_PLANE + bo[b]);
        }
        constexpr int PA[6] = {0, 0, 1, 0, 2, 1}, PB[6] = {0, 1, 0, 2, 0, 1};
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][PA[t]], bfr[b][PB[t]], acc[a][b], 0, 0, 0);
    };

    // prologue: chunks 0 .. S-2 in flight (a missing chunk issues a repeat of the last one so that
    // every wave always has the same number of DMA groups outstanding: the counted waits stay exact)
#pragma unroll
    for (int c = 0; c < S - 1; ++c) issue(min(c, nchunks - 1), c);
    for (int kc = 0; kc < nchunks; ++kc) {
        // chunk kc landed (this wave's 6 pieces; S-2 younger groups may stay in flight) ...
        if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        // ... for every wave, and every wave is done reading stage (kc - 1) % S
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        issue(min(kc + S - 1, nchunks - 1), (kc + S - 1) % S);
        compute(lds + (kc % S) * STAGE);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the trailing repeat DMAs before reusing LDS
    __syncthreads();

    float *cl = reinterpret_cast<float *>(lds);
    constexpr int LDC = BN + 4;
    static_assert(BM * LDC * 4 <= S * STAGE, "C tile must fit in the staging LDS");
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) cl[(wi * 32 + a * 16 + 4 * g + r) * LDC + wj * 32 + b * 16 + i16] = acc[a][b][r];
    __syncthreads();
    epilogue_v4<BM, BN, NT>(P.epi, cl, LDC, m0, n0, P.M, P.N, ep);
}

}  // namespace wd
