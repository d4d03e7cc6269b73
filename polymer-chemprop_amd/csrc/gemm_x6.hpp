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
//   gemm_x6_kernel   fp32 operands split in registers while staging (operands that have no plane copy:
//                    the backward's data gradients, atom-message mode, descriptors); its H2 form splits
//                    into fp16 pairs instead (the message layers' data gradients).
#pragma once
#include "gemm.hpp"
#include "planes.hpp"

#include <type_traits>

namespace wd {

// experiment builds: per-chunk stamps of gemm_x6_kernel (1) or gemm_tn_x6_kernel (2), with WD_STAMPS
#ifndef WD_STAMP_GEMM
#define WD_STAMP_GEMM 0
#endif

struct X6Params {
    const float *a0; int lda0; int ka0;   // A segment 0 [Mp][lda0], K extent ka0 (multiple of BK)
    const float *a1; int lda1; int ka1;   // A segment 1 (ka1 = 0: absent)
    const float *bf; int ldb;             // B fp32 [Np][ldb]
    int M, N;                             // rows / cols written
    int tiles_m, tiles_n;
    Epi epi;
    // H2 (fp16 pairs): A's scale from the max words its producer published, one per 256 consecutive
    // float4 of A (act_bwd_kernel's `words`: word (r * a_cv + c / 4) / 256, a_cv = float4 per A row);
    // B's from one word (W_h's folded max)
    const uint32_t *a_words; int a_cv;
    const uint32_t *b_word;
};

// BM x 64 tile, 4 BM threads = (BM/32) x 2 waves of 32x32 (2x2 16x16x32 accumulators).  BK = 32 or 64
// wide K chunks, two LDS stages, two register sets (prefetch distance 2).  Operand rows are loaded as
// whole 128-byte lines (BK/4 consecutive lanes per row chunk: 8 lanes x 16 B at BK = 32) and each
// float4 is split into three 8-byte plane pieces (ds_write_b64).
//
// H2: the same kernel on fp16 hi / lo pairs (planes.hpp "h2"): two planes per operand and three MFMAs
// (hh, hl, lh) per 16 x 16 x 32 step instead of three planes and six; A scaled by the max of its tile's
// rows (the words its producer published), B by one word; the accumulators are unscaled before the
// epilogue (powers of two: exact).  The data-gradient GEMM dM = Y_t W_h of the fused backward.
template <int BM, int BK, bool H2 = false>
__global__ __launch_bounds__(4 * BM) void gemm_x6_kernel(X6Params P) {
    constexpr int NT = 4 * BM, BN = X6_BN;
    constexpr int NPL = H2 ? 2 : 3;                         // planes per operand
    constexpr int ROWB = 2 * BK;                            // bytes per plane row
    constexpr int APL = BM * ROWB, BPL = BN * ROWB;         // plane bytes
    constexpr int STAGE = NPL * APL + NPL * BPL;
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
    float sa = 1.f, sb = 1.f, inv_sa = 1.f, inv_sb = 1.f;
    if constexpr (H2) {
        const int w0 = (m0 * P.a_cv) >> 8, w1 = ((m0 + BM) * P.a_cv - 1) >> 8;
        const uint32_t ma = max_words(P.a_words + w0, w1 - w0 + 1), mb = P.b_word[0];
        sa = h2_scale(ma); inv_sa = h2_inv_scale(ma);
        sb = h2_scale(mb); inv_sb = h2_inv_scale(mb);
    }

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
    auto put = [&](uint8_t *base, int plane_bytes, int off, const float4 &v, float s) {
        if constexpr (H2) {
            uint32_t h0, l0, h1, l1;
            split_h2(v.x, v.y, s, h0, l0);
            split_h2(v.z, v.w, s, h1, l1);
            *reinterpret_cast<uint2 *>(base + off) = make_uint2(h0, h1);
            *reinterpret_cast<uint2 *>(base + plane_bytes + off) = make_uint2(l0, l1);
        } else {
            uint32_t h0, m0_, l0, h1, m1, l1;
            split_pair(v.x, v.y, h0, m0_, l0);
            split_pair(v.z, v.w, h1, m1, l1);
            *reinterpret_cast<uint2 *>(base + off) = make_uint2(h0, h1);
            *reinterpret_cast<uint2 *>(base + plane_bytes + off) = make_uint2(m0_, m1);
            *reinterpret_cast<uint2 *>(base + 2 * plane_bytes + off) = make_uint2(l0, l1);
        }
    };
    auto store_chunk = [&](const Regs &R, uint8_t *st) {
#pragma unroll
        for (int j = 0; j < AQ; ++j) put(st, APL, dst[j], R.a[j], sa);
#pragma unroll
        for (int j = 0; j < BQ; ++j) put(st + NPL * APL, BPL, dst[j], R.b[j], sb);
    };

    floatx4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](const uint8_t *st) {
        if constexpr (H2) {
#pragma unroll
            for (int s = 0; s < BK / 32; ++s) {
                f16x8 af[2][2], bfr[2][2];
#pragma unroll
                for (int p = 0; p < 2; ++p) {
#pragma unroll
                    for (int a = 0; a < 2; ++a)
                        af[a][p] = *reinterpret_cast<const f16x8 *>(st + p * APL + x6_off<BK>(wi * 32 + a * 16 + i16, 4 * s + g));
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        bfr[b][p] = *reinterpret_cast<const f16x8 *>(st + 2 * APL + p * BPL +
                                                                     x6_off<BK>(wj * 32 + b * 16 + i16, 4 * s + g));
                }
                // hi hi, hi lo, lo hi
                constexpr int PA[3] = {0, 0, 1}, PB[3] = {0, 1, 0};
#pragma unroll
                for (int t = 0; t < 3; ++t)
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int b = 0; b < 2; ++b)
                            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][PA[t]], bfr[b][PB[t]], acc[a][b], 0, 0, 0);
            }
            return;
        }
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
        if (WD_STAMP_GEMM == 1 && wave == 0) wd_lstamp(kc, 0);
        load_chunk(Rfree, min(kc + 2, nchunks - 1));
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this chunk's MFMAs
        compute(lds + (kc & 1) * STAGE);
        if (WD_STAMP_GEMM == 1 && wave == 0) wd_lstamp(kc, 1);
        if (kc + 1 < nchunks) store_chunk(Rnext, lds + ((kc + 1) & 1) * STAGE);
        if (WD_STAMP_GEMM == 1 && wave == 0) wd_lstamp(kc, 2);
        __syncthreads();
        if (WD_STAMP_GEMM == 1 && wave == 0) wd_lstamp(kc, 3);
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
            for (int r = 0; r < 4; ++r)
                cl[(wi * 32 + a * 16 + 4 * g + r) * LDC + wj * 32 + b * 16 + i16] = H2 ? acc[a][b][r] * inv_sa * inv_sb
                                                                                      : acc[a][b][r];
    __syncthreads();
    const uint32_t mx = epilogue_v4<BM, BN, NT>(P.epi, cl, LDC, m0, n0, P.M, P.N, ep);
    if (P.epi.kind == EPI_ACTBWD && P.epi.amax) {
        __shared__ uint32_t red[NT / 64];
        publish_max(mx, P.epi.amax + mt * P.tiles_n + nt, red);
    }
}

// ---------------------------------------------------------------------------------------------
// gemm_tn_x6_kernel — weight gradients as a split-plane GEMM:
//     slab[z][i][j] (+)= sum_{m in split z} A[m][i] B[m][j]     (A = dZ, B = the layer input X)
//     slab[z][i][bias_col] (+)= sum_{m in split z} A[m][i]      (the bias: X's ones column)
// Both operands are row-major in the reduction index m (thousands of bond / atom rows).  A 32-row
// chunk is loaded as 4 rows x 4 columns per thread (16 consecutive lanes read one 256-byte row
// piece), split into bf16x3 planes in registers and stored in the same orientation: LDS image
// [32 m][64 columns] per plane, one conflict-free ds_write_b64 per row and plane.  The MFMA operands
// need 8 consecutive m per lane; ds_read_b64_tr_b16 (MI355X transposed LDS read, cdna_hip_programming
// T10) delivers them from the row-major image, two reads per fragment, conflict-free under the row
// swizzle of tn_unit (brute-forced over both lane halves).  Same products as gemm_x6_kernel (hh hm mh hl
// lh mm).  Threads 0-127 stage A, 128-255 B.  The bias column is not a GEMM tile: the j-tile-0
// workgroups sum their staged rows per column and reduce the eight row groups in a fixed order.
// Deterministic: fixed split ranges, fixed in-tile order, slabs reduced in split order by
// slab_reduce_kernel.
// ---------------------------------------------------------------------------------------------
// byte offset of 8-byte unit u (columns 4u .. 4u+3) of row r in a [32][64] bf16 plane image (128-byte
// rows); the xor spreads the 8 rows of one transposed read over all 64 banks
__device__ __forceinline__ int tn_unit(int r, int u) { return r * 128 + 8 * (u ^ (4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)))); }

typedef short tn_v4s __attribute__((ext_vector_type(4)));
// bf16x8 MFMA fragment of column c (lane-varying), rows 8g .. 8g+7 of a plane image: two transposed reads
__device__ __forceinline__ bf16x8 tn_frag(const uint8_t *plane, int c0, int lane) {
    const int i16 = lane & 15, g = lane >> 4;
    const int u = (c0 >> 2) + (i16 & 3);
    const tn_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) tn_v4s *)(plane + tn_unit(8 * g + (i16 >> 2), u)));
    const tn_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) tn_v4s *)(plane + tn_unit(8 * g + 4 + (i16 >> 2), u)));
    const short v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
}
struct TnX6Params {
    Src A, B;              // A: rows m, cols i (dZ);  B: rows m, cols j (dense segments; the ones column is
                           // the bias and is never read)
    int M, N;              // output rows i (< A.cols_p) / dense output columns j
    int K;                 // reduction rows
    int k_per_split;       // multiple of 32
    int tiles_m, tiles_n;
    float *slab; int ld_slab; long long slab_stride; int accumulate;
    int bias_col;          // slab column of the bias gradient, -1 = none
    const float *bias_src; int bias_ld;  // the bias as column sums of this matrix [K][bias_ld] instead of A (or null)
    // H2 with published scale words instead of the max pass: one scale per operand over the split's rows.
    // A: act_bwd_kernel's words (one per 256 float4, a_cv float4 per row); B: the data-gradient GEMM's
    // (one per b_bm-row x 64-column tile, b_tn column tiles)
    const uint32_t *a_words; int a_cv;
    const uint32_t *b_words; int b_bm, b_tn;
};

// SACT: the activation of a SEG_ACT operand as a compile-time constant (one instantiation per activation:
// a runtime switch over all of them in the staging path bloated the kernel past the instruction cache),
// -1 when no operand is SEG_ACT.  BEXT: the bias sums come from P.bias_src (a compile-time switch: a runtime
// branch around those loads left the compiler's vmcnt waits unable to skip the prefetched chunk's loads)
#ifndef WD_TN_DEPTH
#define WD_TN_DEPTH 2
#endif
#ifndef WD_TN_H2
#define WD_TN_H2 0
#endif
constexpr bool TN_H2 = WD_TN_H2;
constexpr int TN_DEPTH = WD_TN_DEPTH;
// H2: the operands as fp16 hi/lo pairs (planes.hpp split_h2) instead of bf16x3 planes -- two planes per
// operand, three f16 products (hh hl lh) instead of six.  fp16 needs a scale: each of the tile's 128
// operand columns gets its own power-of-two scale from its max |value| over this split's rows (a max pass
// over the split's rows before the GEMM: the values staged are exactly the values maxed, so nothing can
// overflow), and the epilogue multiplies each output by the inverse scales of its row and column (exact:
// powers of two).  Error per product <= 2^-22 of the column maxima (planes.hpp); deterministic.
template <int SACT, bool BEXT, bool H2>
__global__ __launch_bounds__(256) void gemm_tn_x6_kernel(TnX6Params P) {
    constexpr int BM = 64, BN = 64, NT = 256, BKC = 32;
    constexpr int PL = 32 * 128;           // one plane image: 32 rows (m) x 64 columns x 2 B
    constexpr int NPL = H2 ? 2 : 3;        // planes per operand
    constexpr int STAGE = 2 * NPL * PL;    // A planes, then B planes (24 KB; 16 KB with H2)
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
    __shared__ float inv_scale[H2 ? 128 : 1];  // H2: A columns (output rows), then B columns
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave >> 1, wj = wave & 1, g = lane >> 4, i16 = lane & 15;
    // 1-D grid of tiles x splits, XCD-aware (common.hpp xcd_tile): the tiles of one split (same rows of
    // dZ and X) run on one XCD and read those rows through its L2 once
    const int ntile = P.tiles_m * P.tiles_n;
    const int lin = xcd_tile(blockIdx.x, gridDim.x);
    const int split = lin / ntile, tile = lin % ntile;
    const int mt = tile / P.tiles_n, nt = tile % P.tiles_n;
    const int m0 = mt * BM, n0 = nt * BN;
    const int kbeg = split * P.k_per_split;
    const int kend = min(P.K, kbeg + P.k_per_split);
    const int nchunks = kend > kbeg ? (kend - kbeg + BKC - 1) / BKC : 0;
    // staging role: operand (A for tid < 128), column quad q (4 columns), row quad h4 (4 rows of the chunk).
    // The thread's columns are fixed, so its operand segment is resolved once here (no per-load segment
    // search through the kernel arguments).
    const bool isA = tid < 128;
    const int st = tid & 127, q = st & 15, h4 = st >> 4;
    const int col = (isA ? m0 : n0) + 4 * q;
    const int lim = isA ? P.M : P.N;
    const Seg sg = [&] {
        const Src &S = isA ? P.A : P.B;
        int k = 0;
        if (S.nseg > 1 && col >= S.s[1].kp0) k = 1;
        if (S.nseg > 2 && col >= S.s[2].kp0) k = 2;
        return S.s[k];
    }();
    const int kk = col - sg.kp0;
    const bool live = col < lim && kk < sg.K && sg.kind != SEG_ONES;  // (ones columns are the bias, never tiles)
    const bool bias = isA && nt == 0 && P.bias_col >= 0;
    const bool bias_ext = BEXT && bias;
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};
    // LDS byte offsets of this thread's 8-byte pieces (rows 4 h4 + s, columns 4q .. 4q+3) in plane 0
    int dst[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) dst[r] = (isA ? 0 : NPL * PL) + tn_unit(4 * h4 + r, q);
    // branch-free loads: every lane loads (rows past kend clamped to the last row, dead columns from a valid
    // dummy address) and the values are masked when staged, so the loads pipeline ahead of the MFMAs
    const float *abase = live ? sg.src + kk : P.A.s[0].src;
    const int ald = live ? sg.ld : 0;
    const float *bbase = bias_ext && col < lim ? P.bias_src + col : P.A.s[0].src;
    const int bld = bias_ext && col < lim ? P.bias_ld : 0;
    const int rlast = kend - 1;
    const bool base = live;

    struct Regs { float4 v[4], bz[4]; };
    auto load_chunk = [&](Regs &R, int kc) {
        const int r0 = kbeg + kc * BKC + 4 * h4;
#pragma unroll
        for (int s = 0; s < 4; ++s) R.v[s] = ld4(abase + (size_t)min(r0 + s, rlast) * ald);
        if constexpr (BEXT)
#pragma unroll
            for (int s = 0; s < 4; ++s) R.bz[s] = ld4(bbase + (size_t)min(r0 + s, rlast) * bld);
    };
    // rows past kend and dead columns -> 0 (after the loads have landed)
    auto mask_rows = [&](Regs &R, int kc) {
        const int r0 = kbeg + kc * BKC + 4 * h4;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const bool ok = r0 + s < kend;
            if (!(ok && live)) R.v[s] = f4zero();
            if constexpr (BEXT)
                if (!(ok && bld)) R.bz[s] = f4zero();
        }
    };
    // SEG_ACT operands: M = dropout(act(Z)) applied here, when the loads have landed
    auto act_rows = [&](Regs &R, int kc) {
        if constexpr (SACT >= 0) {
            if (sg.kind != SEG_ACT || !base) return;
            const int r0 = kbeg + kc * BKC + 4 * h4;
            const float sl = SACT == ACT_PRELU ? sg.slope[0] : 0.f;
            (void)base;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                float *v = reinterpret_cast<float *>(&R.v[s]);
#pragma unroll
                for (int c = 0; c < 4; ++c) v[c] = act_fwd(SACT, v[c], sl);
                if (sg.p_drop > 0.f)
#pragma unroll
                    for (int c = 0; c < 4; ++c) v[c] *= dropout_scale(sg.seed, sg.layer, r0 + s, kk + c, sg.p_drop);
            }
        }
    };
    float csc[4] = {1.f, 1.f, 1.f, 1.f};  // H2: this thread's column scales
    auto store_chunk = [&](Regs &R, int kc, uint8_t *stg) {
        mask_rows(R, kc);
        act_rows(R, kc);
        // row s of the 4x4 block: columns 4q .. 4q+3 -> packed pairs per plane
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (H2) {
                uint32_t h0, l0, h1, l1;
                split_h2(R.v[r].x, R.v[r].y, csc[0], csc[1], h0, l0);
                split_h2(R.v[r].z, R.v[r].w, csc[2], csc[3], h1, l1);
                *reinterpret_cast<uint2 *>(stg + dst[r]) = make_uint2(h0, h1);
                *reinterpret_cast<uint2 *>(stg + dst[r] + PL) = make_uint2(l0, l1);
            } else {
                uint32_t h0, md0, l0, h1, md1, l1;
                split_pair(R.v[r].x, R.v[r].y, h0, md0, l0);
                split_pair(R.v[r].z, R.v[r].w, h1, md1, l1);
                *reinterpret_cast<uint2 *>(stg + dst[r]) = make_uint2(h0, h1);
                *reinterpret_cast<uint2 *>(stg + dst[r] + PL) = make_uint2(md0, md1);
                *reinterpret_cast<uint2 *>(stg + dst[r] + 2 * PL) = make_uint2(l0, l1);
            }
        }
        if (bias) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const float4 v = BEXT ? R.bz[s] : R.v[s];
                bsum[0] += v.x; bsum[1] += v.y; bsum[2] += v.z; bsum[3] += v.w;
            }
        }
    };
    floatx4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const uint8_t *stg) {
        bf16x8 af[2][NPL], bfr[2][NPL];
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
#pragma unroll
            for (int a = 0; a < 2; ++a) af[a][p] = tn_frag(stg + p * PL, wi * 32 + a * 16, lane);
#pragma unroll
            for (int b = 0; b < 2; ++b) bfr[b][p] = tn_frag(stg + NPL * PL + p * PL, wj * 32 + b * 16, lane);
        }
        if constexpr (H2) {  // hh, hl, lh on fp16 (the same bits read as f16x8)
            constexpr int PA[3] = {0, 0, 1}, PB[3] = {0, 1, 0};
#pragma unroll
            for (int t = 0; t < 3; ++t)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, af[a][PA[t]]),
                                                                           __builtin_bit_cast(f16x8, bfr[b][PB[t]]),
                                                                           acc[a][b], 0, 0, 0);
        } else {
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
    if constexpr (H2) {
        if (P.a_words) {
            // the split's rows' words: one scale per operand (error per product <= 2^-22 of the split maxima,
            // values below 2^-18 of them keep an absolute error <= 2^-39 of the maxima: planes.hpp)
            const int ke = max(kend, kbeg + 1);
            const int wa0 = (kbeg * P.a_cv) >> 8, wa1 = (ke * P.a_cv - 1) >> 8;
            const int rb0 = kbeg / P.b_bm, rb1 = (ke - 1) / P.b_bm;
            const uint32_t ma = max_words(P.a_words + wa0, wa1 - wa0 + 1);
            const uint32_t mb = max_words(P.b_words + rb0 * P.b_tn, (rb1 - rb0 + 1) * P.b_tn);
            const float s = h2_scale(isA ? ma : mb);
#pragma unroll
            for (int c = 0; c < 4; ++c) csc[c] = s;
            if (tid < 128) inv_scale[tid] = h2_inv_scale(tid < 64 ? ma : mb);
            __syncthreads();
        } else {
            // max pass: |value| per column over the split's rows (as staged: masked, activated), two chunks of
            // loads in flight; then per column over the 8 row groups through LDS -> scale and inverse scale
            uint32_t cm[4] = {0u, 0u, 0u, 0u};
            auto maxv = [&](Regs &R, int kc) {
                mask_rows(R, kc);
                act_rows(R, kc);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    cm[0] = max(cm[0], absbits(R.v[r].x)); cm[1] = max(cm[1], absbits(R.v[r].y));
                    cm[2] = max(cm[2], absbits(R.v[r].z)); cm[3] = max(cm[3], absbits(R.v[r].w));
                }
            };
            auto load_v = [&](Regs &R, int kc) {
                const int r0 = kbeg + kc * BKC + 4 * h4;
#pragma unroll
                for (int s = 0; s < 4; ++s) R.v[s] = ld4(abase + (size_t)min(r0 + s, rlast) * ald);
            };
#ifndef WD_TN_NOMAX
            if (nchunks > 0) {
#else
            if (false) {
#endif
                Regs M0, M1;
                load_v(M0, 0);
                load_v(M1, min(1, nchunks - 1));
                int kc = 0;
                for (; kc + 1 < nchunks; kc += 2) {
                    maxv(M0, kc);
                    load_v(M0, min(kc + 2, nchunks - 1));
                    maxv(M1, kc + 1);
                    load_v(M1, min(kc + 3, nchunks - 1));
                }
                if (kc < nchunks) maxv(M0, kc);
            }
            uint32_t *cw = reinterpret_cast<uint32_t *>(lds);  // [2 operands][8 row groups][64 columns]
#pragma unroll
            for (int c = 0; c < 4; ++c) cw[(isA ? 0 : 512) + h4 * 64 + 4 * q + c] = cm[c];
            __syncthreads();
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                uint32_t m = 0;
#pragma unroll
                for (int h = 0; h < 8; ++h) m = max(m, cw[(isA ? 0 : 512) + h * 64 + 4 * q + c]);
                csc[c] = h2_scale(m);
                if (h4 == 0) inv_scale[(isA ? 0 : 64) + 4 * q + c] = h2_inv_scale(m);
            }
            __syncthreads();  // (the words are overwritten by the first chunk's staging)
        }
    }
    if (nchunks > 0) {
        // TN_DEPTH chunks in flight in registers: at step kc chunk kc is in LDS, kc+1 .. kc+D-1 are loading
        // (or landed) in the ring, and kc+D is issued into the set chunk kc left
        constexpr int D = TN_DEPTH;
        Regs R[D];
#pragma unroll
        for (int i = 0; i < D; ++i) load_chunk(R[i], min(i, nchunks - 1));
        store_chunk(R[0], 0, lds);
        __syncthreads();
        auto step = [&](int kc, Regs &Rnext, Regs &Rfree) {
            if (WD_STAMP_GEMM == 2 && BEXT && wave == 0) wd_lstamp(kc, 0);
            // unconditional (the last chunk is reloaded past the end): a skipped load on some path made
            // the compiler's waits for the older chunk drain the fresh prefetch too
            load_chunk(Rfree, min(kc + D, nchunks - 1));
            __builtin_amdgcn_sched_barrier(0);
            compute(lds + (kc & 1) * STAGE);
            if (WD_STAMP_GEMM == 2 && BEXT && wave == 0) wd_lstamp(kc, 1);
            if (kc + 1 < nchunks) store_chunk(Rnext, kc + 1, lds + ((kc + 1) & 1) * STAGE);
            if (WD_STAMP_GEMM == 2 && BEXT && wave == 0) wd_lstamp(kc, 2);
            __syncthreads();
            if (WD_STAMP_GEMM == 2 && BEXT && wave == 0) wd_lstamp(kc, 3);
        };
        int kc = 0;
        for (; kc + D - 1 < nchunks; kc += D) {
#pragma unroll
            for (int i = 0; i < D; ++i) step(kc + i, R[(i + 1) % D], R[i]);
        }
#pragma unroll
        for (int i = 0; i < D - 1; ++i)
            if (kc + i < nchunks) step(kc + i, R[(i + 1) % D], R[i]);
    }
    // epilogue: C tile through LDS, coalesced float4 stores into this split's slab (accumulating over
    // the layers of W_h when asked); the bias sums through LDS in row-group order
    float *cl = reinterpret_cast<float *>(lds);
    constexpr int LDC = BN + 4;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = wi * 32 + a * 16 + 4 * g + r, j = wj * 32 + b * 16 + i16;
                cl[i * LDC + j] = H2 ? acc[a][b][r] * inv_scale[i] * inv_scale[64 + j] : acc[a][b][r];
            }
    float *bl = cl + BM * LDC;  // [8 row groups][64 columns]
    if (bias) {
#pragma unroll
        for (int c = 0; c < 4; ++c) bl[h4 * 64 + 4 * q + c] = bsum[c];
    }
    __syncthreads();
    float *Y = P.slab + (size_t)split * P.slab_stride;
    Epi E{};
    E.kind = EPI_STORE; E.Y = Y; E.ld = P.ld_slab; E.accumulate = P.accumulate;
    EpiPrefetch<BM, BN, NT> ep;
    ep.load(E, m0, n0, P.M, P.N);
    epilogue_v4<BM, BN, NT>(E, cl, LDC, m0, n0, P.M, P.N, ep);
    if (nt == 0 && P.bias_col >= 0 && tid < BM && m0 + tid < P.M) {
        float s = 0.f;
#pragma unroll
        for (int h = 0; h < 8; ++h) s += bl[h * 64 + tid];
        float *d = Y + (size_t)(m0 + tid) * P.ld_slab + P.bias_col;
        *d = P.accumulate ? *d + s : s;
    }
}

// ---------------------------------------------------------------------------------------------
// Split-plane GEMM core on LDS-DMA staged plane tiles (cdna_hip_programming.md §5 "Async
// global->LDS copy"): no staging registers, no arithmetic in the staging path, two LDS stages (one
// chunk in flight behind the one being multiplied), raw s_barrier (a __syncthreads would drain the DMA
// queue).  One wave-instruction fills 1 KB of LDS lane-linearly (16 rows x 64 B of one plane); the
// bank swizzle goes on the per-lane global source address (unit s of row r reads unit
// s ^ ((r >> 1) & 3)).
//
// A K-chunk is 32 columns.  A operand: up to two segments, each a plane-tile matrix with BM-row
// blocks (BR = BM, planes.hpp), so chunk kc of row block rb is ONE contiguous 3 x BM x 64-byte block.
// B operand: plane tiles with 64-row blocks (one 12 KB block per chunk of the column tile).
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void glds16(const void *g, uint8_t *lds_wave_base) {
    __builtin_amdgcn_global_load_lds(g, (lds_void_t *)lds_wave_base, 16, 0, 0);
}

// The same copy issued from inline asm: the compiler does not see it, so it inserts no vmcnt wait for it
// in front of LDS reads of the other stage (for the builtin it waited at every chunk's first fragment
// read, exposing the copy's latency); the caller's explicit vmcnt wait + barrier protocol orders it.  It
// writes no register, so nothing the compiler moves can be overwritten late.  (M0 = the wave's LDS base,
// saved and restored around the copy.)
__device__ __forceinline__ void glds16_untracked(const void *g, uint8_t *lds_wave_base) {
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t *)lds_wave_base);
    uint32_t saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved) : "s"(l), "v"(g) : "memory");
}

struct X6Operands {
    const uint8_t *a0; int nkc0, kc0;   // A segment 0: base of the matrix, its 32-column chunks per row block,
                                        // chunks used (K extent / 32)
    const uint8_t *a1; int nkc1, kc1;   // A segment 1 (kc1 = 0: absent; a1 must still be a valid pointer)
    int rb;                             // A row block (BM rows)
    int a_rows;                         // rows of the block that hold data (<= BM): 16-row groups past it
                                        // are not loaded (their accumulator rows are garbage, never read)
    const uint8_t *b;                   // B: this column tile's first chunk block (3 x BN x 64 B per chunk)
};

template <int BM, int BN>
constexpr int x6_stage_bytes() { return 3 * BM * 64 + 3 * BN * 64; }

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the counter field is an immediate)
__device__ __forceinline__ void wait_vmcnt(int n) {
    switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// acc[TM][TN] (+)= A(rb rows) · B(col tile)ᵀ for a BM x BN tile (BN = 64 or 80), waves WM x WN, wave
// tile (BM / WM) x (BN / WN), S LDS stages (S - 1 chunks in flight behind the one multiplied) of CPS
// chunks each.  Uses lds[0 .. S * CPS * x6_stage_bytes<BM, BN>()); on return every DMA has landed and
// all waves are past their last LDS read (the caller may reuse the LDS after one __syncthreads()).
struct NoHook { __device__ void operator()(int) const {} };

// f(std::integral_constant<int, i>) for i = 0 .. N - 1
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

// f(std::integral_constant<int, n>) for a wave-uniform runtime n in [0, N]
template <int N, typename F>
__device__ __forceinline__ void dispatch_upto(int n, F &&f) {
    if constexpr (N == 0) {
        f(std::integral_constant<int, 0>{});
    } else {
        if (n >= N) f(std::integral_constant<int, N>{});
        else dispatch_upto<N - 1>(n, f);
    }
}

// hook(0): called once, right after the DMA of the second chunk is issued (register prefetches placed
// there land behind the first chunk's MFMAs instead of delaying the first chunk's wait); hook(1): once
// more one chunk later (or right after hook(0) with a single chunk), when hook(0)'s loads have landed --
// for loads whose addresses depend on them

// BPIPE: B fragments one column tile at a time, the next one in flight (two sets of 3 registers x 4
// instead of TN sets): fewer VGPRs for kernels that must co-reside two per CU
template <int BM, int BN, int WM, int WN, int S = 2, int CPS = 1, bool BPIPE = false, typename Hook = NoHook>
__device__ __forceinline__ void x6_mainloop(const X6Operands &O, uint8_t *lds,
                                            floatx4 (&acc)[BM / WM / 16][BN / WN / 16], const Hook &hook = Hook()) {
    constexpr int NW = WM * WN, TM = BM / WM / 16, TN = BN / WN / 16;
    constexpr int APL = BM * 64, BPL = BN * 64, STAGE = x6_stage_bytes<BM, BN>();
    constexpr int AP = 3 * BM / 16, BP = 3 * BN / 16;                 // 1 KB pieces per chunk
    constexpr int APW = (AP + NW - 1) / NW, BPW = (BP + NW - 1) / NW;  // per wave (the last ones predicated)
    static_assert(BM % (16 * WM) == 0 && BN % (16 * WN) == 0, "wave tiles of 16x16 MFMAs");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wi = wave / WN, wj = wave % WN, g = lane >> 4, i16 = lane & 15;

    // piece c of wave w = c * NW + w (interleaved, so that uneven counts fall on the last pieces);
    // lane l -> image unit q = 64 c + l = (plane, row, slot) -> source byte in the chunk block
    int asrc[APW], bsrc[BPW];
#pragma unroll
    for (int j = 0; j < APW; ++j) {
        const int q = 64 * (j * NW + wave) + lane, p = (q / (BM * 4)) % 3, r = (q >> 2) % BM, sl = q & 3;
        asrc[j] = p * APL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
    }
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
        const int q = 64 * (j * NW + wave) + lane, p = (q / (BN * 4)) % 3, r = (q >> 2) % BN, sl = q & 3;
        bsrc[j] = p * BPL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
    }
    const int nchunks = O.kc0 + O.kc1;
    auto issue = [&](int kc, int stage) {
        const bool s1 = kc >= O.kc0;
        const uint8_t *abase = s1 ? O.a1 : O.a0;
        const size_t aoff = ((size_t)O.rb * (s1 ? O.nkc1 : O.nkc0) + (s1 ? kc - O.kc0 : kc)) * (3 * APL);
        const uint8_t *ablk = abase + aoff;
        const uint8_t *bblk = O.b + (size_t)kc * (3 * BPL);
        uint8_t *st = lds + stage * STAGE;
#pragma unroll
        for (int j = 0; j < APW; ++j) {
            const int c = j * NW + wave;  // piece = (plane c / (BM / 16), 16-row group c % (BM / 16))
            if ((AP % NW == 0 || c < AP) && 16 * (c % (BM / 16)) < O.a_rows) glds16(ablk + asrc[j], st + 1024 * c);
        }
#pragma unroll
        for (int j = 0; j < BPW; ++j)
            if (BP % NW == 0 || j * NW + wave < BP) glds16(bblk + bsrc[j], st + 3 * APL + 1024 * (j * NW + wave));
    };
    int ao[TM], bo[TN];
#pragma unroll
    for (int a = 0; a < TM; ++a) ao[a] = x6_slot(wi * (BM / WM) + a * 16 + i16, g);
#pragma unroll
    for (int b = 0; b < TN; ++b) bo[b] = 3 * APL + x6_slot(wj * (BN / WN) + b * 16 + i16, g);
    // only this wave's 16-row A tiles that hold block rows (< a_rows) are read and multiplied: a
    // molecule block is ~3/4 full, and the skipped accumulators stay zero
    const int na = min(TM, max(0, (O.a_rows - wi * (BM / WM) + 15) >> 4));
    auto compute_n = [&](const uint8_t *st, auto na_c) {
        constexpr int NA = decltype(na_c)::value;
        // plane products hh, hm, mh, hl, lh, mm
        constexpr int PA[6] = {0, 0, 1, 0, 2, 1}, PB[6] = {0, 1, 0, 2, 0, 1};
        if constexpr (BPIPE) {
            bf16x8 af[TM][3], bq[2][3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int a = 0; a < NA; ++a) af[a][p] = *reinterpret_cast<const bf16x8 *>(st + p * APL + ao[a]);
                bq[0][p] = *reinterpret_cast<const bf16x8 *>(st + p * BPL + bo[0]);
            }
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                if (b + 1 < TN)
#pragma unroll
                    for (int p = 0; p < 3; ++p) bq[(b + 1) & 1][p] = *reinterpret_cast<const bf16x8 *>(st + p * BPL + bo[b + 1]);
#pragma unroll
                for (int t = 0; t < 6; ++t)
#pragma unroll
                    for (int a = 0; a < NA; ++a)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][PA[t]], bq[b & 1][PB[t]], acc[a][b], 0, 0, 0);
            }
            return;
        }
        bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int a = 0; a < NA; ++a) af[a][p] = *reinterpret_cast<const bf16x8 *>(st + p * APL + ao[a]);
#pragma unroll
            for (int b = 0; b < TN; ++b) bfr[b][p] = *reinterpret_cast<const bf16x8 *>(st + p * BPL + bo[b]);
        }
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a][PA[t]], bfr[b][PB[t]], acc[a][b], 0, 0, 0);
    };
    auto compute = [&](const uint8_t *st) { dispatch_upto<TM>(na, [&](auto c) { compute_n(st, c); }); };
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    // this wave's DMA instructions per chunk (the same for every chunk)
    int mine = 0;
#pragma unroll
    for (int j = 0; j < APW; ++j) {
        const int c = j * NW + wave;
        mine += (AP % NW == 0 || c < AP) && 16 * (c % (BM / 16)) < O.a_rows;
    }
#pragma unroll
    for (int j = 0; j < BPW; ++j) mine += BP % NW == 0 || j * NW + wave < BP;
    if constexpr (CPS > 1) {
        // CPS chunks per stage (two stages): one barrier per CPS chunks; stage s holds the chunk images
        // of super-chunk s back to back
        static_assert(S == 2, "multi-chunk stages use two stages");
        const int nsc = (nchunks + CPS - 1) / CPS;
        auto issue_sc = [&](int sc, int stage) {
#pragma unroll
            for (int q = 0; q < CPS; ++q)
                if (sc * CPS + q < nchunks) issue(sc * CPS + q, stage * CPS + q);
        };
        issue_sc(0, 0);
        for (int sc = 0; sc < nsc; ++sc) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (sc + 1 < nsc) issue_sc(sc + 1, (sc + 1) & 1);
            if (sc == 0) hook(0);
            if (sc == 1 || (sc == 0 && nsc == 1)) hook(1);
#pragma unroll
            for (int q = 0; q < CPS; ++q)
                if (sc * CPS + q < nchunks) compute(lds + ((sc & 1) * CPS + q) * STAGE);
        }
    } else {
#pragma unroll
        for (int c = 0; c < S - 1; ++c)
            if (c < nchunks) issue(c, c);
        for (int kc = 0; kc < nchunks; ++kc) {
            // chunk kc landed for this wave (younger chunks kc+1 .. kc+S-2 may stay in flight), then for
            // every wave; every wave is done reading stage (kc + S - 1) % S (= the one read at kc - 1)
            if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else wait_vmcnt(min(S - 2, nchunks - 1 - kc) * mine);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            // S > 2: the hook's loads go out before the DMA of chunk S - 1, so that the partial
            // vmcnt waits above (which count only DMA instructions) find them among the older ones
            if constexpr (S > 2) {
                if (kc == 0) hook(0);
                if (kc == 1 || (kc == 0 && nchunks == 1)) hook(1);
            }
            if (kc + S - 1 < nchunks) issue(kc + S - 1, (kc + S - 1) % S);
            if constexpr (S == 2) {
                if (kc == 0) hook(0);
                if (kc == 1 || (kc == 0 && nchunks == 1)) hook(1);
            }
            compute(lds + (kc % S) * STAGE);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Warp-specialised fp16-pair GEMM core (the message-passing layer, planes.hpp "h2"): acc (+)= A · Bᵀ
// for a BM x BN tile on 512 threads, two LDS stages of one 32-column chunk, one s_barrier per chunk:
//   waves 0-3 (consumers, one per SIMD) multiply: wave w owns rows 32 w .. 32 w + 31 and all BN
//             columns (2 x BN/16 accumulators), so every B fragment read from LDS feeds two row tiles;
//             three v_mfma_f32_16x16x32_f16 per tile and chunk (hi hi, hi lo, lo hi); before chunk kc's
//             MFMAs they issue the LDS-DMA of chunk kc + 1's B (h2 plane tiles, no registers);
//   waves 4-7 (producers, the consumers' SIMD partners) stage A through registers (AProd: fp32 rows,
//             loads, activation, dropout, scale, fp16 hi / lo split, ds_write), SETS chunks ahead: chunk c
//             lives in register set c % SETS from its loads (issued while chunk c - SETS is multiplied) to
//             its LDS write (while chunk c - 1 is multiplied).
// The two roles run separate loops with the same barrier count, so the register allocator can give the
// producer's staging sets the registers that hold the consumer's accumulators (a shared loop keeps both
// live at once; aliasing them by hand made the compiler wait for the producer's loads inside the
// consumer's MFMAs).
// AProd interface (producer thread t = threadIdx.x & 255): SETS (register sets: chunks in flight); load(set,
// kc) issues chunk kc's loads into register set `set`; init() once the first loads are out (the scale);
// store(set, kc, stage) writes the stage's A image (2 x BM x 64 B: hi plane, lo plane, x6_slot layout).
// On return every wave is past its last LDS access of the stages; the consumers' acc holds the tile
// (the producers' acc is left undefined: the caller reads it in threads 0..255 only).
// ---------------------------------------------------------------------------------------------
// The B (W_h) copies run H2_B_AHEAD chunks ahead of the chunk multiplied (H2_B_AHEAD + 1 B stages); the
// producers store A H2_A_STAGES - 1 chunks ahead (H2_A_STAGES A stages).  (Measured, same box: three A
// stages +1.3 us per launch, B two chunks ahead +0.4 us, all of a chunk's fragments read before its first
// MFMA +0.4 us, 3 / 4 / 6 register sets in flight 16.6 / 17.5 / 22.4 us: tools/prof_libs.sh variants.)
#ifndef WD_H2_B_AHEAD
#define WD_H2_B_AHEAD 1
#endif
constexpr int H2_B_AHEAD = WD_H2_B_AHEAD, H2_A_STAGES = 2;
template <int BM, int BN>
constexpr int h2_lds_bytes() { return H2_A_STAGES * (2 * BM * 64) + (H2_B_AHEAD + 1) * (2 * BN * 64); }

// (Measured, round 6: the K chunks multiplied in an order rotated per molecule block, so that the blocks of an
// XCD do not all read the same W_h chunk at once: 15.9 / 15.5 vs 15.6 / 15.1 us, same box -- no gain.)
template <int BM, int BN, typename AProd>
__device__ __forceinline__ void h2_mainloop_ws(const uint8_t *bsrc_base, int nchunks, int a_rows, uint8_t *lds,
                                               floatx4 (&acc)[BM / 64][BN / 16], AProd &ap) {
    static_assert(BM == 128, "four consumer waves of 32 rows");
    constexpr int TM = BM / 64, TN = BN / 16;
    constexpr int APL = BM * 64, BPL = BN * 64;
    constexpr int ASTAGE = 2 * APL, BSTAGE = 2 * BPL, NA = H2_A_STAGES, NB = H2_B_AHEAD + 1;  // A stages [NA], B [NB]
    constexpr int BP = 2 * BN / 16, BPW = (BP + 3) / 4;  // B: 1 KB DMA pieces per chunk, per consumer wave
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int w4 = wave & 3, g = lane >> 4, i16 = lane & 15;

    if (wave >= 4) {  // ---- producers: chunk c in register set c % NS, loaded NS chunks ahead of its store
        // (compiler-visible loads, issued unconditionally -- past the last chunk they reload it -- so that the
        // compiler's own vmcnt waits before each store are exact: all but the NS - 1 younger sets)
        constexpr int NS = AProd::SETS;
        static_assert(NA - 1 <= NS, "the stages filled ahead come from distinct register sets");
        static_for<NS>([&](auto i) { ap.load(i, min((int)decltype(i)::value, nchunks - 1)); });
        ap.init();  // (after the first loads are out: the scale's words are not on the rows' critical path)
        static_for<NA - 1>([&](auto c) {  // chunks 0 .. NA - 2 before the first barrier
            constexpr int C = decltype(c)::value;
            ap.store(c, C, lds + C * ASTAGE);
            ap.load(c, min(C + NS, nchunks - 1));
        });
        auto produce = [&](int kc, auto set) {  // set = (kc + NA - 1) % NS holds chunk kc + NA - 1
            const int cs = kc + NA - 1;
            if (cs >= nchunks) return;
            if (WD_STAMPS && wave == 4) wd_lstamp(kc, 4);
            ap.store(set, cs, lds + (cs % NA) * ASTAGE);
            if (WD_STAMPS && wave == 4) { __builtin_amdgcn_s_waitcnt(0xc07f); wd_lstamp(kc, 5); }
            ap.load(set, min(cs + NS, nchunks - 1));
        };
        int kc = 0;
        for (; kc + NS <= nchunks; kc += NS)
            static_for<NS>([&](auto j) {
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's stage writes done
                __builtin_amdgcn_s_barrier();
                produce(kc + decltype(j)::value, std::integral_constant<int, (decltype(j)::value + NA - 1) % NS>{});
            });
        static_for<NS>([&](auto j) {
            if (kc + decltype(j)::value < nchunks) {
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_s_barrier();
                produce(kc + decltype(j)::value, std::integral_constant<int, (decltype(j)::value + NA - 1) % NS>{});
            }
        });
        __builtin_amdgcn_s_waitcnt(0xc07f);
        return;
    }
    // ---- consumers: B piece c = 4 j + w4 of the chunk block; lane l -> image unit q = 64 c + l, whose
    // source carries the bank swizzle (the DMA writes LDS lane-linearly)
    int bsrc[BPW];
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
        const int q = 64 * (4 * j + w4) + lane, p = (q / (BN * 4)) % 2, r = (q >> 2) % BN, sl = q & 3;
        bsrc[j] = p * BPL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
    }
    auto issue_b = [&](int kc) {
        const uint8_t *bblk = bsrc_base + (size_t)kc * (2 * BPL);
        uint8_t *st = lds + NA * ASTAGE + (kc % NB) * BSTAGE;
#pragma unroll
        for (int j = 0; j < BPW; ++j)
            if (BP % 4 == 0 || 4 * j + w4 < BP) glds16_untracked(bblk + bsrc[j], st + 1024 * (4 * j + w4));
    };
    int ao[TM], bo[TN];
#pragma unroll
    for (int a = 0; a < TM; ++a) ao[a] = x6_slot(32 * w4 + 16 * a + i16, g);
#pragma unroll
    for (int b = 0; b < TN; ++b) bo[b] = x6_slot(16 * b + i16, g);
    const int na = min(TM, max(0, (a_rows - 32 * w4 + 15) >> 4));
    auto compute_n = [&](const uint8_t *st, const uint8_t *sb, auto na_c) {
        constexpr int NA = decltype(na_c)::value;
        f16x8 af[TM][2], bq[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
            for (int a = 0; a < NA; ++a) af[a][p] = *reinterpret_cast<const f16x8 *>(st + p * APL + ao[a]);
            bq[0][p] = *reinterpret_cast<const f16x8 *>(sb + p * BPL + bo[0]);
        }
        // column tile b: hi hi, the next tile's fragment reads, hi lo and lo hi -- pinned in that order (left
        // to itself the scheduler issued each tile's reads just before their use, and its LDS wait then also
        // covered the reads issued after them)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
#pragma unroll
            for (int a = 0; a < NA; ++a)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[b & 1][0], acc[a][b], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (b + 1 < TN)
#pragma unroll
                for (int p = 0; p < 2; ++p) bq[(b + 1) & 1][p] = *reinterpret_cast<const f16x8 *>(sb + p * BPL + bo[b + 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[b & 1][1], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][1], bq[b & 1][0], acc[a][b], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    // this wave's copies per chunk (uniform)
    int mine = 0;
#pragma unroll
    for (int j = 0; j < BPW; ++j) mine += BP % 4 == 0 || 4 * j + w4 < BP;
#pragma unroll
    for (int c = 0; c < H2_B_AHEAD; ++c)
        if (c < nchunks) issue_b(c);
    for (int kc = 0; kc < nchunks; ++kc) {
        // chunk kc's B landed for this wave (the H2_B_AHEAD - 1 younger chunks may stay in flight), this
        // wave's fragment reads done; then for every wave: A chunk kc staged, B stage (kc + H2_B_AHEAD) % NB
        // read by all (at kc - 1)
        if (WD_STAMPS && wave == 0) wd_lstamp(kc, 0);
        wait_vmcnt(min(H2_B_AHEAD - 1, nchunks - 1 - kc) * mine);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (WD_STAMPS && wave == 0) wd_lstamp(kc, 1);
        __builtin_amdgcn_s_barrier();
        if (WD_STAMPS && wave == 0) wd_lstamp(kc, 2);
        if (kc + H2_B_AHEAD < nchunks) issue_b(kc + H2_B_AHEAD);
        const uint8_t *st = lds + (kc % NA) * ASTAGE, *sb = lds + NA * ASTAGE + (kc % NB) * BSTAGE;
        dispatch_upto<TM>(na, [&](auto c) { compute_n(st, sb, c); });
        if (WD_STAMPS && wave == 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            wd_lstamp(kc, 3);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0070);
}

// ---------------------------------------------------------------------------------------------
// DMA-fed fp16-pair GEMM core (round 6): acc (+)= A · Bᵀ for a BM x BN tile on 512 threads where BOTH
// operands are pre-split fp16 hi / lo pair tiles in HBM -- A = the block's M_{t-1}, written as pairs by
// its producer (the embed, or the previous layer's epilogue) with a power-of-two scale per group of G
// columns (the producer's column tile), B = W_h (wdmpnn_pack_params).  No register staging: waves 4-7
// ("loaders") copy A and B by LDS-DMA NS - 1 chunks ahead into a ring of H2P_STAGES stages, waves 0-3
// (MFMA "consumers", one per SIMD, BM / 4 rows x BN columns each) multiply; one s_barrier per chunk.  The
// two roles run separate loops with the same barrier count, and the consumers' loop is instantiated per
// count of live 16-row tiles: no control flow inside a consumer's chunk, so its accumulators stay in
// place and its MFMAs run on across the barrier into the next chunk (a loop shared by both roles, with
// per-chunk scale steps, made the register allocator copy all 40 accumulators after every chunk -- each
// copy waiting for its MFMA -- 2,200 against 1,200 cycles per chunk, tools/ring_probe.hip).
//
// Scales.  The A groups carry different scales s_g = 2^(se_g - 127) (se = h2_sexp of the group's word).
// Every chunk is multiplied at ONE scale, the block's largest-magnitude group (smallest se, `cur`): each
// lane multiplies its A fragments by 2^-(se_g - cur) in fp16 (v_pk_mul_f16; lanes 32-63 hold k 16..31 of
// a v_mfma_f32_16x16x32_f16 operand, lanes 0-31 k 0..15, so the two 16-column halves of a chunk that
// straddles two producer tiles take their own factors; zero past a difference of 24), rounding at 2^-24
// of the shared scaled unit: the precision of one scale per block, as the register-staged layer's.  An
// all-zero group (word 0) multiplies zeros.  The accumulator's exponent comes back in se_out (-1: no group
// had data; acc is zero).
// Words: lane l of every consumer wave holds word l of the block (nw <= 64, lane_word), group of column
// c = c / G; nchunks <= 64.
// ---------------------------------------------------------------------------------------------
// (2 chunks in flight + the one multiplied; WD_H2P_STAGES 4: 104 KB of LDS, one layer workgroup per CU, measured)
#ifndef WD_H2P_STAGES
#define WD_H2P_STAGES 3
#endif
constexpr int H2P_STAGES = WD_H2P_STAGES;
template <int BM, int BN>
constexpr int h2p_stage_bytes() { return 2 * BM * 64 + 2 * BN * 64; }
template <int BM, int BN>
constexpr int h2p_lds_bytes() { return H2P_STAGES * h2p_stage_bytes<BM, BN>(); }

// FRAG (fragment schedule; tools/ring_probe.hip measures the variants): 0: each column tile's next B
// fragments read after its first MFMAs; 1: read before them; 2: every B fragment of the chunk read before
// the first MFMA
#ifndef WD_H2P_FRAG
#define WD_H2P_FRAG 0
#endif
template <int BM, int BN, int FRAG = WD_H2P_FRAG>
__device__ __forceinline__ void h2_mainloop_pairs(const uint8_t *a_src, const uint8_t *b_src, int nchunks, int a_rows,
                                                  uint32_t wv, int G, uint8_t *lds, floatx4 (&acc)[BM / 64][BN / 16],
                                                  int &se_out) {
    // (acc[BM / 64]: a consumer wave's BM / 4 rows as 16-row tiles; the layout x6_acc_to_lds<BM, BN, 4, 1> reads)
    static_assert(BM == 128 || BM == 64, "four consumer waves of BM / 4 rows");
    constexpr int RW = BM / 4, TM = RW / 16, TN = BN / 16;  // rows per consumer wave, its 16-row tiles
    constexpr int APL = BM * 64, BPL = BN * 64, STAGE = h2p_stage_bytes<BM, BN>(), NS = H2P_STAGES;
    constexpr int AP = 2 * BM / 16, APW = AP / 4;        // A: 16 pieces of 1 KB per chunk, 4 per loader wave
    constexpr int BP = 2 * BN / 16, BPW = (BP + 3) / 4;  // B: 10 pieces, <= 3 per loader wave
    static_assert(AP % 4 == 0, "A pieces split evenly over the loader waves");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, w4 = wave & 3, g = lane >> 4, i16 = lane & 15;
    // chunk kc in stage (kc + roff) % NS, so that the LAST chunk lands in stage 0: the caller may use the
    // tail of stage NS - 1 while the consumers multiply that chunk (mp_layer_kernel's epilogue lists)
    const int roff = (NS - (nchunks - 1) % NS) % NS;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (wave >= 4) {  // ---- loaders
        // this wave's pieces: source offsets in a chunk block (the DMA writes LDS lane-linearly, so the bank
        // swizzle of x6_slot is applied on the source side) and whether each is copied
        int src[APW + BPW], dst[APW + BPW];
        bool on[APW + BPW];
        int mine = 0;
#pragma unroll
        for (int j = 0; j < APW; ++j) {
            const int c = 4 * j + w4, q = 64 * c + lane, p = q / (BM * 4), r = (q >> 2) % BM, sl = q & 3;
            src[j] = p * APL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
            dst[j] = 1024 * c;
            on[j] = 16 * (c % (BM / 16)) < a_rows;  // 16-row groups past the block's rows: not copied
            mine += on[j];
        }
#pragma unroll
        for (int j = 0; j < BPW; ++j) {
            const int c = 4 * j + w4, q = 64 * c + lane, p = (q / (BN * 4)) % 2, r = (q >> 2) % BN, sl = q & 3;
            src[APW + j] = p * BPL + r * 64 + 16 * (sl ^ ((r >> 1) & 3));
            dst[APW + j] = 2 * APL + 1024 * c;
            on[APW + j] = BP % 4 == 0 || c < BP;
            mine += on[APW + j];
        }
        mine = __builtin_amdgcn_readfirstlane(mine);  // (wave-uniform: a scalar wait below)
        auto issue = [&](int kc) {
            uint8_t *st = lds + ((kc + roff) % NS) * STAGE;
            const uint8_t *ablk = a_src + (size_t)kc * (2 * APL), *bblk = b_src + (size_t)kc * (2 * BPL);
#pragma unroll
            for (int j = 0; j < APW; ++j)
                if (on[j]) glds16_untracked(ablk + src[j], st + dst[j]);
#pragma unroll
            for (int j = 0; j < BPW; ++j)
                if (on[APW + j]) glds16_untracked(bblk + src[APW + j], st + dst[APW + j]);
        };
#pragma unroll
        for (int c = 0; c < NS - 1; ++c)
            if (c < nchunks) issue(c);
        // the loop instantiated per copy count (its steady-state wait a constant: a wait on a runtime count
        // is a scalar branch search per chunk, ~300 cycles of the chunk period in tools/ring_probe.hip)
        dispatch_upto<APW + BPW>(mine, [&](auto m_c) {
            constexpr int M = decltype(m_c)::value;
            for (int kc = 0; kc < nchunks; ++kc) {
                // chunk kc landed (chunks kc + 1 .. kc + NS - 2 may stay in flight); after the barrier every
                // consumer is done reading stage (kc + NS - 1 + roff) % NS (chunk kc - 1's)
                if (WD_STAMPS && wave == 4) wd_lstamp(kc, 4);
                if (nchunks - 1 - kc >= NS - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * M) : "memory");
                else wait_vmcnt((nchunks - 1 - kc) * M);
                if (WD_STAMPS && wave == 4) wd_lstamp(kc, 5);
                __builtin_amdgcn_s_barrier();
                if (kc + NS - 1 < nchunks) issue(kc + NS - 1);
            }
        });
        __builtin_amdgcn_s_waitcnt(0x0070);  // (vmcnt(0): every copy of this wave landed)
        se_out = -1;
        return;
    }
    // ---- consumers
    int ao[TM], bo[TN];
#pragma unroll
    for (int a = 0; a < TM; ++a) ao[a] = x6_slot(RW * w4 + 16 * a + i16, g);
#pragma unroll
    for (int b = 0; b < TN; ++b) bo[b] = x6_slot(16 * b + i16, g);
    const int na = min(TM, max(0, (a_rows - RW * w4 + 15) >> 4));
    // the scale exponents of chunk `lane`'s two halves (all-zero group: BIG), the shared one (the smallest
    // over the chunks multiplied) and per chunk (lane) the two halves' fp16 factors 2^-(se - cur), packed
    constexpr int BIG = 1 << 20;
    const int k0 = min((32 * lane) / G, 63), k1 = min((32 * lane + 16) / G, 63);
    const uint32_t lw0 = (uint32_t)__shfl((int)wv, k0, 64), lw1 = (uint32_t)__shfl((int)wv, k1, 64);
    const int s0 = lw0 ? h2_sexp(lw0) : BIG, s1 = lw1 ? h2_sexp(lw1) : BIG;
    const int cur = BIG - (int)wave_max_u32((uint32_t)(BIG - (lane < nchunks ? min(s0, s1) : BIG)));
    auto f16code = [&](int se) -> uint32_t {
        const int d = se - cur;
        return d > 24 ? 0u : (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)__builtin_amdgcn_ldexpf(1.0f, -d));
    };
    const uint32_t fcode = f16code(s0) | (f16code(s1) << 16);
    const int fsh = lane < 32 ? 0 : 16;
    auto compute_n = [&](const uint8_t *st, const uint8_t *sb, auto na_c, _Float16 fl) {
        constexpr int NA = decltype(na_c)::value;
        constexpr int SCH = FRAG & 3, NB = SCH == 2 ? TN : 2;
        f16x8 af[TM][2], bq[NB][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                af[a][p] = *reinterpret_cast<const f16x8 *>(st + p * APL + ao[a]);
                af[a][p] = af[a][p] * fl;
            }
#pragma unroll
            for (int b = 0; b < (SCH == 2 ? TN : 1); ++b) bq[b][p] = *reinterpret_cast<const f16x8 *>(sb + p * BPL + bo[b]);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int cb = SCH == 2 ? b : (b & 1);
            if constexpr (SCH == 1) {
                if (b + 1 < TN)
#pragma unroll
                    for (int p = 0; p < 2; ++p) bq[(b + 1) & 1][p] = *reinterpret_cast<const f16x8 *>(sb + p * BPL + bo[b + 1]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int a = 0; a < NA; ++a)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[cb][0], acc[a][b], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (SCH == 0 && b + 1 < TN)
#pragma unroll
                for (int p = 0; p < 2; ++p) bq[(b + 1) & 1][p] = *reinterpret_cast<const f16x8 *>(sb + p * BPL + bo[b + 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][0], bq[cb][1], acc[a][b], 0, 0, 0);
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[a][1], bq[cb][0], acc[a][b], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    dispatch_upto<TM>(na, [&](auto na_c) {
        for (int kc = 0; kc < nchunks; ++kc) {
            // this wave's fragment reads done (the stage of chunk kc - 1 is refilled after the barrier);
            // after it chunk kc is in LDS
            if (WD_STAMPS && wave == 0) wd_lstamp(kc, 0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (WD_STAMPS && wave == 0) wd_lstamp(kc, 1);
            __builtin_amdgcn_s_barrier();
            if (WD_STAMPS && wave == 0) wd_lstamp(kc, 2);
            const uint8_t *st = lds + ((kc + roff) % NS) * STAGE, *sb = st + 2 * APL;
            const uint32_t fc = __builtin_amdgcn_readlane(fcode, kc);
            const _Float16 fl = __builtin_bit_cast(_Float16, (unsigned short)((fc >> fsh) & 0xffffu));
            compute_n(st, sb, na_c, fl);
            if (WD_STAMPS && wave == 0) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                wd_lstamp(kc, 3);
            }
        }
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    se_out = cur >= BIG ? -1 : cur;
}

// acc tile -> LDS fp32 [BM][BN + 4] (C/D map of 16x16: col = lane & 15, row = 4 (lane >> 4) + reg)
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void x6_acc_to_lds(const floatx4 (&acc)[BM / WM / 16][BN / WN / 16], float *cl) {
    constexpr int TM = BM / WM / 16, TN = BN / WN / 16, LDC = BN + 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wi = wave / WN, wj = wave % WN, g = lane >> 4, i16 = lane & 15;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                cl[(wi * (BM / WM) + a * 16 + 4 * g + r) * LDC + wj * (BN / WN) + b * 16 + i16] = acc[a][b][r];
}

// the same with every value multiplied by sa and then sb (the h2 operands' inverse scales: powers of two,
// exact unless the result is subnormal)
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void x6_acc_to_lds_scaled(const floatx4 (&acc)[BM / WM / 16][BN / WN / 16], float *cl,
                                                     float sa, float sb) {
    constexpr int TM = BM / WM / 16, TN = BN / WN / 16, LDC = BN + 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wi = wave / WN, wj = wave % WN, g = lane >> 4, i16 = lane & 15;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                cl[(wi * (BM / WM) + a * 16 + 4 * g + r) * LDC + wj * (BN / WN) + b * 16 + i16] = acc[a][b][r] * sa * sb;
}

struct X6PParams {
    const uint8_t *a0; int kp0; int ka0;  // A segment 0: plane tiles (64-row blocks) of a [Mp][kp0] matrix, K extent ka0
    const uint8_t *a1; int kp1; int ka1;  // A segment 1 (ka1 = 0: absent)
    const uint8_t *b; int kpb;            // B plane tiles [Np][kpb], kpb == ka0 + ka1
    int M, N;
    int tiles_m, tiles_n;
    Epi epi;
};

// C[Mp][Np] = epi([A0 | A1] · Bᵀ): 64x64 tile, 8 waves of 16x32 (more waves issuing loads: a CU's
// L2 -> LDS rate grows with them, tools/gemm_lab stream), fused bias/residual/activation/dropout
// epilogue (epilogue_v4: fp32 Z / Y and optionally the next layer's plane tiles).
__global__ __launch_bounds__(512) void gemm_x6g_kernel(X6PParams P) {
    constexpr int BM = 64, NT = 512;
    // two LDS stages (three measured slower: 11.1 vs 11.0 us here, 9.6 vs 8.5 us on QM9-shaped batches)
    constexpr int S = 2;
    __shared__ __attribute__((aligned(16))) uint8_t lds[S * x6_stage_bytes<BM, 64>()];
    const int tile = xcd_tile(blockIdx.x, P.tiles_m * P.tiles_n);
    const int mt = tile / P.tiles_n, nt = tile % P.tiles_n;
    const int m0 = mt * BM, n0 = nt * X6_BN;
    EpiPrefetch<BM, X6_BN, NT> ep;
    ep.load(P.epi, m0, n0, P.M, P.N);
    X6Operands O{};
    O.a0 = P.a0; O.nkc0 = P.kp0 >> 5; O.kc0 = P.ka0 >> 5;
    O.a1 = P.a1; O.nkc1 = P.kp1 >> 5; O.kc1 = P.ka1 >> 5;
    O.rb = mt;
    O.a_rows = BM;
    O.b = P.b + (size_t)nt * (P.kpb >> 5) * X6_BLOCK;
    floatx4 acc[1][2];
    x6_mainloop<BM, 64, 4, 2, S>(O, lds, acc);
    __syncthreads();
    float *cl = reinterpret_cast<float *>(lds);
    x6_acc_to_lds<BM, 64, 4, 2>(acc, cl);
    __syncthreads();
    const uint32_t mx = epilogue_v4<BM, X6_BN, NT>(P.epi, cl, 68, m0, n0, P.M, P.N, ep);
    if (P.epi.kind == EPI_ACT && P.epi.amax && n0 < P.epi.amax_cols) {  // (workgroup-uniform)
        __shared__ uint32_t red[NT / 64];
        publish_max(mx, P.epi.amax + (size_t)mt * (P.epi.amax_cols / X6_BN) + nt, red);
    }
}

}  // namespace wd
