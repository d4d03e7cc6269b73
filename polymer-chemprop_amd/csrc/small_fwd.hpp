// small_fwd.hpp — the whole inference forward of a small molecule block in ONE workgroup (QM9-sized
// molecules, one batch in flight: chemprop/train/predict.py:30-40 runs one forward per batch).
//
// The molecule-blocked forward (fused_mp.hpp) is four launches: embed, T - 1 layers, W_o + readout.  A
// QM9 batch of 64 molecules is cut into ~64 blocks of ~14 bond rows, and each of those launches is a
// latency chain of its own (launch ramp, weight streaming, barriers) over a grid that barely fills the
// chip: 37 us per forward with one batch in flight (BENCH_r04.json).  Molecule blocks are independent
// through every layer (block-diagonal batches, featurization.py:782-800), so one workgroup can carry its
// block from the input layer to the readout with every intermediate in LDS and no other workgroup's
// data: one launch, no HBM round trips.  Per block (bond rows <= 32, atoms <= 32, Hk = 320):
//
//   inp  = f_bonds W_i^T (+ b_i)            sums of W_i columns from the codes (mpn.py:92-95)
//   for t = 1 .. T-1:                       (mpn.py:100-124)
//     M  = act(Z_{t-1})  -> fp16 hi / lo pair image (scale from the block's max, planes.hpp h2)
//     P  = M W_h^T                          fp16-pair MFMA GEMM, W_h fragments streamed from L2
//     A  = sum_{b into a} w_b P[b];  Z_t = inp + (A[src] - P[rev] + b_h)
//   M_T = act(Z_{T-1}); A = sum w_b M_T[b]  (mpn.py:126-131) -> bf16x3 image
//   h   = act(A W_o[:, Fa:]^T + f_atoms W_o[:, :Fa]^T + b_o)  (mpn.py:132-134)
//   out = readout of the block's molecules   (mpn.py:145-171)
//
// Every step is the fused path's arithmetic in the fused path's order (the same splits, MFMA product
// order per accumulator and chunk, gather order, residual / bias order, readout lane tree), so the
// result is bitwise the four-launch forward's: tests compare the two paths with torch.equal.
// LDS (124 KB + lists): three fp32 row tiles [32][Hk + 4] -- inp, P / Z, and the GEMM operand image
// (which also holds the atom sums and Ea); the W_o operand image (bf16x3, 60 KB) spans the last two.
#pragma once
#include "fused_mp.hpp"

namespace wd {

constexpr int SF_THREADS = 512, SF_ROWS = 32, SF_ATOMS = 32, SF_HK = 320;
constexpr int SF_LDI = SF_HK + 4;  // fp32 row stride of the LDS tiles

struct SmallFwdP {
    const int32_t *blocks;
    const WdAtomCode *codes;       // natural atom rows
    const uint8_t *src_blk;        // per natural bond row: block-local source atom
    const uint16_t *tail;          // per natural bond row: bond columns as bits
    const int32_t *rev;            // b2revb (natural ids)
    const uint8_t *aell_idx; const float *aell_coef;   // atom gather, block-local ELL (in-bonds, w_bonds)
    const int32_t *aptr, *aidx; const float *acoef;     // its CSR (natural ids) for rows past the ELL width
    const float *w_atoms; const int32_t *mol_start, *mol_size; const float *xn;
    const float *wit;              // W_i^T [>= Fb][Hk]
    const float *woat;             // W_o[:, :Fa]^T [>= Fa][Hk]
    const float *bi, *bh, *bo;     // padded biases (bi / bh may be null)
    const uint8_t *wh; const uint32_t *wh_amax; int whbr;  // W_h fp16-pair tiles (BR-row blocks) + scale word
    const uint8_t *wo; int wobr, kcw;                       // W_o bf16x3 tiles [Hk][Fak + Hk], BR-row blocks
    int Fa, Fb, T, undirected, agg; float norm;
    const float *zero_vec; const float *slope;
    float *out; int ncols;
};

// acc[j][r] (+)= A(rows 16 r ..) . B(column tile wave + 8 j)^T over NKC 32-column chunks, for the NRG
// 16-row groups holding rows and this wave's NTL column tiles (20 tiles over 8 waves: waves 0-3 three, 4-7
// two).  A: an LDS image of NP planes per chunk (x6_slot layout, SF_ROWS rows); B: NP-plane tiles in global
// memory with br-row blocks of nkc_tot chunks, the GEMM's chunks starting at kc_off.  NP = 2: fp16 hi / lo,
// products hh, hl, lh (the fused layer's order); NP = 3: bf16x3, products hh, hm, mh, hl, lh, mm
// (x6_mainloop's).  B fragments are buffer-loaded into registers PF chunks ahead (compile-time chunk loop:
// the compiler's vmcnt waits are exact).  Row groups and tiles are template arguments, dispatched once per
// GEMM: MFMAs under runtime predicates made the compiler keep every combination's registers (spills).
template <int NP, int NKC, int PF, int NRG, int NTL>
__device__ __forceinline__ void sf_gemm_body(const uint8_t *a_img, const uint8_t *bmat, int br, int nkc_tot, int kc_off,
                                             floatx4 (&acc)[3][2]) {
    using V = std::conditional_t<NP == 2, f16x8, bf16x8>;
    constexpr int NPROD = NP == 2 ? 3 : 6;
    constexpr int PA[6] = {0, 0, 1, 0, 2, 1}, PB[6] = {0, 1, 0, 2, 0, 1};
    constexpr int PA2[3] = {0, 0, 1}, PB2[3] = {0, 1, 0};
    constexpr int ACHUNK = NP * SF_ROWS * 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
    // one 32-bit lane offset per tile, the chunk / plane offsets as scalars (64-bit addresses per unrolled
    // load held ~200 VGPRs and spilled)
    const int bstep = NP * br * 64;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(bmat), 0, 0x7ffffff0, 0x00020000);
    int bo[NTL];
#pragma unroll
    for (int j = 0; j < NTL; ++j) {
        const int n = 16 * (wave + 8 * j) + i16;
        bo[j] = ((n / br) * nkc_tot + kc_off) * bstep + (n % br) * 64 + 16 * g;
    }
    V bq[PF][NTL][NP];
    auto load = [&](int s, int kc) {
#pragma unroll
        for (int j = 0; j < NTL; ++j)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                bq[s][j][p] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs, bo[j], kc * bstep + p * br * 64, 0));
    };
#pragma unroll
    for (int s = 0; s < PF; ++s)
        if (s < NKC) load(s, s);
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
        const int s = kc % PF;
        V af[NRG][NP];
#pragma unroll
        for (int r = 0; r < NRG; ++r)
#pragma unroll
            for (int p = 0; p < NP; ++p)
                af[r][p] = *reinterpret_cast<const V *>(a_img + kc * ACHUNK + p * SF_ROWS * 64 + x6_slot(16 * r + i16, g));
#pragma unroll
        for (int t = 0; t < NPROD; ++t)
#pragma unroll
            for (int j = 0; j < NTL; ++j)
#pragma unroll
                for (int r = 0; r < NRG; ++r) {
                    if constexpr (NP == 2)
                        acc[j][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r][PA2[t]], bq[s][j][PB2[t]], acc[j][r], 0, 0, 0);
                    else
                        acc[j][r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[r][PA[t]], bq[s][j][PB[t]], acc[j][r], 0, 0, 0);
                }
        if (kc + PF < NKC) load(s, kc + PF);
        __builtin_amdgcn_sched_barrier(0);  // (chunk by chunk: hoisting later chunks' loads spilled registers)
    }
}

// rg: 16-row groups of A that hold rows (1 or 2); accumulators the body does not touch stay zero
template <int NP, int NKC, int PF>
__device__ __forceinline__ void sf_gemm(const uint8_t *a_img, int rg, const uint8_t *bmat, int br, int nkc_tot,
                                        int kc_off, floatx4 (&acc)[3][2]) {
    static_assert(2 * NKC > 16 && 2 * NKC <= 24, "two or three column tiles per wave");
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[j][r] = floatx4{0.f, 0.f, 0.f, 0.f};
    const bool three = (int)(threadIdx.x >> 6) < 2 * NKC - 16;
    if (rg <= 1) {
        if (three) sf_gemm_body<NP, NKC, PF, 1, 3>(a_img, bmat, br, nkc_tot, kc_off, acc);
        else sf_gemm_body<NP, NKC, PF, 1, 2>(a_img, bmat, br, nkc_tot, kc_off, acc);
    } else {
        if (three) sf_gemm_body<NP, NKC, PF, 2, 3>(a_img, bmat, br, nkc_tot, kc_off, acc);
        else sf_gemm_body<NP, NKC, PF, 2, 2>(a_img, bmat, br, nkc_tot, kc_off, acc);
    }
}

// code_sum over a global (L2-resident) table, branch-free: every slot loads a row (an unused slot row 0,
// added as +0), so the nine loads of a unit go out together -- the same sums as code_sum
template <int LDT>
__device__ __forceinline__ float4 code_sum_g(const WdAtomCode &cd, const float *T, int Fa, int c) {
    float4 w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = ld4(T + (cd.col[q] == 0xFF ? 0 : (int)cd.col[q]) * LDT + c);
    const float4 wl = ld4(T + (Fa - 1) * LDT + c);
    float4 s = f4zero();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const bool ok = cd.col[q] != 0xFF;
        s.x += ok ? w[q].x : 0.f; s.y += ok ? w[q].y : 0.f; s.z += ok ? w[q].z : 0.f; s.w += ok ? w[q].w : 0.f;
    }
    fma4(s, cd.last, wl);
    return s;
}

// acc -> fp32 LDS tile T[row][SF_LDI] (x sa x sb, in that order: the fused layer's x6_acc_to_lds_scaled)
template <bool SCALED>
__device__ __forceinline__ void sf_acc_store(const floatx4 (&acc)[3][2], float *T, float sa, float sb) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, i16 = lane & 15;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int ct = wave + 8 * j;
        if (ct >= SF_HK / 16) continue;
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    T[(16 * r + 4 * g + e) * SF_LDI + 16 * ct + i16] = SCALED ? acc[j][r][e] * sa * sb : acc[j][r][e];
    }
}

// s = sum over atom la's in-bond entries (ELL slots, then the CSR rest) of w * T[bond][c .. c+7]: the fused
// epilogue's row_sum (fmaf chain from zero in slot order)
__device__ __forceinline__ void sf_atom_sum(const SmallFwdP &P, const EllRow &E, int a, int bs, int c, const float *T,
                                            float4 &s0, float4 &s1) {
    s0 = s1 = f4zero();
#pragma unroll
    for (int k = 0; k < ELLW; ++k)
        if (E.w[k] != 0.f) lds_term<SF_LDI>(T, ell_idx(E, k), c, E.w[k], s0, s1);
    if (ell_more(E))
        for (int q = P.aptr[a] + ELLW; q < P.aptr[a + 1]; ++q) {
            const int li = P.aidx[q] - bs;
            if (li >= 0) lds_term<SF_LDI>(T, li, c, P.acoef ? P.acoef[q] : 1.0f, s0, s1);
        }
}

// the block's max |act(Z)| over its rows -> the fp16-pair image of M = act(Z) (rows past bn zero)
template <int ACT>
__device__ __forceinline__ float sf_stage_h2(const float *Z, int bn, uint8_t *img, float slope, uint32_t *red) {
    constexpr int NKC = SF_HK / 32, UN = SF_ROWS * NKC * 4;  // (row, chunk, 8-column unit)
    const int tid = threadIdx.x;
    uint32_t mx = 0;
    for (int v = tid; v < bn * (SF_HK / 4); v += SF_THREADS) {
        const float4 z = ld4(Z + (v / (SF_HK / 4)) * SF_LDI + 4 * (v % (SF_HK / 4)));
        mx = max(mx, max(max(absbits(act_fwd(ACT, z.x, slope)), absbits(act_fwd(ACT, z.y, slope))),
                         max(absbits(act_fwd(ACT, z.z, slope)), absbits(act_fwd(ACT, z.w, slope)))));
    }
    mx = wave_max_u32(mx);
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = red[0];
#pragma unroll
    for (int w = 1; w < SF_THREADS / 64; ++w) mx = max(mx, red[w]);
    const float s = h2_scale(mx);
    for (int v = tid; v < UN; v += SF_THREADS) {
        const int r = v / (NKC * 4), kc = (v / 4) % NKC, u = v % 4;
        uint32_t hh[4] = {0u, 0u, 0u, 0u}, ll[4] = {0u, 0u, 0u, 0u};
        if (r < bn) {
            const float *zr = Z + r * SF_LDI + 32 * kc + 8 * u;
            const float4 a = ld4(zr), b = ld4(zr + 4);
            float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = act_fwd(ACT, x[q], slope);
#pragma unroll
            for (int q = 0; q < 4; ++q) split_h2(x[2 * q], x[2 * q + 1], s, hh[q], ll[q]);
        }
        uint8_t *d = img + kc * (2 * SF_ROWS * 64) + x6_slot(r, u);
        *reinterpret_cast<u32x4 *>(d) = u32x4{hh[0], hh[1], hh[2], hh[3]};
        *reinterpret_cast<u32x4 *>(d + SF_ROWS * 64) = u32x4{ll[0], ll[1], ll[2], ll[3]};
    }
    return h2_inv_scale(mx);
}

// one workgroup per molecule block (grid = n_blocks), SF_THREADS threads; blocks must hold <= SF_ROWS bond
// rows and <= SF_ATOMS atoms (the host checks WdGraph.blk_max_*), Hk == SF_HK
template <int ACT>
__global__ __launch_bounds__(SF_THREADS) void small_forward_kernel(const SmallFwdP P) {
    constexpr int NT = SF_THREADS, LDI = SF_LDI, HK = SF_HK, C4 = HK / 4, NKC = HK / 32;
    constexpr int TILE = SF_ROWS * LDI;  // floats per fp32 row tile
    __shared__ __attribute__((aligned(16))) float lds[3 * TILE];
    __shared__ __attribute__((aligned(16))) WdAtomCode s_code[SF_ATOMS];
    __shared__ EllRow s_ell[SF_ATOMS];
    __shared__ int s_src[SF_ROWS], s_rev[SF_ROWS];
    __shared__ uint32_t s_tail[SF_ROWS], s_red[NT / 64];
    __shared__ float s_wat[SF_ATOMS], s_ml[3 * BLK_MOLS];
    static_assert(SF_ATOMS <= SF_ROWS && NKC * 2 * SF_ROWS * 64 <= TILE * 4 && NKC * 3 * SF_ROWS * 64 <= 2 * TILE * 4,
                  "operand images fit their regions");
    float *INP = lds, *ZP = lds + TILE, *X = lds + 2 * TILE;
    const int tid = threadIdx.x;
    wd_stamp(0);
    const BlockRow B = load_block(P.blocks, blockIdx.x);
    const int nm = min(B.mh - B.ml, BLK_MOLS);
    const float slope = ACT == ACT_PRELU ? P.slope[0] : 0.f;
    // ---- the block's graph: atom codes, gather lists, atom weights, bonds' source / reverse / tail, molecules
    if (tid < B.an) {
        reinterpret_cast<u32x4 *>(s_code)[tid] = reinterpret_cast<const u32x4 *>(P.codes)[B.as + tid];
        s_ell[tid] = ell_load(P.aell_idx, P.aell_coef, (size_t)B.as + tid);
        s_wat[tid] = P.w_atoms[B.as + tid];
    }
    if (tid >= 64 && tid - 64 < B.bn) {
        const int lb = tid - 64;
        s_src[lb] = P.src_blk[B.bs + lb];
        s_rev[lb] = P.rev[B.bs + lb] - B.bs;
        s_tail[lb] = P.tail[B.bs + lb];
    }
    if (tid >= 128 && tid - 128 < nm) {
        const int im = tid - 128;
        s_ml[im] = __int_as_float(P.mol_start[B.ml + im]);
        s_ml[BLK_MOLS + im] = __int_as_float(P.mol_size[B.ml + im]);
        s_ml[2 * BLK_MOLS + im] = P.xn[B.ml + im];
    }
    __syncthreads();
    wd_stamp(1);
    // ---- input layer: Ea[a] = sum_{c in code(a)} W_i[:, c] + last W_i[:, Fa-1] (into X), then per bond
    // inp[b] = Ea[src] + sum_{k in tail} W_i[:, Fa + k] (+ b_i)  (embed_kernel's sums)
    // (the bond columns' rows of W_i^T staged in ZP: the tail loop below reads them per set bit, and from
    // global memory each would be a dependent L2 round trip)
    for (int v = tid; v < (P.Fb - P.Fa) * C4; v += NT)
        st4(ZP + (v / C4) * LDI + 4 * (v % C4), ld4(P.wit + (size_t)(P.Fa + v / C4) * HK + 4 * (v % C4)));
    for (int v = tid; v < B.an * C4; v += NT) {
        const int la = v / C4, c = 4 * (v % C4);
        st4(X + la * LDI + c, code_sum_g<HK>(s_code[la], P.wit, P.Fa, c));
    }
    __syncthreads();
    wd_stamp(2);
    for (int v = tid; v < B.bn * C4; v += NT) {
        const int lb = v / C4, c = 4 * (v % C4);
        float4 z = ld4(X + s_src[lb] * LDI + c);
        for (uint32_t m = s_tail[lb]; m; m &= m - 1) {
            const float4 w = ld4(ZP + __builtin_ctz(m) * LDI + c);
            z.x += w.x; z.y += w.y; z.z += w.z; z.w += w.w;
        }
        const float4 b = P.bi ? ld4(P.bi + c) : f4zero();
        z.x += b.x; z.y += b.y; z.z += b.z; z.w += b.w;
        st4(INP + lb * LDI + c, z);
    }
    __syncthreads();
    wd_stamp(3);
    // ---- message passing (mpn.py:100-124)
    const float iw = h2_inv_scale(*P.wh_amax);
    const float *Z = INP;
    constexpr int UPT = (SF_ROWS * C4 + NT - 1) / NT;  // (row, float4) units per thread
    for (int t = 1; t < P.T; ++t) {
        const float ia = sf_stage_h2<ACT>(Z, B.bn, reinterpret_cast<uint8_t *>(X), slope, s_red);
        __syncthreads();  // the operand image is complete; Z (in ZP from the second layer on) is dead
        const int sl = 4 + 4 * min(t - 1, 1);
        wd_stamp(sl);
        floatx4 acc[3][2];
        sf_gemm<2, NKC, 4>(reinterpret_cast<const uint8_t *>(X), (B.bn + 15) >> 4, P.wh, P.whbr, NKC, 0, acc);
        sf_acc_store<true>(acc, ZP, ia, iw);
        wd_stamp(sl + 1);
        __syncthreads();
        if (P.undirected) {  // P <- (P + P[rev]) / 2 (mpn.py:101-102), once per reverse pair
            for (int v = tid; v < B.bn * C4; v += NT) {
                const int lr = v / C4, c = 4 * (v % C4), rl = s_rev[lr];
                if (lr < rl) {
                    float4 p = ld4(ZP + lr * LDI + c);
                    const float4 q = ld4(ZP + rl * LDI + c);
                    p.x = (p.x + q.x) / 2.0f; p.y = (p.y + q.y) / 2.0f; p.z = (p.z + q.z) / 2.0f; p.w = (p.w + q.w) / 2.0f;
                    st4(ZP + lr * LDI + c, p);
                    st4(ZP + rl * LDI + c, p);
                }
            }
            __syncthreads();
        }
        // A[a] = sum_{b into a} w_b P[b] (mpn.py:112-118), into X (the operand image is dead)
        for (int v = tid; v < B.an * (HK / 8); v += NT) {
            const int la = v / (HK / 8), c = 8 * (v % (HK / 8));
            float4 s0, s1;
            sf_atom_sum(P, s_ell[la], B.as + la, B.bs, c, ZP, s0, s1);
            st4(X + la * LDI + c, s0);
            st4(X + la * LDI + c + 4, s1);
        }
        __syncthreads();
        wd_stamp(sl + 2);
        // Z_t = inp + (A[src] - P[rev] + b_h) (mpn.py:119-123), held in registers until every P read is done
        float4 zn[UPT];
#pragma unroll
        for (int i = 0; i < UPT; ++i) {
            const int v = tid + NT * i, lr = v / C4, c = 4 * (v % C4);
            zn[i] = f4zero();
            if (lr < B.bn) {
                const float4 a = ld4(X + s_src[lr] * LDI + c), q = ld4(ZP + s_rev[lr] * LDI + c);
                const float4 r = ld4(INP + lr * LDI + c);
                const float4 b = P.bh ? ld4(P.bh + c) : f4zero();
                zn[i] = make_float4(r.x + ((a.x - q.x) + b.x), r.y + ((a.y - q.y) + b.y), r.z + ((a.z - q.z) + b.z),
                                    r.w + ((a.w - q.w) + b.w));
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < UPT; ++i) {
            const int v = tid + NT * i, lr = v / C4, c = 4 * (v % C4);
            if (lr < B.bn) st4(ZP + lr * LDI + c, zn[i]);
        }
        __syncthreads();
        wd_stamp(sl + 3);
        Z = ZP;
    }
    // ---- atom aggregate of M_T = act(Z_{T-1}) (mpn.py:126-131): act in place, then A into INP (inp is dead)
    for (int v = tid; v < B.bn * C4; v += NT) {
        float *zr = ZP + (v / C4) * LDI + 4 * (v % C4);
        float4 z = ld4(zr);
        z = make_float4(act_fwd(ACT, z.x, slope), act_fwd(ACT, z.y, slope), act_fwd(ACT, z.z, slope), act_fwd(ACT, z.w, slope));
        st4(zr, z);
    }
    __syncthreads();
    for (int v = tid; v < B.an * (HK / 8); v += NT) {
        const int la = v / (HK / 8), c = 8 * (v % (HK / 8));
        float4 s0, s1;
        sf_atom_sum(P, s_ell[la], B.as + la, B.bs, c, ZP, s0, s1);
        st4(INP + la * LDI + c, s0);
        st4(INP + la * LDI + c + 4, s1);
    }
    __syncthreads();
    // A -> bf16x3 image (the last layer's x6_store8_blk split) over ZP and X; rows past the atoms zero
    uint8_t *AO = reinterpret_cast<uint8_t *>(ZP);
    for (int v = tid; v < SF_ROWS * NKC * 4; v += NT) {
        const int r = v / (NKC * 4), kc = (v / 4) % NKC, u = v % 4;
        uint32_t h[4] = {0u, 0u, 0u, 0u}, m[4] = {0u, 0u, 0u, 0u}, l[4] = {0u, 0u, 0u, 0u};
        if (r < B.an) {
            const float4 lo = ld4(INP + r * LDI + 32 * kc + 8 * u), hi = ld4(INP + r * LDI + 32 * kc + 8 * u + 4);
            split_pair(lo.x, lo.y, h[0], m[0], l[0]);
            split_pair(lo.z, lo.w, h[1], m[1], l[1]);
            split_pair(hi.x, hi.y, h[2], m[2], l[2]);
            split_pair(hi.z, hi.w, h[3], m[3], l[3]);
        }
        uint8_t *d = AO + kc * (3 * SF_ROWS * 64) + x6_slot(r, u);
        *reinterpret_cast<u32x4 *>(d) = u32x4{h[0], h[1], h[2], h[3]};
        *reinterpret_cast<u32x4 *>(d + SF_ROWS * 64) = u32x4{m[0], m[1], m[2], m[3]};
        *reinterpret_cast<u32x4 *>(d + 2 * SF_ROWS * 64) = u32x4{l[0], l[1], l[2], l[3]};
    }
    __syncthreads();
    wd_stamp(12);
    // ---- h = act(A W_o[:, Fa:]^T + Eo + b_o) (mpn.py:132-134; Eo = the codes' W_o columns, embed_kernel's sums)
    {
        floatx4 acc[3][2];
        sf_gemm<3, NKC, 3>(AO, (B.an + 15) >> 4, P.wo, P.wobr, P.kcw + NKC, P.kcw, acc);
        sf_acc_store<false>(acc, INP, 1.f, 1.f);
    }
    wd_stamp(13);
    __syncthreads();
    for (int v = tid; v < B.an * C4; v += NT) {
        const int la = v / C4, c = 4 * (v % C4);
        float4 hv = ld4(INP + la * LDI + c);
        const float4 eo = code_sum_g<HK>(s_code[la], P.woat, P.Fa, c);
        const float4 bb = ld4(P.bo + c);
        hv.x += eo.x; hv.y += eo.y; hv.z += eo.z; hv.w += eo.w;
        float z[4] = {hv.x + bb.x, hv.y + bb.y, hv.z + bb.z, hv.w + bb.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) z[q] = act_fwd(ACT, z[q], slope);
        st4(INP + la * LDI + c, make_float4(z[0], z[1], z[2], z[3]));
    }
    __syncthreads();
    wd_stamp(14);
    // ---- readout (mpn.py:145-171): wo_readout_kernel's eight-lane sums and xor tree, all Hk columns
    constexpr int RP = 8;
    for (int t = tid; t < nm * HK * RP; t += NT) {
        const int part = t % RP, u = t / RP, im = u / HK, i = B.ml + im, col = u % HK;
        const int n = __float_as_int(s_ml[BLK_MOLS + im]);
        float s = 0.f, wsum = 0.f;
        const int a0 = __float_as_int(s_ml[im]) - B.as;
        for (int a = part; a < n; a += RP) {
            const float w = s_wat[a0 + a];
            s = fmaf(w, INP[(a0 + a) * LDI + col], s);
            wsum += w;
        }
#pragma unroll
        for (int off = 1; off < RP; off <<= 1) {
            s += __shfl_xor(s, off, 64);
            wsum += __shfl_xor(wsum, off, 64);
        }
        if (part != 0 || col >= P.ncols) continue;
        float v;
        if (n == 0) {
            v = P.zero_vec[col];
        } else {
            const float m = P.agg == 0 ? s / wsum : (P.agg == 2 ? s / P.norm : s);
            v = s_ml[2 * BLK_MOLS + im] * m;
        }
        P.out[(size_t)i * P.ncols + col] = v;
    }
    wd_stamp(15);
}

}  // namespace wd
