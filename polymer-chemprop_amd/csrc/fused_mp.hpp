// fused_mp.hpp — molecule-blocked fused message passing (inference forward, bond messages).
//
// Molecules are independent (block-diagonal batches, featurization.py:782-800), so a workgroup that
// owns whole molecules needs no other workgroup's rows.  The host packer groups consecutive molecules
// into blocks of <= 128 bond rows and <= 64 atom rows (WdGraph.blocks).  Intermediates live in
// molecule-blocked plane tiles (planes.hpp, BR = 128 for bond rows, BR = 64 for atom rows), and
// every stage after W_i is ONE launch per (block, 64- or 80-column tile):
//
//   mp_layer_kernel   P = M_{t-1} W_hᵀ (bf16x6 split-plane GEMM on the block's 128 rows; the first layer
//                       stages M_0 = act(inp) from the fp32 inp rows itself), then the CSR gather of P
//                       inside the block (GEMM first, gather second: X_t W_hᵀ = (G M_{t-1}) W_hᵀ =
//                       G (M_{t-1} W_hᵀ), column-separable, mpn.py:110-124), bias, residual inp and
//                       activation: M_t = act(inp + G P (+ b_h)) -> plane tiles of the next layer.  The last layer also forms the atom aggregate
//                       A = Σ_{b into a} w_b M_t[b] (mpn.py:126-131) for its columns -> atom plane tiles.
//   wo_readout_kernel   h = act([f_atoms | A] W_oᵀ + b_o) (mpn.py:132-134) on the block's atoms, then the
//                       molecule readout (mpn.py:145-171) of those columns straight to out[mol].
//
// So the forward is W_i + (T - 1) layer launches + 1, with no gather kernels, no M_0 round trip through
// HBM and no separate readout.  Arithmetic per output element: the P and h GEMMs
// are fp32-accurate (gemm_x6.hpp), the gathers add in CSR order (the reference's slot order).
#pragma once
#include "gemm_x6.hpp"
#include "kernels.hpp"
#include "wdmpnn.h"

namespace wd {


constexpr int BLK_BONDS = 128, BLK_ATOMS = 64;  // block capacity (rows of the blocked layouts)
constexpr int BLK_MOLS = 64;                     // molecules per block (empty molecules have no rows)
// gather entries per row in the block-local ELL form (WdGraph.*_ell_*, WDMPNN_ELL_WIDTH; 12 measured
// no faster than 8 on the polymer benchmark, whose longest rows have 9 entries)
constexpr int ELLW = 8;
static_assert(ELLW % 4 == 0, "ELL rows of whole 4-byte index words and float4 weight groups");

// one prefetched ELL row: ELLW uint8 indices (bit 7 of the last = "more entries in the CSR list") and
// ELLW weights (0 = empty slot)
struct EllRow {
    uint32_t ix[ELLW / 4];
    float w[ELLW];
};
__device__ __forceinline__ EllRow ell_zero() {
    EllRow e;
    for (int k = 0; k < ELLW / 4; ++k) e.ix[k] = 0;
    for (int k = 0; k < ELLW; ++k) e.w[k] = 0.f;
    return e;
}
__device__ __forceinline__ EllRow ell_load(const uint8_t *idx, const float *coef, size_t row) {
    EllRow e;
    const uint32_t *ip = reinterpret_cast<const uint32_t *>(idx + ELLW * row);
    const float *cp = coef + ELLW * row;
#pragma unroll
    for (int q = 0; q < ELLW / 4; ++q) {
        e.ix[q] = ip[q];
        const float4 w = ld4(cp + 4 * q);
        e.w[4 * q] = w.x; e.w[4 * q + 1] = w.y; e.w[4 * q + 2] = w.z; e.w[4 * q + 3] = w.w;
    }
    return e;
}
__device__ __forceinline__ int ell_idx(const EllRow &e, int k) { return (e.ix[k >> 2] >> (8 * (k & 3))) & 0x7f; }
__device__ __forceinline__ bool ell_more(const EllRow &e) { return e.ix[ELLW / 4 - 1] & 0x80000000u; }

// WdGraph.blocks row: {bond_start, bond_count, atom_start, atom_count, mol_lo, mol_hi, -, -}
struct BlockRow { int bs, bn, as, an, ml, mh; };
__device__ __forceinline__ BlockRow load_block(const int32_t *blocks, int i) {
    const int4 a = *reinterpret_cast<const int4 *>(blocks + 8 * i);
    const int2 b = *reinterpret_cast<const int2 *>(blocks + 8 * i + 4);
    return BlockRow{a.x, a.y, a.z, a.w, b.x, b.y};
}

// s += w * T[j][c .. c+7] (LDS tile, row stride LDC)
template <int LDC>
__device__ __forceinline__ void lds_term(const float *T, int j, int c, float w, float4 &s0, float4 &s1) {
    fma4(s0, w, ld4(T + j * LDC + c));
    fma4(s1, w, ld4(T + j * LDC + c + 4));
}

struct MpLayerP {
    const float *zin;           // Z_{t-1}: fp32 natural bond rows [Rp][kp] (the first layer: inp, mpn.py:95); the
                                // GEMM operand is M_{t-1} = dropout(act(Z_{t-1})) (mpn.py:97, 123-124), formed
                                // while staging
    const uint32_t *amax_in;    // its scale words (planes.hpp h2): [nblk][amax_in_n] maxima of |M_{t-1}|,
    int amax_in_n;              // published per (block, tile) by the embed or by layer t - 1; amax_rt > 0:
    int amax_rt;                //   per (amax_rt-row tile of zin, column tile) by the input GEMM (gemm_x6g's
                                //   Epi.amax): the words of the row tiles the block's rows overlap
    int ldz, ldr;               // row strides of zin and of the residual inp (Hk, or wider for column slices)
    float p_drop_in;            // the dropout of M_{t-1} (0 for M_0: mpn.py:97 drops nothing)
    float *zout;                // Z_t, same layout (null in the last layer)
    uint32_t *amax_out;         // [nblk][n_tiles]: max |dropout(act(Z_t))| of each workgroup (not the last layer)
    int kp;                     // Hk
    const uint8_t *wh;          // W_h h2 plane tiles [Hk][Hk] with BN-row blocks
    const uint32_t *wh_amax;    // their scale word (max |W_h|, wdmpnn_pack_params)
    const float *inp;           // fp32 [Rp][Hk] natural rows (mpn.py:95 input)
    const float *bias;          // b_h (padded) or null
    const int32_t *blocks;
    const int32_t *rev;         // b2revb (natural bond ids)
    const uint8_t *src_blk;     // per natural bond row: block-local source atom (b2a)
    int undirected;             // mpn.py:101-102
    int act; const float *slope; float p_drop; uint64_t seed; uint32_t layer;
    const int32_t *aptr, *aidx; const float *acoef;  // atom gather (natural atom rows -> natural bond rows)
    const uint8_t *aell_idx; const float *aell_coef; // its first ELLW entries per row, block-local (WdGraph)
    uint8_t *aplanes;           // A: blocked atom plane tiles [nblk * 64][kp] (the last layer)
    int n_tiles;                // Hk / BN
    // training forward (save_for_backward) or null, the last layer only (the others' Z_t is zout): its
    // pre-activation Z_t (mpn.py:123) as fp32 natural bond rows [Rp][kp] and the atom aggregate A
    // (mpn.py:126-131) as fp32 natural atom rows [Vap][kp] (the backward's operands)
    float *zsave, *asave;
    // atom-message mode (mpn.py:47-53, 93-94, 104-108; the template's ATOM): the message rows are the
    // block's atoms, inp is the residual inp + (sum over a2b of the bond features) W_h[:, H:]^T, and the
    // gather is the a2a neighbour sum X[a] = sum_{a' in nbr(a)} P[a'] (no reverse term), from these lists
    // (block-local ELL over atom rows); aptr / aell above stay the final
    // aggregate (mpn.py:126-131).  The ELL lists drop the a2a pad slots (atom 0, whose message is zero
    // without biases); rows longer than the ELL width continue in the CSR list msg_gather, whose pad-slot
    // entry (atom 0, outside every block) is skipped
    const uint8_t *mell_idx; const float *mell_coef;
    const int32_t *mptr, *midx; const float *mcoef;
    // pair-operand layers (the template's PAIRS, round 6): M_{t-1} comes as fp16 hi / lo pair tiles of the
    // molecule blocks ([nblk][Hk / 32 chunks][2 planes][128 rows][64 B]), scaled per group of ain_g columns
    // by the words amax_in [nblk][amax_in_n] (the embed: 32-column groups; a layer: its BN-column tiles),
    // and the layer writes M_t the same way into aout (not the last layer), scaled by its tile's max
    const uint8_t *ain; int ain_g;
    uint8_t *aout;
    // ... and the last layer writes the atom aggregate A as pair tiles of the blocks' atom rows ([nblk][Hk / 32]
    // [2][64][64 B], W_o's A operand: wo_readout_kernel<..., PAIRS>), scaled by its tile's max, published in
    // amax_out [nblk][n_tiles]
    uint8_t *apairs;
};

// The GEMM operand M_{t-1} = dropout(act(Z_{t-1})), formed while staging from the fp32 Z rows (the
// producer waves of h2_mainloop_ws), so that no message tensor goes through HBM in split form: producer
// thread t (0..255) stages rows t / 4 and t / 4 + 64 of the block, columns 8 (t % 4) .. +7 of each
// 32-column chunk, applies the activation and dropout, scales and splits into fp16 hi / lo.  The rows are
// read through a buffer resource that ends at the block's last bond: rows past it come back as zeros
// without touching memory (a QM9 block holds ~14 of the 128 rows), with the same instruction stream in
// every wave, so the compiler's vmcnt waits stay exact; only the 16-row tiles the consumers multiply are
// converted and stored.  (8 lanes per row, one 16-byte load each, measured +0.5 us per launch.)
template <int BM, int AACT>
struct H2Prod {
    static constexpr int U = BM / 64;                    // rows per producer thread
    static constexpr int SETS = 3;                       // register sets (chunks in flight)
    __amdgpu_buffer_rsrc_t rs;              // the block's Z rows
    int off[U];                             // byte offset of this thread's columns in row r0 + 64 i
    uint32_t grow[U];                       // natural bond row (dropout counter)
    int r0, u, live16;                      // live16: rows of the 16-row tiles holding bonds
    float slope, scale, pd;
    uint64_t seed;
    uint32_t layer;
    uint32_t wv;                            // this lane's scale word (lane_word, loaded by the caller)
    u32x4 v[SETS][U][2];                    // register sets (raw fp32 bits)
    __device__ __forceinline__ void init() { scale = h2_scale(wave_max_u32(wv)); }
    // rows rs .. rs + rn - 1 of zin (the block's bonds, or its atoms in atom-message mode)
    __device__ __forceinline__ H2Prod(const MpLayerP &P, int rs0, int rn, uint32_t words) {
        const int t = threadIdx.x & 255;
        r0 = t >> 2; u = t & 3;
        rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(P.zin + (size_t)rs0 * P.ldz), 0,
                                               rn > 0 ? ((rn - 1) * P.ldz + P.kp) * 4 : 0, 0x00020000);
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const int r = r0 + 64 * i;
            grow[i] = r < rn ? rs0 + r : 0;
            off[i] = (r * P.ldz + 8 * u) * 4;
        }
        live16 = (rn + 15) & ~15;
        slope = AACT == ACT_PRELU ? P.slope[0] : 0.f;
        wv = words;
        scale = 1.f;
        pd = P.p_drop_in;
        seed = P.seed;
        layer = P.layer - 1;
    }
    template <typename S>
    __device__ __forceinline__ void load(S, int kc) {
#pragma unroll
        for (int i = 0; i < U; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                v[S::value][i][h] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off[i] + 128 * kc + 16 * h, 0, 0));
    }
    template <typename S>
    __device__ __forceinline__ void store(S, int kc, uint8_t *st) {
        // (a use of every register of the set outside the row branch below: the compiler otherwise sank
        // the first set's second-row loads into that branch, right in front of their use)
#pragma unroll
        for (int i = 0; i < U; ++i)
#pragma unroll
            for (int h = 0; h < 2; ++h) asm volatile("" ::"v"(v[S::value][i][h]));
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const int r = r0 + 64 * i;
            if (r >= live16) continue;  // (the consumers skip those 16-row tiles)
            float x[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const u32x4 a = v[S::value][i][h];
                x[4 * h] = __uint_as_float(a.x); x[4 * h + 1] = __uint_as_float(a.y);
                x[4 * h + 2] = __uint_as_float(a.z); x[4 * h + 3] = __uint_as_float(a.w);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = act_fwd(AACT, x[q], slope);
            if (pd > 0.f)
#pragma unroll
                for (int q = 0; q < 8; ++q) x[q] *= dropout_scale(seed, layer, grow[i], 32 * kc + 8 * u + q, pd);
            uint32_t hh[4], ll[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) split_h2(x[2 * q], x[2 * q + 1], scale, hh[q], ll[q]);
            uint8_t *d = st + x6_slot(r, u);
            *reinterpret_cast<u32x4 *>(d) = u32x4{hh[0], hh[1], hh[2], hh[3]};
            *reinterpret_cast<u32x4 *>(d + BM * 64) = u32x4{ll[0], ll[1], ll[2], ll[3]};
        }
    }
};

// cache policy of the Z_t row stores: default write-back.  Write-through, as the planes use, measured
// slower on the first polymer layer (17.46 us against 16.50, same box)
#ifndef WD_ZWT
#define WD_ZWT 0
#endif

// The fused layer kernel runs 512 threads, warp-specialised: 4 MFMA waves of 32 rows x all BN columns and
// their 4 staging partners (gemm_x6.hpp h2_mainloop_ws); the epilogue runs on all 512.  80-column tiles
// give 4 tiles for Hk = 320 and so exactly one workgroup per CU at the benchmark size (64 blocks x 4 =
// 256): a grid of 1.25 workgroups per CU left a quarter of the CUs with twice the bytes to stream.
constexpr int MP_THREADS = 512;

// mp_layer epilogue: the gather G applied to the P = M_{t-1} W_h^T tile in LDS in the reference's two
// steps (mpn.py:110-120), then bias, residual and the fp32 stores of Z_t (with the maximum of
// dropout(act(Z_t)) published for the next layer's scale) -- or, in the last layer, activation, dropout
// and the atom aggregate of M_t (mpn.py:126-131):
//     (undirected: P <- (P + P[rev]) / 2, mpn.py:101-102)
//     A[a] = sum_{b into a} w_b P[b]      (the block's atoms, slot order, into LDS)
//     X[b] = A[src(b)] - P[rev(b)]
// Only the atom gather lists and the rows' source / reverse ids are prefetched during the GEMM (a few
// registers: with <= 128 VGPRs two layer workgroups co-reside on a CU -- one's epilogue beside the
// other's GEMM when batches are in flight on two streams); the residual rows are loaded when the
// epilogue starts and land behind the atom sums.
template <int BN, int NT, bool LAST, bool ATOM = false, bool POUT = false>
struct MpEpilogue {
    static constexpr int BM = BLK_BONDS, LDC = BN + 4;
    static constexpr int UPR = BN / 8, UNITS = BM * UPR, UPT = (UNITS + NT - 1) / NT;  // 8-column units
    static constexpr int AUNITS = BLK_ATOMS * UPR, AUPT = (AUNITS + NT - 1) / NT;
    static constexpr int LDS_FLOATS = (BM + BLK_ATOMS) * LDC;  // P tile, then the atom sums
    static constexpr int YPT = ATOM ? AUPT : UPT;              // units of M_t per thread (rows: atoms | bonds)
    EllRow aell[AUPT];               // bond mode: the atom gather; atom mode: the a2a neighbour lists
    EllRow gell[ATOM && LAST ? AUPT : 1];  // atom mode, last layer: the final aggregate's lists
    int32_t rv[ATOM ? 1 : UPT];
    uint32_t sa[ATOM ? 1 : UPT];

    // during the GEMM: the gather rows of this thread's atom units (unit v = tid + NT i: atom v / UPR) and,
    // in bond mode, the source / reverse ids of its bond units (unit v: row v / UPR) -- loads only, no
    // arithmetic on what they return (that would wait for them inside the GEMM)
    __device__ __forceinline__ void prefetch(const MpLayerP &P, const BlockRow &B) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int i = 0; i < AUPT; ++i) {
            const int v = tid + NT * i;
            const bool ok = v < AUNITS && v / UPR < B.an;
            aell[i] = ell_zero();
            if (ok) aell[i] = ATOM ? ell_load(P.mell_idx, P.mell_coef, (size_t)B.as + v / UPR)
                                   : ell_load(P.aell_idx, P.aell_coef, (size_t)B.as + v / UPR);
            if constexpr (ATOM && LAST) {
                gell[i] = ell_zero();
                if (ok) gell[i] = ell_load(P.aell_idx, P.aell_coef, (size_t)B.as + v / UPR);
            }
        }
        if constexpr (!ATOM)
#pragma unroll
            for (int i = 0; i < UPT; ++i) {
                const int v = tid + NT * i, lr = v / UPR;
                rv[i] = 0;
                sa[i] = 0;
                if (v < UNITS && lr < B.bn) {
                    rv[i] = P.rev[B.bs + lr];
                    sa[i] = P.src_blk[B.bs + lr];
                }
            }
    }

    // The same lists handed over through LDS (WD_EPI_PRE): the staging waves, done one chunk before the MFMA
    // waves, load them for the whole block while the last chunk is multiplied (fill_pre), and every thread
    // reads its units' rows from LDS after the barrier (take_pre) -- no memory latency after the GEMM.
    static constexpr int PRE_ELL = BLK_ATOMS * (int)sizeof(EllRow);
    static constexpr int PRE_BYTES = PRE_ELL * (ATOM && LAST ? 2 : 1) + (ATOM ? 0 : BM * 8);
    __device__ __forceinline__ void fill_pre(const MpLayerP &P, const BlockRow &B, uint8_t *pre) {
        const int t = threadIdx.x - MP_THREADS / 2;  // (staging threads 0 .. 255)
        if (t < BLK_ATOMS) {
            EllRow e = ell_zero();
            if (t < B.an) e = ATOM ? ell_load(P.mell_idx, P.mell_coef, (size_t)B.as + t)
                                   : ell_load(P.aell_idx, P.aell_coef, (size_t)B.as + t);
            reinterpret_cast<EllRow *>(pre)[t] = e;
            if constexpr (ATOM && LAST) {
                EllRow f = ell_zero();
                if (t < B.an) f = ell_load(P.aell_idx, P.aell_coef, (size_t)B.as + t);
                reinterpret_cast<EllRow *>(pre + PRE_ELL)[t] = f;
            }
        }
        if constexpr (!ATOM)
            if (t < BM) {
                int2 q = make_int2(0, 0);
                if (t < B.bn) q = make_int2(P.rev[B.bs + t], (int)P.src_blk[B.bs + t]);
                reinterpret_cast<int2 *>(pre + PRE_ELL)[t] = q;
            }
    }
    __device__ __forceinline__ void take_pre(const BlockRow &B, const uint8_t *pre) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int i = 0; i < AUPT; ++i) {
            const int v = tid + NT * i, la = min(v / UPR, BLK_ATOMS - 1);
            aell[i] = reinterpret_cast<const EllRow *>(pre)[la];
            if constexpr (ATOM && LAST) gell[i] = reinterpret_cast<const EllRow *>(pre + PRE_ELL)[la];
        }
        if constexpr (!ATOM)
#pragma unroll
            for (int i = 0; i < UPT; ++i) {
                const int v = tid + NT * i, lr = min(v / UPR, BM - 1);
                const int2 q = reinterpret_cast<const int2 *>(pre + PRE_ELL)[lr];
                rv[i] = q.x;
                sa[i] = (uint32_t)q.y;
            }
    }

    // s = sum over the row's entries (ELL slots, then the CSR rest: natural ids, base = the block's first
    // row of the gathered kind; entries below it -- the atom-message pad slot -- skipped) of w * T[entry][c .. c + 7]
    __device__ __forceinline__ void row_sum(const int32_t *ptr, const int32_t *idx, const float *coef, int row, int base,
                                            const EllRow &E, int c, const float *T, float4 &s0, float4 &s1) {
        s0 = s1 = f4zero();
#pragma unroll
        for (int k = 0; k < ELLW; ++k)
            if (E.w[k] != 0.f) lds_term<LDC>(T, ell_idx(E, k), c, E.w[k], s0, s1);
        if (ell_more(E))
            for (int q = ptr[row] + ELLW; q < ptr[row + 1]; ++q) {
                const int li = idx[q] - base;
                if (li >= 0) lds_term<LDC>(T, li, c, coef ? coef[q] : 1.0f, s0, s1);
            }
    }
    // A[la][c..c+7] = sum over the atom's in-bonds of w * T[bond] (bond mode's atom gather)
    __device__ __forceinline__ void atom_sum(const MpLayerP &P, const BlockRow &B, const EllRow &E, int la, int c,
                                             const float *T, float4 &s0, float4 &s1) {
        row_sum(P.aptr, P.aidx, P.acoef, B.as + la, ATOM ? B.as : B.bs, E, c, T, s0, s1);
    }

    // Pt: the P tile [BM][LDC] fp32 in LDS (every write of it done and synchronised); At = Pt + BM * LDC
    template <int ACT>
    __device__ __forceinline__ void run(const MpLayerP &P, const BlockRow &B, int blk, int n0, float *Pt) {
        const int tid = threadIdx.x;
        float *At = Pt + BM * LDC;
        // message rows of this block: bonds, or atoms in atom-message mode
        const int rs = ATOM ? B.as : B.bs, rn = ATOM ? B.an : B.bn;
        constexpr int NU = ATOM ? AUNITS : UNITS, PT = ATOM ? AUPT : UPT;
        // residual rows (mpn.py:123 input): issued now, consumed after the gathers
        float4 res[PT][2];
#pragma unroll
        for (int i = 0; i < PT; ++i) {
            const int v = tid + NT * i, lr = v / UPR, c = 8 * (v % UPR);
            res[i][0] = res[i][1] = f4zero();
            if (v < NU && lr < rn) {
                const float *s = P.inp + (size_t)(rs + lr) * P.ldr + n0 + c;
                res[i][0] = ld4(s);
                res[i][1] = ld4(s + 4);
            }
        }
        if constexpr (!ATOM) {
            if (P.undirected) {  // P <- (P + P[rev]) / 2, one thread per reverse pair (the lower row)
#pragma unroll
                for (int i = 0; i < UPT; ++i) {
                    const int v = tid + NT * i, lr = v / UPR, c = 8 * (v % UPR);
                    const int rl = rv[i] - B.bs;
                    if (v < UNITS && lr < B.bn && lr < rl) {
                        float4 p0 = ld4(Pt + lr * LDC + c), p1 = ld4(Pt + lr * LDC + c + 4);
                        const float4 q0 = ld4(Pt + rl * LDC + c), q1 = ld4(Pt + rl * LDC + c + 4);
                        p0.x = (p0.x + q0.x) / 2.0f; p0.y = (p0.y + q0.y) / 2.0f;
                        p0.z = (p0.z + q0.z) / 2.0f; p0.w = (p0.w + q0.w) / 2.0f;
                        p1.x = (p1.x + q1.x) / 2.0f; p1.y = (p1.y + q1.y) / 2.0f;
                        p1.z = (p1.z + q1.z) / 2.0f; p1.w = (p1.w + q1.w) / 2.0f;
                        st4(Pt + lr * LDC + c, p0); st4(Pt + lr * LDC + c + 4, p1);
                        st4(Pt + rl * LDC + c, p0); st4(Pt + rl * LDC + c + 4, p1);
                    }
                }
                __syncthreads();
            }
            wd_stamp(4 + 8 * LAST);
            // A[a] = sum_{b into a} w_b P[b] (mpn.py:112-118)
#pragma unroll
            for (int i = 0; i < AUPT; ++i) {
                const int v = tid + NT * i, la = v / UPR, c = 8 * (v % UPR);
                if (v >= AUNITS || la >= B.an) break;
                float4 s0, s1;
                atom_sum(P, B, aell[i], la, c, Pt, s0, s1);
                st4(At + la * LDC + c, s0);
                st4(At + la * LDC + c + 4, s1);
            }
            __syncthreads();
            wd_stamp(5 + 8 * LAST);
        }
        const float slope = ACT == ACT_PRELU ? P.slope[0] : 0.f;
        float4 ym[LAST || POUT ? YPT : 1][2];  // LAST: this thread's M_t units until P is dead; POUT: until the scale is known
        // Z_t rows of this block (the training forward's save in the last layer)
        float *zr = LAST ? P.zsave : P.zout;
        const __amdgpu_buffer_rsrc_t zrs = __builtin_amdgcn_make_buffer_rsrc(zr ? (void *)(zr + (size_t)rs * P.kp) : (void *)P.inp, 0,
                                                                            BM * P.kp * 4, 0x00020000);
        uint32_t mx = 0;               // max |dropout(act(Z_t))| of this thread's units (not LAST)
#pragma unroll
        for (int i = 0; i < PT; ++i) {
            const int v = tid + NT * i, lr = v / UPR, c = 8 * (v % UPR);
            if (v >= NU) break;
            float4 y0 = f4zero(), y1 = f4zero();
            if (lr < rn) {
                const int b = rs + lr;
                float z[8];
                if constexpr (ATOM) {
                    // X[a] = sum_{a' in nbr(a)} P[a'] (mpn.py:104-108, the W_h[:, :H] part; the bond-feature
                    // part is in the residual)
                    float4 s0, s1;
                    row_sum(P.mptr, P.midx, P.mcoef, b, B.as, aell[i], c, Pt, s0, s1);
                    z[0] = s0.x; z[1] = s0.y; z[2] = s0.z; z[3] = s0.w; z[4] = s1.x; z[5] = s1.y; z[6] = s1.z; z[7] = s1.w;
                } else {
                    const int rl = rv[i] - B.bs, a = (int)sa[i];
                    // X[b] = A[src(b)] - P[rev(b)] (mpn.py:119-120)
                    const float4 a0 = ld4(At + a * LDC + c), a1 = ld4(At + a * LDC + c + 4);
                    const float4 q0 = ld4(Pt + rl * LDC + c), q1 = ld4(Pt + rl * LDC + c + 4);
                    z[0] = a0.x - q0.x; z[1] = a0.y - q0.y; z[2] = a0.z - q0.z; z[3] = a0.w - q0.w;
                    z[4] = a1.x - q1.x; z[5] = a1.y - q1.y; z[6] = a1.z - q1.z; z[7] = a1.w - q1.w;
                }
                float4 b0 = f4zero(), b1 = f4zero();
                if (P.bias) { b0 = ld4(P.bias + n0 + c); b1 = ld4(P.bias + n0 + c + 4); }
                const float r8[8] = {res[i][0].x, res[i][0].y, res[i][0].z, res[i][0].w,
                                     res[i][1].x, res[i][1].y, res[i][1].z, res[i][1].w};
                const float b8[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
                for (int q = 0; q < 8; ++q) z[q] = r8[q] + (z[q] + b8[q]);  // mpn.py:122-123
                if (zr) {  // (16-byte buffer stores)
                    const int o = (lr * P.kp + n0 + c) * 4;
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(z[0]), __float_as_uint(z[1]),
                                                                 __float_as_uint(z[2]), __float_as_uint(z[3])}, zrs, o, 0, WD_ZWT);
                    __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(z[4]), __float_as_uint(z[5]),
                                                                 __float_as_uint(z[6]), __float_as_uint(z[7])}, zrs, o + 16, 0, WD_ZWT);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) z[q] = act_fwd(ACT, z[q], slope);
                if (P.p_drop > 0.f)
#pragma unroll
                    for (int q = 0; q < 8; ++q) z[q] *= dropout_scale(P.seed, P.layer, b, n0 + c + q, P.p_drop);
                if constexpr (!LAST)
#pragma unroll
                    for (int q = 0; q < 8; ++q) mx = max(mx, absbits(z[q]));
                y0 = make_float4(z[0], z[1], z[2], z[3]);
                y1 = make_float4(z[4], z[5], z[6], z[7]);
            }
            if constexpr (LAST || POUT) {
                ym[i][0] = y0;
                ym[i][1] = y1;
            }
        }
        if constexpr (!LAST && POUT) {
            // M_t as fp16 pairs scaled by this tile's max (the next layer's A operand, copied by LDS-DMA)
            __shared__ uint32_t red[MP_THREADS / 64];
            const float s = h2_scale(publish_max_all(mx, P.amax_out + (size_t)blk * P.n_tiles + n0 / BN, red));
            constexpr int CH = 2 * BM * 64;
            const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
                P.aout + (size_t)blk * (P.kp >> 5) * CH, 0, (P.kp >> 5) * CH, 0x00020000);
#pragma unroll
            for (int i = 0; i < PT; ++i) {
                const int v = tid + NT * i, lr = v / UPR, c = 8 * (v % UPR);
                // (rows up to the end of the last 16-row group the consumers multiply: zeros past the block)
                if (v >= NU || lr >= ((rn + 15) & ~15)) break;
                h2_store8(prs, h2_blk_off<BM>(lr, n0 + c), BM * 64, ym[i][0], ym[i][1], s);
            }
        } else if constexpr (!LAST) {
            __shared__ uint32_t red[MP_THREADS / 64];
            publish_max(mx, P.amax_out + (size_t)blk * P.n_tiles + n0 / BN, red);
        }
        if constexpr (LAST) {
            __syncthreads();  // every read of P done: M_t replaces it
            float *Mt = Pt;
#pragma unroll
            for (int i = 0; i < PT; ++i) {
                const int v = tid + NT * i, lr = v / UPR, c = 8 * (v % UPR);
                if (v >= NU) break;
                st4(Mt + lr * LDC + c, ym[i][0]);
                st4(Mt + lr * LDC + c + 4, ym[i][1]);
            }
            __syncthreads();
            // atom aggregate of this column tile: A[a] = sum_{x into a} w M_t[x] (mpn.py:126-131; x: the
            // atom's in-bonds, or its a2a neighbours in atom-message mode)
            if (POUT && P.apairs) {
                // A as fp16 pairs scaled by this tile's max (rows to the end of the last 16-row group: zeros)
                float4 as[AUPT][2];
                uint32_t amx = 0;
#pragma unroll
                for (int i = 0; i < AUPT; ++i) {
                    const int v = tid + NT * i, la = v / UPR, c = 8 * (v % UPR);
                    as[i][0] = as[i][1] = f4zero();
                    if (v < AUNITS && la < B.an) {
                        atom_sum(P, B, aell[i], la, c, Mt, as[i][0], as[i][1]);
                        const float q[8] = {as[i][0].x, as[i][0].y, as[i][0].z, as[i][0].w,
                                            as[i][1].x, as[i][1].y, as[i][1].z, as[i][1].w};
#pragma unroll
                        for (int k = 0; k < 8; ++k) amx = max(amx, absbits(q[k]));
                    }
                }
                __shared__ uint32_t red[MP_THREADS / 64];
                const float s = h2_scale(publish_max_all(amx, P.amax_out + (size_t)blk * P.n_tiles + n0 / BN, red));
                constexpr int CHA = 2 * BLK_ATOMS * 64;
                const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
                    P.apairs + (size_t)blk * (P.kp >> 5) * CHA, 0, (P.kp >> 5) * CHA, 0x00020000);
#pragma unroll
                for (int i = 0; i < AUPT; ++i) {
                    const int v = tid + NT * i, la = v / UPR, c = 8 * (v % UPR);
                    if (v >= AUNITS || la >= ((B.an + 15) & ~15)) break;
                    h2_store8(prs, h2_blk_off<BLK_ATOMS>(la, n0 + c), BLK_ATOMS * 64, as[i][0], as[i][1], s);
                }
            } else {
            const __amdgpu_buffer_rsrc_t ars = x6_block_rsrc<BLK_ATOMS>(P.aplanes, P.kp, blk);
#pragma unroll
            for (int i = 0; i < AUPT; ++i) {
                const int v = tid + NT * i, la = v / UPR, c = 8 * (v % UPR);
                if (v >= AUNITS || la >= B.an) break;  // rows past the block's atoms are never loaded
                float4 s0, s1;
                if constexpr (ATOM) atom_sum(P, B, gell[i], la, c, Mt, s0, s1);
                else atom_sum(P, B, aell[i], la, c, Mt, s0, s1);
                x6_store8_blk<BLK_ATOMS>(ars, la, n0 + c, s0, s1);
                if (P.asave) {
                    float *ar = P.asave + (size_t)(B.as + la) * P.kp + n0 + c;
                    st4(ar, s0);
                    st4(ar + 4, s1);
                }
            }
            }
        }
    }
};

// grid = nblk * n_tiles (XCD-grouped: the column tiles of a block share an XCD), MP_THREADS threads.
// LDS: two GEMM stages, reused by the epilogue as P [128][BN + 4] fp32 + the atom sums; the last layer
// then overwrites P with M_t (held in registers across a barrier) for the atom aggregate.
// ACT: the activation (one instantiation each: the staging of M_{t-1} and the epilogue fold it to
// straight-line code).
template <int BN, bool LAST, int ACT, bool ATOM = false, int NJ = WD_MULTI, bool PAIRS = false>
// (__launch_bounds__ min 4 waves per SIMD: <= 128 VGPRs, so that two layer workgroups -- batches in flight
// on two streams -- co-reside on a CU)
__global__ __launch_bounds__(MP_THREADS, 4) void mp_layer_kernel(const Multi<MpLayerP, NJ> MP) {
    constexpr int BM = BLK_BONDS;
    using Epi_ = MpEpilogue<BN, MP_THREADS, LAST, ATOM, PAIRS>;
    constexpr int EPI_BYTES = Epi_::LDS_FLOATS * 4;  // P tile + the atom sums
    constexpr int STG_BYTES = PAIRS ? h2p_lds_bytes<BM, BN>() : h2_lds_bytes<BM, BN>();
    constexpr int LDS_BYTES = EPI_BYTES > STG_BYTES ? EPI_BYTES : STG_BYTES;
    static_assert(LDS_BYTES <= (PAIRS && H2P_STAGES > 3 ? 160 : 80) * 1024, "two workgroups per CU");
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    int tile;
    wd_stamp(0 + 8 * LAST);
    const MpLayerP &P = multi_pick(MP, xcd_tile(blockIdx.x, gridDim.x), tile);
    const int blk = tile / P.n_tiles, nt = tile % P.n_tiles, n0 = nt * BN;
    const BlockRow B = load_block(P.blocks, blk);
    Epi_ E;
    float *Pt = reinterpret_cast<float *>(lds);
    const int rs = ATOM ? B.as : B.bs, rn = ATOM ? B.an : B.bn;  // the block's message rows
    if constexpr (PAIRS) {
        static_assert(!ATOM, "pair operands: bond messages");
        // the epilogue's gather lists and ids, staged by the loader waves while the consumers multiply the
        // last chunk, in the tail of ring stage 2 (the last chunk lands in stage 0): clear of the P tile and
        // the atom sums the epilogue writes
        static_assert(EPI_BYTES + Epi_::PRE_BYTES <= STG_BYTES, "epilogue lists beside the P tile");
        uint8_t *pre = lds + STG_BYTES - Epi_::PRE_BYTES;
        const uint32_t wv = lane_word(P.amax_in + (size_t)blk * P.amax_in_n, P.amax_in_n);
        const uint32_t whm = *P.wh_amax;
        wd_stamp(1 + 8 * LAST);
        floatx4 acc[BM / 64][BN / 16];
        int se;
        constexpr int CH = 2 * BM * 64;
        h2_mainloop_pairs<BM, BN>(P.ain + (size_t)blk * (P.kp >> 5) * CH, P.wh + (size_t)nt * (P.kp >> 5) * (2 * BN * 64),
                                  P.kp >> 5, rn, wv, P.ain_g, lds, acc, se);
        wd_stamp(2 + 8 * LAST);
        if (threadIdx.x >= MP_THREADS / 2) E.fill_pre(P, B, pre);
        __syncthreads();
        E.take_pre(B, pre);
        wd_stamp(3 + 8 * LAST);
        if (threadIdx.x < 256) {  // (the consumer waves hold the tile)
            const float ia = se >= 0 ? __uint_as_float((uint32_t)(254 - se) << 23) : 1.f;
            x6_acc_to_lds_scaled<BM, BN, 4, 1>(acc, Pt, ia, h2_inv_scale(whm));
        }
        __syncthreads();
        E.template run<ACT>(P, B, blk, n0, Pt);
        wd_stamp(6 + 8 * LAST);
        if (blk == 0 && threadIdx.x < BN / 4) {  // (pad rows, as below)
            float *zr = LAST ? P.zsave : P.zout;
            if (zr) st4(zr + n0 + 4 * threadIdx.x, f4zero());
            if (LAST && P.asave) st4(P.asave + n0 + 4 * threadIdx.x, f4zero());
        }
    } else {
    // the block's scale words of M_{t-1} (<= 64, one per lane) and W_h's: loaded before the GEMM's first
    // loads, reduced by the producers before their first stage and by the consumers after the GEMM
    int w0 = blk * P.amax_in_n, wn = P.amax_in_n;
    if (P.amax_rt > 0) {  // (the row tiles of the block's rows)
        const int t0 = rs / P.amax_rt, t1 = (rs + max(rn, 1) - 1) / P.amax_rt;
        w0 = t0 * P.amax_in_n;
        wn = (t1 - t0 + 1) * P.amax_in_n;
    }
    const uint32_t wv = lane_word(P.amax_in + w0, wn);
    const uint32_t whm = *P.wh_amax;
    H2Prod<BM, ACT> ap(P, rs, rn, wv);
    wd_stamp(1 + 8 * LAST);
    floatx4 acc[BM / 64][BN / 16];
    h2_mainloop_ws<BM, BN>(P.wh + (size_t)nt * (P.kp >> 5) * (2 * BN * 64), P.kp >> 5, rn, lds, acc, ap);
    // the epilogue's gather lists and ids: not during the GEMM (live across the GEMM loop they pushed the
    // consumers' accumulators and fragments past 128 VGPRs); the staging waves load them into LDS while the
    // MFMA waves finish the last chunk
    wd_stamp(2 + 8 * LAST);
#ifndef WD_EPI_PRE
#define WD_EPI_PRE 1
#endif
    __shared__ __attribute__((aligned(16))) uint8_t pre[WD_EPI_PRE ? Epi_::PRE_BYTES : 16];
    static_assert(LDS_BYTES + (WD_EPI_PRE ? Epi_::PRE_BYTES : 0) + 64 <= 80 * 1024, "two workgroups per CU");
    if (WD_EPI_PRE) {
        if (threadIdx.x >= MP_THREADS / 2) E.fill_pre(P, B, pre);
    } else {
        E.prefetch(P, B);
    }
    __syncthreads();
    if (WD_EPI_PRE) E.take_pre(B, pre);
    wd_stamp(3 + 8 * LAST);
    const float ia = h2_inv_scale(wave_max_u32(wv));  // (the producers' scale)
    const float iw = h2_inv_scale(whm);
    if (threadIdx.x < 256) x6_acc_to_lds_scaled<BM, BN, 4, 1>(acc, Pt, ia, iw);  // (the consumer waves hold the tile)
    __syncthreads();
    E.template run<ACT>(P, B, blk, n0, Pt);
    wd_stamp(6 + 8 * LAST);
    // the pad row 0 (bond and atom) belongs to no block: its Z rows are written as zeros (the backward
    // multiplies them by its zero gradients, where an uninitialised NaN would poison them)
    if (blk == 0 && threadIdx.x < BN / 4) {
        float *zr = LAST ? P.zsave : P.zout;
        if (zr) st4(zr + n0 + 4 * threadIdx.x, f4zero());
        if (LAST && P.asave) st4(P.asave + n0 + 4 * threadIdx.x, f4zero());
    }
    }  // (register-staged path)
}

// ------------------------------------------------------------------------------------------------
// embed_kernel: the input layer (mpn.py:92-97) of a compact batch without a GEMM.  Every f_bonds row is
// its source atom's one-hot row + the bond's binary columns (+ mass * 0.01 in the atom's last column,
// featurization.py:190-250, 467-468), so f_bonds[b] W_i^T is a sum of W_i columns:
//     Ea[a]  = sum_{c in code(a)} W_i[:, c] + last(a) W_i[:, Fa-1]          (per atom of the block)
//     inp[b] = Ea[src(b)] + sum_{k in tail(b)} W_i[:, Fa + k] (+ b_i)       (per bond)
//     Eo[a]  = sum_{c in code(a)} W_o[:, c] + last(a) W_o[:, Fa-1]          (the f_atoms half of W_o)
// One workgroup per (block, BN-column tile), the tile's W_o[:, :Fa]^T and then W_i^T rows staged in LDS.
// Writes inp (fp32, natural rows: the residual of every layer, and the first layer's A operand, which
// applies the activation M_0 = act(inp) while staging) and Eo (fp32, blocked atom rows) for
// wo_readout_kernel's epilogue.  Every global load of the workgroup (atom
// codes, both weight tiles, the bonds' source atoms and tail bits) is issued up front, so the kernel
// waits for memory once.
// ------------------------------------------------------------------------------------------------
struct EmbedP {
    const WdAtomCode *codes;     // natural atom rows
    const uint8_t *src_blk;      // per natural bond row: block-local source atom
    const uint16_t *tail;        // per natural bond row: bond columns as bits
    const float *wt;             // W_i^T [>= Fb][Hk] (fp32, packed)
    const float *woat;           // W_o[:, :Fa]^T [>= Fa][Hk] (fp32, packed)
    float *eo;                   // [atom rows][Hk] (natural rows)
    const float *bias;           // b_i (padded) or null
    const int32_t *blocks;
    int Fa, Fb, Hk, n_tiles;
    float *inp;                  // [Rp][Hk]
    const float *slope;          // PReLU slope (or null)
    uint32_t *amax;              // [nblk][n_tiles]: max |act(inp)| per workgroup (the first layer's scale, planes.hpp h2)
    uint8_t *m0;                 // the template's PAIRS: M_0 = act(inp) as fp16 pair tiles of the molecule blocks
                                 // ([nblk][Hk / 32][2][128][64 B]), scaled by this workgroup's word (the first
                                 // layer's A operand, copied by LDS-DMA: mp_layer_kernel<..., PAIRS>)
};

// s = sum_{c in code} T[c][c4 .. c4+3] + last * T[Fa - 1][c4 ..] (ascending columns, then the mass column:
// the order of the f_atoms row's dot product terms that are not zero)
template <int LDT>
__device__ __forceinline__ float4 code_sum(const WdAtomCode &cd, const float *T, int Fa, int c) {
    float4 s = f4zero();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (cd.col[q] == 0xFF) continue;
        const float4 w = ld4(T + cd.col[q] * LDT + c);
        s.x += w.x; s.y += w.y; s.z += w.z; s.w += w.w;
    }
    fma4(s, cd.last, ld4(T + (Fa - 1) * LDT + c));
    return s;
}

// (EO_LAST measured, same box: embed 10.00 vs 10.25 us, the bench's single stream 119.2 vs 125.2 M, headline
// 202.7 vs 204.8 M -- not kept)
#ifndef WD_EMBED_EO_LAST
#define WD_EMBED_EO_LAST 0
#endif
template <int BN, int ACT, int NJ = WD_MULTI, bool PAIRS = false>
__global__ __launch_bounds__(512) void embed_kernel(const Multi<EmbedP, NJ> MP) {
    constexpr bool EO_LAST = WD_EMBED_EO_LAST;
    static_assert(!PAIRS || BN % 16 == 0, "pair groups of whole 16-column halves");
    constexpr int NT = 512, LDC = BN + 4, C4 = BN / 4, U8 = BN / 8, MAXK = 160, PER = (MAXK * C4 + NT - 1) / NT;
    constexpr int BU = (BLK_BONDS * U8 + NT - 1) / NT;  // bond units (8 columns of a row) per thread
    __shared__ __attribute__((aligned(16))) float wt[MAXK * BN];        // the staged W_i^T tile
    __shared__ __attribute__((aligned(16))) float ea[BLK_ATOMS * LDC];  // Ea of the block's atoms
    __shared__ __attribute__((aligned(16))) float bb[BN];
    __shared__ WdAtomCode code[BLK_ATOMS];
    static_assert(sizeof(float) * (MAXK * BN + BLK_ATOMS * LDC + BN) + sizeof(WdAtomCode) * BLK_ATOMS <= 80 * 1024,
                  "LDS of two co-resident workgroups");
    int tile;
    wd_estamp(0);
    const EmbedP &P = multi_pick(MP, xcd_tile(blockIdx.x, gridDim.x), tile);
    const int blk = tile / P.n_tiles, nt = tile % P.n_tiles, n0 = nt * BN;
    const BlockRow B = load_block(P.blocks, blk);
    const int tid = threadIdx.x;
    // every load up front, in the order their values are needed (codes and bias, the weight tile, the
    // bonds' source atoms and tails): each wait then covers only what it needs
    static_assert(sizeof(WdAtomCode) == 16, "codes move as one 16-byte word");
    u32x4 cd = {0u, 0u, 0u, 0u};  // (raw words: a struct with a byte array went to scratch)
    if (tid < B.an) cd = reinterpret_cast<const u32x4 *>(P.codes)[B.as + tid];
    float4 bq = f4zero();
    if (tid >= NT - C4 && P.bias) bq = ld4(P.bias + n0 + 4 * (tid - (NT - C4)));
    float4 ro[PER], ri[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int v = tid + NT * q, k = v / C4, c = 4 * (v % C4);
        ro[q] = k < P.Fa ? ld4(P.woat + (size_t)k * P.Hk + n0 + c) : f4zero();
        ri[q] = k < P.Fb ? ld4(P.wt + (size_t)k * P.Hk + n0 + c) : f4zero();
    }
    uint32_t sa[BU], tl[BU];
#pragma unroll
    for (int u = 0; u < BU; ++u) {
        const int v = tid + NT * u, lb = v / U8;
        sa[u] = tl[u] = 0;
        if (lb < B.bn) {
            sa[u] = P.src_blk[B.bs + lb];
            tl[u] = P.tail[B.bs + lb];
        }
    }
    if (tid < B.an) reinterpret_cast<u32x4 *>(code)[tid] = cd;
    if (tid >= NT - C4) st4(bb + 4 * (tid - (NT - C4)), bq);
    // (EO_LAST: the W_i tile and the layers' operand first, the f_atoms half of W_o -- for wo_readout, two
    // launches later -- while the M_0 stores drain)
    auto eo_half = [&]() {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int v = tid + NT * q, k = v / C4, c = 4 * (v % C4);
            if (k < P.Fa) st4(wt + k * BN + c, ro[q]);
        }
        __syncthreads();
        // Eo[a] = sum_{c in code(a)} W_o[:, c] + last(a) W_o[:, Fa-1] (the f_atoms half of W_o)
        for (int v = tid; v < B.an * C4; v += NT) {
            const int la = v / C4, c = 4 * (v % C4);
            st4(P.eo + (size_t)(B.as + la) * P.Hk + n0 + c, code_sum<BN>(code[la], wt, P.Fa, c));
        }
    };
    if constexpr (!EO_LAST) {
        eo_half();
        __syncthreads();  // every read of the W_o tile done
    }
    wd_estamp(2);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int v = tid + NT * q, k = v / C4, c = 4 * (v % C4);
        if (k < P.Fb) st4(wt + k * BN + c, ri[q]);
    }
    __syncthreads();
    wd_estamp(3);
    // Ea[a] = sum_{c in code(a)} W_i[:, c] + last(a) W_i[:, Fa-1]
    for (int v = tid; v < B.an * C4; v += NT) {
        const int la = v / C4, c = 4 * (v % C4);
        st4(ea + la * LDC + c, code_sum<BN>(code[la], wt, P.Fa, c));
    }
    __syncthreads();
    wd_estamp(4);
    const float slope = ACT == ACT_PRELU ? P.slope[0] : 0.f;
    uint32_t mx = 0;
    float4 ym[PAIRS ? BU : 1][2];  // PAIRS: this thread's act(inp) units until the scale is known
#pragma unroll
    for (int u = 0; u < (PAIRS ? BU : 1); ++u) ym[u][0] = ym[u][1] = f4zero();
#pragma unroll
    for (int u = 0; u < BU; ++u) {
        const int v = tid + NT * u, lb = v / U8, c = 8 * (v % U8), b = B.bs + lb;
        if (lb >= B.bn) break;
        const int s_ = (int)sa[u];
        float4 z0 = ld4(ea + s_ * LDC + c), z1 = ld4(ea + s_ * LDC + c + 4);
        for (uint32_t m = tl[u]; m; m &= m - 1) {
            const float *w = wt + (P.Fa + __builtin_ctz(m)) * BN + c;
            const float4 w0 = ld4(w), w1 = ld4(w + 4);
            z0.x += w0.x; z0.y += w0.y; z0.z += w0.z; z0.w += w0.w;
            z1.x += w1.x; z1.y += w1.y; z1.z += w1.z; z1.w += w1.w;
        }
        const float4 b0 = ld4(bb + c), b1 = ld4(bb + c + 4);
        z0.x += b0.x; z0.y += b0.y; z0.z += b0.z; z0.w += b0.w;
        z1.x += b1.x; z1.y += b1.y; z1.z += b1.z; z1.w += b1.w;
        float *zr = P.inp + (size_t)b * P.Hk + n0 + c;
        st4(zr, z0);
        st4(zr + 4, z1);
        float zz[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            zz[q] = act_fwd(ACT, zz[q], slope);
            mx = max(mx, absbits(zz[q]));
        }
        if constexpr (PAIRS) {
            ym[u][0] = make_float4(zz[0], zz[1], zz[2], zz[3]);
            ym[u][1] = make_float4(zz[4], zz[5], zz[6], zz[7]);
        }
    }
    if (blk == 0 && tid < C4) st4(P.inp + n0 + 4 * tid, f4zero());  // pad row 0 (Z_0 of the backward)
    wd_estamp(5);
    __shared__ uint32_t red[NT / 64];
    if constexpr (PAIRS) {
        // M_0 = act(inp) as fp16 pairs scaled by this tile's max (rows up to the end of the last 16-row group
        // the layer multiplies: zeros past the block)
        const float s = h2_scale(publish_max_all(mx, P.amax + (size_t)blk * P.n_tiles + nt, red));
        wd_estamp(6);
        constexpr int CH = 2 * BLK_BONDS * 64;
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            P.m0 + (size_t)blk * (P.Hk >> 5) * CH, 0, (P.Hk >> 5) * CH, 0x00020000);
#pragma unroll
        for (int u = 0; u < BU; ++u) {
            const int v = tid + NT * u, lb = v / U8, c = 8 * (v % U8);
            if (lb >= ((B.bn + 15) & ~15)) break;
            h2_store8(prs, h2_blk_off<BLK_BONDS>(lb, n0 + c), BLK_BONDS * 64, ym[u][0], ym[u][1], s);
        }
        wd_estamp(7);
    } else {
        publish_max(mx, P.amax + (size_t)blk * P.n_tiles + nt, red);
    }
    if constexpr (EO_LAST) {
        __syncthreads();  // every read of the W_i tile done (the bond units' tail sums)
        eo_half();
    }
}

constexpr int WO_MAXK = 160;  // f_atoms / f_bonds columns embed_kernel stages (Fa, Fb <= 160)

struct WoReadoutP {
    const uint8_t *fa; int kpa; int kca;     // f_atoms: blocked atom plane tiles [nblk * 64][kpa], kca chunks used
    int kcw;                                 // f_atoms chunks in the W_o plane tiles (Fak / 32; kca = 0 or kcw)
    const uint8_t *ag; int kp;               // A: blocked atom plane tiles [nblk * 64][kp = Hk]
    const uint8_t *wo;                       // W_o plane tiles [Hk][Fak + Hk] with BN-row blocks
    const float *bias;                       // b_o (padded)
    const int32_t *blocks;
    const float *w_atoms; const int32_t *mol_start, *mol_size; const float *xn;
    int agg; float norm; const float *zero_vec;
    int act; const float *slope; float p_drop; uint64_t seed; uint32_t layer;
    float *out; int ncols;                   // out [B][ncols] (ncols = H)
    int n_tiles;
    // kca = 0: the f_atoms half of [f_atoms | A] W_o^T, precomputed per atom (by embed_kernel as sums of
    // W_o columns, or by the atom-message input GEMM): fp32 natural atom rows, row stride ldeo (null: GEMM
    // segment)
    const float *eo;
    int Hk, ldeo;
    float *zosave;  // training forward or null: the W_o pre-activation (mpn.py:133) as fp32 natural atom rows [Vap][Hk]
    // the template's PAIRS (round 6): A as fp16 pair tiles of the blocks' atom rows ([nblk][Hk / 32][2][64][64 B],
    // written by the last layer) with its words [nblk][a_nw] (groups of a_g columns), and W_o[:, Fa:] as fp16
    // pair tiles with BN-row blocks scaled by the word wo_amax (wdmpnn_pack_params)
    const uint8_t *apairs; const uint32_t *a_amax; int a_nw, a_g;
    const uint8_t *woh; const uint32_t *wo_amax;
};

template <int BN> struct WoWaves;
template <> struct WoWaves<64> { static constexpr int WM = 4, WN = 2; };
template <> struct WoWaves<80> { static constexpr int WM = 2, WN = 5; };

// grid = nblk * n_tiles: 64 atom rows x BN columns per workgroup.  CPS: K chunks per LDS stage (one
// barrier per CPS chunks; two stages).  80-column tiles: CPS 2 (W_o's 64-row chunks are short: one barrier
// per chunk cost 0.6 us alone on the chip, 12.5 vs 13.1 us) for launches of several batches, where
// workgroups queue per CU; CPS 1 (55 KB of LDS) for one batch, whose 256 workgroups then co-reside
// with the layer kernels of batches in flight on other streams (+5 % with two streams, same-box A/B,
// profiles/round3_*).  64-column tiles: CPS 1.
// PAIRS (round 6): the GEMM on fp16 pair tiles of A and W_o (gemm_x6.hpp h2_mainloop_pairs: 4 MFMA waves of
// 16 atom rows, 4 waves copying A; three products per fp32 product instead of the planes' six), 512 threads.
template <int BN, int CPS, int NJ = WD_MULTI, bool PAIRS = false>
// (PAIRS: <= 128 VGPRs, two workgroups per CU beside other streams' layers)
__global__ __launch_bounds__(PAIRS ? 512 : 64 * WoWaves<BN>::WM * WoWaves<BN>::WN, PAIRS ? 4 : 1) void wo_readout_kernel(const Multi<WoReadoutP, NJ> MP) {
    // (PAIRS: WM x WN = 4 x 1 MFMA waves, and four more copying A: NT = 512)
    constexpr int BM = BLK_ATOMS, LDC = BN + 4, WM = PAIRS ? 4 : WoWaves<BN>::WM, WN = PAIRS ? 1 : WoWaves<BN>::WN;
    constexpr int NT = PAIRS ? 512 : 64 * WM * WN;
    // (deeper single-chunk pipelines, with the mainloop hook's loads ordered ahead of the partial vmcnt
    // waits, measured slower: three / four stages 15.1 / 14.8 us here, 12.8 / 11.8 against 9.7 us on
    // QM9-shaped batches)
    constexpr int WS = 2;  // LDS stages
    constexpr int EPI_BYTES = (BM * LDC + BM + 3 * BLK_MOLS + BN) * 4;  // (+ the bias columns: PAIRS)
    constexpr int LDS_BYTES = PAIRS ? (h2p_lds_bytes<BM, BN>() > EPI_BYTES ? h2p_lds_bytes<BM, BN>() : EPI_BYTES)
                                    : WS * CPS * x6_stage_bytes<BM, BN>();
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    int tile;
    const WoReadoutP &P = multi_pick(MP, xcd_tile(blockIdx.x, gridDim.x), tile);
    const int blk = tile / P.n_tiles, nt = tile % P.n_tiles, n0 = nt * BN;
    const BlockRow B = load_block(P.blocks, blk);
    const int tid = threadIdx.x;
    X6Operands O{};
    O.a0 = P.fa; O.nkc0 = P.kpa >> 5; O.kc0 = P.kca;
    O.a1 = P.ag; O.nkc1 = P.kp >> 5; O.kc1 = P.kp >> 5;
    O.rb = blk;
    O.a_rows = B.an;
    // W_o planes: per BN-row block, kcw f_atoms chunks then kp / 32 A chunks; the f_atoms chunks are
    // skipped when the codes path adds that half in the epilogue (kca = 0)
    O.b = P.wo + ((size_t)nt * (P.kcw + (P.kp >> 5)) + (P.kcw - P.kca)) * (3 * BN * 64);
    // prefetched during the GEMM (mainloop hook): this thread's bias columns, the block's atom weights
    // (thread a < an: w_atoms[as + a]) and its molecules' scope / Xn (thread i < nm)
    constexpr int C4 = BN / 4;
    static_assert((PAIRS || NT % C4 == 0) && BM <= NT, "one bias group per thread, one atom weight per thread");
    const int nm = min(B.mh - B.ml, BLK_MOLS);  // (the packer never exceeds BLK_MOLS)
    if (P.zosave && blk == 0 && tid < BN / 4) st4(P.zosave + n0 + 4 * tid, f4zero());  // pad atom row 0
    float4 bb = f4zero();
    float watom = 0.f, mxn = 0.f;
    int mstart = 0, msize = 0;
    // codes path: this thread's rows of the precomputed f_atoms W_o[:, :Fa]^T (the epilogue units below)
    constexpr int EPU = (BM * C4 + NT - 1) / NT;
    float4 eo[EPU];
    auto prefetch = [&](int phase) {
        if (phase != 0) return;
        if (!PAIRS || tid < C4) bb = ld4(P.bias + n0 + 4 * (tid % C4));  // (PAIRS: staged through LDS below)
        if (tid < B.an) watom = P.w_atoms[B.as + tid];
#pragma unroll
        for (int j = 0; j < EPU; ++j) {
            const int v = tid + NT * j, la = v / C4, c = 4 * (v % C4);
            eo[j] = P.eo && v < BM * C4 && la < B.an ? ld4(P.eo + (size_t)(B.as + la) * P.ldeo + n0 + c) : f4zero();
        }
        if (tid < nm) {
            mstart = P.mol_start[B.ml + tid];
            msize = P.mol_size[B.ml + tid];
            mxn = P.xn[B.ml + tid];
        }
    };
    float *H = reinterpret_cast<float *>(lds);
    floatx4 acc[BM / WM / 16][BN / WN / 16];
    if constexpr (PAIRS) {
        prefetch(0);  // (registers across the GEMM: 16 rows per MFMA wave leave room)
        const uint32_t wv = threadIdx.x < 256 ? lane_word(P.a_amax + (size_t)blk * P.a_nw, P.a_nw) : 0u;
        int se;
        h2_mainloop_pairs<BM, BN>(P.apairs + (size_t)blk * (P.kp >> 5) * (2 * BM * 64),
                                  P.woh + (size_t)nt * (P.kp >> 5) * (2 * BN * 64), P.kp >> 5, B.an, wv, P.a_g, lds,
                                  acc, se);
        __syncthreads();
        if (threadIdx.x < 256)
            x6_acc_to_lds_scaled<BM, BN, 4, 1>(acc, H, se >= 0 ? __uint_as_float((uint32_t)(254 - se) << 23) : 1.f,
                                               h2_inv_scale(*P.wo_amax));
    } else {
        x6_mainloop<BM, BN, WM, WN, WS, CPS>(O, lds, acc, prefetch);
        __syncthreads();
        x6_acc_to_lds<BM, BN, WM, WN>(acc, H);
    }
    float *Wl = H + BM * LDC;           // [BM] atom weights of the block
    float *Ml = Wl + BM;                // [3][BLK_MOLS] per molecule: start (as float bits), size, Xn
    static_assert(EPI_BYTES <= LDS_BYTES, "readout staging fits");
    static_assert(BLK_MOLS <= NT, "one molecule per thread in the prefetch");
    if (tid < BM) Wl[tid] = watom;
    if (PAIRS && tid < C4) st4(Ml + 3 * BLK_MOLS + 4 * tid, bb);
    if (tid < nm) {
        Ml[tid] = __int_as_float(mstart);
        Ml[BLK_MOLS + tid] = __int_as_float(msize);
        Ml[2 * BLK_MOLS + tid] = mxn;
    }
    __syncthreads();
    // h = act(. + b_o) (* dropout), in place (mpn.py:133-134)
    with_act(P.act, [&](auto act_c) {
        constexpr int ACT = decltype(act_c)::value;
        const float slope = ACT == ACT_PRELU ? P.slope[0] : 0.f;
#pragma unroll
        for (int j = 0; j < EPU; ++j) {
            const int v = tid + NT * j;
            if (v >= BM * C4) break;
            const int la = v / C4, c = 4 * (v % C4);
            float4 hv = ld4(H + la * LDC + c);
            hv.x += eo[j].x; hv.y += eo[j].y; hv.z += eo[j].z; hv.w += eo[j].w;  // (0 without codes)
            // (PAIRS, 512 threads: NT % C4 != 0, each unit its own bias columns, from LDS)
            const float4 b4 = PAIRS ? ld4(Ml + 3 * BLK_MOLS + c) : bb;
            float z[4] = {hv.x + b4.x, hv.y + b4.y, hv.z + b4.z, hv.w + b4.w};
            if (P.zosave && la < B.an) st4(P.zosave + (size_t)(B.as + la) * P.Hk + n0 + c, make_float4(z[0], z[1], z[2], z[3]));
#pragma unroll
            for (int q = 0; q < 4; ++q) z[q] = act_fwd(ACT, z[q], slope);
            if (P.p_drop > 0.f && la < B.an)
#pragma unroll
                for (int q = 0; q < 4; ++q) z[q] *= dropout_scale(P.seed, P.layer, B.as + la, n0 + c + q, P.p_drop);
            st4(H + la * LDC + c, make_float4(z[0], z[1], z[2], z[3]));
        }
    });
    __syncthreads();
    // readout (mpn.py:145-171) of this block's molecules, columns n0 .. n0 + BN - 1: eight lanes per
    // (molecule, column), lane j summing the molecule's atoms j, j + 8, ... from LDS, then a fixed xor
    // butterfly over the eight lanes (deterministic; every lane ends with the same sum)
    constexpr int RP = 8;
    static_assert(NT % RP == 0 && 64 % RP == 0, "lane groups stay inside a wave");
    for (int t = tid; t < nm * BN * RP; t += NT) {
        const int part = t % RP, u = t / RP, im = u / BN, i = B.ml + im, cc = u % BN, col = n0 + cc;
        const int n = __float_as_int(Ml[BLK_MOLS + im]);
        float s = 0.f, wsum = 0.f;
        const int a0 = __float_as_int(Ml[im]) - B.as;
        for (int a = part; a < n; a += RP) {
            const float w = Wl[a0 + a];
            s = fmaf(w, H[(a0 + a) * LDC + cc], s);
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
            v = P.zero_vec[col];  // cached_zero_vector, no Xn factor (mpn.py:148-149)
        } else {
            const float m = P.agg == 0 ? s / wsum : (P.agg == 2 ? s / P.norm : s);
            v = Ml[2 * BLK_MOLS + im] * m;
        }
        P.out[(size_t)i * P.ncols + col] = v;
    }
}

}  // namespace wd
