// graph_build.hpp — the whole device graph (WdGraph) of a compact batch, built on the GPU in one launch
// (format: include/wdmpnn.h "Compact graphs").
//
// One workgroup per molecule block (<= 128 directed bonds, <= 64 atoms, <= 64 molecules: every index of
// the block is block-local, so the in-lists are built in LDS) plus one workgroup for the pad rows.
// It reproduces, value for value and entry for entry, what the host path builds:
//   * feature rows: f_atoms[a] = one-hot columns from the atom code + the last column's value
//     (featurization.py:190-211), f_bonds[b] = f_atoms[src(b)] ‖ bond columns (featurization.py:467-468,
//     545-546, 616-617), fp32 with 16-byte aligned rows, and their bf16x3 plane tiles (planes.hpp):
//     natural rows (BR 64) and, for atoms, the molecule-blocked layout of the fused W_o;
//   * in(a) = the bonds into a in creation order (= a2b[a], featurization.py:471-476, 624-627);
//   * msg_gather row b (mpn.py:112-120): j in in(src(b)), coefficient w_j - [j == rev(b)] (w - 1 is a
//     single fp32 rounding, as the host's double-then-float), zero coefficients dropped;
//     atom_gather row a (mpn.py:126-131): j in in(a), coefficient w_j != 0;
//     their transposes (the backward's gathers): msg_gather_t row j = the rows b with src(b) = dst(j) in
//     increasing b, atom_gather_t row j = (dst(j), w_j);
//   * the ELL-8 rows, the block maps, b2revb, w_atoms and the molecule scope arrays.
// A lean graph (WDMPNN_GRAPH_LEAN) gets only what the fused inference forward reads: the atom gather
// (CSR + ELL), the block maps, b2revb, the bonds' source atoms and tails, the scope arrays.
// Pair structure: bond ids 1 + 2p and 2 + 2p are pair p's b1 = a1 -> a2 and b2 = a2 -> a1 (pad bond 0),
// so every molecule's first bond id is odd and a block-local bond index lb has rev(lb) = lb ^ 1.
#pragma once
#include "planes.hpp"
#include "wdmpnn.h"

namespace wd {

constexpr int GB_BONDS = 128, GB_ATOMS = 64, GB_MOLS = 64, GB_ELLW = 8, GB_CSR_PAD = 8;
// workgroups per block for a full (non-lean) build: slice 0 builds the block's structure (in-lists, CSR,
// ELL, maps) and every slice writes a quarter of its feature rows and planes -- with one workgroup per
// block a B = 64 batch (65 workgroups) wrote its ~30 MB from a quarter of the CUs (48 us, 0.08 of HBM)
constexpr int GB_SLICES = 4;

struct GraphBuildP {
    WdCompact c;
    int Fa, Fb, lda, ldb, Vap, Rbp;
    float *f_atoms, *f_bonds;
    uint8_t *fa_x6, *fb_x6, *fa_blk_x6;
    float *w_atoms, *xn;
    int32_t *mol_start, *mol_size, *b2revb, *blocks, *bond_blk_row, *atom_blk_row;
    uint8_t *bond_src_blk;
    uint16_t *bond_tail;
    uint8_t *msg_ell_idx, *agg_ell_idx;
    float *msg_ell_coef, *agg_ell_coef;
    int32_t *msg_ptr, *msg_idx, *agg_ptr, *agg_idx, *msgt_ptr, *msgt_idx, *aggt_ptr, *aggt_idx;
    float *msg_coef, *agg_coef, *msgt_coef, *aggt_coef;
    int lean;    // 1: no dense feature rows / planes and no transposed gathers (inference-only graph)
    int planes;  // 0: no plane tiles of the feature rows (WDMPNN_GRAPH_NO_PLANES)
};

// value of f_atoms column c for an atom code (c < Fa)
__device__ __forceinline__ float code_value(const WdAtomCode &a, int c, int Fa) {
    if (c == Fa - 1) return a.last;
    bool hit = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) hit |= a.col[k] == c;
    return hit ? 1.f : 0.f;
}

// 8 consecutive columns c0 .. c0 + 7 of a natural fp32 row + its plane tiles (BR 64; planes null: none)
__device__ __forceinline__ void put_row8(float *row_f32, uint8_t *planes, int ld, int r, int c0, const float (&v)[8]) {
    const float4 lo = make_float4(v[0], v[1], v[2], v[3]), hi = make_float4(v[4], v[5], v[6], v[7]);
    st4(row_f32 + c0, lo);
    st4(row_f32 + c0 + 4, hi);
    if (planes) x6_store8<64>(planes, ld, r, c0, lo, hi);
}

// the block's in-lists, gather CSRs (+ transposes) and ELL rows (slice 0 of a block's workgroups; the
// endpoint arrays are in LDS, every thread of the workgroup calls this)
__device__ __forceinline__ void build_structure(const GraphBuildP &P, int k, int bs, int bn, int as, int an,
                                                const uint8_t *s_src, const uint8_t *s_dst, uint8_t *s_in,
                                                uint8_t *s_out, const float *s_w, int *s_start, int *s_pm, int *s_pt,
                                                int *s_pg, int *s_pa, const int *s_off) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    (void)k;
    // in(a) / out(a) in creation order by counting sort: a bond's slot = start of its atom + the number of
    // earlier bonds with the same endpoint (16-byte broadcast reads of the endpoint arrays: no serial
    // loops over the block's bonds); every pair gives each endpoint one in- and one out-bond, so
    // |in(a)| = |out(a)| = deg(a)
    auto count_eq = [](const uint8_t *arr, int v, int below) {
        int n = 0;
        for (int q = 0; q < GB_BONDS / 16 && 16 * q < below; ++q) {
            const uint4 w = *reinterpret_cast<const uint4 *>(arr + 16 * q);
            const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int u = 0; u < 16; ++u)
                n += ((wd[u >> 2] >> (8 * (u & 3))) & 0xFF) == (uint32_t)v && 16 * q + u < below;
        }
        return n;
    };
    if (wave == 0) {  // deg + exclusive prefix over the atoms (one wave)
        const int d = lane < an ? count_eq(s_dst, lane, bn) : 0;
        int incl = d;
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        if (lane < an) s_start[lane] = incl - d;
        if (lane == 63) s_start[an] = incl;  // (an <= 64: lanes >= an add 0)
    }
    __syncthreads();
    if (tid < bn) {
        s_in[s_start[s_dst[tid]] + count_eq(s_dst, s_dst[tid], tid)] = (uint8_t)tid;
        s_out[s_start[s_src[tid]] + count_eq(s_src, s_src[tid], tid)] = (uint8_t)tid;
    }
    __syncthreads();
    // entry counts: msg row, msg_t row, agg_t row (bonds); agg row (atoms)
    if (tid < bn) {
        const int s = s_src[tid], rev = tid ^ 1;
        int cm = 0;
        for (int e = s_start[s]; e < s_start[s + 1]; ++e) {
            const int j = s_in[e];
            cm += (j == rev ? s_w[j] - 1.0f : s_w[j]) != 0.f;
        }
        // msg_t row: the rows lb in out(dst(tid)); every one has coefficient w - [lb == rev(tid)], and
        // rev(tid) is among them (src(rev) = dst(tid))
        const int nout = s_start[s_dst[tid] + 1] - s_start[s_dst[tid]];
        s_pm[tid + 1] = cm;
        s_pt[tid + 1] = (nout - 1) * (s_w[tid] != 0.f) + (s_w[tid] - 1.0f != 0.f);
        s_pg[tid + 1] = s_w[tid] != 0.f;
    }
    if (tid < an) {
        int ca = 0;
        for (int e = s_start[tid]; e < s_start[tid + 1]; ++e) ca += s_w[s_in[e]] != 0.f;
        s_pa[tid + 1] = ca;
    }
    __syncthreads();
    if (wave < 4) {  // four exclusive prefix sums, one wave each (two elements per lane)
        int *pre = wave == 0 ? s_pm : wave == 1 ? s_pt : wave == 2 ? s_pg : s_pa;
        const int n = wave == 3 ? an : bn;
        const int e0 = 2 * lane + 1, e1 = 2 * lane + 2;
        const int a = e0 <= n ? pre[e0] : 0, c = e1 <= n ? pre[e1] : 0;
        int incl = a + c;
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o, 64);
            if (lane >= o) incl += t;
        }
        const int base = incl - a - c;
        if (e0 <= n) pre[e0] = base + a;
        if (e1 <= n) pre[e1] = base + a + c;
        if (lane == 0) pre[0] = 0;
    }
    __syncthreads();
    const int om = s_off[0], oa = s_off[1];
    if (tid < bn && !P.lean) {  // (a lean graph serves only the fused forward, which gathers by src / rev)
        const int b = bs + tid, s = s_src[tid], rev = tid ^ 1;
        // msg_gather row b + its ELL-8 row
        int o = om + s_pm[tid], n = 0;
        uint8_t eidx[GB_ELLW];
        float ecoef[GB_ELLW];
#pragma unroll
        for (int q = 0; q < GB_ELLW; ++q) { eidx[q] = 0; ecoef[q] = 0.f; }
        for (int e = s_start[s]; e < s_start[s + 1]; ++e) {
            const int j = s_in[e];
            const float c = j == rev ? s_w[j] - 1.0f : s_w[j];
            if (c == 0.f) continue;
            P.msg_idx[o] = bs + j;
            P.msg_coef[o] = c;
            ++o;
            if (n < GB_ELLW) { eidx[n] = (uint8_t)j; ecoef[n] = c; }
            ++n;
        }
        P.msg_ptr[b + 1] = om + s_pm[tid + 1];
        if (n > GB_ELLW) eidx[GB_ELLW - 1] |= 0x80;
#pragma unroll
        for (int q = 0; q < GB_ELLW; ++q) {
            P.msg_ell_idx[(size_t)GB_ELLW * b + q] = eidx[q];
            P.msg_ell_coef[(size_t)GB_ELLW * b + q] = ecoef[q];
        }
        {
            // msg_gather_t row b: the rows lb in out(dst(b)), increasing lb
            o = om + s_pt[tid];
            const int d = s_dst[tid];
            for (int e = s_start[d]; e < s_start[d + 1]; ++e) {
                const int lb = s_out[e];
                const float c = tid == (lb ^ 1) ? s_w[tid] - 1.0f : s_w[tid];
                if (c == 0.f) continue;
                P.msgt_idx[o] = bs + lb;
                P.msgt_coef[o] = c;
                ++o;
            }
            P.msgt_ptr[b + 1] = om + s_pt[tid + 1];
            // atom_gather_t row b: (dst(b), w_b)
            if (s_w[tid] != 0.f) {
                P.aggt_idx[oa + s_pg[tid]] = as + s_dst[tid];
                P.aggt_coef[oa + s_pg[tid]] = s_w[tid];
            }
            P.aggt_ptr[b + 1] = oa + s_pg[tid + 1];
        }
    }
    if (tid < an) {  // atom_gather row a + its ELL-8 row
        const int a = as + tid;
        int o = oa + s_pa[tid], n = 0;
        uint8_t eidx[GB_ELLW];
        float ecoef[GB_ELLW];
#pragma unroll
        for (int q = 0; q < GB_ELLW; ++q) { eidx[q] = 0; ecoef[q] = 0.f; }
        for (int e = s_start[tid]; e < s_start[tid + 1]; ++e) {
            const int j = s_in[e];
            if (s_w[j] == 0.f) continue;
            P.agg_idx[o] = bs + j;
            P.agg_coef[o] = s_w[j];
            ++o;
            if (n < GB_ELLW) { eidx[n] = (uint8_t)j; ecoef[n] = s_w[j]; }
            ++n;
        }
        P.agg_ptr[a + 1] = oa + s_pa[tid + 1];
        if (n > GB_ELLW) eidx[GB_ELLW - 1] |= 0x80;
#pragma unroll
        for (int q = 0; q < GB_ELLW; ++q) {
            P.agg_ell_idx[(size_t)GB_ELLW * a + q] = eidx[q];
            P.agg_ell_coef[(size_t)GB_ELLW * a + q] = ecoef[q];
        }
    }
}

// grid: per batch its n_blocks + 1 workgroups (Multi: up to WD_MULTI batches per launch) x gridDim.y
// slices (GB_SLICES for full builds, 1 for lean ones)
__global__ __launch_bounds__(256) void graph_build_kernel(const Multi<GraphBuildP> MP) {
    int k;
    const GraphBuildP &P = multi_pick(MP, (int)blockIdx.x, k);
    const int tid = threadIdx.x, sl = blockIdx.y, nsl = gridDim.y;
    const WdCompact &C = P.c;
    const int Fa = P.Fa, Fb = P.Fb, UA = P.lda / 8, UB = P.ldb / 8;
    if (k == C.n_blocks && sl != 0) return;
    if (k == C.n_blocks) {  // pad rows: atom / bond row 0, the rows up to the padded extents, CSR heads and tails
        const int V1 = C.n_atoms, E1 = C.n_bonds;
        const int na_pad = 1 + (P.Vap - V1), nb_pad = 1 + (P.Rbp - E1);
        const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int u = tid; u < (P.lean ? 0 : na_pad * UA); u += 256) {
            const int i = u / UA, r = i == 0 ? 0 : V1 + i - 1, c0 = (u % UA) * 8;
            put_row8(P.f_atoms + (size_t)r * P.lda, P.fa_x6, P.lda, r, c0, z);
        }
        for (int u = tid; u < (P.lean ? 0 : nb_pad * UB); u += 256) {
            const int i = u / UB, r = i == 0 ? 0 : E1 + i - 1, c0 = (u % UB) * 8;
            put_row8(P.f_bonds + (size_t)r * P.ldb, P.fb_x6, P.ldb, r, c0, z);
        }
        for (int i = tid; i < na_pad; i += 256) {
            const int r = i == 0 ? 0 : V1 + i - 1;
            P.atom_blk_row[r] = -1;
            for (int s = 0; s < GB_ELLW; ++s) { P.agg_ell_idx[GB_ELLW * r + s] = 0; P.agg_ell_coef[GB_ELLW * r + s] = 0.f; }
        }
        for (int i = tid; i < nb_pad; i += 256) {
            const int r = i == 0 ? 0 : E1 + i - 1;
            P.bond_blk_row[r] = -1;
            P.bond_src_blk[r] = 0;
            P.bond_tail[r] = 0;
            if (!P.lean)
                for (int s = 0; s < GB_ELLW; ++s) { P.msg_ell_idx[GB_ELLW * r + s] = 0; P.msg_ell_coef[GB_ELLW * r + s] = 0.f; }
        }
        if (tid < 2) {  // row 0 (pad atom / bond) has no entries
            P.agg_ptr[tid] = 0;
            if (!P.lean) { P.msg_ptr[tid] = 0; P.msgt_ptr[tid] = 0; P.aggt_ptr[tid] = 0; }
        }
        if (tid == 0) { P.w_atoms[0] = 0.f; P.b2revb[0] = 0; }
        if (tid < GB_CSR_PAD) {  // readable dummy entries past the end (WdCsr)
            P.agg_idx[C.nnz_agg + tid] = 0; P.agg_coef[C.nnz_agg + tid] = 0.f;
            if (!P.lean) {
                P.msg_idx[C.nnz_msg + tid] = 0; P.msg_coef[C.nnz_msg + tid] = 0.f;
                P.msgt_idx[C.nnz_msg + tid] = 0; P.msgt_coef[C.nnz_msg + tid] = 0.f;
                P.aggt_idx[C.nnz_agg + tid] = 0; P.aggt_coef[C.nnz_agg + tid] = 0.f;
            }
        }
        return;
    }

    __shared__ int s_blk[8];
    __shared__ int s_mas[GB_MOLS], s_mbs[GB_MOLS];
    __shared__ WdAtomCode s_code[GB_ATOMS];
    __shared__ __attribute__((aligned(16))) uint8_t s_src[GB_BONDS], s_dst[GB_BONDS];
    __shared__ uint8_t s_in[GB_BONDS], s_out[GB_BONDS];
    __shared__ uint16_t s_tail[GB_BONDS];
    __shared__ float s_w[GB_BONDS];
    __shared__ int s_start[GB_ATOMS + 1];  // in(a) = s_in[s_start[a] ..), out(a) = s_out[s_start[a] ..)
    __shared__ int s_pm[GB_BONDS + 1], s_pt[GB_BONDS + 1], s_pg[GB_BONDS + 1], s_pa[GB_ATOMS + 1];
    __shared__ int s_off[2];
    if (tid < 8) s_blk[tid] = C.blocks[8 * k + tid];
    if (tid < 2) s_off[tid] = C.block_nnz[2 * k + tid];
    __syncthreads();
    const int bs = s_blk[0], bn = s_blk[1], as = s_blk[2], an = s_blk[3], ml = s_blk[4], nm = s_blk[5] - s_blk[4];
    if (bn > GB_BONDS || an > GB_ATOMS || nm > GB_MOLS || nm < 0) return;  // the host plan never does this
    const bool head = sl == 0;  // the slice that writes the block's structure
    if (tid < nm) {
        s_mas[tid] = C.mols[4 * (ml + tid)];
        s_mbs[tid] = C.mols[4 * (ml + tid) + 2];
        if (head) {
            P.mol_start[ml + tid] = C.mols[4 * (ml + tid)];
            P.mol_size[ml + tid] = C.mols[4 * (ml + tid) + 1];
            P.xn[ml + tid] = C.xn[ml + tid];
        }
    }
    if (tid < an) {
        s_code[tid] = C.atoms[as + tid];
        if (head) {
            P.w_atoms[as + tid] = s_code[tid].w;
            P.atom_blk_row[as + tid] = GB_ATOMS * k + tid;
        }
    }
    if (tid < 8 && head) P.blocks[8 * k + tid] = s_blk[tid];
    if (tid >= bn && tid < GB_BONDS) s_src[tid] = s_dst[tid] = 0xFF;  // never equal to an atom of the block
    __syncthreads();
    if (tid < bn) {  // endpoints of bond b = bs + tid
        const int b = bs + tid;
        int lo = 0, hi = nm - 1;  // the molecule: last one whose first bond is <= b
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_mbs[mid] <= b) lo = mid; else hi = mid - 1;
        }
        const int p = (b - 1) >> 1, dir = (b - 1) & 1;
        const WdBondPair q = C.pairs[p];
        const int l1 = s_mas[lo] + q.a1 - as, l2 = s_mas[lo] + q.a2 - as;
        s_src[tid] = (uint8_t)(dir ? l2 : l1);
        s_dst[tid] = (uint8_t)(dir ? l1 : l2);
        s_w[tid] = dir ? q.w21 : q.w12;
        s_tail[tid] = q.tail;
        if (head) {
            P.b2revb[b] = dir ? b - 1 : b + 1;
            P.bond_blk_row[b] = GB_BONDS * k + tid;
            P.bond_src_blk[b] = (uint8_t)(dir ? l2 : l1);
            P.bond_tail[b] = q.tail;
        }
    }
    __syncthreads();
    if (head) build_structure(P, k, bs, bn, as, an, s_src, s_dst, s_in, s_out, s_w, s_start, s_pm, s_pt, s_pg, s_pa, s_off);
    if (P.lean) return;
    // feature rows (8 columns per thread-step, slice sl of them): atoms natural + blocked (zero rows past
    // an), bonds natural
    for (int u = tid + 256 * sl; u < GB_ATOMS * UA; u += 256 * nsl) {
        const int la = u / UA, c0 = (u % UA) * 8;
        float v[8];
        if (la < an) {
            const WdAtomCode &cd = s_code[la];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = c0 + q < Fa ? code_value(cd, c0 + q, Fa) : 0.f;
            put_row8(P.f_atoms + (size_t)(as + la) * P.lda, P.fa_x6, P.lda, as + la, c0, v);
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = 0.f;
        }
        if (P.fa_blk_x6)
            x6_store8<64>(P.fa_blk_x6, P.lda, GB_ATOMS * k + la, c0, make_float4(v[0], v[1], v[2], v[3]),
                          make_float4(v[4], v[5], v[6], v[7]));
    }
    for (int u = tid + 256 * sl; u < bn * UB; u += 256 * nsl) {
        const int lb = u / UB, c0 = (u % UB) * 8;
        const WdAtomCode &cd = s_code[s_src[lb]];
        const int tail = s_tail[lb];
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int c = c0 + q;
            v[q] = c < Fa ? code_value(cd, c, Fa) : (c < Fb ? (float)((tail >> (c - Fa)) & 1) : 0.f);
        }
        put_row8(P.f_bonds + (size_t)(bs + lb) * P.ldb, P.fb_x6, P.ldb, bs + lb, c0, v);
    }
}

}  // namespace wd
