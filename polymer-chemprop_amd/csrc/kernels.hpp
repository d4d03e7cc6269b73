// kernels.hpp — bandwidth-bound kernels of the wD-MPNN encoder: CSR row gathers (the padded
// index_select_ND + weighted sum of mpn.py:112-131), the molecule readout (mpn.py:145-171), the
// activation/gather backward, weight packing and the deterministic slab reduction.
#pragma once
#include "common.hpp"
#include "planes.hpp"
#include "wdmpnn.h"

namespace wd {

// ---------------------------------------------------------------------------------------------
// Row gather (the padded index_select_ND + weighted sum of mpn.py:112-131 as one CSR list per output
// row), 8 columns per thread, first G8 CSR entries fetched together:
//   out[r][c..c+7] = sum_{e in [ptr[r], ptr[r+1])} coef[e] * S(idx[e], c..c+7)
//   S(j, c) = src[j][c]  or  (src[j][c] + src[rev[j]][c]) / 2 with sym_rev (mpn.py:101-102)
// The idx / coef of entries e0 .. e0+7 are loaded unconditionally (WdCsr lists are readable 8 entries
// past their end; dead entries point at row 0 and are not added), then all their source rows are
// loaded at once: a row costs three dependent hops (ptr -> idx -> rows) instead of one per entry.
// Entries are added in CSR order (fixed order: deterministic, the order of the reference's slot sum).
// Output: fp32 rows (out) and/or the plane tiles of the next split GEMM (planes, columns
// pcol0 + c of a [rows_p][kp] plane-tile matrix).  Rows [rows, rows_p) are written as zeros.
// ---------------------------------------------------------------------------------------------
constexpr int G8 = 8;

struct Gather8P {
    const float *src; int ld_src; int K;   // K: columns gathered (multiple of 8)
    const int32_t *ptr; const int32_t *idx; const float *coef;
    const int32_t *sym_rev;
    float *out; int ld_out;
    uint8_t *planes; int kp; int pcol0;
    int rows, rows_p;
};

__global__ __launch_bounds__(256) void gather8_kernel(Gather8P P) {
    const int nu = P.K >> 3;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P.rows_p * nu) return;
    const int r = t / nu, c = (t % nu) * 8;
    float4 lo = f4zero(), hi = f4zero();
    if (r < P.rows) {
        const int e0 = P.ptr[r], e1 = P.ptr[r + 1];
        int j[G8];
        float w[G8];
#pragma unroll
        for (int k = 0; k < G8; ++k) {
            const bool ok = e0 + k < e1;
            const int jj = P.idx[e0 + k];
            const float ww = P.coef ? P.coef[e0 + k] : 1.0f;
            j[k] = ok ? jj : 0;
            w[k] = ww;
        }
        float4 xa[G8], xb[G8];
#pragma unroll
        for (int k = 0; k < G8; ++k) {
            const float *s = P.src + (size_t)j[k] * P.ld_src + c;
            xa[k] = ld4(s);
            xb[k] = ld4(s + 4);
        }
        if (P.sym_rev) {
#pragma unroll
            for (int k = 0; k < G8; ++k) {
                const float *s = P.src + (size_t)P.sym_rev[j[k]] * P.ld_src + c;
                const float4 ua = ld4(s), ub = ld4(s + 4);
                xa[k].x = (xa[k].x + ua.x) / 2.0f; xa[k].y = (xa[k].y + ua.y) / 2.0f;
                xa[k].z = (xa[k].z + ua.z) / 2.0f; xa[k].w = (xa[k].w + ua.w) / 2.0f;
                xb[k].x = (xb[k].x + ub.x) / 2.0f; xb[k].y = (xb[k].y + ub.y) / 2.0f;
                xb[k].z = (xb[k].z + ub.z) / 2.0f; xb[k].w = (xb[k].w + ub.w) / 2.0f;
            }
        }
#pragma unroll
        for (int k = 0; k < G8; ++k)
            if (e0 + k < e1) {
                fma4(lo, w[k], xa[k]);
                fma4(hi, w[k], xb[k]);
            }
        for (int e = e0 + G8; e < e1; ++e) {  // rows with more than G8 entries
            const int jj = P.idx[e];
            const float ww = P.coef ? P.coef[e] : 1.0f;
            const float *s = P.src + (size_t)jj * P.ld_src + c;
            float4 ya = ld4(s), yb = ld4(s + 4);
            if (P.sym_rev) {
                const float *u = P.src + (size_t)P.sym_rev[jj] * P.ld_src + c;
                const float4 ua = ld4(u), ub = ld4(u + 4);
                ya.x = (ya.x + ua.x) / 2.0f; ya.y = (ya.y + ua.y) / 2.0f;
                ya.z = (ya.z + ua.z) / 2.0f; ya.w = (ya.w + ua.w) / 2.0f;
                yb.x = (yb.x + ub.x) / 2.0f; yb.y = (yb.y + ub.y) / 2.0f;
                yb.z = (yb.z + ub.z) / 2.0f; yb.w = (yb.w + ub.w) / 2.0f;
            }
            fma4(lo, ww, ya);
            fma4(hi, ww, yb);
        }
    }
    if (P.out) {
        float *o = P.out + (size_t)r * P.ld_out + c;
        st4(o, lo);
        st4(o + 4, hi);
    }
    if (P.planes) x6_store8(P.planes, P.kp, r, P.pcol0 + c, lo, hi);
}

constexpr int RO_BWD_COLS = 1024;  // columns per workgroup of readout_bwd_kernel (256 threads x 4)

// ---------------------------------------------------------------------------------------------
// Readout (mpn.py:145-171): out_i = Xn_i * (sum_a w_a h_a) / sum_a w_a  (mean) | sum | / norm.
// One workgroup per molecule; lanes = (atom slot, float4 column); atom slots reduced through LDS
// in a fixed order.
// ---------------------------------------------------------------------------------------------
struct ReadoutP {
    const float *h; int ldh; int ncols;
    const float *w_atoms; const int32_t *mol_start; const int32_t *mol_size; const float *xn;
    int agg; float norm;
    const float *zero_vec;
    float *out;
};

constexpr int RO_THREADS = 256;
constexpr int RO_QW = 16;                    // float4 columns per workgroup
constexpr int RO_SLOTS = RO_THREADS / RO_QW;  // atom slots per workgroup

// grid = (molecules, ceil(ncols / (4 * RO_QW))); lane = (atom slot, float4 column); the 16 slot
// partial sums are added in slot order (deterministic).
__global__ __launch_bounds__(RO_THREADS) void readout_kernel(ReadoutP P) {
    __shared__ float4 part[RO_THREADS];
    const int i = blockIdx.x;
    const int a0 = P.mol_start[i], n = P.mol_size[i];
    const int slot = threadIdx.x / RO_QW, ql = threadIdx.x % RO_QW;
    const int q = blockIdx.y * RO_QW + ql;
    float *out = P.out + (size_t)i * P.ncols;
    if (n == 0) {  // mpn.py:148-149 cached_zero_vector (no Xn factor)
        if (slot == 0)
            for (int e = 0; e < 4; ++e)
                if (4 * q + e < P.ncols) out[4 * q + e] = P.zero_vec[4 * q + e];
        return;
    }
    float4 s = f4zero();
    if (4 * q < P.ncols)
        for (int a = slot; a < n; a += RO_SLOTS) fma4(s, P.w_atoms[a0 + a], ld4(P.h + (size_t)(a0 + a) * P.ldh + 4 * q));
    part[threadIdx.x] = s;
    __syncthreads();
    if (slot != 0 || 4 * q >= P.ncols) return;
    float4 t = part[ql];
    for (int k = 1; k < RO_SLOTS; ++k) {
        const float4 u = part[k * RO_QW + ql];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    float wsum = 0.f;  // sequential, identical order in every thread
    for (int a = 0; a < n; ++a) wsum += P.w_atoms[a0 + a];
    const float x = P.xn[i];
    const float v[4] = {t.x, t.y, t.z, t.w};
    for (int e = 0; e < 4; ++e) {
        const int c = 4 * q + e;
        if (c >= P.ncols) break;
        const float m = P.agg == 0 ? v[e] / wsum : (P.agg == 2 ? v[e] / P.norm : v[e]);
        out[c] = x * m;
    }
}

// d readout / d h: dh[a] = dout[i] * Xn_i * w_a * (1/sum w | 1 | 1/norm); rows outside every scope
// stay 0 (caller memsets).  grid = (molecules, ceil(ncols / (NT * MAXC))): blockIdx.y picks a chunk of
// RO_BWD_COLS columns (any hidden + descriptor width).
__global__ __launch_bounds__(256) void readout_bwd_kernel(ReadoutP P, const float *__restrict__ dout,
                                                          float *__restrict__ dh) {
    const int i = blockIdx.x;
    const int a0 = P.mol_start[i], n = P.mol_size[i];
    if (n == 0) return;
    // Σ w_a as a fixed-shape tree over the block (deterministic), the atom weights staged in LDS, and
    // each thread's column gradient kept in registers: the store loop issues no global loads (the
    // previous element-per-iteration form waited on two dependent loads per element, ~19 us per call)
    constexpr int NT = 256, MAXC = 4;  // columns per thread in this workgroup's chunk
    __shared__ float red[NT];
    __shared__ float wl[NT];
    const int tid = threadIdx.x;
    float w = 0.f;
    for (int a = tid; a < n; a += NT) w += P.w_atoms[a0 + a];
    red[tid] = w;
    __syncthreads();
    for (int k = NT / 2; k > 0; k >>= 1) {
        if (tid < k) red[tid] += red[tid + k];
        __syncthreads();
    }
    const float wsum = red[0];
    const float x = P.xn[i];
    float gs[MAXC];
    const int c0 = blockIdx.y * NT * MAXC;
#pragma unroll
    for (int q = 0; q < MAXC; ++q) {
        const int c = c0 + tid + NT * q;
        const float g = c < P.ncols ? dout[(size_t)i * P.ncols + c] * x : 0.f;
        gs[q] = P.agg == 0 ? g / wsum : (P.agg == 2 ? g / P.norm : g);
    }
    for (int base = 0; base < n; base += NT) {
        const int m = min(NT, n - base);
        __syncthreads();
        if (tid < m) wl[tid] = P.w_atoms[a0 + base + tid];
        __syncthreads();
        float *row = dh + (size_t)(a0 + base) * P.ldh;
        for (int a = 0; a < m; ++a, row += P.ldh) {
            const float wa = wl[a];
#pragma unroll
            for (int q = 0; q < MAXC; ++q) {
                const int c = c0 + tid + NT * q;
                if (c < P.ncols) row[c] = gs[q] * wa;
            }
        }
    }
}

// The readout backward fused with the backward of the W_o activation (mpn.py:133-134, 145-171) when the
// readout reads h directly (no descriptor layer):
//     dZo[a] = (dout[i] Xn_i w_a (1/sum w | 1 | 1/norm)) * dropout_scale * act'(Zo[a])
// the same arithmetic, in the same order, as readout_bwd_kernel + act_bwd_kernel, without dh's round trip
// through HBM and without its memset: workgroups (i < B, y) write molecule i's atom rows (all ld columns,
// zeros past ncols; the (atom, float4) units strided over the RO_ACT_Y workgroups of the molecule), the
// workgroups (B, y) the rows of no molecule (the pad row 0 and [rows, rows_p)).  Each thread loads its
// RO_ACT_U units' Zo before computing any (the loop of load-then-store units waited one memory latency per
// unit).  grid = (B + 1, RO_ACT_Y), 256 threads; ld <= RO_ACT_MAXLD, a multiple of 4.
struct RoActBwd {
    const float *Z; int ld;                 // Zo [rows_p][ld]
    int act; const float *slope; float p_drop; uint64_t seed; uint32_t layer;
    float *out;                             // dZo [rows_p][ld]
    int rows, rows_p;
    float *prelu_part;                      // [gridDim.x * gridDim.y] or null
};
#ifndef WD_RO_ACT_Y
#define WD_RO_ACT_Y 16  // (workgroups per molecule: 4 / 8 / 16 took 7.5 / 6.5 / 6.4 us at B = 128)
#endif
constexpr int RO_ACT_MAXLD = 2560, RO_ACT_Y = WD_RO_ACT_Y, RO_ACT_U = 4;

__global__ __launch_bounds__(256) void readout_act_bwd_kernel(ReadoutP P, const float *__restrict__ dout, RoActBwd A) {
    constexpr int NT = 256, U = RO_ACT_U;
    __shared__ float red[NT];
    __shared__ float4 gsl[RO_ACT_MAXLD / 4];
    const int tid = threadIdx.x, i = blockIdx.x, Q = A.ld / 4;
    const int t0 = blockIdx.y * NT + tid, ts = NT * gridDim.y;  // this thread's units t0, t0 + ts, ...
    const float slope = A.act == ACT_PRELU ? A.slope[0] : 0.f;
    float ppart = 0.f;
    if (i == (int)gridDim.x - 1) {
        const int extra = A.rows_p - A.rows;
        for (int t = t0; t < (1 + extra) * Q; t += ts) {
            const int k = t / Q, q = t % Q, r = k == 0 ? 0 : A.rows + k - 1;
            st4(A.out + (size_t)r * A.ld + 4 * q, f4zero());
        }
    } else if (P.mol_size[i] > 0) {
        const int a0 = P.mol_start[i], n = P.mol_size[i];
        float w = 0.f;  // sum w_a: the tree of readout_bwd_kernel
        for (int a = tid; a < n; a += NT) w += P.w_atoms[a0 + a];
        red[tid] = w;
        __syncthreads();
        for (int k = NT / 2; k > 0; k >>= 1) {
            if (tid < k) red[tid] += red[tid + k];
            __syncthreads();
        }
        const float wsum = red[0], x = P.xn[i];
        for (int q = tid; q < Q; q += NT) {
            float gs[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = 4 * q + e;
                const float g = c < P.ncols ? dout[(size_t)i * P.ncols + c] * x : 0.f;
                gs[e] = P.agg == 0 ? g / wsum : (P.agg == 2 ? g / P.norm : g);
            }
            gsl[q] = make_float4(gs[0], gs[1], gs[2], gs[3]);
        }
        __syncthreads();
        for (int tb = t0; tb < n * Q; tb += U * ts) {
            float4 z4[U];
            float wa[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = tb + u * ts, a = t / Q, q = t % Q;
                z4[u] = f4zero();
                wa[u] = 0.f;
                if (t < n * Q) {
                    z4[u] = ld4(A.Z + (size_t)(a0 + a) * A.ld + 4 * q);
                    wa[u] = P.w_atoms[a0 + a];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = tb + u * ts, a = t / Q, q = t % Q, r = a0 + a;
                if (t >= n * Q) break;
                const float4 g4 = gsl[q];
                const float g[4] = {g4.x * wa[u], g4.y * wa[u], g4.z * wa[u], g4.w * wa[u]};
                const float z[4] = {z4[u].x, z4[u].y, z4[u].z, z4[u].w};
                float dz[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float s = A.p_drop > 0.f ? dropout_scale(A.seed, A.layer, r, 4 * q + e, A.p_drop) : 1.f;
                    dz[e] = g[e] * s * act_grad(A.act, z[e], slope);
                    if (A.act == ACT_PRELU && !(z[e] > 0.f)) ppart += z[e] * g[e] * s;
                }
                st4(A.out + (size_t)r * A.ld + 4 * q, make_float4(dz[0], dz[1], dz[2], dz[3]));
            }
        }
    }
    if (A.prelu_part) {
        __syncthreads();
        red[tid] = ppart;
        __syncthreads();
        for (int s = NT / 2; s > 0; s >>= 1) {
            if (tid < s) red[tid] += red[tid + s];
            __syncthreads();
        }
        if (tid == 0) A.prelu_part[blockIdx.y * gridDim.x + blockIdx.x] = red[0];
    }
}

// ---------------------------------------------------------------------------------------------
// Backward of one activation layer, fused with the gather that produces its incoming gradient:
//   g   = sum_e coef[e] * G[idx[e]]  (csr) | (G[r] + G[rev[r]]) / 2 (sym) | G[r] (dense)
//   dz  = g * dropout_scale * act'(z)          (Z == null: dz = g)
//   dz += add_in[r];  res_out (=|+=) dz;  PReLU partial sum of z * g * scale over z <= 0
// Rows [rows, rows_p) are written as 0.
// ---------------------------------------------------------------------------------------------
struct ActBwd {
    const float *G; int ldg;
    const int32_t *ptr; const int32_t *idx; const float *coef;
    const int32_t *sym_rev;
    const float *Z; int act; const float *slope; float p_drop; uint64_t seed; uint32_t layer;
    const float *add_in;
    float *res_out; int res_init;
    float *out;
    float *prelu_part;
    int rows, rows_p, cols, ld;  // cols: padded width (zero columns stay zero)
    // max |dz| of every 256 consecutive vectors (t / 256) as u32 bits: the scale words of the fp16-pair
    // GEMM that consumes `out` (gemm_x6_kernel<H2>); needs V = 4 and rows_p * cols / 4 % 256 == 0 (every
    // workgroup's trip count uniform)
    uint32_t *words;
};

// V consecutive columns per thread (V = 4 when cols, ld, ldg are multiples of 4: 16-byte loads and
// stores); 32-bit index math (rows_p * cols < 2^31 is checked by the launcher).  The CSR sum runs in
// entry order per element, so V does not change any result bit.
template <int V>
__global__ __launch_bounds__(256) void act_bwd_kernel(ActBwd P) {
    typedef float __attribute__((ext_vector_type(V))) fv;
    __shared__ float red[256];
    __shared__ uint32_t wred[2][4];
    const float slope = (P.Z && P.act == ACT_PRELU) ? P.slope[0] : 0.f;
    float ppart = 0.f;
    const int cv = P.cols / V;
    const int total = P.rows_p * cv;
    int it = 0;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x, ++it) {
        const int r = t / cv, c = (t - r * cv) * V;
        const size_t o = (size_t)r * P.ld + c;
        fv dz = (fv)0.f;
        if (r < P.rows) {
            fv g;
            if (P.ptr) {
                // the first GE entries' ids and weights fetched together (WdCsr lists are readable 8 entries
                // past their end; dead entries read row 0 and are not added), then all their rows: three
                // dependent hops per row instead of two per entry; entries added in CSR order
                constexpr int GE = 4;
                g = (fv)0.f;
                const int e0 = P.ptr[r], e1 = P.ptr[r + 1];
                int j[GE];
                float w[GE];
#pragma unroll
                for (int k = 0; k < GE; ++k) {
                    const int jj = P.idx[e0 + k];
                    j[k] = e0 + k < e1 ? jj : 0;
                    w[k] = P.coef ? P.coef[e0 + k] : 1.f;
                }
                fv x[GE];
#pragma unroll
                for (int k = 0; k < GE; ++k) x[k] = *(const fv *)(P.G + (size_t)j[k] * P.ldg + c);
#pragma unroll
                for (int k = 0; k < GE; ++k)
                    if (e0 + k < e1)
                        for (int q = 0; q < V; ++q) g[q] = fmaf(w[k], x[k][q], g[q]);
                for (int e = e0 + GE; e < e1; ++e) {
                    const float we = P.coef ? P.coef[e] : 1.f;
                    const fv xe = *(const fv *)(P.G + (size_t)P.idx[e] * P.ldg + c);
                    for (int q = 0; q < V; ++q) g[q] = fmaf(we, xe[q], g[q]);
                }
            } else if (P.sym_rev) {
                const fv a = *(const fv *)(P.G + (size_t)r * P.ldg + c);
                const fv b = *(const fv *)(P.G + (size_t)P.sym_rev[r] * P.ldg + c);
                for (int q = 0; q < V; ++q) g[q] = (a[q] + b[q]) * 0.5f;
            } else {
                g = *(const fv *)(P.G + (size_t)r * P.ldg + c);
            }
            dz = g;
            if (P.Z) {
                const fv z = *(const fv *)(P.Z + o);
                for (int q = 0; q < V; ++q) {
                    const float s = P.p_drop > 0.f ? dropout_scale(P.seed, P.layer, r, c + q, P.p_drop) : 1.f;
                    dz[q] = g[q] * s * act_grad(P.act, z[q], slope);
                    if (P.act == ACT_PRELU && !(z[q] > 0.f)) ppart += z[q] * g[q] * s;
                }
            }
            if (P.add_in) dz += *(const fv *)(P.add_in + o);
        }
        if (P.res_out) *(fv *)(P.res_out + o) = P.res_init ? dz : *(const fv *)(P.res_out + o) + dz;
        *(fv *)(P.out + o) = dz;
        if (P.words) {
            // (two LDS slots alternating: the next iteration's writes cannot pass thread 0's read, which
            // precedes its barrier)
            uint32_t m = 0u;
            for (int q = 0; q < V; ++q) m = max(m, absbits(dz[q]));
            m = wave_max_u32(m);
            if ((threadIdx.x & 63) == 0) wred[it & 1][threadIdx.x >> 6] = m;
            __syncthreads();
            if (threadIdx.x == 0)
                P.words[t >> 8] = max(max(wred[it & 1][0], wred[it & 1][1]), max(wred[it & 1][2], wred[it & 1][3]));
        }
    }
    if (P.prelu_part) {
        red[threadIdx.x] = ppart;
        __syncthreads();
        for (int s = 128; s > 0; s >>= 1) {
            if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
            __syncthreads();
        }
        if (threadIdx.x == 0) P.prelu_part[blockIdx.x] = red[0];
    }
}

// ---------------------------------------------------------------------------------------------
// Weight packing: nn.Linear weights -> zero-padded GEMM operands (and transposes for the data
// gradients).  dst[r][c], r < rows_p, c < cols_p:
//   plain:      segment s with dst cols [dc0_s, dc0_s + K_s): src[r][sc0_s + c - dc0_s]  (r < nrows)
//   transpose:  src[c][sc0_0 + r]  for r < nrows (= K_0 source cols), c < K_0 (source rows)
// ---------------------------------------------------------------------------------------------
struct PackJob {
    float *dst; int rows_p, cols_p;
    const float *src; int ld_src;
    int transpose, nrows, nseg;
    int dc0[2], sc0[2], K[2];
    uint32_t *amax;  // or null: max |dst| of workgroup x -> amax[x] (the h2 scale of split_h2_kernel)
    const float *src1; int ld_src1;  // or null: segment 1's source (plain jobs; else every segment reads src)
};
struct PackJobs { PackJob j[16]; int n; };

__global__ __launch_bounds__(256) void pack_kernel(PackJobs J) {
    const PackJob &P = J.j[blockIdx.y];
    const size_t total = (size_t)P.rows_p * P.cols_p;
    uint32_t mx = 0;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / P.cols_p), c = (int)(t % P.cols_p);
        float v = 0.f;
        if (P.src && r < P.nrows) {
            if (P.transpose) {
                if (c < P.K[0]) v = P.src[(size_t)c * P.ld_src + P.sc0[0] + r];
            } else {
                for (int s = 0; s < P.nseg; ++s)
                    if (c >= P.dc0[s] && c < P.dc0[s] + P.K[s]) {
                        const bool one = s == 1 && P.src1;
                        v = (one ? P.src1 : P.src)[(size_t)r * (one ? P.ld_src1 : P.ld_src) + P.sc0[s] + c - P.dc0[s]];
                    }
            }
        }
        P.dst[t] = v;
        mx = max(mx, absbits(v));
    }
    if (P.amax) {  // (uniform per workgroup)
        __shared__ uint32_t red[4];
        publish_max(mx, P.amax + blockIdx.x, red);
    }
}

// per molecule block (WdGraph.blocks row {bond_start, bond_count, ...}, workgroup = block): max |act(x)|
// over the block's rows of x [.][ld], columns [0, cols) -> out[block] (the first fused layer's operand
// scale when the input layer ran as a GEMM instead of the embed)
template <int ACT>
__global__ __launch_bounds__(256) void absmax_blocks_kernel(const float *x, int ld, int cols, const int32_t *blocks,
                                                            const float *slope_p, uint32_t *out, int atom_rows) {
    const float slope = ACT == ACT_PRELU ? slope_p[0] : 0.f;
    // the block's bond rows (or its atom rows: atom-message mode)
    const int bs = blocks[8 * blockIdx.x + 2 * atom_rows], bn = blocks[8 * blockIdx.x + 1 + 2 * atom_rows];
    const int c4 = cols / 4;
    uint32_t mx = 0;
    for (int t = threadIdx.x; t < bn * c4; t += blockDim.x) {
        const float4 v = ld4(x + (size_t)(bs + t / c4) * ld + 4 * (t % c4));
        mx = max(mx, max(max(absbits(act_fwd(ACT, v.x, slope)), absbits(act_fwd(ACT, v.y, slope))),
                         max(absbits(act_fwd(ACT, v.z, slope)), absbits(act_fwd(ACT, v.w, slope)))));
    }
    __shared__ uint32_t red[4];
    publish_max(mx, out + blockIdx.x, red);
}

// ---------------------------------------------------------------------------------------------
// Slab reduction of the weight-gradient GEMMs (fixed split order: deterministic).
//   dW[n][w0_s + kk] = sum_z slab[z][n][c0_s + kk],  db[n] = sum_z slab[z][n][bias_col]
// ---------------------------------------------------------------------------------------------
struct SlabReduce {
    const float *slab; int nsplit; long long slab_stride; int ld_slab;
    int rows;
    int nseg; int c0[3], w0[3], K[3];
    float *dW; int ldw;
    float *db; int bias_col;
};

// grid (column groups of 64, row groups of 4), 256 threads: one output element per thread (the
// bias is the extra column after the segments).  Every thread sums its column over the splits in
// split order z = 0, 1, ... (eight independent loads in flight, then eight ordered adds), so the
// result does not depend on the launch shape.
// several reductions in one launch (the training backward's W_o, W_h and W_i gradients, each from its own
// slab area): job k owns the 1-D grid range [blk0[k], blk0[k + 1]), each range a (column groups x row
// groups) grid of the single-job form
constexpr int SLAB_MAX = 4;
struct SlabReduceJobs {
    SlabReduce j[SLAB_MAX];
    int cgroups[SLAB_MAX];
    int blk0[SLAB_MAX + 1];
    int n;
};

__device__ __forceinline__ void slab_reduce_elem(const SlabReduce &P, int n, int j);

__global__ __launch_bounds__(256) void slab_reduce_multi_kernel(SlabReduceJobs J) {
    int k = 0;
    while (k + 1 < J.n && (int)blockIdx.x >= J.blk0[k + 1]) ++k;
    const int b = blockIdx.x - J.blk0[k];
    slab_reduce_elem(J.j[k], (b / J.cgroups[k]) * 4 + (threadIdx.x >> 6), (b % J.cgroups[k]) * 64 + (threadIdx.x & 63));
}

__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabReduce P) {
    slab_reduce_elem(P, blockIdx.y * 4 + (threadIdx.x >> 6), blockIdx.x * 64 + (threadIdx.x & 63));
}

__device__ __forceinline__ void slab_reduce_elem(const SlabReduce &P, int n, int j) {
    if (n >= P.rows) return;
    int src = -1;
    float *dst = nullptr;
    if (P.dW) {
        for (int s = 0; s < P.nseg; ++s) {
            if (j < P.K[s]) {
                src = P.c0[s] + j;
                dst = P.dW + (size_t)n * P.ldw + P.w0[s] + j;
                break;
            }
            j -= P.K[s];
        }
    }
    if (!dst && P.db && j == 0) {
        src = P.bias_col;
        dst = P.db + n;
    }
    if (!dst) return;
    const float *col = P.slab + (size_t)n * P.ld_slab + src;
    float acc = 0.f;
    int z = 0;
    for (; z + 8 <= P.nsplit; z += 8) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = col[(size_t)(z + q) * P.slab_stride];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q];
    }
    for (; z < P.nsplit; ++z) acc += col[(size_t)z * P.slab_stride];
    *dst = acc;
}

__global__ void sum_kernel(const float *__restrict__ x, int n, float *__restrict__ out) {
    __shared__ float red[256];
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0];
}

// nn_utils.py:50-67 index_select_ND on rows.
__global__ __launch_bounds__(256) void index_select_rows_kernel(const float *__restrict__ src, int64_t row_len,
                                                                const int64_t *__restrict__ index, int64_t n_index,
                                                                float *__restrict__ out) {
    const int64_t total = n_index * row_len;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / row_len, c = t % row_len;
        out[t] = src[index[i] * row_len + c];
    }
}

// Gradient of index_select_rows: dsrc[j] = sum over positions p with index[p] == j of grad[p], added in
// increasing p (deterministic, no atomics).  perm = positions sorted stably by index, ptr[j] .. ptr[j+1]
// the positions of row j in perm; one thread per output value.
__global__ __launch_bounds__(256) void index_select_rows_bwd_kernel(const float *__restrict__ grad, int64_t row_len,
                                                                    const int64_t *__restrict__ perm,
                                                                    const int64_t *__restrict__ ptr, int64_t n_src,
                                                                    float *__restrict__ dsrc) {
    const int64_t total = n_src * row_len;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = t / row_len, c = t % row_len;
        float s = 0.f;
        for (int64_t e = ptr[j]; e < ptr[j + 1]; ++e) s += grad[perm[e] * row_len + c];
        dsrc[t] = s;
    }
}

// f_bonds[r] = f_atoms[b2a[r]] ‖ bond_tail[r] ‖ 0 (featurization.py:467-468, 545-546, 616-617 build each
// directed bond row as its source atom's features followed by the bond's own), one thread per output
// value.  An out-of-range source atom writes NaN to the row (never read past f_atoms).
__global__ __launch_bounds__(256) void build_bond_features_kernel(const float *__restrict__ fa, int lda, int Fa,
                                                                  int atom_rows, const int32_t *__restrict__ b2a,
                                                                  const float *__restrict__ tail, int ldt, int Ft,
                                                                  int rows, float *__restrict__ fb, int ldb) {
    const size_t total = (size_t)rows * ldb;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / ldb), c = (int)(t % ldb);
        float v = 0.f;
        if (c < Fa) {
            const int a = b2a[r];
            v = (a >= 0 && a < atom_rows) ? fa[(size_t)a * lda + c] : __builtin_nanf("");
        } else if (c < Fa + Ft) {
            v = tail[(size_t)r * ldt + (c - Fa)];
        }
        fb[t] = v;
    }
}

}  // namespace wd

// One Adam / AdamW step over up to ADAM_MAX tensors in one launch (the optimizer step of train.py:84,
// torch.optim.Adam / AdamW as built by utils.py:295-310).  Each tensor owns a contiguous range of
// workgroups (blk0), each workgroup 1024 elements (4 per thread, strided by 256: coalesced), so the
// tensor lookup is a uniform scan of the launch table.  Same per-element arithmetic as torch's fused
// Adam: L2 weight decay folded into the gradient (AdamW: decoupled, on the parameter), moments as
// beta * m + (1 - beta) * g, denom = sqrt(v) / sqrt(bc2) + eps, p -= (lr / bc1) * m / denom.
namespace wd {
constexpr int ADAM_MAX = 16, ADAM_PER_BLOCK = 1024, ADAM_OUTS = 16, ADAM_TJ = 6, ADAM_TILE = 32;
// An extra destination of a weight's updated values (wdmpnn_adam_step_repack: the training step's packed
// weight copies written by the optimizer itself instead of a repack before the next forward).  Source
// element (r, c) of a [rows][cols] weight, for the column segment s holding c (c in [sc0[s], sc0[s] + K[s])):
//   AO_PLAIN      dst[r * ld + dc0[s] + c - sc0[s]]            (pack_kernel's plain jobs)
//   AO_TRANSPOSE  dst[(c - sc0[s]) * ld + r]                   (its transposes)
//   AO_PLANES     bf16x3 plane tiles of the padded plain matrix (row blocks of br, kp = ld padded columns),
//                 the value split exactly as split_pair / x6_store8 split it
enum { AO_PLAIN = 0, AO_TRANSPOSE = 1, AO_PLANES = 2 };
struct AdamOut {
    void *dst;
    int kind, ld, nseg, br;
    int sc0[2], dc0[2], K[2];
};
// a repacked weight, updated in 32 x 32 tiles (one workgroup each): the transposed copies leave through
// LDS as whole 128-byte rows, and each tile publishes max |w| (W_h's fp16-pair scale) as one word
struct AdamTileJob {
    int t;                  // its tensor in AdamLaunch::t
    int rows, cols, tiles_c, blk0;
    int o0, o1;             // its outputs out[o0 .. o1)
    uint32_t *amax;         // one word per tile, or null
};
struct AdamLaunch {
    WdAdamTensor t[ADAM_MAX];
    int blk0[ADAM_MAX + 1];  // element-wise blocks per tensor (none for a tile job's tensor)
    int n;
    float beta1, beta2, eps, wd, lr, step_size, bc2_sqrt;
    int decoupled;
    AdamTileJob tj[ADAM_TJ];
    int ntj, tile_blocks;    // tile blocks first, then the element-wise blocks
    AdamOut out[ADAM_OUTS];
};

// one element's update (torch.optim.Adam / AdamW): p, m, v in place from p, g, m, v
__device__ __forceinline__ void adam_math(const AdamLaunch &A, float &p, float g, float &m, float &v) {
#pragma clang fp contract(off)
    if (A.wd != 0.f) {
        if (A.decoupled) p -= A.lr * A.wd * p;
        else g += p * A.wd;
    }
    m = A.beta1 * m + (1.f - A.beta1) * g;
    v = A.beta2 * v + (1.f - A.beta2) * g * g;
    const float denom = sqrtf(v) / A.bc2_sqrt + A.eps;
    p = p - A.step_size * m / denom;
}

__device__ __forceinline__ int ao_seg(const AdamOut &O, int c) { return O.nseg > 1 && c >= O.sc0[1] ? 1 : 0; }

__device__ void adam_tile(const AdamLaunch &A, int b) {
    __shared__ float tl[ADAM_TILE][ADAM_TILE + 1];  // [source column][source row]
    __shared__ uint32_t red[4];
    int j = 0;
    while (j + 1 < A.ntj && b >= A.tj[j + 1].blk0) ++j;
    const AdamTileJob &J = A.tj[j];
    const WdAdamTensor &T = A.t[J.t];
    const int tile = b - J.blk0, tr = tile / J.tiles_c, tc = tile % J.tiles_c;
    const int lr = threadIdx.x >> 3, lc = 4 * (threadIdx.x & 7);
    const int r = tr * ADAM_TILE + lr;
    uint32_t mx = 0;
    bool transposes = false;
    // all four elements' operands loaded before any store (the stores could alias the loads of the next
    // element as far as the compiler knows: interleaved, each element paid a memory latency)
    float pv[4], gv[4], mv[4], vv[4];
    const int64_t i0 = (int64_t)r * J.cols + tc * ADAM_TILE + lc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool ok = r < J.rows && tc * ADAM_TILE + lc + q < J.cols;
        const int64_t i = ok ? i0 + q : 0;
        pv[q] = T.param[i]; gv[q] = T.grad[i]; mv[q] = T.exp_avg[i]; vv[q] = T.exp_avg_sq[i];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) adam_math(A, pv[q], gv[q], mv[q], vv[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int c = tc * ADAM_TILE + lc + q;
        float pn = 0.f;
        if (r < J.rows && c < J.cols) {
            pn = pv[q];
            T.param[i0 + q] = pn;
            T.exp_avg[i0 + q] = mv[q];
            T.exp_avg_sq[i0 + q] = vv[q];
            mx = max(mx, absbits(pn));
            for (int o = J.o0; o < J.o1; ++o) {
                const AdamOut &O = A.out[o];
                const int s = ao_seg(O, c), cc = c - O.sc0[s];
                if (O.kind == AO_TRANSPOSE || cc < 0 || cc >= O.K[s]) continue;
                if (O.kind == AO_PLAIN) {
                    reinterpret_cast<float *>(O.dst)[(int64_t)r * O.ld + O.dc0[s] + cc] = pn;
                } else {
                    const int k = O.dc0[s] + cc;
                    const uint32_t h = cvt_pk_bf16(pn, 0.f);
                    const float v1 = pn - bf_lo(h);
                    const uint32_t m = cvt_pk_bf16(v1, 0.f);
                    const uint32_t l = cvt_pk_bf16(v1 - bf_lo(m), 0.f);
                    uint8_t *d = reinterpret_cast<uint8_t *>(O.dst) +
                                 ((int64_t)(r / O.br) * (O.ld >> 5) + (k >> 5)) * (3 * O.br * 64) + (r % O.br) * 64 +
                                 2 * (k & 31);
                    *reinterpret_cast<uint16_t *>(d) = (uint16_t)h;
                    *reinterpret_cast<uint16_t *>(d + O.br * 64) = (uint16_t)m;
                    *reinterpret_cast<uint16_t *>(d + 2 * O.br * 64) = (uint16_t)l;
                }
            }
        }
        tl[lc + q][lr] = pn;
    }
    for (int o = J.o0; o < J.o1; ++o) transposes |= A.out[o].kind == AO_TRANSPOSE;
    if (transposes) {  // (uniform) column lc8 of the tile as 4 consecutive rows of the transposed copy
        __syncthreads();
        const int cl = threadIdx.x >> 3, rl = 4 * (threadIdx.x & 7);
        const int c = tc * ADAM_TILE + cl;
        for (int o = J.o0; o < J.o1; ++o) {
            const AdamOut &O = A.out[o];
            if (O.kind != AO_TRANSPOSE) continue;
            const int s = ao_seg(O, c), cc = c - O.sc0[s];
            if (c >= J.cols || cc < 0 || cc >= O.K[s]) continue;
            float *d = reinterpret_cast<float *>(O.dst) + (int64_t)cc * O.ld + tr * ADAM_TILE + rl;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (tr * ADAM_TILE + rl + q < J.rows) d[q] = tl[cl][rl + q];
        }
    }
    if (J.amax) publish_max(mx, J.amax + tile, red);  // (uniform per workgroup)
}

template <bool REPACK>
__global__ __launch_bounds__(256) void adam_kernel(AdamLaunch A) {
    int b = blockIdx.x;
    if (REPACK) {
        if (b < A.tile_blocks) {
            adam_tile(A, b);
            return;
        }
        b -= A.tile_blocks;
    }
    int k = 0;
    while (k + 1 < A.n && b >= A.blk0[k + 1]) ++k;
    const WdAdamTensor &T = A.t[k];
    const int64_t i0 = (int64_t)(b - A.blk0[k]) * ADAM_PER_BLOCK + threadIdx.x;
    constexpr int PT = ADAM_PER_BLOCK / 256;
    float pv[PT], gv[PT], mv[PT], vv[PT];
#pragma unroll
    for (int j = 0; j < PT; ++j) {  // (loads first: see adam_tile)
        const int64_t i = min(i0 + 256 * j, T.numel - 1);
        pv[j] = T.param[i]; gv[j] = T.grad[i]; mv[j] = T.exp_avg[i]; vv[j] = T.exp_avg_sq[i];
    }
#pragma unroll
    for (int j = 0; j < PT; ++j) {
        const int64_t i = i0 + 256 * j;
        adam_math(A, pv[j], gv[j], mv[j], vv[j]);
        if (i < T.numel) { T.param[i] = pv[j]; T.exp_avg[i] = mv[j]; T.exp_avg_sq[i] = vv[j]; }
    }
}
}  // namespace wd

// ------------------------------------------------------------------------------------------------
// The training step's FFN head and masked loss (model.py:57-121 with ffn_num_layers = 2, no dropout;
// train.py:55-74 with MSELoss): per molecule row x (the encoder output),
//     h = W1 x + b1, a = act(h), out = W2 a + b2,
//     loss = sum_rows sum_t w[t] (out[t] - y[t])^2 / n      (w = target weight * data weight * mask)
// and, in the same pass, the gradients of that loss: dout = 2 w (out - y) / n, dh = act'(h) W2^T dout,
// dx = W1^T dh, dW1 = sum_rows dh x^T, db1 = sum dh, dW2 = sum dout a^T, db2 = sum dout.  Three launches:
// the H GEMM, one wave per row for the loss and dh, then the dX and dW1 GEMMs and the small sums (fixed
// summation orders).  fp32 FMA throughout (the GEMMs are 128 x 300 x 300: latency, not FLOPs).
// ------------------------------------------------------------------------------------------------
namespace wd {
constexpr int HEAD_MAX_F = 4096, HEAD_MAX_H = 4096, HEAD_MAX_T = 64;

__device__ __forceinline__ float wave_sum(float s) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

// C[i][j] (+ bias[j]) = sum_k A(i, k) B(k, j) for one 32 x 32 tile of C (M x N), 256 threads (2 x 2
// outputs each), K in 32-wide chunks through LDS.  Strided operands: A(i, k) = A[i sai + k sak],
// B(k, j) = B[k sbk + j sbj] -- the head's three small GEMMs (X W1^T, dH W1, dH^T X) differ only in
// their strides; every operand is L2-resident (<= 0.5 MB).
struct SmallGemm {
    const float *A; long long sai, sak;
    const float *B; long long sbk, sbj;
    const float *bias;
    float *C; long long ldc;
    int M, N, K;
};
// TS x TS output tile per workgroup of 4 waves: both operands' K-slices of SG_KC staged k-major in LDS
// (every load of the stage in flight at once: these GEMMs are load-latency-bound, 128 x 300 x 300), wave w
// multiplies the w-th quarter of the stage's K (lane: R x R outputs, R = TS / 8, from two R-float reads per
// k), and the four partial tiles are added in wave order (deterministic; every output's arithmetic is
// the same for either tile size).  TS = 16: 4x the workgroups of 32 x 32 tiles, each loading
// half the operand rows: head_h_kernel's 128 x 300 output as 40 tiles of 32 x 32 took 12.8 us, as 152 of
// 16 x 16 6.9 us; head_grads_kernel's dX = dH W1 (K = 300) on 16 x 16 too, its dW1 = dH^T X (K = B = 128,
// half of a 320-deep stage) on 32 x 32 (all of it on 16 x 16: 13.0 against 11.0 us).
constexpr int SG_KC = 320;
template <int TS>
struct alignas(16) SmallGemmLds {
    static constexpr int LD = TS + 4;  // (row stride TS + 4: R-float aligned, bank spread for the staging)
    float as[SG_KC][LD];
    float bs[SG_KC][LD];
};
static_assert(sizeof(SmallGemmLds<16>) <= sizeof(SmallGemmLds<32>), "head_grads_kernel shares one LDS area");
// AK: A's k index contiguous (sak == 1, else sai == 1); BJ: B's j index contiguous (sbj == 1, else sbk == 1)
template <int TS, bool AK, bool BJ>
__device__ __forceinline__ void small_gemm_tile_t(const SmallGemm &G, int tile, SmallGemmLds<TS> &L) {
    constexpr int R = TS / 8;
    typedef float fR __attribute__((ext_vector_type(R)));
    const int tn = (G.N + TS - 1) / TS, i0 = (tile / tn) * TS, j0 = (tile % tn) * TS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, ri = R * (lane >> 3), cj = R * (lane & 7);
    constexpr int PER = TS * SG_KC / 256;
    float c[R][R] = {};
    float ra[PER], rb[PER];
    auto load = [&](int k0) {  // consecutive lanes along each operand's contiguous index (coalesced)
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + 256 * q;
            const int ia = i0 + (AK ? e / SG_KC : e % TS), ka = k0 + (AK ? e % SG_KC : e / TS);
            ra[q] = ia < G.M && ka < G.K ? G.A[ia * G.sai + ka * G.sak] : 0.f;
            const int kb = k0 + (BJ ? e / TS : e % SG_KC), jb = j0 + (BJ ? e % TS : e / SG_KC);
            rb[q] = kb < G.K && jb < G.N ? G.B[kb * G.sbk + jb * G.sbj] : 0.f;
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int e = tid + 256 * q;
            if (AK) L.as[e % SG_KC][e / SG_KC] = ra[q];
            else L.as[e / TS][e % TS] = ra[q];
            if (BJ) L.bs[e / TS][e % TS] = rb[q];
            else L.bs[e % SG_KC][e / SG_KC] = rb[q];
        }
    };
    load(0);
    for (int k0 = 0; k0 < G.K; k0 += SG_KC) {
        store();
        __syncthreads();
        if (k0 + SG_KC < G.K) load(k0 + SG_KC);
        const int kn = min(SG_KC, G.K - k0), kq = (kn + 3) / 4, kb = wave * kq, ke = min(kn, kb + kq);
#pragma unroll 4
        for (int k = kb; k < ke; ++k) {
            const fR a = *reinterpret_cast<const fR *>(&L.as[k][ri]);
            const fR b = *reinterpret_cast<const fR *>(&L.bs[k][cj]);
#pragma unroll
            for (int x = 0; x < R; ++x)
#pragma unroll
                for (int y = 0; y < R; ++y) c[x][y] = fmaf(a[x], b[y], c[x][y]);
        }
        __syncthreads();
    }
    // the four waves' partial tiles (in as, free after the last barrier), added in wave order
    float *part = &L.as[0][0];
    static_assert(4 * TS * TS <= SG_KC * SmallGemmLds<TS>::LD, "partial tiles must fit in the A stage");
#pragma unroll
    for (int x = 0; x < R; ++x) {
        fR v;
#pragma unroll
        for (int y = 0; y < R; ++y) v[y] = c[x][y];
        *reinterpret_cast<fR *>(part + wave * TS * TS + (ri + x) * TS + cj) = v;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TS * TS / 256; ++q) {
        const int o = tid + 256 * q, i = i0 + o / TS, j = j0 + o % TS;
        const float v = ((part[o] + part[TS * TS + o]) + part[2 * TS * TS + o]) + part[3 * TS * TS + o];
        if (i < G.M && j < G.N) G.C[i * G.ldc + j] = v + (G.bias ? G.bias[j] : 0.f);
    }
}
template <int TS>
__device__ __forceinline__ void small_gemm_tile(const SmallGemm &G, int tile, SmallGemmLds<TS> &L) {
    if (G.sak == 1) {
        if (G.sbj == 1) small_gemm_tile_t<TS, true, true>(G, tile, L);
        else small_gemm_tile_t<TS, true, false>(G, tile, L);
    } else {
        if (G.sbj == 1) small_gemm_tile_t<TS, false, true>(G, tile, L);
        else small_gemm_tile_t<TS, false, false>(G, tile, L);
    }
}

// sum_{r < B} x[r * ld] (+ fma with y[r * ldy] when y): rows in order, RU loads in flight
__device__ __forceinline__ float row_sum(const float *x, long long ld, const float *y, long long ldy, int B) {
    float s = 0.f;
    int r = 0;
    constexpr int RU = 32;  // rows in flight (8 paid a memory latency per 8 rows: B = 128 -> 16 in a row)
    for (; r + RU <= B; r += RU) {
        float v[RU], w[RU];
#pragma unroll
        for (int q = 0; q < RU; ++q) {
            v[q] = x[(r + q) * ld];
            w[q] = y ? y[(r + q) * ldy] : 1.f;
        }
#pragma unroll
        for (int q = 0; q < RU; ++q) s = y ? fmaf(v[q], w[q], s) : s + v[q];
    }
    for (; r < B; ++r) s = y ? fmaf(x[r * ld], y[r * ldy], s) : s + x[r * ld];
    return s;
}
// tile sizes of the head's GEMMs and the launch sizes they give
constexpr int HEAD_H_TS = 16, HEAD_G_TS = 32;
__host__ __device__ inline int head_tiles(int M, int N, int ts) { return ((M + ts - 1) / ts) * ((N + ts - 1) / ts); }

// head step 1: H = X W1^T + b1 -> P.a (pre-activation, [B][Hf])
__global__ __launch_bounds__(256) void head_h_kernel(WdHead P) {
    __shared__ SmallGemmLds<HEAD_H_TS> L;
    SmallGemm G{P.x, P.ld_x, 1, P.W1, 1, P.F, P.b1, P.a, P.Hf, P.B, P.Hf, P.F};
    small_gemm_tile(G, blockIdx.x, L);
}

// head step 2, one wave per row: out = W2 act(h) + b2, the row's loss terms, dout = 2 w (out - y) / n,
// dh = act'(h) * (W2^T dout); act(h) replaces h in P.a (for dW2)
__global__ __launch_bounds__(256) void head_rows_kernel(WdHead P) {
    __shared__ float dsh[4][HEAD_MAX_T];  // the row's dout (every lane writes the same value; LDS keeps a wave's order)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, row = blockIdx.x * 4 + wave;
    if (row >= P.B) return;
    const int Hf = P.Hf, T = P.T;
    float *h = P.a + (size_t)row * Hf;
    const float *tab = P.table + (size_t)row * P.ld_table;
    // the row's targets | weights, one per lane, loaded first: the table may be read from pinned host
    // memory (train.py's zero-copy loss table), whose latency then overlaps the dot products below
    const bool tlane = 2 * T <= 64;
    const float tv = tlane && lane < 2 * T ? tab[lane] : 0.f;
    with_act(P.act, [&](auto act_c) {
        constexpr int ACT = decltype(act_c)::value;
        float l = 0.f;
        for (int t = 0; t < T; ++t) {
            const float *w2 = P.W2 + (size_t)t * Hf;
            float s = 0.f;
            for (int j = lane; j < Hf; j += 64) s = fmaf(w2[j], act_fwd(ACT, h[j], 0.f), s);
            s = wave_sum(s) + (P.b2 ? P.b2[t] : 0.f);
            const float y = tlane ? __shfl(tv, t, 64) : tab[t], w = tlane ? __shfl(tv, T + t, 64) : tab[T + t];
            float d;
            if (P.loss_kind == 0) {  // MSE: w (s - y)^2, d/ds = 2 w (s - y)
                const float r = s - y;
                l = fmaf(w * r, r, l);
                d = 2.f * w * r * P.inv_n;
            } else {  // BCE with logits: w (max(s, 0) - s y + log(1 + e^-|s|)), d/ds = w (sigmoid(s) - y)
                l = fmaf(w, fmaxf(s, 0.f) - s * y + log1pf(expf(-fabsf(s))), l);
                d = w * (1.f / (1.f + expf(-s)) - y) * P.inv_n;
            }
            dsh[wave][t] = d;
            if (lane == 0) P.dout[(size_t)row * T + t] = d;
        }
        if (lane == 0) P.lossrow[row] = l;
        for (int j = lane; j < Hf; j += 64) {
            float s = 0.f;
            for (int t = 0; t < T; ++t) s = fmaf(dsh[wave][t], P.W2[(size_t)t * Hf + j], s);
            const float z = h[j];
            P.dh[(size_t)row * Hf + j] = s * act_grad(ACT, z, 0.f);
            h[j] = act_fwd(ACT, z, 0.f);
        }
    });
}

// head step 3: dX = dH W1 (tiles 0 .. n1), dW1 = dH^T X (next n2 tiles), then db1, dW2, db2 and the loss
// (one thread per element, rows summed in order)
__global__ __launch_bounds__(256) void head_grads_kernel(WdHead P) {
    __shared__ SmallGemmLds<HEAD_G_TS> L;
    const SmallGemm GX{P.dh, P.Hf, 1, P.W1, P.F, 1, nullptr, P.dx, P.ld_x, P.B, P.F, P.Hf};
    const SmallGemm GW{P.dh, 1, P.Hf, P.x, P.ld_x, 1, nullptr, P.dW1, P.F, P.Hf, P.F, P.B};
    const int n1 = head_tiles(GX.M, GX.N, HEAD_H_TS), n2 = head_tiles(GW.M, GW.N, HEAD_G_TS);
    const int b = blockIdx.x;
    if (b < n1) { small_gemm_tile(GX, b, *reinterpret_cast<SmallGemmLds<HEAD_H_TS> *>(&L)); return; }
    if (b < n1 + n2) { small_gemm_tile(GW, b - n1, L); return; }
    const int Hf = P.Hf, T = P.T, B = P.B;
    const long long q = (long long)(b - n1 - n2) * 256 + threadIdx.x;
    if (q < Hf) {
        const float s = row_sum(P.dh + q, Hf, nullptr, 0, B);
        if (P.db1) P.db1[q] = s;
    } else if (q < Hf + (long long)T * Hf) {
        const int u = (int)(q - Hf), t = u / Hf, j = u % Hf;
        P.dW2[u] = row_sum(P.dout + t, T, P.a + j, Hf, B);
    } else if (q < Hf + (long long)T * Hf + T) {
        const int t = (int)(q - Hf - (long long)T * Hf);
        const float s = row_sum(P.dout + t, T, nullptr, 0, B);
        if (P.db2) P.db2[t] = s;
    } else if (q == Hf + (long long)T * Hf + T) {
        P.loss[0] = row_sum(P.lossrow, 1, nullptr, 0, B) * P.inv_n;
    }
}


// y_i *= s[0] for up to 8 buffers (the head's gradients times the incoming gradient of the loss)
struct ScaleJobs {
    float *p[8];
    long long n[8];
    int k;
    const float *s;
};
__global__ __launch_bounds__(256) void scale_kernel(ScaleJobs J) {
    const float s = J.s[0];
    for (int i = 0; i < J.k; ++i)
        for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < J.n[i]; e += (long long)gridDim.x * 256)
            J.p[i][e] *= s;
}
}  // namespace wd
