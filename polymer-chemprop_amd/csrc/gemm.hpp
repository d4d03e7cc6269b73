// gemm.hpp — fp32 MFMA GEMMs of the wD-MPNN encoder (v_mfma_f32_32x32x2_f32, exact f32 fma chain,
// 64 FLOP/clk/SIMD = the fp32 dense peak of MI355X).
//
// gemm_nt16_kernel  C[m][n] = epi( sum_k A(m,k) * B[n][k] )      unblocked forward layers (f32 A/B
//                                                                 variant) + backward data gradients
//     A = one or two dense row-major segments laid side by side along k (mpn.py:132's concat without a
//     copy), B = a packed weight [Np][Kp].  Every buffer is padded (rows to the 64-row tile, columns
//     and K to the 32-wide chunk, padding zero), so the loads are unconditional float4 and the
//     segment of a K-chunk is uniform over the workgroup: no per-element branches or waits in the
//     K loop.
// Src / Seg  the row-major operands of the weight-gradient GEMM (gemm_x6.hpp gemm_tn_x6_kernel):
//     segments laid side by side along the columns, plus a ones column for the bias.
//
// Tiles: BM x BN per workgroup of WM x WN waves; K in chunks of 32 staged through LDS (row stride 36
// floats, conflict-free for ds_read_b128 and ds_write_b128: checked by brute force over the lane
// groups of MI355X_MICROARCH.md §LDS).
#pragma once
#include "common.hpp"
#include "planes.hpp"

namespace wd {

constexpr int BK = 32;

// EPI_ACTBWD: the activation backward of the layer below fused into a data-gradient GEMM (the elementwise
// branch of act_bwd_kernel): Y = dZ = C * dropout * act'(Z) (+ add_in), res_out (+)= dZ, PReLU slope partials
enum EpiKind : int { EPI_ACT = 0, EPI_STORE = 1, EPI_ACTBWD = 2 };

struct Epi {
    int kind;
    const float *bias;     // [N] (EPI_ACT; packed, zero padded)
    const float *resid;    // [M][ld] or null (mpn.py:123 `input + message`)
    float *Z;              // pre-activation out or null
    float *Y;              // output (EPI_ACT: may be null when `planes` is set)
    int ld;                // row stride of resid / Z / Y
    uint8_t *planes;       // EPI_ACT: also store Y as bf16x3 plane tiles with 128-row blocks (the
    const int32_t *plane_row;  //   molecule-blocked bond layout) at row plane_row[i] (< 0: skipped)
    int planes_kp;         //   column extent of that plane-tile matrix
    long long slab_stride; // EPI_STORE (tn): Y += blockIdx.y * slab_stride
    int accumulate;        // EPI_STORE: Y += C
    int act;
    const float *slope;    // PReLU slope (device)
    float p_drop;
    uint64_t seed;
    uint32_t layer;
    // EPI_ACTBWD
    const float *add_in;   // [M][ld] or null
    float *res_out;        // [M][ld] or null: res_out = (res_init ? 0 : res_out) + dZ
    int res_init;
    int rows_valid;        // rows >= rows_valid get dZ = 0
    float *prelu_part;     // per-workgroup PReLU slope partial (indexed by blockIdx.x) or null
    // EPI_ACT, gemm_x6g only: per (64-row tile, 64-column tile) the max |amax_act(z)| of the output columns
    // < amax_cols -> amax[row tile * amax_cols / 64 + column tile] (the h2 scale words of a fused layer's
    // first operand, planes.hpp; slope: PReLU's).  EPI_ACTBWD, gemm_x6_kernel: per output tile the max
    // |dropout(act(Z))| -> amax[row tile * tiles_n + column tile]
    uint32_t *amax;
    int amax_cols, amax_act;
};

template <int ACT, int TM, int TN>
__device__ __forceinline__ void epilogue_act(const Epi &E, floatx16 (&acc)[TM][TN], int i0, int j0, int h, int l32,
                                             int M, int N, float *Y) {
    const float slope = (E.kind == EPI_ACT && E.act == ACT_PRELU) ? E.slope[0] : 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const int j = j0 + b * 32 + l32;
            if (j >= N) continue;
            const float bias = (E.kind == EPI_ACT && E.bias) ? E.bias[j] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = i0 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (i >= M) continue;
                const size_t o = (size_t)i * E.ld + j;
                const float v = acc[a][b][r];
                if (E.kind == EPI_ACT) {
                    float z = v + bias;
                    if (E.resid) z += E.resid[o];
                    if (E.Z) E.Z[o] = z;
                    float y = act_fwd(ACT, z, slope);
                    if (E.p_drop > 0.f) y *= dropout_scale(E.seed, E.layer, i, j, E.p_drop);
                    Y[o] = y;
                } else {
                    Y[o] = E.accumulate ? Y[o] + v : v;
                }
            }
        }
}

// ---------------------------------------------------------------------------------------------
// NT kernel over padded dense operands
// ---------------------------------------------------------------------------------------------
struct NtParams {
    const float *a0; int lda0; int ka0;   // A segment 0: [Mp][lda0], K extent ka0 (multiple of 32)
    const float *a1; int lda1; int ka1;   // A segment 1 (ka1 = 0: absent)
    const float *b; int ldb;              // B packed [Np][ldb], ldb >= ka0 + ka1
    int M, N;                             // valid output rows / cols written (<= padded extents)
    int tiles_m, tiles_n;
    Epi epi;
};

// ---------------------------------------------------------------------------------------------
// NT GEMM on f32 MFMA: the wave's 32x32 block is 2x2 v_mfma_f32_16x16x4_f32 tiles (4 independent
// accumulator chains), two-chunk register prefetch, two LDS stages.  Lane l = (i = l&15,
// g = l>>4) supplies k = 8g + s at step s (0..7 per 32-chunk): two ds_read_b128 per operand tile.
// C/D map of 16x16: col = l&15, row = 4*(l>>4) + reg.
// ---------------------------------------------------------------------------------------------
typedef float floatx4 __attribute__((ext_vector_type(4)));

// Row-major float4 epilogue of a BM x BN tile over NT threads: thread t owns float4 column c4 =
// t % (BN/4) of rows t / (BN/4) + p * (NT*4/BN).  Requires ld % 4 == 0 and 16-byte aligned
// resid / Z / Y (checked by the launcher).
template <int BM, int BN, int NT>
struct EpiPrefetch {
    static constexpr int C4 = BN / 4, RS = NT / C4, NP = BM / RS;
    float4 resid[NP];
    float4 bias;
    __device__ __forceinline__ void load(const Epi &E, int m0, int n0, int M, int N) {
        const int t = threadIdx.x, c = n0 + (t % C4) * 4;
        bias = f4zero();
        if (E.kind == EPI_ACT && E.bias && c < N) bias = ld4(E.bias + c);
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const int i = m0 + t / C4 + p * RS;
            resid[p] = (E.kind == EPI_ACT && E.resid && i < M && c < N) ? ld4(E.resid + (size_t)i * E.ld + c)
                                                                       : f4zero();
        }
    }
};

// returns this thread's max |amax_act(z)| (Epi.amax; 0 without)
template <int ACT, int BM, int BN, int NT>
__device__ __forceinline__ uint32_t epilogue_v4_act(const Epi &E, const float *C, int ldc, int m0, int n0, int M, int N,
                                                    const EpiPrefetch<BM, BN, NT> &ep) {
    using EP = EpiPrefetch<BM, BN, NT>;
    const int t = threadIdx.x, cl = (t % EP::C4) * 4, j = n0 + cl;
    uint32_t mx = 0;
    if (j >= N) return mx;
    const float slope = (E.kind == EPI_ACT && E.act == ACT_PRELU) ? E.slope[0] : 0.f;
    const bool amx = E.kind == EPI_ACT && E.amax && j < E.amax_cols;
    const float aslope = amx && E.amax_act == ACT_PRELU ? E.slope[0] : 0.f;
#pragma unroll
    for (int p = 0; p < EP::NP; ++p) {
        const int rl = t / EP::C4 + p * EP::RS, i = m0 + rl;
        if (i >= M) continue;
        const float4 v = ld4(C + rl * ldc + cl);
        const size_t o = (size_t)i * E.ld + j;
        float vv[4] = {v.x, v.y, v.z, v.w};
        float out[4];
        if (E.kind == EPI_ACT) {
            const float bb[4] = {ep.bias.x, ep.bias.y, ep.bias.z, ep.bias.w};
            const float rr[4] = {ep.resid[p].x, ep.resid[p].y, ep.resid[p].z, ep.resid[p].w};
            float z[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                z[q] = vv[q] + bb[q] + rr[q];
                float y = act_fwd(ACT, z[q], slope);
                if (E.p_drop > 0.f) y *= dropout_scale(E.seed, E.layer, i, j + q, E.p_drop);
                out[q] = y;
                if (amx) mx = max(mx, absbits(act_fwd(E.amax_act, z[q], aslope)));
            }
            if (j + 4 <= N) {
                if (E.Z) st4(E.Z + o, make_float4(z[0], z[1], z[2], z[3]));
                if (E.Y) gst16(E.Y + o, u32x4{__float_as_uint(out[0]), __float_as_uint(out[1]), __float_as_uint(out[2]),
                                               __float_as_uint(out[3])});
            } else {
                for (int q = 0; q < N - j; ++q) {
                    if (E.Z) E.Z[o + q] = z[q];
                    if (E.Y) E.Y[o + q] = out[q];
                }
            }
            if (E.planes) {  // padded columns (>= N) of the plane tiles hold act(0) = 0 from the zero padding
                const int pr = E.plane_row[i];
                if (pr >= 0) x6_store4<128>(E.planes, E.planes_kp, pr, j, make_float4(out[0], out[1], out[2], out[3]));
            }
        } else {
            if (j + 4 <= N) {
                float4 r = v;
                if (E.accumulate) {
                    const float4 y0 = ld4(E.Y + o);
                    r.x += y0.x; r.y += y0.y; r.z += y0.z; r.w += y0.w;
                }
                st4(E.Y + o, r);
            } else {
                for (int q = 0; q < N - j; ++q) E.Y[o + q] = E.accumulate ? E.Y[o + q] + vv[q] : vv[q];
            }
        }
    }
    return mx;
}


// returns this thread's max |dropout(act(Z))| when E.amax is set (the layer input M the weight-gradient
// GEMM restages from Z: its fp16-pair scale words), else 0
template <int ACT, int BM, int BN, int NT>
__device__ __forceinline__ uint32_t epilogue_v4_actbwd(const Epi &E, const float *C, int ldc, int m0, int n0, int M,
                                                       int N) {
    using EP = EpiPrefetch<BM, BN, NT>;
    const int t = threadIdx.x, cl = (t % EP::C4) * 4, j = n0 + cl;
    const float slope = ACT == ACT_PRELU ? E.slope[0] : 0.f;
    float pp = 0.f;
    uint32_t mx = 0;
    if (j < N) {  // (N % 4 == 0: checked by the launcher)
#pragma unroll
        for (int p = 0; p < EP::NP; ++p) {
            const int rl = t / EP::C4 + p * EP::RS, i = m0 + rl;
            if (i >= M) continue;
            const size_t o = (size_t)i * E.ld + j;
            const float4 g = ld4(C + rl * ldc + cl);
            float4 dz = f4zero();
            if (i < E.rows_valid) {
                const float4 z = ld4(E.Z + o);
                const float gg[4] = {g.x, g.y, g.z, g.w}, zz[4] = {z.x, z.y, z.z, z.w};
                float d[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float sd = E.p_drop > 0.f ? dropout_scale(E.seed, E.layer, i, j + q, E.p_drop) : 1.f;
                    d[q] = gg[q] * sd * act_grad(ACT, zz[q], slope);
                    if (ACT == ACT_PRELU && !(zz[q] > 0.f)) pp += zz[q] * gg[q] * sd;
                    if (E.amax) mx = max(mx, absbits(act_fwd(ACT, zz[q], slope) * sd));
                }
                dz = make_float4(d[0], d[1], d[2], d[3]);
                if (E.add_in) {
                    const float4 a = ld4(E.add_in + o);
                    dz.x += a.x; dz.y += a.y; dz.z += a.z; dz.w += a.w;
                }
            }
            if (E.res_out) {
                float4 r = dz;
                if (!E.res_init) {
                    const float4 r0 = ld4(E.res_out + o);
                    r.x += r0.x; r.y += r0.y; r.z += r0.z; r.w += r0.w;
                }
                st4(E.res_out + o, r);
            }
            st4(E.Y + o, dz);
        }
    }
    if (ACT == ACT_PRELU && E.prelu_part) {  // fixed-order block sum (deterministic)
        __shared__ float red[NT];
        red[t] = pp;
        __syncthreads();
        for (int s2 = NT / 2; s2 > 0; s2 >>= 1) {
            if (t < s2) red[t] += red[t + s2];
            __syncthreads();
        }
        if (t == 0) E.prelu_part[blockIdx.x] = red[0];
    }
    return mx;
}

// the epilogues with the activation dispatched once per call (common.hpp with_act)
template <int TM, int TN>
__device__ __forceinline__ void epilogue(const Epi &E, floatx16 (&acc)[TM][TN], int i0, int j0, int h, int l32,
                                         int M, int N, float *Y) {
    if (E.kind == EPI_ACT)
        with_act(E.act, [&](auto a) { epilogue_act<decltype(a)::value>(E, acc, i0, j0, h, l32, M, N, Y); });
    else
        epilogue_act<ACT_IDENTITY>(E, acc, i0, j0, h, l32, M, N, Y);
}
template <int BM, int BN, int NT>
__device__ __forceinline__ uint32_t epilogue_v4(const Epi &E, const float *C, int ldc, int m0, int n0, int M, int N,
                                                const EpiPrefetch<BM, BN, NT> &ep) {
    uint32_t mx = 0;
    if (E.kind == EPI_ACT)
        with_act(E.act, [&](auto a) { mx = epilogue_v4_act<decltype(a)::value>(E, C, ldc, m0, n0, M, N, ep); });
    else if (E.kind == EPI_ACTBWD)
        with_act(E.act, [&](auto a) { mx = epilogue_v4_actbwd<decltype(a)::value, BM, BN, NT>(E, C, ldc, m0, n0, M, N); });
    else
        mx = epilogue_v4_act<ACT_IDENTITY>(E, C, ldc, m0, n0, M, N, ep);
    return mx;
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void gemm_nt16_kernel(NtParams P) {
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
    constexpr int LD = BK + 4;
    constexpr int A_V4 = BM * 8, B_V4 = BN * 8;
    constexpr int PA = A_V4 / NT, PB = B_V4 / NT;
    constexpr int STAGE = (BM + BN) * LD;
    static_assert(A_V4 % NT == 0 && B_V4 % NT == 0, "tile must divide evenly over threads");
    __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave / WN, wj = wave % WN, g = lane >> 4, i16 = lane & 15;
    const int tile = xcd_tile(blockIdx.x, P.tiles_m * P.tiles_n);
    const int mt = tile / P.tiles_n, nt = tile % P.tiles_n;
    const int m0 = mt * BM, n0 = nt * BN;
    const int K = P.ka0 + P.ka1;
    EpiPrefetch<BM, BN, NT> ep;
    ep.load(P.epi, m0, n0, P.M, P.N);

    floatx4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

    const float *pb[PB];
#pragma unroll
    for (int p = 0; p < PB; ++p) {
        const int q = tid + p * NT, r = q >> 3, c = (q & 7) * 4;
        pb[p] = P.b + (size_t)(n0 + r) * P.ldb + c;
    }
    struct Regs { float4 a[PA], b[PB]; };
    auto load_chunk = [&](Regs &R, int k0) {
        const bool seg1 = k0 >= P.ka0;
        const float *base = seg1 ? P.a1 : P.a0;
        const int ld = seg1 ? P.lda1 : P.lda0;
        const int kk = seg1 ? k0 - P.ka0 : k0;
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int q = tid + p * NT, r = q >> 3, c = (q & 7) * 4;
            R.a[p] = ld4(base + (size_t)(m0 + r) * ld + kk + c);
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) R.b[p] = ld4(pb[p] + k0);
    };
    auto store_chunk = [&](const Regs &R, float *st) {
#pragma unroll
        for (int p = 0; p < PA; ++p) {
            const int q = tid + p * NT, r = q >> 3, c = (q & 7) * 4;
            st4(st + r * LD + c, R.a[p]);
        }
#pragma unroll
        for (int p = 0; p < PB; ++p) {
            const int q = tid + p * NT, r = q >> 3, c = (q & 7) * 4;
            st4(st + BM * LD + r * LD + c, R.b[p]);
        }
    };
    auto compute = [&](const float *As) {
        const float *Bs = As + BM * LD;
        float af[TM][8], bf[TN][8];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
            const float *src = As + (wi * (BM / WM) + a * 16 + i16) * LD + 8 * g;
            const float4 v0 = ld4(src), v1 = ld4(src + 4);
            af[a][0] = v0.x; af[a][1] = v0.y; af[a][2] = v0.z; af[a][3] = v0.w;
            af[a][4] = v1.x; af[a][5] = v1.y; af[a][6] = v1.z; af[a][7] = v1.w;
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
            const float *src = Bs + (wj * (BN / WN) + b * 16 + i16) * LD + 8 * g;
            const float4 v0 = ld4(src), v1 = ld4(src + 4);
            bf[b][0] = v0.x; bf[b][1] = v0.y; bf[b][2] = v0.z; bf[b][3] = v0.w;
            bf[b][4] = v1.x; bf[b][5] = v1.y; bf[b][6] = v1.z; bf[b][7] = v1.w;
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < TN; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
    };
    const int nchunks = K / BK;
    Regs R0, R1;
    load_chunk(R0, 0);
    load_chunk(R1, min(1, nchunks - 1) * BK);
    store_chunk(R0, lds);
    __syncthreads();
    auto step = [&](int kc, Regs &Rnext, Regs &Rfree) {
        load_chunk(Rfree, min(kc + 2, nchunks - 1) * BK);
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

    // epilogue: the C tile goes through LDS (row stride BN + 4: conflict-free for the 16x16 C/D
    // layout) so that every lane loads resid and stores Z / Y as coalesced float4 (the scalar-store
    // tail was store-issue bound); resid and bias were prefetched before the K loop.
    constexpr int LDC = BN + 4;
    static_assert(BM * LDC <= 2 * STAGE, "C tile must fit in the staging LDS");
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                lds[(wi * (BM / WM) + a * 16 + 4 * g + r) * LDC + wj * (BN / WN) + b * 16 + i16] = acc[a][b][r];
    __syncthreads();
    epilogue_v4<BM, BN, NT>(P.epi, lds, LDC, m0, n0, P.M, P.N, ep);
}

// ---------------------------------------------------------------------------------------------
// Weight-gradient operands: both k-major (rows = m), masked at the split's row range.
// ---------------------------------------------------------------------------------------------
// SEG_ACT: the activations M = dropout(act(Z)) recomputed from the saved pre-activations Z while
// loading (the fused training forward keeps Z_t, not M_t: mpn.py:97, 123-124)
enum SegKind : int { SEG_DENSE = 0, SEG_ACT = 1, SEG_ONES = 2 };

struct Seg {
    const float *src;
    int ld;
    int K;      // width (padded extent; zeros beyond the real width are fine)
    int kp0;    // first column in the operand's column space (multiple of 4)
    int kind;
    int act; const float *slope; float p_drop; uint64_t seed; uint32_t layer;  // SEG_ACT
};

struct Src {
    Seg s[3];
    int nseg;
    int rows;      // valid rows
    int cols_p;    // column extent (multiple of 4)
};

__device__ __forceinline__ float4 seg_load4(const Seg &g, int r, int kk) {
    if (kk >= g.K) return f4zero();
    if (g.kind == SEG_ONES) return kk == 0 ? make_float4(1.f, 0.f, 0.f, 0.f) : f4zero();
    float4 v = ld4(g.src + (size_t)r * g.ld + kk);
    if (g.kind == SEG_ACT) {
        const float sl = g.act == ACT_PRELU ? g.slope[0] : 0.f;
        v.x = act_fwd(g.act, v.x, sl); v.y = act_fwd(g.act, v.y, sl);
        v.z = act_fwd(g.act, v.z, sl); v.w = act_fwd(g.act, v.w, sl);
        if (g.p_drop > 0.f) {
            v.x *= dropout_scale(g.seed, g.layer, r, kk, g.p_drop);
            v.y *= dropout_scale(g.seed, g.layer, r, kk + 1, g.p_drop);
            v.z *= dropout_scale(g.seed, g.layer, r, kk + 2, g.p_drop);
            v.w *= dropout_scale(g.seed, g.layer, r, kk + 3, g.p_drop);
        }
    }
    return v;
}

__device__ __forceinline__ float4 src_load4(const Src &S, int r, int cp, int rlim) {
    if (r >= rlim || cp >= S.cols_p) return f4zero();
    int s = 0;
    if (S.nseg > 1 && cp >= S.s[1].kp0) s = 1;
    if (S.nseg > 2 && cp >= S.s[2].kp0) s = 2;
    const Seg &g = s == 0 ? S.s[0] : (s == 1 ? S.s[1] : S.s[2]);
    return seg_load4(g, r, cp - g.kp0);
}


}  // namespace wd
