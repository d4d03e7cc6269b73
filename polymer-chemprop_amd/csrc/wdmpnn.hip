// wdmpnn.hip — MI355X (gfx950) wD-MPNN encoder: kernels + C-ABI (include/wdmpnn.h).
//
// Forward = MPNEncoder.forward (chemprop/models/mpn.py:66-173) as depth+2 (+1 with atom descriptors)
// launches of one fused gather-GEMM kernel (gemm_gather.hpp) and one readout kernel:
//
//   L0        M0 = act(f_bonds W_i^T (+b_i))                          mpn.py:92-97
//   L1..T-1   M_t = act(Z0 + X_t W_h^T (+b_h)),                        mpn.py:100-124
//             X_t[b] = sum_{j in in(b2a[b])} w_j M_{t-1}[j] - M_{t-1}[b2revb[b]]
//             (gathered into LDS inside the GEMM; the reverse term is folded into the gather list
//              as coefficient w_rev - 1, dropped when it is 0)
//   LT        h = act([f_atoms | sum_{j in in(a)} w_j M_{T-1}[j]] W_o^T + b_o)   mpn.py:126-134
//   (LT+1     hd = [h | desc] W_d^T + b_d                              mpn.py:136-143)
//   readout   out_i = Xn_i * sum_a w_a h_a / sum_a w_a  (mean|sum|norm)  mpn.py:145-171
//
// Backward = the autograd graph of the same (used by train.py:79) with deterministic, atomics-free
// kernels: transposed gather lists for the scatter-adds, split-K slabs + ordered reduction for the
// weight gradients.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gemm_gather.hpp"
#include "wdmpnn.h"

using namespace wd;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define WD_CHECK_LAUNCH(what)                                                              \
    do {                                                                                   \
        hipError_t e_ = hipGetLastError();                                                 \
        if (e_ != hipSuccess) return fail(-(int)e_, "%s: %s", what, hipGetErrorString(e_)); \
    } while (0)

inline int round4(int x) { return (x + 3) & ~3; }
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ------------------------------------------------------------------------------------------------
// small kernels
// ------------------------------------------------------------------------------------------------

// mpn.py:145-171: per-molecule weighted readout.  One workgroup per molecule, columns over lanes.
__global__ __launch_bounds__(128) void readout_kernel(const float *__restrict__ h, int ldh, int ncols,
                                                      const float *__restrict__ w_atoms,
                                                      const int32_t *__restrict__ mol_start,
                                                      const int32_t *__restrict__ mol_size,
                                                      const float *__restrict__ xn, int agg, float norm,
                                                      const float *__restrict__ zero_vec,
                                                      float *__restrict__ out) {
    const int i = blockIdx.x;
    const int a0 = mol_start[i], n = mol_size[i];
    if (n == 0) {  // mpn.py:148-149 cached_zero_vector (no Xn factor)
        for (int c = threadIdx.x; c < ncols; c += blockDim.x) out[(size_t)i * ncols + c] = zero_vec[c];
        return;
    }
    float wsum = 0.f;
    for (int a = 0; a < n; ++a) wsum += w_atoms[a0 + a];
    const float x = xn[i];
    for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
        float s = 0.f;
        for (int a = 0; a < n; ++a) s += w_atoms[a0 + a] * h[(size_t)(a0 + a) * ldh + c];
        float v = agg == WD_AGG_MEAN ? s / wsum : (agg == WD_AGG_NORM ? s / norm : s);
        out[(size_t)i * ncols + c] = x * v;
    }
}

// d readout / d h: dh[a] = dout[i] * Xn_i * w_a * (1/sum w | 1 | 1/norm); rows outside every scope
// stay 0 (caller memsets).
__global__ __launch_bounds__(128) void readout_bwd_kernel(const float *__restrict__ dout, int ncols,
                                                          const float *__restrict__ w_atoms,
                                                          const int32_t *__restrict__ mol_start,
                                                          const int32_t *__restrict__ mol_size,
                                                          const float *__restrict__ xn, int agg, float norm,
                                                          float *__restrict__ dh, int lddh) {
    const int i = blockIdx.x;
    const int a0 = mol_start[i], n = mol_size[i];
    if (n == 0) return;
    float wsum = 0.f;
    for (int a = 0; a < n; ++a) wsum += w_atoms[a0 + a];
    const float x = xn[i];
    const float scale = agg == WD_AGG_MEAN ? 1.f / wsum : (agg == WD_AGG_NORM ? 1.f / norm : 1.f);
    for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
        const float g = dout[(size_t)i * ncols + c] * x;
        const float gs = agg == WD_AGG_MEAN ? g / wsum : g * scale;
        for (int a = 0; a < n; ++a) dh[(size_t)(a0 + a) * lddh + c] = gs * w_atoms[a0 + a];
    }
}

// mpn.py:101-102: message = (message + message[b2revb]) / 2
__global__ __launch_bounds__(256) void symmetrize_kernel(const float *__restrict__ m, const int32_t *__restrict__ rev,
                                                         int rows, int cols, float *__restrict__ out) {
    const size_t total = (size_t)rows * cols;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / cols), c = (int)(t % cols);
        out[t] = (m[t] + m[(size_t)rev[r] * cols + c]) / 2.0f;
    }
}

// Backward of one activation layer, fused with the gather that produces its incoming gradient:
//   g   = sum_e coef[e] * G[idx[e]]         (csr) | 0.5*(G[r] + G[rev[r]]) (sym) | G[r] (dense)
//   dz  = g * dropout_scale * act'(z)        (Z == null: dz = g, gather only)
//   dz += add_in[r]                           (residual gradient of mpn.py:123 reaching input)
//   res_out (=|+=) dz                         (accumulate the residual gradient)
//   prelu partial: sum over z<=0 of z * g * dropout_scale
struct ActBwd {
    const float *G; int ldg;
    const int32_t *ptr; const int32_t *idx; const float *coef;
    const int32_t *sym_rev;
    const float *Z; int act; const float *slope; float p_drop; uint64_t seed; uint32_t layer;
    const float *add_in;
    float *res_out; int res_init;
    float *out;
    float *prelu_part;
    int rows, cols;
};

__global__ __launch_bounds__(256) void act_bwd_kernel(ActBwd P) {
    __shared__ float red[256];
    const float slope = (P.Z && P.act == ACT_PRELU) ? P.slope[0] : 0.f;
    float ppart = 0.f;
    const size_t total = (size_t)P.rows * P.cols;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(t / P.cols), c = (int)(t % P.cols);
        float g;
        if (P.ptr) {
            g = 0.f;
            for (int e = P.ptr[r]; e < P.ptr[r + 1]; ++e)
                g = fmaf(P.coef ? P.coef[e] : 1.f, P.G[(size_t)P.idx[e] * P.ldg + c], g);
        } else if (P.sym_rev) {
            g = (P.G[(size_t)r * P.ldg + c] + P.G[(size_t)P.sym_rev[r] * P.ldg + c]) * 0.5f;
        } else {
            g = P.G[(size_t)r * P.ldg + c];
        }
        float dz = g;
        if (P.Z) {
            const float z = P.Z[t];
            const float s = P.p_drop > 0.f ? dropout_scale(P.seed, P.layer, r, c, P.p_drop) : 1.f;
            dz = g * s * act_grad(P.act, z, slope);
            if (P.act == ACT_PRELU && !(z > 0.f)) ppart += z * g * s;
        }
        if (P.add_in) dz += P.add_in[t];
        if (P.res_out) P.res_out[t] = P.res_init ? dz : P.res_out[t] + dz;
        P.out[t] = dz;
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

struct SlabSeg { int kp0, K, wcol, kind; float *dst; };
struct SlabReduce {
    const float *slab; int nsplit; long long slab_stride; int ld_slab;
    int rows;  // output rows (n)
    SlabSeg s[3]; int nseg;
    int ldw;
};

// dW[n][wcol + kk] = sum_z slab[z][n][kp0 + kk]  (fixed split order: deterministic)
__global__ __launch_bounds__(256) void slab_reduce_kernel(SlabReduce P) {
    const int n = blockIdx.x;
    for (int si = 0; si < P.nseg; ++si) {
        const SlabSeg g = P.s[si];
        if (!g.dst) continue;
        for (int kk = threadIdx.x; kk < g.K; kk += blockDim.x) {
            float acc = 0.f;
            for (int z = 0; z < P.nsplit; ++z)
                acc += P.slab[(size_t)z * P.slab_stride + (size_t)n * P.ld_slab + g.kp0 + kk];
            if (g.kind == SEG_ONES) g.dst[n] = acc;
            else g.dst[(size_t)n * P.ldw + g.wcol + kk] = acc;
        }
    }
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

// ------------------------------------------------------------------------------------------------
// host helpers
// ------------------------------------------------------------------------------------------------
bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

Seg seg_dense(const float *src, int ld, int K, int kp0) {
    Seg s{};
    s.src = src; s.ld = ld; s.K = K; s.kp0 = kp0; s.kind = SEG_DENSE;
    s.vec = (ld % 4 == 0) && aligned16(src);
    return s;
}

Seg seg_gather(const float *src, int ld, int K, int kp0, const WdCsr &csr) {
    Seg s = seg_dense(src, ld, K, kp0);
    s.kind = SEG_GATHER; s.ptr = csr.ptr; s.idx = csr.idx; s.coef = csr.coef;
    return s;
}

Seg seg_ones(int kp0) {
    Seg s{};
    s.K = 1; s.kp0 = kp0; s.kind = SEG_ONES; s.ld = 1;
    return s;
}

Src make_src(int rows, std::initializer_list<Seg> segs) {
    Src S{};
    S.rows = rows;
    S.nseg = 0;
    int kp = 0;
    for (const Seg &g : segs) {
        S.s[S.nseg] = g;
        S.s[S.nseg].kp0 = kp;
        kp += round4(g.K);
        ++S.nseg;
    }
    S.cols_p = kp;
    return S;
}

// B operand of an NT layer: the weight matrix W[n][wcol + k] laid out with the same padded column
// segments as the A operand.
Src weight_src_like(const Src &A, const float *W, int ldw, int nrows, const int *wcol) {
    Src S{};
    S.rows = nrows; S.nseg = A.nseg; S.cols_p = A.cols_p;
    for (int i = 0; i < A.nseg; ++i) S.s[i] = seg_dense(W + wcol[i], ldw, A.s[i].K, A.s[i].kp0);
    return S;
}

Epi epi_act(int act, const float *slope, const float *bias, const float *resid, int ld_resid, float *Z, float *Y,
            int ld, const WdConfig *c, uint32_t layer) {
    Epi e{};
    e.kind = EPI_ACT; e.act = act; e.slope = slope; e.bias = bias; e.resid = resid; e.ld_resid = ld_resid;
    e.Z = Z; e.ld_z = ld; e.Y = Y; e.ld_y = ld;
    e.p_drop = c->dropout; e.seed = c->seed; e.layer = layer;
    return e;
}

Epi epi_store(float *Y, int ld, long long slab_stride, int accumulate) {
    Epi e{};
    e.kind = EPI_STORE; e.Y = Y; e.ld_y = ld; e.slab_stride = slab_stride; e.accumulate = accumulate;
    return e;
}

constexpr int GBM = 64, GBN = 64, GWM = 2, GWN = 2;

int gemm_nt(const Src &A, const Src &B, int M, int N, const Epi &epi, hipStream_t st) {
    if (M <= 0 || N <= 0) return 0;
    GemmParams P{};
    P.A = A; P.B = B; P.M = M; P.N = N; P.K = A.cols_p; P.k_per_split = ((A.cols_p + BK - 1) / BK) * BK;
    P.tiles_n = (N + GBN - 1) / GBN;
    P.epi = epi;
    dim3 grid(((M + GBM - 1) / GBM) * P.tiles_n, 1);
    hipLaunchKernelGGL((gemm_kernel<GBM, GBN, GWM, GWN, false, false>), grid, dim3(64 * GWM * GWN), 0, st, P);
    WD_CHECK_LAUNCH("gemm_nt");
    return 0;
}

// C[m][n] = sum_k A[m][k] * W[k][wcol + n]  (A dense rows, B = rows k of W)
int gemm_nn(const Src &A, const float *W, int ldw, int wcol, int M, int N, int K, const Epi &epi, hipStream_t st) {
    if (M <= 0 || N <= 0) return 0;
    GemmParams P{};
    P.A = A;
    P.B = make_src(K, {seg_dense(W + wcol, ldw, N, 0)});
    P.M = M; P.N = N; P.K = K; P.k_per_split = ((K + BK - 1) / BK) * BK;
    P.tiles_n = (N + GBN - 1) / GBN;
    P.epi = epi;
    dim3 grid(((M + GBM - 1) / GBM) * P.tiles_n, 1);
    hipLaunchKernelGGL((gemm_kernel<GBM, GBN, GWM, GWN, false, true>), grid, dim3(64 * GWM * GWN), 0, st, P);
    WD_CHECK_LAUNCH("gemm_nn");
    return 0;
}

// slab[z][n][j] (+)= sum_{m in split z} dZ[m][n] * X(m, j)
struct TnPlan { int nsplit; int k_per_split; long long slab_stride; int ld_slab; };

TnPlan tn_plan(int n_out, int cols_p, int m_rows) {
    TnPlan t{};
    const int tiles = ((n_out + GBM - 1) / GBM) * ((cols_p + GBN - 1) / GBN);
    int chunks = (m_rows + BK - 1) / BK;
    int ns = (1024 + tiles - 1) / tiles;
    if (ns > chunks) ns = chunks;
    if (ns < 1) ns = 1;
    int cps = (chunks + ns - 1) / ns;
    t.k_per_split = cps * BK;
    t.nsplit = (m_rows + t.k_per_split - 1) / t.k_per_split;
    if (t.nsplit < 1) t.nsplit = 1;
    t.ld_slab = cols_p;
    t.slab_stride = (long long)n_out * cols_p;
    return t;
}

int gemm_tn(const Src &dZ, const Src &X, int n_out, int m_rows, const TnPlan &tp, float *slab, int accumulate,
            hipStream_t st) {
    if (n_out <= 0 || m_rows <= 0) return 0;
    GemmParams P{};
    P.A = dZ; P.B = X; P.M = n_out; P.N = X.cols_p; P.K = m_rows; P.k_per_split = tp.k_per_split;
    P.tiles_n = (X.cols_p + GBN - 1) / GBN;
    P.epi = epi_store(slab, tp.ld_slab, tp.slab_stride, accumulate);
    dim3 grid(((n_out + GBM - 1) / GBM) * P.tiles_n, tp.nsplit);
    hipLaunchKernelGGL((gemm_kernel<GBM, GBN, GWM, GWN, true, true>), grid, dim3(64 * GWM * GWN), 0, st, P);
    WD_CHECK_LAUNCH("gemm_tn");
    return 0;
}

int slab_reduce(const TnPlan &tp, const float *slab, int n_out, const Src &X, float *dW, int ldw, const int *wcol,
                float *db, hipStream_t st) {
    SlabReduce R{};
    R.slab = slab; R.nsplit = tp.nsplit; R.slab_stride = tp.slab_stride; R.ld_slab = tp.ld_slab; R.rows = n_out;
    R.nseg = X.nseg; R.ldw = ldw;
    for (int i = 0; i < X.nseg; ++i) {
        R.s[i].kp0 = X.s[i].kp0; R.s[i].K = X.s[i].K; R.s[i].kind = X.s[i].kind;
        R.s[i].wcol = X.s[i].kind == SEG_ONES ? 0 : wcol[i];
        R.s[i].dst = X.s[i].kind == SEG_ONES ? db : dW;
    }
    if (!dW && !db) return 0;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(n_out), dim3(256), 0, st, R);
    WD_CHECK_LAUNCH("slab_reduce");
    return 0;
}

int ew_blocks(size_t total) {
    size_t b = (total + 255) / 256;
    if (b > 4096) b = 4096;
    if (b < 1) b = 1;
    return (int)b;
}

// ------------------------------------------------------------------------------------------------
// workspace layouts
// ------------------------------------------------------------------------------------------------
struct Dims {
    int H, T, R, Va, B, Fa, Fb, d, Hout, Kin;
    bool atom, undirected, save, desc;
};

int get_dims(const WdGraph *g, const WdParams *p, const WdConfig *c, Dims &D) {
    if (!g || !p || !c) return fail(WD_ERR_ARG, "null graph/params/config");
    if (c->depth < 1) return fail(WD_ERR_ARG, "depth must be >= 1 (got %d)", c->depth);
    if (p->hidden <= 0) return fail(WD_ERR_ARG, "hidden_size must be > 0");
    if (g->n_atoms < 1 || g->n_bonds < 1) return fail(WD_ERR_SHAPE, "n_atoms/n_bonds must include the pad row");
    if (c->activation < 0 || c->activation > WD_ACT_IDENTITY) return fail(WD_ERR_ARG, "bad activation %d", c->activation);
    if (c->aggregation < 0 || c->aggregation > WD_AGG_NORM) return fail(WD_ERR_ARG, "bad aggregation %d", c->aggregation);
    if (c->activation == WD_ACT_PRELU && !p->prelu) return fail(WD_ERR_ARG, "PReLU needs a slope pointer");
    if (!(c->dropout >= 0.f && c->dropout < 1.f)) return fail(WD_ERR_ARG, "dropout must be in [0, 1)");
    D.H = p->hidden; D.T = c->depth; D.Va = g->n_atoms; D.B = g->n_mols;
    D.atom = g->atom_messages != 0; D.undirected = c->undirected != 0; D.save = c->save_for_backward != 0;
    D.R = D.atom ? g->n_atoms : g->n_bonds;
    D.Fa = g->atom_fdim; D.Fb = g->bond_fdim;
    D.desc = g->atom_desc != nullptr && g->desc_dim > 0;
    D.d = D.desc ? g->desc_dim : 0;
    D.Hout = D.H + D.d;
    D.Kin = D.atom ? D.Fa : D.Fb;
    if (D.atom && D.undirected)
        return fail(WD_ERR_UNSUPPORTED, "undirected with atom_messages (the reference indexes atom messages "
                                        "with b2revb, mpn.py:101-102)");
    if (D.desc && (!p->W_d || !p->b_d)) return fail(WD_ERR_ARG, "atom descriptors need W_d and b_d");
    if (!p->W_i || !p->W_h || !p->W_o || !p->b_o || !p->zero_vec) return fail(WD_ERR_ARG, "missing weights");
    return 0;
}

struct FwdLayout {
    std::vector<size_t> Z, M, Ms;
    size_t Zo = 0, h = 0, Zd = 0, hd = 0, total = 0;
};

FwdLayout fwd_layout(const Dims &D) {
    FwdLayout L;
    size_t off = 0;
    auto take = [&](size_t floats) { size_t o = off; off = align256(off + floats * 4); return o; };
    const size_t msg = (size_t)D.R * D.H, atm = (size_t)D.Va * D.H, atd = (size_t)D.Va * D.Hout;
    const int nZ = D.save ? D.T : 1;
    for (int t = 0; t < nZ; ++t) L.Z.push_back(take(msg));
    const int nM = D.save ? D.T : (D.T > 1 ? 2 : 1);
    for (int t = 0; t < nM; ++t) L.M.push_back(take(msg));
    if (D.undirected) {
        const int nS = D.save ? D.T : 1;
        for (int t = 0; t < nS; ++t) L.Ms.push_back(take(msg));
    }
    if (D.save) L.Zo = take(atm);
    L.h = take(atm);
    if (D.desc) {
        if (D.save) L.Zd = take(atd);
        L.hd = take(atd);
    }
    L.total = off;
    return L;
}

struct BwdLayout {
    size_t dH = 0, dZd = 0, dHo = 0, dZo = 0, dA = 0, dZ0 = 0, dZ1 = 0, dRes = 0, dX = 0, dMs = 0, slab = 0,
           prelu = 0, total = 0;
    size_t slab_floats = 0, prelu_floats = 0;
};

// TN plans of the three weight-gradient GEMMs
Src x_src_in(const WdGraph *g, const Dims &D) {  // rows of W_i's input
    return D.atom ? make_src(D.R, {seg_dense(g->f_atoms, g->ld_atoms, D.Fa, 0), seg_ones(0)})
                  : make_src(D.R, {seg_dense(g->f_bonds + g->bond_col0, g->ld_bonds, D.Fb, 0), seg_ones(0)});
}
Src x_src_h(const WdGraph *g, const Dims &D, const float *srcM, bool ones) {  // gathered W_h input X_t
    if (D.atom) {
        Seg a = seg_gather(srcM, D.H, D.H, 0, g->msg_gather);
        Seg b = seg_gather(g->f_bonds + g->bond_col0, g->ld_bonds, D.Fb, 0, g->bond_feat_gather);
        return ones ? make_src(D.R, {a, b, seg_ones(0)}) : make_src(D.R, {a, b});
    }
    Seg a = seg_gather(srcM, D.H, D.H, 0, g->msg_gather);
    return ones ? make_src(D.R, {a, seg_ones(0)}) : make_src(D.R, {a});
}
Src x_src_o(const WdGraph *g, const Dims &D, const float *M_last, bool ones) {  // [f_atoms | A]
    Seg a = seg_dense(g->f_atoms, g->ld_atoms, D.Fa, 0);
    Seg b = seg_gather(M_last, D.H, D.H, 0, g->atom_gather);
    return ones ? make_src(D.Va, {a, b, seg_ones(0)}) : make_src(D.Va, {a, b});
}
Src x_src_d(const WdGraph *g, const Dims &D, const float *h, bool ones) {  // [h | desc]
    Seg a = seg_dense(h, D.H, D.H, 0);
    Seg b = seg_dense(g->atom_desc, D.d, D.d, 0);
    return ones ? make_src(D.Va, {a, b, seg_ones(0)}) : make_src(D.Va, {a, b});
}

BwdLayout bwd_layout(const WdGraph *g, const Dims &D) {
    BwdLayout L;
    size_t off = 0;
    auto take = [&](size_t floats) { size_t o = off; off = align256(off + floats * 4); return o; };
    const size_t msg = (size_t)D.R * D.H, atm = (size_t)D.Va * D.H;
    L.dH = take((size_t)D.Va * D.Hout);
    if (D.desc) { L.dZd = take((size_t)D.Va * D.Hout); L.dHo = take(atm); }
    L.dZo = take(atm);
    L.dA = take(atm);
    L.dZ0 = take(msg);
    L.dZ1 = take(msg);
    L.dRes = take(msg);
    L.dX = take(msg);
    if (D.undirected) L.dMs = take(msg);
    size_t slab = 0;
    auto upd = [&](int n_out, const Src &X, int m_rows) {
        TnPlan tp = tn_plan(n_out, X.cols_p, m_rows);
        size_t s = (size_t)tp.nsplit * tp.slab_stride;
        if (s > slab) slab = s;
    };
    upd(D.H, x_src_in(g, D), D.R);
    upd(D.H, x_src_h(g, D, nullptr, true), D.R);
    upd(D.H, x_src_o(g, D, nullptr, true), D.Va);
    if (D.desc) upd(D.Hout, x_src_d(g, D, nullptr, true), D.Va);
    L.slab_floats = slab;
    L.slab = take(slab);
    L.prelu_floats = (size_t)(D.T + 2) * 4096;
    L.prelu = take(L.prelu_floats);
    L.total = off;
    return L;
}

struct EventPool {
    int n = 0;
    std::vector<hipEvent_t> ev;  // 2 per pair
};

int record_prof(const WdConfig *c, int pair, int which, hipStream_t st) {
    if (!c->prof_pool) return 0;
    EventPool *pool = (EventPool *)c->prof_pool;
    const int slot = c->prof_slot + pair;
    if (slot < 0 || slot >= pool->n) return 0;
    if (hipEventRecord(pool->ev[2 * slot + which], st) != hipSuccess) return fail(WD_ERR_ARG, "hipEventRecord failed");
    return 0;
}

}  // namespace

// ================================================================================================
// C-ABI
// ================================================================================================
extern "C" {

int wdmpnn_abi_version(void) { return WDMPNN_ABI_VERSION; }

const char *wdmpnn_last_error(void) { return g_err.c_str(); }

int wdmpnn_workspace_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes) {
    Dims D;
    int rc = get_dims(g, p, c, D);
    if (rc) return rc;
    if (!bytes) return fail(WD_ERR_ARG, "null bytes");
    *bytes = fwd_layout(D).total;
    return 0;
}

int wdmpnn_backward_workspace_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes) {
    Dims D;
    int rc = get_dims(g, p, c, D);
    if (rc) return rc;
    if (!bytes) return fail(WD_ERR_ARG, "null bytes");
    *bytes = bwd_layout(g, D).total;
    return 0;
}

int wdmpnn_forward(const WdGraph *g, const WdParams *p, const WdConfig *c, void *workspace, size_t workspace_bytes,
                   float *out, void *stream) {
    Dims D;
    int rc = get_dims(g, p, c, D);
    if (rc) return rc;
    const FwdLayout L = fwd_layout(D);
    if (!workspace || workspace_bytes < L.total)
        return fail(WD_ERR_WORKSPACE, "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
    if (!out) return fail(WD_ERR_ARG, "null out");
    hipStream_t st = (hipStream_t)stream;
    char *ws = (char *)workspace;
    auto F = [&](size_t off) { return (float *)(ws + off); };
    const int H = D.H;

    // L0: input layer (mpn.py:92-97)
    {
        Src A = D.atom ? make_src(D.R, {seg_dense(g->f_atoms, g->ld_atoms, D.Fa, 0)})
                       : make_src(D.R, {seg_dense(g->f_bonds + g->bond_col0, g->ld_bonds, D.Fb, 0)});
        const int wcol[1] = {0};
        Src B = weight_src_like(A, p->W_i, D.Kin, H, wcol);
        rc = gemm_nt(A, B, D.R, H, epi_act(c->activation, p->prelu, p->b_i, nullptr, 0, F(L.Z[0]), F(L.M[0]), H, c, 0),
                     st);
        if (rc) return rc;
    }
    // L1..T-1: message passing (mpn.py:100-124)
    int cur = 0;
    for (int t = 1; t < D.T; ++t) {
        const int prev = D.save ? t - 1 : cur;
        const int next = D.save ? t : 1 - cur;
        const float *srcM = F(L.M[prev]);
        if (D.undirected) {
            float *ms = F(L.Ms[D.save ? t : 0]);
            const size_t total = (size_t)D.R * H;
            hipLaunchKernelGGL(symmetrize_kernel, dim3(ew_blocks(total)), dim3(256), 0, st, srcM, g->b2revb, D.R, H, ms);
            WD_CHECK_LAUNCH("symmetrize");
            srcM = ms;
        }
        Src A = x_src_h(g, D, srcM, false);
        const int wcol[2] = {0, H};
        Src B = weight_src_like(A, p->W_h, D.atom ? H + D.Fb : H, H, wcol);
        float *Zt = D.save ? F(L.Z[t]) : nullptr;
        if ((rc = record_prof(c, t - 1, 0, st))) return rc;
        rc = gemm_nt(A, B, D.R, H, epi_act(c->activation, p->prelu, p->b_h, F(L.Z[0]), H, Zt, F(L.M[next]), H, c, t),
                     st);
        if (rc) return rc;
        if ((rc = record_prof(c, t - 1, 1, st))) return rc;
        cur = next;
    }
    const float *M_last = F(L.M[D.save ? D.T - 1 : cur]);
    // LT: atom hidden states (mpn.py:126-134)
    {
        Src A = x_src_o(g, D, M_last, false);
        const int wcol[2] = {0, D.Fa};
        Src B = weight_src_like(A, p->W_o, D.Fa + H, H, wcol);
        float *Zo = D.save ? F(L.Zo) : nullptr;
        rc = gemm_nt(A, B, D.Va, H, epi_act(c->activation, p->prelu, p->b_o, nullptr, 0, Zo, F(L.h), H, c, D.T), st);
        if (rc) return rc;
    }
    const float *hfin = F(L.h);
    // LT+1: atom descriptors layer (mpn.py:136-143): Linear + dropout, no activation
    if (D.desc) {
        Src A = x_src_d(g, D, F(L.h), false);
        const int wcol[2] = {0, H};
        Src B = weight_src_like(A, p->W_d, D.Hout, D.Hout, wcol);
        float *Zd = D.save ? F(L.Zd) : nullptr;
        rc = gemm_nt(A, B, D.Va, D.Hout,
                     epi_act(WD_ACT_IDENTITY, nullptr, p->b_d, nullptr, 0, Zd, F(L.hd), D.Hout, c, D.T + 1), st);
        if (rc) return rc;
        hfin = F(L.hd);
    }
    // readout (mpn.py:145-171)
    if (D.B > 0) {
        hipLaunchKernelGGL(readout_kernel, dim3(D.B), dim3(128), 0, st, hfin, D.Hout, D.Hout, g->w_atoms, g->mol_start,
                           g->mol_size, g->degree_of_polym, c->aggregation, c->aggregation_norm, p->zero_vec, out);
        WD_CHECK_LAUNCH("readout");
    }
    return 0;
}

int wdmpnn_backward(const WdGraph *g, const WdParams *p, const WdConfig *c, const void *workspace,
                    size_t workspace_bytes, const float *dout, void *scratch, size_t scratch_bytes,
                    const WdGrads *grads, void *stream) {
    Dims D;
    int rc = get_dims(g, p, c, D);
    if (rc) return rc;
    if (!D.save) return fail(WD_ERR_ARG, "backward needs a forward run with save_for_backward=1");
    const FwdLayout L = fwd_layout(D);
    const BwdLayout Bl = bwd_layout(g, D);
    if (!workspace || workspace_bytes < L.total) return fail(WD_ERR_WORKSPACE, "forward workspace too small");
    if (!scratch || scratch_bytes < Bl.total)
        return fail(WD_ERR_WORKSPACE, "backward scratch too small: need %zu bytes, got %zu", Bl.total, scratch_bytes);
    if (!dout || !grads) return fail(WD_ERR_ARG, "null dout/grads");
    hipStream_t st = (hipStream_t)stream;
    const char *ws = (const char *)workspace;
    char *sc = (char *)scratch;
    auto F = [&](size_t off) { return (float *)(ws + off); };
    auto S = [&](size_t off) { return (float *)(sc + off); };
    const int H = D.H;
    const bool prelu = c->activation == WD_ACT_PRELU;
    float *prelu_part = S(Bl.prelu);
    int prelu_used = 0;
    if (prelu && hipMemsetAsync(prelu_part, 0, Bl.prelu_floats * 4, st) != hipSuccess)
        return fail(WD_ERR_ARG, "memset failed");

    auto act_bwd = [&](ActBwd P) -> int {
        const size_t total = (size_t)P.rows * P.cols;
        const int nb = ew_blocks(total);
        if (prelu && P.Z) { P.prelu_part = prelu_part + prelu_used; prelu_used += nb; }
        hipLaunchKernelGGL(act_bwd_kernel, dim3(nb), dim3(256), 0, st, P);
        WD_CHECK_LAUNCH("act_bwd");
        return 0;
    };
    auto base_bwd = [&](const float *Z, uint32_t layer, int act, int rows, int cols, float *out) {
        ActBwd P{};
        P.Z = Z; P.act = act; P.slope = p->prelu; P.p_drop = c->dropout; P.seed = c->seed; P.layer = layer;
        P.rows = rows; P.cols = cols; P.out = out;
        return P;
    };

    // readout backward -> dH [Va, Hout]
    float *dH = S(Bl.dH);
    if (hipMemsetAsync(dH, 0, (size_t)D.Va * D.Hout * 4, st) != hipSuccess) return fail(WD_ERR_ARG, "memset failed");
    if (D.B > 0) {
        hipLaunchKernelGGL(readout_bwd_kernel, dim3(D.B), dim3(128), 0, st, dout, D.Hout, g->w_atoms, g->mol_start,
                           g->mol_size, g->degree_of_polym, c->aggregation, c->aggregation_norm, dH, D.Hout);
        WD_CHECK_LAUNCH("readout_bwd");
    }
    const float *M_last = F(L.M[D.T - 1]);
    const float *dh = dH;
    if (D.desc) {  // hd = Zd * s (identity act)
        ActBwd P = base_bwd(F(L.Zd), D.T + 1, WD_ACT_IDENTITY, D.Va, D.Hout, S(Bl.dZd));
        P.G = dH; P.ldg = D.Hout;
        if ((rc = act_bwd(P))) return rc;
        Src dZ = make_src(D.Va, {seg_dense(S(Bl.dZd), D.Hout, D.Hout, 0)});
        Src X = x_src_d(g, D, F(L.h), true);
        TnPlan tp = tn_plan(D.Hout, X.cols_p, D.Va);
        if ((rc = gemm_tn(dZ, X, D.Hout, D.Va, tp, S(Bl.slab), 0, st))) return rc;
        const int wcol[3] = {0, H, 0};
        if ((rc = slab_reduce(tp, S(Bl.slab), D.Hout, X, grads->W_d, D.Hout, wcol, grads->b_d, st))) return rc;
        // dh = dZd @ W_d[:, :H]
        Src A = make_src(D.Va, {seg_dense(S(Bl.dZd), D.Hout, D.Hout, 0)});
        if ((rc = gemm_nn(A, p->W_d, D.Hout, 0, D.Va, H, D.Hout, epi_store(S(Bl.dHo), H, 0, 0), st))) return rc;
        dh = S(Bl.dHo);
    }
    // W_o layer
    {
        ActBwd P = base_bwd(F(L.Zo), D.T, c->activation, D.Va, H, S(Bl.dZo));
        P.G = dh; P.ldg = H;
        if ((rc = act_bwd(P))) return rc;
        Src dZ = make_src(D.Va, {seg_dense(S(Bl.dZo), H, H, 0)});
        Src X = x_src_o(g, D, M_last, true);
        TnPlan tp = tn_plan(H, X.cols_p, D.Va);
        if ((rc = gemm_tn(dZ, X, H, D.Va, tp, S(Bl.slab), 0, st))) return rc;
        const int wcol[3] = {0, D.Fa, 0};
        if ((rc = slab_reduce(tp, S(Bl.slab), H, X, grads->W_o, D.Fa + H, wcol, grads->b_o, st))) return rc;
        // dA = dZo @ W_o[:, Fa:]
        if ((rc = gemm_nn(dZ, p->W_o, D.Fa + H, D.Fa, D.Va, H, H, epi_store(S(Bl.dA), H, 0, 0), st))) return rc;
    }
    // gradient reaching M_{T-1} through the final aggregation, then the message layers
    float *dZbuf[2] = {S(Bl.dZ0), S(Bl.dZ1)};
    int cur = 0;
    {
        ActBwd P = base_bwd(F(L.Z[D.T - 1]), D.T - 1, c->activation, D.R, H, dZbuf[cur]);
        P.G = S(Bl.dA); P.ldg = H;
        P.ptr = g->atom_gather_t.ptr; P.idx = g->atom_gather_t.idx; P.coef = g->atom_gather_t.coef;
        if (D.T > 1) { P.res_out = S(Bl.dRes); P.res_init = 1; }
        if ((rc = act_bwd(P))) return rc;
    }
    TnPlan tph{};
    Src Xh0 = x_src_h(g, D, nullptr, true);
    tph = tn_plan(H, Xh0.cols_p, D.R);
    for (int t = D.T - 1; t >= 1; --t) {
        float *dZt = dZbuf[cur];
        const float *srcM = D.undirected ? F(L.Ms[t]) : F(L.M[t - 1]);
        // dW_h, db_h (+)= dZ_t^T [X_t | 1]
        Src dZ = make_src(D.R, {seg_dense(dZt, H, H, 0)});
        Src X = x_src_h(g, D, srcM, true);
        if ((rc = gemm_tn(dZ, X, H, D.R, tph, S(Bl.slab), t != D.T - 1, st))) return rc;
        // dX = dZ_t @ W_h[:, :H]
        const int ldwh = D.atom ? H + D.Fb : H;
        if ((rc = gemm_nn(dZ, p->W_h, ldwh, 0, D.R, H, H, epi_store(S(Bl.dX), H, 0, 0), st))) return rc;
        // dM_{t-1} = gather^T(dX) (+ symmetrize), then through act of layer t-1
        const int nxt = 1 - cur;
        ActBwd P = base_bwd(F(L.Z[t - 1]), t - 1, c->activation, D.R, H, dZbuf[nxt]);
        if (D.undirected) {
            ActBwd Q{};
            Q.G = S(Bl.dX); Q.ldg = H;
            Q.ptr = g->msg_gather_t.ptr; Q.idx = g->msg_gather_t.idx; Q.coef = g->msg_gather_t.coef;
            Q.rows = D.R; Q.cols = H; Q.out = S(Bl.dMs);
            if ((rc = act_bwd(Q))) return rc;
            P.G = S(Bl.dMs); P.ldg = H; P.sym_rev = g->b2revb;
        } else {
            P.G = S(Bl.dX); P.ldg = H;
            P.ptr = g->msg_gather_t.ptr; P.idx = g->msg_gather_t.idx; P.coef = g->msg_gather_t.coef;
        }
        if (t - 1 == 0) P.add_in = S(Bl.dRes);
        else { P.res_out = S(Bl.dRes); P.res_init = 0; }
        if ((rc = act_bwd(P))) return rc;
        cur = nxt;
    }
    if (D.T > 1) {
        const int ldwh = D.atom ? H + D.Fb : H;
        const int wcol[3] = {0, H, 0};
        if ((rc = slab_reduce(tph, S(Bl.slab), H, Xh0, grads->W_h, ldwh, wcol, grads->b_h, st))) return rc;
    }
    // input layer: dW_i, db_i = dZ_0^T [f | 1]
    {
        Src dZ = make_src(D.R, {seg_dense(dZbuf[cur], H, H, 0)});
        Src X = x_src_in(g, D);
        TnPlan tp = tn_plan(H, X.cols_p, D.R);
        if ((rc = gemm_tn(dZ, X, H, D.R, tp, S(Bl.slab), 0, st))) return rc;
        const int wcol[2] = {0, 0};
        if ((rc = slab_reduce(tp, S(Bl.slab), H, X, grads->W_i, D.Kin, wcol, grads->b_i, st))) return rc;
    }
    if (prelu && grads->prelu) {
        hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, st, prelu_part, prelu_used, grads->prelu);
        WD_CHECK_LAUNCH("prelu sum");
    }
    return 0;
}

int wdmpnn_event_pool_create(int32_t n_pairs, void **pool) {
    if (n_pairs <= 0 || !pool) return fail(WD_ERR_ARG, "bad event pool request");
    EventPool *p = new EventPool();
    p->n = n_pairs;
    p->ev.resize(2 * (size_t)n_pairs);
    for (auto &e : p->ev)
        if (hipEventCreate(&e) != hipSuccess) return fail(WD_ERR_ARG, "hipEventCreate failed");
    *pool = p;
    return 0;
}

int wdmpnn_event_pool_destroy(void *pool) {
    EventPool *p = (EventPool *)pool;
    if (!p) return 0;
    for (auto &e : p->ev) (void)hipEventDestroy(e);
    delete p;
    return 0;
}

int wdmpnn_event_pool_elapsed_ms(void *pool, int32_t first, int32_t count, float *total_ms) {
    EventPool *p = (EventPool *)pool;
    if (!p || !total_ms || first < 0 || count < 0 || first + count > p->n) return fail(WD_ERR_ARG, "bad pool range");
    double tot = 0.0;
    for (int i = first; i < first + count; ++i) {
        float ms = 0.f;
        if (hipEventSynchronize(p->ev[2 * i + 1]) != hipSuccess ||
            hipEventElapsedTime(&ms, p->ev[2 * i], p->ev[2 * i + 1]) != hipSuccess)
            return fail(WD_ERR_ARG, "event pair %d not recorded", i);
        tot += ms;
    }
    *total_ms = (float)tot;
    return 0;
}

int wdmpnn_index_select_rows(const float *src, int64_t n_src_rows, int64_t row_len, const int64_t *index,
                             int64_t n_index, float *out, void *stream) {
    if (n_index < 0 || row_len < 0 || n_src_rows < 0) return fail(WD_ERR_ARG, "negative size");
    if (n_index == 0 || row_len == 0) return 0;
    if (!src || !index || !out) return fail(WD_ERR_ARG, "null pointer");
    const size_t total = (size_t)n_index * row_len;
    hipLaunchKernelGGL(index_select_rows_kernel, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, src,
                       row_len, index, n_index, out);
    WD_CHECK_LAUNCH("index_select_rows");
    return 0;
}

}  // extern "C"
