// wdmpnn.hip — MI355X (gfx950) wD-MPNN encoder: C-ABI (include/wdmpnn.h) and launch orchestration.
//
// Forward = MPNEncoder.forward (chemprop/models/mpn.py:66-173):
//
//   L0        Z0 = f_bonds W_i^T (+b_i);  M0 = act(Z0)                      mpn.py:92-97
//   t=1..T-1  X_t = gather(M_{t-1})        X_t[b] = sum_{j in in(b2a[b])} w_j M_j - M_{b2revb[b]}
//                                         (reverse term folded into the list as w_rev - 1)
//             M_t = act(Z0 + X_t W_h^T (+b_h))                             mpn.py:100-124
//   LT        A = gather(M_{T-1}) (sum_{j in in(a)} w_j M_j);  h = act([f_atoms | A] W_o^T + b_o)
//                                                                           mpn.py:126-134
//  (LT+1      hd = [h | desc] W_d^T + b_d                                   mpn.py:136-143)
//   readout   out_i = Xn_i * sum_a w_a h_a / sum_a w_a (mean | sum | norm)   mpn.py:145-171
//
// Buffers are padded: rows to 128 (GEMM row tile), hidden columns to 64, K extents to 32, padding
// zero; weights are packed once per parameter version (wdmpnn_pack_params) into the same padded
// shapes (+ transposes for the backward data gradients).  Backward = the autograd graph of the
// above with deterministic, atomics-free kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "feed.hpp"
#include "fused_mp.hpp"
#include "gemm.hpp"
#include "gemm_x6.hpp"
#include "graph_build.hpp"
#include "kernels.hpp"
#include "selfcheck.hpp"
#include "small_fwd.hpp"
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

// Load-time kernel check (selfcheck.hpp): run once per process, before the first launch of any entry point;
// a library whose gfx950 code object lacks a kernel its host code launches fails every call with
// WD_ERR_UNSUPPORTED instead of aborting the process inside the HIP launch.
int self_check_once();
#define WD_KERNELS_OK() WD_TRY(self_check_once())

#define WD_CHECK_LAUNCH(what)                                                                  \
    do {                                                                                       \
        hipError_t e_ = hipGetLastError();                                                     \
        if (e_ != hipSuccess) return fail(-(int)e_, "%s: %s", what, hipGetErrorString(e_));   \
    } while (0)
#define WD_TRY(x)             \
    do {                      \
        int rc_ = (x);        \
        if (rc_) return rc_;  \
    } while (0)

struct SelfCheck {
    int rc;
    std::string why;
    int n_host, n_dev;
};
const SelfCheck &self_check_result() {
    static const SelfCheck r = [] {
        SelfCheck c{};
        c.rc = code_object_check(reinterpret_cast<const void *>(&self_check_result), c.why, c.n_host, c.n_dev);
        return c;
    }();
    return r;
}
int self_check_once() {
    const SelfCheck &c = self_check_result();
    return c.rc ? fail(WD_ERR_UNSUPPORTED, "libwdmpnn self-check: %s", c.why.c_str()) : 0;
}

// W_o + readout on fp16 pair tiles (1; the last pair layer writes A as pairs) or on bf16x3 planes (0) in the
// pair-operand forward
#ifndef WD_WO_PAIRS
#define WD_WO_PAIRS 1
#endif

// feed events that host threads wait for: hipEventBlockingSync (the waiting thread sleeps) or 0 (polls;
// experiments)
#ifndef WD_FEED_EVENT_SYNC
#define WD_FEED_EVENT_SYNC hipEventBlockingSync
#endif

// the fused backward's data-gradient GEMMs dM = Y_t W_h on fp16 pairs (1) or bf16x3 planes (0)
#ifndef WD_BWD_H2
#define WD_BWD_H2 1
#endif

inline int rup(int x, int m) { return (x + m - 1) / m * m; }


inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }
bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

int ew_blocks(size_t total) {
    size_t b = (total + 255) / 256;
    if (b > 4096) b = 4096;
    if (b < 1) b = 1;
    return (int)b;
}

// ------------------------------------------------------------------------------------------------
// dimensions
// ------------------------------------------------------------------------------------------------
struct Dims {
    int H, Hk, T, R, Rp, Va, Vap, B, Fa, Fak, Fb, Fbk, d, dk, Hd, Hdk, Kin, Kink;
    int ldx, Ko, Kd;
    bool atom, undirected, save, desc;
    bool f32;  // WdConfig.gemm_variant 9: f32-MFMA GEMMs (gemm_nt16_kernel) on the unblocked path
    bool x6;   // plane-tile pipeline: gathers emit bf16x3 plane tiles, GEMMs run gemm_x6g_kernel
    bool blocked;  // molecule-blocked fused inference forward (fused_mp.hpp)
    bool small;    // ... as ONE launch, a workgroup per block (small_fwd.hpp: blocks <= 32 rows, Hk 320)
    bool pairs;    // ... hands M_t between the launches as fp16 pair tiles (LDS-DMA layer operands): the
                   // workspace holds them (fused_forward: unless gemm_variant 12)
    bool pack_pairs;  // the packed weights hold W_o's pair tiles (a function of the encoder and config only:
                      // one inference pack serves every graph)
    int nblk;
};

// WdConfig.gemm_variant values that run the fused forward's layers on fp16 pair operands where the layout
// allows (all but 9, the f32-MFMA A/B, and 12, the register-staged layers)
inline bool pair_variant(int v) { return v != 9 && v != 12; }
#ifndef WD_EMBED_PAIR_BN
#define WD_EMBED_PAIR_BN 32
#endif
constexpr int EPB = WD_EMBED_PAIR_BN;  // the pair path's embed tile width (a multiple of 16 dividing every Hk: 32, 64)

int get_dims(const WdGraph *g, const WdParams *p, const WdConfig *c, Dims &D) {
    if (!g || !p || !c) return fail(WD_ERR_ARG, "null graph/params/config");
    if (c->depth < 1) return fail(WD_ERR_ARG, "depth must be >= 1 (got %d)", c->depth);
    if (p->hidden <= 0) return fail(WD_ERR_ARG, "hidden_size must be > 0");
    if (g->n_atoms < 1 || g->n_bonds < 1) return fail(WD_ERR_SHAPE, "n_atoms/n_bonds must include the pad row");
    if (c->activation < 0 || c->activation > WD_ACT_IDENTITY) return fail(WD_ERR_ARG, "bad activation %d", c->activation);
    if (c->aggregation < 0 || c->aggregation > WD_AGG_NORM) return fail(WD_ERR_ARG, "bad aggregation %d", c->aggregation);
    if (c->activation == WD_ACT_PRELU && !p->prelu) return fail(WD_ERR_ARG, "PReLU needs a slope pointer");
    if (!(c->dropout >= 0.f && c->dropout < 1.f)) return fail(WD_ERR_ARG, "dropout must be in [0, 1)");
    D.H = p->hidden; D.Hk = rup(D.H, 64); D.T = c->depth;
    D.atom = g->atom_messages != 0; D.undirected = c->undirected != 0; D.save = c->save_for_backward != 0;
    D.Va = g->n_atoms; D.Vap = rup(D.Va, 128); D.B = g->n_mols;
    D.R = D.atom ? g->n_atoms : g->n_bonds; D.Rp = rup(D.R, 128);
    D.Fa = g->atom_fdim; D.Fak = rup(D.Fa, 32); D.Fb = g->bond_fdim; D.Fbk = rup(D.Fb, 32);
    D.desc = g->atom_desc != nullptr && g->desc_dim > 0;
    D.d = D.desc ? g->desc_dim : 0; D.dk = rup(D.d, 32);
    D.Hd = D.H + D.d; D.Hdk = rup(D.Hd, 64);
    D.Kin = D.atom ? D.Fa : D.Fb; D.Kink = D.atom ? D.Fak : D.Fbk;
    D.ldx = D.atom ? D.Hk + D.Fbk : D.Hk;
    D.Ko = D.Fak + D.Hk;
    D.Kd = D.Hk + D.dk;
    // default (0) = 10: bf16x6 split-plane GEMMs (fp32-accurate)
    D.f32 = c->gemm_variant == 9;
    D.x6 = !D.f32 && !D.atom;
    // molecule-blocked fused forward, also for training (the fused kernels then save Z_t, A and Zo in
    // natural rows for the backward)
    // (an embed-capable graph -- categorical codes -- needs no feature planes)
    const bool codes = g->atom_codes && g->bond_src_blk && g->bond_tail && D.Fb <= WO_MAXK && D.Fa <= WO_MAXK;
    // (any Hk: a consumer folds its block's h2 scale words 64 at a time, planes.hpp lane_word)
    const bool blk_common = !D.desc && D.T >= 2 && g->n_blocks > 0 && g->blocks &&
                            g->atom_ell_idx && g->atom_ell_coef;
    // atom-message mode (inference): the a2a gather's pad slots read atom 0, whose message is act(b_i) and
    // later act(b_i + W_h(...)) -- zero without biases, so the block-local lists drop them; with biases,
    // or for training, the unblocked path runs
    const bool atom_blk = D.atom && !D.f32 && !D.save && !D.undirected && !p->b_i && !p->b_h &&
                          g->f_atoms_x6 &&
                          g->f_atoms_blk_x6 && g->bond_feat_gather.ptr && g->msg_ell_idx && g->msg_ell_coef &&
                          g->msg_gather.ptr && D.Fbk == 32;
    D.blocked = blk_common && (atom_blk || (D.x6 && g->bond_blk_row && (codes || (g->f_atoms_blk_x6 && g->f_bonds_x6)) &&
                                            g->bond_src_blk && g->b2revb));
    D.nblk = D.blocked ? g->n_blocks : 0;
    // QM9-sized blocks, inference: the one-launch forward (WdConfig.gemm_variant 11 / 12 / 13 keep the four launches)
    D.small = D.blocked && codes && !D.atom && !D.save && c->dropout == 0.f && D.Hk == SF_HK && !D.undirected &&
              c->gemm_variant != 11 && c->gemm_variant != 12 && c->gemm_variant != 13 && c->gemm_variant < 100 &&
              g->blk_max_bonds > 0 && g->blk_max_bonds <= SF_ROWS &&
              g->blk_max_atoms <= SF_ATOMS && D.Fa <= WO_MAXK && D.Fb <= WO_MAXK && D.Fb - D.Fa <= SF_ROWS;
    // inference through the embed (codes), bond messages, 80-column layer tiles, <= 64 embed words per block:
    // the layers read M_{t-1} as fp16 pair tiles written by its producer (fused_mp.hpp PAIRS; WdConfig.gemm_variant
    // 12 keeps the register-staged layers that read Z_t, 13 the pair layers also for QM9-sized blocks)
    D.pack_pairs = !D.atom && !D.save && D.Hk % 80 == 0 && D.Hk / 32 <= 64 && pair_variant(c->gemm_variant);
    // (debug variants 1ab: a = 1 pair layers / 2 register-staged layers, the fused forward stopped after stage
    // b = 1 embed, 2 first layer, ...: intermediate buffers left for tools/debug_pairs.py)
    D.pairs = D.pack_pairs && D.blocked && codes;
    if (D.atom && D.undirected)
        return fail(WD_ERR_UNSUPPORTED, "undirected with atom_messages (the reference indexes atom messages "
                                        "with b2revb, mpn.py:101-102)");
    // (a lean graph has neither table; two distinct arrays of a real graph cannot both sit at address 0 --
    // host-only tests pass buffer offsets as pointers)
    if (!g->f_atoms && !g->f_bonds && !(D.blocked && codes && !D.save))
        return fail(WD_ERR_UNSUPPORTED, "graph built without feature rows (WDMPNN_GRAPH_LEAN): only the fused "
                                        "inference forward runs on it");
    if (D.desc && (!p->W_d || !p->b_d)) return fail(WD_ERR_ARG, "atom descriptors need W_d and b_d");
    if (!p->W_i || !p->W_h || !p->W_o || !p->b_o || !p->zero_vec) return fail(WD_ERR_ARG, "missing weights");
    if (g->ld_atoms < D.Fak || g->ld_atoms % 4 || g->ld_bonds < D.Fbk || g->ld_bonds % 4 || g->bond_col0 != 0)
        return fail(WD_ERR_SHAPE, "f_atoms / f_bonds must be zero padded to 32 columns (ld %d/%d, need %d/%d) "
                                  "with bond_col0 == 0", g->ld_atoms, g->ld_bonds, D.Fak, D.Fbk);
    if (!aligned16(g->f_atoms) || !aligned16(g->f_bonds) || (D.desc && !aligned16(g->atom_desc)))
        return fail(WD_ERR_ARG, "feature arrays must be 16-byte aligned");
    return 0;
}

// ------------------------------------------------------------------------------------------------
// packed parameters
// ------------------------------------------------------------------------------------------------
struct PackLayout {
    size_t Wi = 0, bi = 0, Wh = 0, bh = 0, Wo = 0, bo = 0, Wd = 0, bd = 0, WhT = 0, WoT = 0, WdT = 0, total = 0;
    size_t WiX = 0, WhX = 0, WoX = 0;  // bf16x3 plane tiles (64-row blocks) of W_i / W_h / W_o
    size_t WhX80 = 0, WoX80 = 0;       // the same with 80-row blocks (fused forward, Hk % 80 == 0)
    size_t WiT = 0, WoaT = 0;          // W_i^T [Kink][Hk] and W_o[:, :Fa]^T [Fak][Hk]: weight columns as rows
                                       // (the categorical-code embedding of the fused forward)
    size_t WhH = 0;                    // h2 plane tiles of W_h (fused layers; BN-row blocks, BN = fused_bn)
    size_t amax = 0;                   // W_h's h2 scale: pack_kernel's 64 per-workgroup maxima + their max (u32)
    // atom-message mode: the fused forward's input GEMM [f_atoms | Fs] B^T with B [3 Hk][Fak + Fbk] =
    // [[W_i, 0], [W_i, W_h[:, H:]], [W_o[:, :Fa], 0]] -> inp | inp + Fs W_h[:, H:]^T | f_atoms W_o[:, :Fa]^T
    size_t WiA = 0, WiAX = 0;          // fp32, and its bf16x3 plane tiles (64-row blocks)
    // inference with pair operands (D.pairs; no training pack holds them): W_o[:, Fa:] as fp16 pair tiles with
    // 80-row blocks (wo_readout_kernel<..., PAIRS>'s B) and its scale: pack_kernel's 64 maxima + their max
    size_t WoH = 0, wo_amax = 0;
};

// column tile of the fused kernels: 80 when it divides Hk (Hk = 320: 4 tiles, one workgroup per CU at the
// benchmark size), else 64
int fused_bn(int Hk) { return Hk % 80 == 0 ? 80 : 64; }

PackLayout pack_layout(const Dims &D) {
    PackLayout L;
    size_t off = 0;
    auto take = [&](size_t floats) { size_t o = off; off = align256(off + floats * 4); return o; };
    L.Wi = take((size_t)D.Hk * D.Kink);
    L.bi = take(D.Hk);
    L.Wh = take((size_t)D.Hk * D.ldx);
    L.bh = take(D.Hk);
    L.Wo = take((size_t)D.Hk * D.Ko);
    L.bo = take(D.Hk);
    L.WhT = take((size_t)D.Hk * D.Hk);
    L.WoT = take((size_t)D.Hk * D.Hk);
    L.WiT = take((size_t)D.Kink * D.Hk);
    L.WoaT = take((size_t)D.Fak * D.Hk);
    L.WiX = take((size_t)D.Hk * D.Kink * 3 / 2);  // 3 bf16 planes = 1.5 floats per value
    L.WhX = take((size_t)D.Hk * D.ldx * 3 / 2);
    L.WoX = take((size_t)D.Hk * D.Ko * 3 / 2);
    if (D.Hk % 80 == 0) {
        L.WhX80 = take((size_t)D.Hk * D.ldx * 3 / 2);
        L.WoX80 = take((size_t)D.Hk * D.Ko * 3 / 2);
    }
    L.WhH = take((size_t)D.Hk * D.Hk);  // 2 fp16 per value
    // W_h's h2 scale words: pack_kernel's 64 per-workgroup maxima, their max (word 64, read by the fused
    // layers), then one word per 32 x 32 tile of W_h from adam_kernel (wdmpnn_adam_step_repack)
    L.amax = take(65 + (size_t)((D.H + ADAM_TILE - 1) / ADAM_TILE) * ((D.H + (D.atom ? D.Fb : 0) + ADAM_TILE - 1) / ADAM_TILE));
    if (D.atom) {
        L.WiA = take((size_t)3 * D.Hk * (D.Fak + D.Fbk));
        L.WiAX = take((size_t)3 * D.Hk * (D.Fak + D.Fbk) * 3 / 2);
    }
    if (D.pack_pairs) {
        L.WoH = take((size_t)D.Hk * D.Hk);  // 2 fp16 per value
        L.wo_amax = take(65);
    }
    if (D.desc) {
        L.Wd = take((size_t)D.Hdk * D.Kd);
        L.bd = take(D.Hdk);
        L.WdT = take((size_t)D.Hk * D.Hdk);
    }
    L.total = off;
    return L;
}

PackJob job_plain(float *dst, int rows_p, int cols_p, const float *src, int ld, int nrows,
                  std::initializer_list<std::array<int, 3>> segs) {  // {dst_col0, src_col0, K}
    PackJob j{};
    j.dst = dst; j.rows_p = rows_p; j.cols_p = cols_p; j.src = src; j.ld_src = ld; j.nrows = nrows;
    for (const auto &s : segs) {
        j.dc0[j.nseg] = s[0]; j.sc0[j.nseg] = s[1]; j.K[j.nseg] = s[2];
        ++j.nseg;
    }
    return j;
}

PackJob job_transpose(float *dst, int rows_p, int cols_p, const float *src, int ld, int src_col0, int nrows,
                      int src_rows) {
    PackJob j{};
    j.dst = dst; j.rows_p = rows_p; j.cols_p = cols_p; j.src = src; j.ld_src = ld; j.transpose = 1;
    j.nrows = nrows; j.nseg = 1; j.sc0[0] = src_col0; j.K[0] = src_rows;
    return j;
}

int pack_params(const Dims &D, const WdParams *p, char *base, hipStream_t st) {
    const PackLayout L = pack_layout(D);
    auto F = [&](size_t off) { return (float *)(base + off); };
    const int H = D.H;
    PackJobs J{};
    auto add = [&](const PackJob &j) { J.j[J.n++] = j; };
    add(job_plain(F(L.Wi), D.Hk, D.Kink, p->W_i, D.Kin, H, {{0, 0, D.Kin}}));
    add(job_plain(F(L.bi), 1, D.Hk, p->b_i, H, 1, {{0, 0, H}}));
    uint32_t *wh_amax = (uint32_t *)(base + L.amax);
    if (D.atom)
        add(job_plain(F(L.Wh), D.Hk, D.ldx, p->W_h, H + D.Fb, H, {{0, 0, H}, {D.Hk, H, D.Fb}}));
    else
        add(job_plain(F(L.Wh), D.Hk, D.ldx, p->W_h, H, H, {{0, 0, H}}));
    J.j[J.n - 1].amax = wh_amax;  // (pack_kernel's grid: 64 workgroups per job)
    add(job_plain(F(L.bh), 1, D.Hk, p->b_h, H, 1, {{0, 0, H}}));
    add(job_plain(F(L.Wo), D.Hk, D.Ko, p->W_o, D.Fa + H, H, {{0, 0, D.Fa}, {D.Fak, D.Fa, H}}));
    add(job_plain(F(L.bo), 1, D.Hk, p->b_o, H, 1, {{0, 0, H}}));
    // transposes for dX = dZ W_h[:, :H] and dA = dZo W_o[:, Fa:]
    add(job_transpose(F(L.WhT), D.Hk, D.Hk, p->W_h, D.atom ? H + D.Fb : H, 0, H, H));
    add(job_transpose(F(L.WoT), D.Hk, D.Hk, p->W_o, D.Fa + H, D.Fa, H, H));
    if (D.pack_pairs) J.j[J.n - 1].amax = (uint32_t *)(base + L.wo_amax);  // (max |W_o[:, Fa:]|: the pair tiles' scale)
    // weight columns as rows for the categorical-code embedding (fused_mp.hpp embed_kernel / wo_readout)
    add(job_transpose(F(L.WiT), D.Kink, D.Hk, p->W_i, D.Kin, 0, D.Kin, H));
    add(job_transpose(F(L.WoaT), D.Fak, D.Hk, p->W_o, D.Fa + H, 0, D.Fa, H));
    if (D.atom) {
        const int Kc = D.Fak + D.Fbk;
        const size_t band = (size_t)D.Hk * Kc;
        add(job_plain(F(L.WiA), D.Hk, Kc, p->W_i, D.Fa, H, {{0, 0, D.Fa}}));
        PackJob b1 = job_plain(F(L.WiA) + band, D.Hk, Kc, p->W_i, D.Fa, H, {{0, 0, D.Fa}, {D.Fak, H, D.Fb}});
        b1.src1 = p->W_h; b1.ld_src1 = H + D.Fb;
        add(b1);
        add(job_plain(F(L.WiA) + 2 * band, D.Hk, Kc, p->W_o, D.Fa + H, H, {{0, 0, D.Fa}}));
    }
    if (D.desc) {
        add(job_plain(F(L.Wd), D.Hdk, D.Kd, p->W_d, D.Hd, D.Hd, {{0, 0, H}, {D.Hk, H, D.d}}));
        add(job_plain(F(L.bd), 1, D.Hdk, p->b_d, D.Hd, 1, {{0, 0, D.Hd}}));
        add(job_transpose(F(L.WdT), D.Hk, D.Hdk, p->W_d, D.Hd, 0, H, D.Hd));
    }
    hipLaunchKernelGGL(pack_kernel, dim3(64, J.n), dim3(256), 0, st, J);
    WD_CHECK_LAUNCH("pack_params");
    // bf16x3 plane tiles of the padded W_i / W_h / W_o copies (B operands of gemm_x6g_kernel; BR 80
    // copies of W_h / W_o for the fused layer and W_o kernels), one launch
    SplitJobs X{};
    auto split = [&](size_t from, size_t to, int kp, int br) {
        X.j[X.n++] = SplitJob{(const float *)(base + from), (uint8_t *)(base + to), kp, D.Hk, kp, br};
    };
    split(L.Wi, L.WiX, D.Kink, 64);
    split(L.Wh, L.WhX, D.ldx, 64);
    split(L.Wo, L.WoX, D.Ko, 64);
    if (D.Hk % 80 == 0) {
        split(L.Wh, L.WhX80, D.ldx, 80);
        split(L.Wo, L.WoX80, D.Ko, 80);
    }
    int kmax = std::max(D.Kink, std::max(D.ldx, D.Ko));
    if (D.atom) {
        X.j[X.n++] = SplitJob{(const float *)(base + L.WiA), (uint8_t *)(base + L.WiAX), D.Fak + D.Fbk, 3 * D.Hk,
                              D.Fak + D.Fbk, 64};
        kmax = std::max(kmax, D.Fak + D.Fbk);
    }
    hipLaunchKernelGGL(split_tiles_batch_kernel, dim3(ew_blocks((size_t)D.Hk * kmax / 8), X.n), dim3(256), 0, st, X);
    WD_CHECK_LAUNCH("pack_params planes");
    // fp16 hi / lo tiles of W_h[:, :Hk] for the fused layers, scaled by its published maximum
    hipLaunchKernelGGL(split_h2_kernel, dim3(ew_blocks((size_t)D.Hk * D.Hk / 8)), dim3(256), 0, st, (const float *)F(L.Wh),
                       D.ldx, D.Hk, D.Hk, fused_bn(D.Hk), (uint8_t *)(base + L.WhH), wh_amax, 64, wh_amax + 64);
    WD_CHECK_LAUNCH("pack_params h2");
    if (D.pack_pairs) {  // W_o[:, Fa:] (columns Fak.. of the padded copy) as fp16 pair tiles, 80-row blocks
        hipLaunchKernelGGL(split_h2_kernel, dim3(ew_blocks((size_t)D.Hk * D.Hk / 8)), dim3(256), 0, st,
                           (const float *)F(L.Wo) + D.Fak, D.Ko, D.Hk, D.Hk, 80, (uint8_t *)(base + L.WoH),
                           (const uint32_t *)(base + L.wo_amax), 64, (uint32_t *)(base + L.wo_amax) + 64);
        WD_CHECK_LAUNCH("pack_params W_o h2");
    }
    return 0;
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
Epi epi_act(int act, const float *slope, const float *bias, const float *resid, float *Z, float *Y, int ld,
            const WdConfig *c, uint32_t layer) {
    Epi e{};
    e.kind = EPI_ACT; e.act = act; e.slope = slope; e.bias = bias; e.resid = resid; e.Z = Z; e.Y = Y; e.ld = ld;
    // dropout follows every W_h update, W_o and the descriptor layer (mpn.py:124, 134, 143), never the
    // input layer's message = act(input) (mpn.py:97): layer 0 is not dropped
    e.p_drop = layer == 0 ? 0.f : c->dropout; e.seed = c->seed; e.layer = layer;
    return e;
}

Epi epi_store(float *Y, int ld, long long slab_stride = 0, int accumulate = 0) {
    Epi e{};
    e.kind = EPI_STORE; e.Y = Y; e.ld = ld; e.slab_stride = slab_stride; e.accumulate = accumulate;
    return e;
}

constexpr int NBM = 64, NBN = 64;

bool epi_aligned(const Epi &epi) {
    const uintptr_t al = (uintptr_t)epi.Y | (uintptr_t)epi.Z | (uintptr_t)epi.resid | (uintptr_t)epi.bias |
                         (uintptr_t)epi.add_in | (uintptr_t)epi.res_out;
    return epi.ld % 4 == 0 && al % 16 == 0;
}

// C[Mp][Np] = epi([A0 | A1] B^T) on fp32 operands; A segments [Mp][lda], K extents multiples of 32, B
// [Np][ldb].  split: bf16x6 GEMM with the operands split into planes in the kernel (gemm_x6_kernel,
// 128- or 64-row tiles; fp32-accurate), else f32 MFMA (gemm_nt16_kernel, 64x64 tiles).
// gemm_x6_kernel's row tile (its grid, PReLU partials and TN scale-word rows follow it).  (64-row tiles for
// grids under 256 workgroups, the training batch's atom-row GEMM: 12.80 vs 12.76 us, not taken)
inline int x6_bm(int Mp) { return Mp % 128 == 0 ? 128 : 64; }

// a_words / b_word (split only): fp16 pairs instead of bf16x3 planes (gemm_x6_kernel<H2>), A scaled by the
// max words act_bwd_kernel published for it (a_cv float4 per A row), B by one word.
int gemm_nt(const float *a0, int lda0, int ka0, const float *a1, int lda1, int ka1, const float *b, int ldb, int Mp,
            int Np, const Epi &epi, hipStream_t st, bool split = false, const uint32_t *a_words = nullptr,
            int a_cv = 0, const uint32_t *b_word = nullptr) {
    if (Mp <= 0 || Np <= 0) return 0;
    if (Mp % NBM || Np % NBN || ka0 % BK || ka1 % BK || ka0 <= 0 || lda0 % 4 || (ka1 && lda1 % 4) || ldb % 4 ||
        !epi_aligned(epi))
        return fail(WD_ERR_SHAPE, "gemm_nt: unpadded or unaligned operand (Mp %d Np %d ka %d/%d)", Mp, Np, ka0, ka1);
    if (split) {
        X6Params X{};
        X.a0 = a0; X.lda0 = lda0; X.ka0 = ka0; X.a1 = a1; X.lda1 = lda1; X.ka1 = ka1;
        X.bf = b; X.ldb = ldb;
        X.M = Mp; X.N = Np; X.epi = epi; X.tiles_n = Np / X6_BN;
        const int bm = x6_bm(Mp);
        X.tiles_m = Mp / bm;
        const dim3 grid(X.tiles_m * X.tiles_n), blk(4 * bm);
        const bool h2 = a_words != nullptr;
        if (h2) {
            if (!b_word || a1 || a_cv <= 0 || ((size_t)Mp * a_cv) % 256)
                return fail(WD_ERR_SHAPE, "gemm_nt: fp16-pair operands need A's words (Mp %d, %d float4 per row)", Mp,
                            a_cv);
            X.a_words = a_words; X.a_cv = a_cv; X.b_word = b_word;
        }
        if (bm == 128) {
            if (h2) hipLaunchKernelGGL((gemm_x6_kernel<128, 32, true>), grid, blk, 0, st, X);
            else hipLaunchKernelGGL((gemm_x6_kernel<128, 32>), grid, blk, 0, st, X);
        } else {
            if (h2) hipLaunchKernelGGL((gemm_x6_kernel<64, 32, true>), grid, blk, 0, st, X);
            else hipLaunchKernelGGL((gemm_x6_kernel<64, 32>), grid, blk, 0, st, X);
        }
        WD_CHECK_LAUNCH("gemm_x6");
        return 0;
    }
    NtParams P{};
    P.a0 = a0; P.lda0 = lda0; P.ka0 = ka0; P.a1 = a1; P.lda1 = lda1; P.ka1 = ka1; P.b = b; P.ldb = ldb;
    P.M = Mp; P.N = Np; P.epi = epi;
    P.tiles_m = Mp / 64; P.tiles_n = Np / 64;
    hipLaunchKernelGGL((gemm_nt16_kernel<64, 64, 2, 2>), dim3(P.tiles_m * P.tiles_n), dim3(256), 0, st, P);
    WD_CHECK_LAUNCH("gemm_nt16");
    return 0;
}

// C[Mp][Np] = epi([A0 | A1] B^T) with every operand in plane tiles (planes.hpp): A segment i is the
// first ka_i columns of a [Mp][kp_i] plane-tile matrix, B a [Np][ka0 + ka1] one.
bool x6g_eligible(const Epi &epi) { return epi_aligned(epi); }

int gemm_x6g(const void *a0, int kp0, int ka0, const void *a1, int kp1, int ka1, const void *b, int Mp, int Np,
             const Epi &epi, hipStream_t st) {
    if (Mp <= 0 || Np <= 0) return 0;
    if (Mp % 64 || Np % 64 || ka0 <= 0 || ka0 % 32 || ka1 % 32 || kp0 % 32 || (ka1 && kp1 % 32) || ka0 > kp0 ||
        ka1 > kp1 || !x6g_eligible(epi))
        return fail(WD_ERR_SHAPE, "gemm_x6g: operand not in plane tiles (Mp %d Np %d ka %d/%d)", Mp, Np, ka0, ka1);
    X6PParams X{};
    X.a0 = (const uint8_t *)a0; X.kp0 = kp0; X.ka0 = ka0;
    X.a1 = (const uint8_t *)(a1 ? a1 : a0); X.kp1 = a1 ? kp1 : kp0; X.ka1 = ka1;
    X.b = (const uint8_t *)b; X.kpb = ka0 + ka1;
    X.M = Mp; X.N = Np; X.epi = epi; X.tiles_m = Mp / 64; X.tiles_n = Np / X6_BN;
    hipLaunchKernelGGL(gemm_x6g_kernel, dim3(X.tiles_m * X.tiles_n), dim3(512), 0, st, X);
    WD_CHECK_LAUNCH("gemm_x6g");
    return 0;
}

// gather8_kernel: fp32 rows into out (may be null) and/or plane tiles (planes, columns pcol0.. of a
// [rows_p][kp] plane-tile matrix; may be null)
int gather8(const float *src, int ld_src, int K, const WdCsr &csr, const int32_t *sym_rev, float *out, int ld_out,
            void *planes, int kp, int pcol0, int rows, int rows_p, hipStream_t st) {
    if (rows_p <= 0 || K <= 0) return 0;
    if (K % 8 || ld_src % 4 || (out && ld_out % 4) || (planes && (rows_p % 64 || kp % 32 || pcol0 % 32)))
        return fail(WD_ERR_SHAPE, "gather8: unaligned operand (K %d)", K);
    Gather8P P{};
    P.src = src; P.ld_src = ld_src; P.K = K; P.ptr = csr.ptr; P.idx = csr.idx; P.coef = csr.coef;
    P.sym_rev = sym_rev; P.out = out; P.ld_out = ld_out; P.planes = (uint8_t *)planes; P.kp = kp; P.pcol0 = pcol0;
    P.rows = rows; P.rows_p = rows_p;
    const size_t total = (size_t)rows_p * (K / 8);
    hipLaunchKernelGGL(gather8_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, P);
    WD_CHECK_LAUNCH("gather8");
    return 0;
}

Seg seg_dense(const float *src, int ld, int K) {
    Seg s{};
    s.src = src; s.ld = ld; s.K = K; s.kind = SEG_DENSE;
    return s;
}
Seg seg_ones() {
    Seg s{};
    s.K = 1; s.kind = SEG_ONES;
    return s;
}
Src make_src(int rows, std::initializer_list<Seg> segs) {
    Src S{};
    S.rows = rows;
    int kp = 0;
    for (const Seg &g : segs) {
        S.s[S.nseg] = g;
        S.s[S.nseg].kp0 = kp;
        kp += rup(g.K, 4);
        ++S.nseg;
    }
    S.cols_p = kp;
    return S;
}

struct TnPlan { int nsplit; int k_per_split; long long slab_stride; int ld_slab; int n_dense; int bias_col; };

// columns of X that are GEMM tiles (its dense segments) and the slab column of the bias (its ones
// segment, summed from dZ by gemm_tn_x6_kernel), -1 without one
void tn_cols(const Src &X, int &n_dense, int &bias_col) {
    const bool ones = X.nseg > 0 && X.s[X.nseg - 1].kind == SEG_ONES;
    n_dense = ones ? X.s[X.nseg - 1].kp0 : X.cols_p;
    bias_col = ones ? X.s[X.nseg - 1].kp0 : -1;
}

// split-K plan of the weight-gradient GEMM: at most TN_TARGET workgroups (512 = two per CU, the kernel's
// occupancy: a grid just past it runs a second, nearly empty round) over the output tiles (64 x 64 of
// [n_out][n_dense]), 32-row chunks; the slabs keep X's padded column space [n_out][cols_p]
TnPlan tn_plan(int n_out, const Src &X, int m_rows) {
    static const int target = [] {
        const char *e = getenv("WDMPNN_TN_TARGET");
        return e ? std::max(1, atoi(e)) : 512;
    }();
    TnPlan t{};
    tn_cols(X, t.n_dense, t.bias_col);
    const int tiles = ((n_out + 63) / 64) * ((t.n_dense + 63) / 64);
    const int chunks = (m_rows + 31) / 32;
    int ns = target / tiles;
    if (ns > chunks) ns = chunks;
    if (ns < 1) ns = 1;
    const int cps = (chunks + ns - 1) / ns;
    t.k_per_split = cps * 32;
    t.nsplit = (m_rows + t.k_per_split - 1) / t.k_per_split;
    if (t.nsplit < 1) t.nsplit = 1;
    t.ld_slab = X.cols_p;
    t.slab_stride = (long long)n_out * X.cols_p;
    return t;
}

// slab[z][n][j] (+)= sum_{m in split z} dZ[m][n] * X[m][j]  (bias column: sum_m dZ[m][n], or of bias_src
// [m_rows][dZ's ld] when given)
// a_words / b_words: fp16 pairs scaled by those published words (gemm_tn_x6_kernel<..., true>; SEG_ACT operands
// only), else bf16x3 planes (or TN_H2's max-pass pairs)
int gemm_tn(const Src &dZ, const Src &X, int n_out, int m_rows, const TnPlan &tp, float *slab, int accumulate,
            hipStream_t st, const float *bias_src = nullptr, const uint32_t *a_words = nullptr, int a_cv = 0,
            const uint32_t *b_words = nullptr, int b_bm = 0, int b_tn = 0) {
    if (n_out <= 0 || m_rows <= 0) return 0;
    TnX6Params P{};
    P.A = dZ; P.B = X; P.M = n_out; P.N = tp.n_dense; P.K = m_rows; P.k_per_split = tp.k_per_split;
    P.tiles_m = (n_out + 63) / 64; P.tiles_n = (tp.n_dense + 63) / 64;
    P.slab = slab; P.ld_slab = tp.ld_slab; P.slab_stride = tp.slab_stride; P.accumulate = accumulate;
    P.bias_col = tp.bias_col;
    P.bias_src = bias_src; P.bias_ld = dZ.s[0].ld;
    if (tp.ld_slab % 4 || tp.slab_stride % 4 || ((uintptr_t)slab & 15))
        return fail(WD_ERR_SHAPE, "gemm_tn: unaligned slab");
    const dim3 grid(P.tiles_m * P.tiles_n * tp.nsplit);
    int sact = -1;
    for (int q = 0; q < X.nseg; ++q)
        if (X.s[q].kind == SEG_ACT) sact = X.s[q].act;
    if (sact >= 0 && !bias_src) return fail(WD_ERR_ARG, "gemm_tn: a SEG_ACT operand needs its bias source");
    if (bias_src && sact < 0) return fail(WD_ERR_ARG, "gemm_tn: an external bias source goes with a SEG_ACT operand");
    if (a_words) {
        if (sact < 0 || !b_words || a_cv <= 0 || b_bm <= 0 || b_tn <= 0)
            return fail(WD_ERR_ARG, "gemm_tn: fp16-pair words need a SEG_ACT operand and both word arrays");
        P.a_words = a_words; P.a_cv = a_cv; P.b_words = b_words; P.b_bm = b_bm; P.b_tn = b_tn;
        switch (sact) {
        case ACT_RELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_RELU, true, true>), grid, dim3(256), 0, st, P); break;
        case ACT_LEAKY: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_LEAKY, true, true>), grid, dim3(256), 0, st, P); break;
        case ACT_PRELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_PRELU, true, true>), grid, dim3(256), 0, st, P); break;
        case ACT_TANH: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_TANH, true, true>), grid, dim3(256), 0, st, P); break;
        case ACT_SELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_SELU, true, true>), grid, dim3(256), 0, st, P); break;
        case ACT_ELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_ELU, true, true>), grid, dim3(256), 0, st, P); break;
        default: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_IDENTITY, true, true>), grid, dim3(256), 0, st, P); break;
        }
        WD_CHECK_LAUNCH("gemm_tn");
        return 0;
    }
    constexpr bool H2 = TN_H2;
    switch (sact) {
    case -1: hipLaunchKernelGGL((gemm_tn_x6_kernel<-1, false, H2>), grid, dim3(256), 0, st, P); break;
    case ACT_RELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_RELU, true, H2>), grid, dim3(256), 0, st, P); break;
    case ACT_LEAKY: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_LEAKY, true, H2>), grid, dim3(256), 0, st, P); break;
    case ACT_PRELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_PRELU, true, H2>), grid, dim3(256), 0, st, P); break;
    case ACT_TANH: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_TANH, true, H2>), grid, dim3(256), 0, st, P); break;
    case ACT_SELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_SELU, true, H2>), grid, dim3(256), 0, st, P); break;
    case ACT_ELU: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_ELU, true, H2>), grid, dim3(256), 0, st, P); break;
    default: hipLaunchKernelGGL((gemm_tn_x6_kernel<ACT_IDENTITY, true, H2>), grid, dim3(256), 0, st, P); break;
    }
    WD_CHECK_LAUNCH("gemm_tn");
    return 0;
}

// dW[n][w0 + kk] = sum_z slab[z][n][c0 + kk] per mapping {c0, w0, K}; db[n] = slab bias column
SlabReduce slab_job(const TnPlan &tp, const float *slab, int n_rows, std::initializer_list<std::array<int, 3>> map,
                    float *dW, int ldw, float *db, int bias_col) {
    SlabReduce R{};
    R.slab = slab; R.nsplit = tp.nsplit; R.slab_stride = tp.slab_stride; R.ld_slab = tp.ld_slab; R.rows = n_rows;
    for (const auto &m : map) {
        R.c0[R.nseg] = m[0]; R.w0[R.nseg] = m[1]; R.K[R.nseg] = m[2];
        ++R.nseg;
    }
    R.dW = dW; R.ldw = ldw; R.db = db; R.bias_col = bias_col;
    return R;
}
// the reductions of several gradients in one launch (jobs without dW and db skipped)
int slab_reduce_multi(const SlabReduce *jobs, int n, hipStream_t st) {
    SlabReduceJobs J{};
    int blocks = 0;
    for (int k = 0; k < n; ++k) {
        const SlabReduce &R = jobs[k];
        if (!R.dW && !R.db) continue;
        if (J.n == SLAB_MAX) return fail(WD_ERR_ARG, "slab_reduce_multi: more than %d jobs", SLAB_MAX);
        int cols = 0;
        if (R.dW)
            for (int q = 0; q < R.nseg; ++q) cols += R.K[q];
        if (R.db) cols += 1;
        J.j[J.n] = R;
        J.cgroups[J.n] = (cols + 63) / 64;
        J.blk0[J.n] = blocks;
        blocks += J.cgroups[J.n] * ((R.rows + 3) / 4);
        ++J.n;
    }
    if (!J.n) return 0;
    J.blk0[J.n] = blocks;
    hipLaunchKernelGGL(slab_reduce_multi_kernel, dim3(blocks), dim3(256), 0, st, J);
    WD_CHECK_LAUNCH("slab_reduce_multi");
    return 0;
}
int slab_reduce(const TnPlan &tp, const float *slab, int n_rows, std::initializer_list<std::array<int, 3>> map,
                float *dW, int ldw, float *db, int bias_col, hipStream_t st) {
    if (!dW && !db) return 0;
    SlabReduce R{};
    R.slab = slab; R.nsplit = tp.nsplit; R.slab_stride = tp.slab_stride; R.ld_slab = tp.ld_slab; R.rows = n_rows;
    for (const auto &m : map) {
        R.c0[R.nseg] = m[0]; R.w0[R.nseg] = m[1]; R.K[R.nseg] = m[2];
        ++R.nseg;
    }
    R.dW = dW; R.ldw = ldw; R.db = db; R.bias_col = bias_col;
    int cols = 0;
    if (dW)
        for (int q = 0; q < R.nseg; ++q) cols += R.K[q];
    if (db) cols += 1;  // the bias column after the segments
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((cols + 63) / 64, (n_rows + 3) / 4), dim3(256), 0, st, R);
    WD_CHECK_LAUNCH("slab_reduce");
    return 0;
}

ReadoutP readout_params(const WdGraph *g, const WdParams *p, const WdConfig *c, const float *h, int ldh, int ncols,
                        float *out) {
    ReadoutP R{};
    R.h = h; R.ldh = ldh; R.ncols = ncols; R.w_atoms = g->w_atoms; R.mol_start = g->mol_start;
    R.mol_size = g->mol_size; R.xn = g->degree_of_polym; R.agg = c->aggregation; R.norm = c->aggregation_norm;
    R.zero_vec = p->zero_vec; R.out = out;
    return R;
}

// ------------------------------------------------------------------------------------------------
// workspace layouts
// ------------------------------------------------------------------------------------------------
struct FwdLayout {
    std::vector<size_t> Z, M, X;
    size_t packed = 0, A = 0, Zo = 0, h = 0, Zd = 0, hd = 0, total = 0;
    size_t Xp = 0, Ap = 0;  // plane tiles of X_t and A (D.x6)
    size_t Zb[2] = {0, 0}, Ab = 0;  // D.blocked inference: Z_t fp32 rows (ping-pong); A as blocked plane tiles
    size_t amax[2] = {0, 0};        // D.blocked: h2 scale words of M_t, ping-pong [nblk][tiles] (planes.hpp)
    size_t Mp[2] = {0, 0};          // D.pairs: M_t as fp16 pair tiles of the molecule blocks, ping-pong
                                    // [nblk][Hk / 32][2][128][64 B] (the embed writes M_0)
    size_t Eo = 0;                  // D.blocked: f_atoms W_o[:, :Fa]^T per blocked atom row (compact codes)
    size_t Fs = 0, In3 = 0;         // D.blocked atom-message mode: per atom the sum of its in-bonds' features
                                    // (plane tiles [Vap][Fbk]), and the input GEMM's [Vap][3 Hk] output
                                    // inp | inp + Fs W_h[:, H:]^T (the layers' residual) | Eo
    bool own_pack = false;
};

FwdLayout fwd_layout(const Dims &D, bool own_pack) {
    FwdLayout L;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
    const size_t msg = (size_t)D.Rp * D.Hk * 4, atm = (size_t)D.Vap * D.Hk * 4, atd = (size_t)D.Vap * D.Hdk * 4;
    L.own_pack = own_pack;
    if (own_pack) L.packed = take(pack_layout(D).total);
    for (int t = 0; t < (D.save ? D.T : 1); ++t) L.Z.push_back(take(msg));
    if (!D.blocked) {  // (the fused kernels keep M_t in plane tiles and never form X_t)
        for (int t = 0; t < (D.save ? D.T : (D.T > 1 ? 2 : 1)); ++t) L.M.push_back(take(msg));
        if (D.T > 1)
            for (int t = 0; t < (D.save ? D.T - 1 : 1); ++t) L.X.push_back(take((size_t)D.Rp * D.ldx * 4));
    }
    L.A = take(atm);
    if (D.blocked) {
        // Z_t, ping-pong (layer t writes Zb[t & 1]; the first reads inp, the last writes none; a training
        // forward writes L.Z[t] instead)
        if (!D.save)
            for (int i = 0; i < 2 && i < D.T - 2; ++i) L.Zb[1 - i] = take(msg);
        if (D.pairs)  // (M_0 .. M_{T-2}: the last layer writes none)
            for (int i = 0; i < 2 && i < D.T - 1; ++i) L.Mp[i] = take((size_t)D.nblk * BLK_BONDS * D.Hk * 4);
        // (<= 64 tiles per block; the atom-message input GEMM: one word per 64 x 64 tile of inp)
        const size_t words = std::max((size_t)D.nblk * 64, (size_t)(D.Rp / 64) * (D.Hk / 64));
        for (int i = 0; i < 2; ++i) L.amax[i] = take(words * 4);
        // A: bf16x3 plane tiles, or fp16 pair tiles (D.pairs), of the blocks' atom rows
        L.Ab = take((size_t)D.nblk * BLK_ATOMS * D.Hk * 6);  // (6 bytes per value: also room for pairs)
        if (D.atom) {
            L.Fs = take((size_t)D.Vap * D.Fbk * 6);
            L.In3 = take((size_t)D.Rp * 3 * D.Hk * 4);
        } else {
            L.Eo = take((size_t)D.Vap * D.Hk * 4);
        }
    } else if (D.x6) {
        if (D.T > 1) L.Xp = take((size_t)D.Rp * D.Hk * 6);
        L.Ap = take((size_t)D.Vap * D.Hk * 6);
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
           slab_h = 0, slab_i = 0, prelu = 0, words = 0, mwords = 0, total = 0;  // slab: W_o's (and W_d's) split-K slabs; W_h's, W_i's
    size_t prelu_floats = 0;
};

Src x_in(const WdGraph *g, const Dims &D) {
    return D.atom ? make_src(D.R, {seg_dense(g->f_atoms, g->ld_atoms, D.Fak), seg_ones()})
                  : make_src(D.R, {seg_dense(g->f_bonds, g->ld_bonds, D.Fbk), seg_ones()});
}
Src x_h(const Dims &D, const float *X) { return make_src(D.R, {seg_dense(X, D.ldx, D.ldx), seg_ones()}); }
Src x_o(const WdGraph *g, const Dims &D, const float *A) {
    return make_src(D.Va, {seg_dense(g->f_atoms, g->ld_atoms, D.Fak), seg_dense(A, D.Hk, D.Hk), seg_ones()});
}
Src x_d(const WdGraph *g, const Dims &D, const float *h) {
    return make_src(D.Va, {seg_dense(h, D.Hk, D.Hk), seg_dense(g->atom_desc, D.dk, D.dk), seg_ones()});
}

BwdLayout bwd_layout(const WdGraph *g, const Dims &D) {
    BwdLayout L;
    size_t off = 0;
    auto take = [&](size_t floats) { size_t o = off; off = align256(off + floats * 4); return o; };
    const size_t msg = (size_t)D.Rp * D.Hk, atm = (size_t)D.Vap * D.Hk, atd = (size_t)D.Vap * D.Hdk;
    L.dH = take(D.desc ? atd : atm);
    if (D.desc) { L.dZd = take(atd); L.dHo = take(atm); }
    L.dZo = take(atm);
    L.dA = take(atm);
    L.dZ0 = take(msg);
    L.dZ1 = take(msg);
    L.dRes = take(msg);
    L.dX = take(msg);
    if (D.undirected) L.dMs = take(msg);
    // split-K slabs: W_o's (shared with the descriptor layer's, reduced before W_o's GEMM), W_h's and W_i's
    // apart, so that one launch at the end reduces all three (slab_reduce_multi)
    auto slab_of = [&](int n_out, const Src &X, int m_rows) {
        TnPlan tp = tn_plan(n_out, X, m_rows);
        return (size_t)tp.nsplit * (size_t)tp.slab_stride;
    };
    size_t so = slab_of(D.Hk, x_o(g, D, nullptr), D.Va);
    if (D.desc) so = std::max(so, slab_of(D.Hdk, x_d(g, D, nullptr), D.Va));
    L.slab = take(so);
    L.slab_h = take(slab_of(D.Hk, x_h(D, nullptr), D.R));
    L.slab_i = take(slab_of(D.Hk, x_in(g, D), D.R));
    L.prelu_floats = (size_t)(D.T + 2) * std::max(4096, (D.Rp / 64) * (D.Hk / 64));  // (64-row tiles at most)
    L.prelu = take(L.prelu_floats);
    L.words = take((msg / 4 + 255) / 256);  // Y_t's scale words (act_bwd_kernel -> gemm_x6_kernel<H2>, gemm_tn)
    L.mwords = take((size_t)(D.Rp / 64) * (D.Hk / 64));  // M_{t-1}'s (the data-gradient GEMM -> gemm_tn)
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

// ------------------------------------------------------------------------------------------------
// device graph of a compact batch (graph_build.hpp)
// ------------------------------------------------------------------------------------------------
struct GraphLayout {
    int lda = 0, ldb = 0, Vap = 0, Rbp = 0;
    size_t f_atoms = 0, f_bonds = 0, fa_x6 = 0, fb_x6 = 0, fa_blk_x6 = 0, w_atoms = 0, mol_start = 0, mol_size = 0,
           xn = 0, b2revb = 0, blocks = 0, bond_blk_row = 0, atom_blk_row = 0, bond_src_blk = 0, bond_tail = 0,
           msg_ell_idx = 0, msg_ell_coef = 0,
           agg_ell_idx = 0, agg_ell_coef = 0, csr[4][3] = {}, total = 0;
};

int graph_layout(const WdCompact *c, GraphLayout &L) {
    if (!c) return fail(WD_ERR_ARG, "null compact graph");
    if (c->n_atoms < 1 || c->n_bonds < 1 || c->n_mols < 0 || c->n_blocks < 0 || (c->n_bonds - 1) % 2 ||
        c->nnz_msg < 0 || c->nnz_agg < 0)
        return fail(WD_ERR_SHAPE, "compact graph: bad counts (atoms %d bonds %d mols %d blocks %d)", c->n_atoms,
                    c->n_bonds, c->n_mols, c->n_blocks);
    if (c->atom_fdim < 2 || c->atom_fdim > 255 || c->bond_fdim < c->atom_fdim || c->bond_fdim - c->atom_fdim > 16)
        return fail(WD_ERR_SHAPE, "compact graph: atom_fdim %d / bond_fdim %d out of range", c->atom_fdim, c->bond_fdim);
    L.lda = rup(c->atom_fdim, 32); L.ldb = rup(c->bond_fdim, 32);
    L.Vap = rup(c->n_atoms, 128); L.Rbp = rup(c->n_bonds, 128);
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
    L.f_atoms = take((size_t)L.Vap * L.lda * 4);
    L.f_bonds = take((size_t)L.Rbp * L.ldb * 4);
    L.fa_x6 = take((size_t)L.Vap * L.lda * 6);
    L.fb_x6 = take((size_t)L.Rbp * L.ldb * 6);
    L.fa_blk_x6 = take((size_t)std::max(c->n_blocks, 1) * BLK_ATOMS * L.lda * 6);
    L.w_atoms = take((size_t)c->n_atoms * 4);
    L.mol_start = take((size_t)c->n_mols * 4 + 4);
    L.mol_size = take((size_t)c->n_mols * 4 + 4);
    L.xn = take((size_t)c->n_mols * 4 + 4);
    L.b2revb = take((size_t)c->n_bonds * 4);
    L.blocks = take((size_t)c->n_blocks * 32 + 32);
    L.bond_blk_row = take((size_t)L.Rbp * 4);
    L.atom_blk_row = take((size_t)L.Vap * 4);
    L.bond_src_blk = take((size_t)L.Rbp);
    L.bond_tail = take((size_t)L.Rbp * 2);
    L.msg_ell_idx = take((size_t)L.Rbp * GB_ELLW);
    L.msg_ell_coef = take((size_t)L.Rbp * GB_ELLW * 4);
    L.agg_ell_idx = take((size_t)L.Vap * GB_ELLW);
    L.agg_ell_coef = take((size_t)L.Vap * GB_ELLW * 4);
    // msg, agg, msg_t, agg_t: {ptr, idx, coef}
    const int rows[4] = {c->n_bonds, c->n_atoms, c->n_bonds, c->n_bonds};
    const int nnz[4] = {c->nnz_msg, c->nnz_agg, c->nnz_msg, c->nnz_agg};
    for (int q = 0; q < 4; ++q) {
        L.csr[q][0] = take((size_t)(rows[q] + 1) * 4);
        L.csr[q][1] = take((size_t)(nnz[q] + GB_CSR_PAD) * 4);
        L.csr[q][2] = take((size_t)(nnz[q] + GB_CSR_PAD) * 4);
    }
    L.total = off;
    return 0;
}

// ------------------------------------------------------------------------------------------------
// molecule-blocked fused forward (fused_mp.hpp): embed (or the W_i GEMM) -> (T-1) x mp_layer ->
// wo_readout, for up to WD_MULTI independent batches per launch (wdmpnn_forward_many; one batch for
// wdmpnn_forward).  Every job shares the parameters, the configuration and the packed weights.
// ------------------------------------------------------------------------------------------------
struct FusedJob {
    const WdGraph *g;
    Dims D;
    FwdLayout L;
    char *ws;
    float *out;
};

bool fused_codes(const WdGraph *g, const Dims &D) {
    return g->atom_codes && g->bond_src_blk && g->bond_tail && D.Fb <= WO_MAXK && D.Fa <= WO_MAXK;
}

template <typename T, typename Fill>
int launch_multi(const FusedJob *jobs, int n, int tiles_per_blk, Fill &&fill, Multi<T> &M, int &grid) {
    M = Multi<T>{};
    M.n = n;
    int t = 0;
    for (int j = 0; j < n; ++j) {
        M.t0[j] = t;
        fill(M.p[j], jobs[j]);
        t += jobs[j].D.nblk * tiles_per_blk;
    }
    for (int j = n; j <= WD_MULTI; ++j) M.t0[j] = t;
    grid = t;
    return 0;
}
// the one-batch form of a filled Multi (a launch's host cost grows with its kernel-argument bytes)
template <typename T>
Multi<T, 1> one_job(const Multi<T> &M) {
    Multi<T, 1> o{};
    o.p[0] = M.p[0]; o.t0[0] = M.t0[0]; o.t0[1] = M.t0[1]; o.n = 1;
    return o;
}

int fused_forward(const FusedJob *jobs, int n, const WdParams *p, const WdConfig *c, const PackLayout &PL,
                  const char *pk, hipStream_t st) {
    if (n < 1 || n > WD_MULTI) return fail(WD_ERR_ARG, "fused forward: %d jobs per launch (1..%d)", n, WD_MULTI);
    const Dims &D0 = jobs[0].D;
    if (D0.atom && n > 1)  // (the atom-row layer kernel is instantiated for one batch per launch only)
        return fail(WD_ERR_UNSUPPORTED, "fused forward: atom messages run one batch per launch");
    auto W = [&](size_t off) { return (const float *)(pk + off); };
    auto F = [](const FusedJob &J, size_t off) { return (float *)(J.ws + off); };
    const int Hk = D0.Hk;
    // 80-column tiles when they divide Hk (Hk = 320: 4 tiles, one workgroup per CU at the benchmark
    // size), else 64
    const bool bn80 = Hk % 80 == 0;
    const int BNf = bn80 ? 80 : 64;
    // categorical codes (compact graphs): the input layer and the f_atoms half of W_o as sums of weight
    // columns instead of GEMMs over the one-hot rows (fused_mp.hpp embed_kernel)
    const bool codes = fused_codes(jobs[0].g, D0);
    for (int j = 1; j < n; ++j)
        if (fused_codes(jobs[j].g, jobs[j].D) != codes || jobs[j].D.Hk != Hk || jobs[j].D.T != D0.T ||
            jobs[j].D.atom != D0.atom ||
            jobs[j].D.Fa != D0.Fa || jobs[j].D.Fb != D0.Fb || jobs[j].D.save != D0.save)
            return fail(WD_ERR_UNSUPPORTED, "fused forward: batches of one launch differ in layout");
    // h2 scale words of M_t (written by the embed for t = 0, by layer t after): [nblk][tiles of the producer]
    auto slot = [&](const FusedJob &J, int t) { return (uint32_t *)(J.ws + J.L.amax[t & 1]); };
    // 40-column tiles for the embed when they divide Hk: twice the workgroups of the layer tiling (two per
    // CU at the benchmark size, 37 KB of LDS each), so one's staging overlaps the other's sums
#ifndef WD_EMBED40
#define WD_EMBED40 1
#endif
    // (the pair path: EPB-column embed tiles, one scale word per tile of M_0; measured, same box: 64-column
    // tiles -- 320 workgroups, one round at B = 64 -- 11.29 vs 9.63 us for 32, 186.5 vs 194.0 M edges/s)
    // The pair-operand layers (M_t as fp16 pair tiles, written by its producer and copied by LDS-DMA; DESIGN.md
    // §4 "Pair operands") wherever the layout allows (D.pairs; gemm_variant 12 keeps the register-staged layers):
    // round 6, one box, 190.1 vs 178.8 M edges/s three batches in flight, 121.2 vs 118.1 M one, 203.0 vs 175.0 M
    // forward_many(4) (profiles/round6_pairs_default_ab.txt)
    bool pairs = D0.pairs;
    if (c->gemm_variant >= 100) pairs = D0.pairs && (c->gemm_variant / 10) % 10 == 1;  // (debug stops)
    for (int j = 1; j < n; ++j)
        if (jobs[j].D.pairs != D0.pairs) return fail(WD_ERR_UNSUPPORTED, "fused forward: batches of one launch differ in layout");
    const bool bn40 = WD_EMBED40 && Hk % 40 == 0 && !pairs;
    const int embed_tiles = Hk / (pairs ? EPB : (bn40 ? 40 : BNf));
    if (codes) {
        const int nt = embed_tiles;
        Multi<EmbedP> M;
        int grid;
        launch_multi(jobs, n, nt, [&](EmbedP &E, const FusedJob &J) {
            const WdGraph *g = J.g;
            E.codes = g->atom_codes; E.src_blk = g->bond_src_blk; E.tail = g->bond_tail;
            E.wt = W(PL.WiT); E.woat = W(PL.WoaT); E.eo = F(J, J.L.Eo); E.bias = p->b_i ? W(PL.bi) : nullptr;
            E.blocks = g->blocks;
            E.Fa = J.D.Fa; E.Fb = J.D.Fb; E.Hk = Hk; E.n_tiles = nt;
            E.inp = F(J, J.L.Z[0]);
            E.slope = p->prelu; E.amax = slot(J, 0);
            E.m0 = pairs ? (uint8_t *)(J.ws + J.L.Mp[0]) : nullptr;
        }, M, grid);
        host_with_act(c->activation, [&](auto act_c) {
            constexpr int A = decltype(act_c)::value;
            if (pairs) {
                if (n == 1) hipLaunchKernelGGL((embed_kernel<EPB, A, 1, true>), dim3(grid), dim3(512), 0, st, one_job(M));
                else hipLaunchKernelGGL((embed_kernel<EPB, A, WD_MULTI, true>), dim3(grid), dim3(512), 0, st, M);
            } else if (n == 1) {
                const Multi<EmbedP, 1> M1 = one_job(M);
                if (bn40) hipLaunchKernelGGL((embed_kernel<40, A, 1>), dim3(grid), dim3(512), 0, st, M1);
                else if (bn80) hipLaunchKernelGGL((embed_kernel<80, A, 1>), dim3(grid), dim3(512), 0, st, M1);
                else hipLaunchKernelGGL((embed_kernel<64, A, 1>), dim3(grid), dim3(512), 0, st, M1);
            } else if (bn40) hipLaunchKernelGGL((embed_kernel<40, A>), dim3(grid), dim3(512), 0, st, M);
            else if (bn80) hipLaunchKernelGGL((embed_kernel<80, A>), dim3(grid), dim3(512), 0, st, M);
            else hipLaunchKernelGGL((embed_kernel<64, A>), dim3(grid), dim3(512), 0, st, M);
        });
        WD_CHECK_LAUNCH("embed");
        if (c->gemm_variant >= 100 && c->gemm_variant % 10 == 1) return 0;
    } else {
        for (int j = 0; j < n; ++j) {
            const FusedJob &J = jobs[j];
            if (J.D.atom) {
                // atom messages: per atom Fs = the sum of its in-bonds' feature rows (mpn.py:105-107, as plane
                // tiles), then ONE GEMM [f_atoms | Fs] [[W_i, 0], [W_i, W_h[:, H:]], [W_o[:, :Fa], 0]]^T ->
                // inp (mpn.py:93) | inp + Fs W_h[:, H:]^T (every layer's residual: the bond-feature half of
                // W_h is the same in each layer) | f_atoms W_o[:, :Fa]^T (the f_atoms half of W_o), whose
                // epilogue also publishes the first layer's h2 scale words per 64 x 64 tile of inp
                const void *fs = J.g->atom_feat_sum_x6;  // (built with the graph, or gathered here)
                int kpf = J.g->ld_bonds;
                if (!fs) {
                    kpf = J.D.Fbk;
                    WD_TRY(gather8(J.g->f_bonds, J.g->ld_bonds, J.D.Fbk, J.g->bond_feat_gather, nullptr, nullptr, 0,
                                   J.ws + J.L.Fs, J.D.Fbk, 0, J.D.R, J.D.Rp, st));
                    fs = J.ws + J.L.Fs;
                }
                Epi e = epi_act(ACT_IDENTITY, nullptr, nullptr, nullptr, nullptr, F(J, J.L.In3), 3 * Hk, c, 0);
                e.amax = slot(J, 0); e.amax_cols = Hk; e.amax_act = c->activation; e.slope = p->prelu;
                if (!x6g_eligible(e)) return fail(WD_ERR_SHAPE, "fused forward: unaligned buffers");
                WD_TRY(gemm_x6g(J.g->f_atoms_x6, J.g->ld_atoms, J.D.Fak, fs, kpf, J.D.Fbk, pk + PL.WiAX,
                                J.D.Rp, 3 * Hk, e, st));
                continue;
            }
            // inp only: the first layer stages M_0 = act(inp) itself
            Epi e = epi_act(ACT_IDENTITY, nullptr, W(PL.bi), nullptr, F(J, J.L.Z[0]), nullptr, Hk, c, 0);
            if (!x6g_eligible(e)) return fail(WD_ERR_SHAPE, "fused forward: unaligned buffers");
            WD_TRY(gemm_x6g(J.g->f_bonds_x6, J.g->ld_bonds, J.D.Kink, nullptr, 0, 0, pk + PL.WiX, J.D.Rp, Hk, e, st));
            host_with_act(c->activation, [&](auto act_c) {
                hipLaunchKernelGGL(absmax_blocks_kernel<decltype(act_c)::value>, dim3(J.D.nblk), dim3(256), 0, st,
                                   (const float *)F(J, J.L.Z[0]), Hk, Hk, J.g->blocks, p->prelu, slot(J, 0), 0);
            });
            WD_CHECK_LAUNCH("absmax");

        }
    }
    const int T = D0.T;
    for (int t = 1; t < T; ++t) {
        const bool last = t == T - 1;
        Multi<MpLayerP> M;
        int grid;
        launch_multi(jobs, n, Hk / BNf, [&](MpLayerP &Q, const FusedJob &J) {
            const WdGraph *g = J.g;
            // Z_{t-1} in, Z_t out (the last layer: none): a training forward keeps every Z_t (L.Z), inference
            // ping-pongs two buffers after inp
            auto zbuf = [&](int k) { return k == 0 || J.D.save ? F(J, J.L.Z[k]) : F(J, J.L.Zb[k & 1]); };
            const bool a3 = J.D.atom && t == 1;  // (the atom-message input GEMM's inp columns)
            Q.zin = a3 ? F(J, J.L.In3) : zbuf(t - 1);
            Q.ldz = a3 ? 3 * Hk : Hk;
            Q.amax_in = slot(J, t - 1);
            Q.amax_in_n = t > 1 ? Hk / BNf : (codes ? embed_tiles : (J.D.atom ? Hk / 64 : 1));
            Q.amax_rt = a3 ? 64 : 0;
            Q.p_drop_in = t - 1 == 0 ? 0.f : c->dropout;
            Q.zout = last ? nullptr : zbuf(t);
            Q.amax_out = last ? nullptr : slot(J, t);
            Q.kp = Hk;
            Q.wh = (const uint8_t *)(pk + PL.WhH); Q.wh_amax = (const uint32_t *)(pk + PL.amax) + 64;
            Q.inp = J.D.atom ? F(J, J.L.In3) + Hk : F(J, J.L.Z[0]);
            Q.ldr = J.D.atom ? 3 * Hk : Hk;
            Q.bias = p->b_h ? W(PL.bh) : nullptr;
            Q.mell_idx = g->msg_ell_idx; Q.mell_coef = g->msg_ell_coef;
            Q.mptr = g->msg_gather.ptr; Q.midx = g->msg_gather.idx; Q.mcoef = g->msg_gather.coef;
            Q.blocks = g->blocks;
            Q.rev = g->b2revb; Q.src_blk = g->bond_src_blk; Q.undirected = J.D.undirected;
            Q.act = c->activation; Q.slope = p->prelu; Q.p_drop = c->dropout; Q.seed = c->seed; Q.layer = t;
            Q.aptr = g->atom_gather.ptr; Q.aidx = g->atom_gather.idx; Q.acoef = g->atom_gather.coef;
            Q.aell_idx = g->atom_ell_idx; Q.aell_coef = g->atom_ell_coef;
            Q.aplanes = (uint8_t *)(J.ws + J.L.Ab);
            Q.n_tiles = Hk / BNf;
            Q.zsave = J.D.save && last ? F(J, J.L.Z[t]) : nullptr;
            Q.asave = J.D.save && last ? F(J, J.L.A) : nullptr;
            if (pairs) {  // M_{t-1} from the pair tiles of its producer (no Z_t in inference)
                Q.ain = (const uint8_t *)(J.ws + J.L.Mp[(t - 1) & 1]);
                Q.ain_g = t == 1 ? EPB : BNf;
                Q.aout = last ? nullptr : (uint8_t *)(J.ws + J.L.Mp[t & 1]);
                Q.zin = nullptr;
                Q.zout = nullptr;
                // the last layer: A as pair tiles (W_o on pairs, WD_WO_PAIRS), its words in the slot this layer
                // does not read; else bf16x3 plane tiles
                Q.apairs = last && WD_WO_PAIRS ? (uint8_t *)(J.ws + J.L.Ab) : nullptr;
                Q.amax_out = slot(J, t);
            }
        }, M, grid);
        if (t == 1) WD_TRY(record_prof(c, 0, 0, st));  // one pair around all the layers
        // one instantiation per (tile width, last layer, activation)
        auto go = [&](auto bn_c, auto last_c) {
            constexpr int BN = decltype(bn_c)::value;
            constexpr bool LAST = decltype(last_c)::value;
            host_with_act(c->activation, [&](auto act_c) {
                constexpr int A = decltype(act_c)::value;
                if constexpr (BN == 80) {
                    if (pairs) {
                        if (n == 1)
                            hipLaunchKernelGGL((mp_layer_kernel<BN, LAST, A, false, 1, true>), dim3(grid), dim3(MP_THREADS), 0, st, one_job(M));
                        else
                            hipLaunchKernelGGL((mp_layer_kernel<BN, LAST, A, false, WD_MULTI, true>), dim3(grid), dim3(MP_THREADS), 0, st, M);
                        return;
                    }
                }
                if (n == 1 && D0.atom)
                    hipLaunchKernelGGL((mp_layer_kernel<BN, LAST, A, true, 1>), dim3(grid), dim3(MP_THREADS), 0, st, one_job(M));
                else if (n == 1)
                    hipLaunchKernelGGL((mp_layer_kernel<BN, LAST, A, false, 1>), dim3(grid), dim3(MP_THREADS), 0, st, one_job(M));
                else
                    hipLaunchKernelGGL((mp_layer_kernel<BN, LAST, A, false>), dim3(grid), dim3(MP_THREADS), 0, st, M);
            });
        };
        using I80 = std::integral_constant<int, 80>;
        using I64 = std::integral_constant<int, 64>;
        if (bn80) { if (last) go(I80{}, std::true_type{}); else go(I80{}, std::false_type{}); }
        else { if (last) go(I64{}, std::true_type{}); else go(I64{}, std::false_type{}); }
        WD_CHECK_LAUNCH("mp_layer");
        if (last) WD_TRY(record_prof(c, 0, 1, st));
        if (c->gemm_variant >= 100 && c->gemm_variant % 10 == t + 1) return 0;
    }
    // W_o + readout (empty batches -- no molecules -- have no blocks and write nothing)
    Multi<WoReadoutP> M;
    int grid;
    launch_multi(jobs, n, Hk / BNf, [&](WoReadoutP &R, const FusedJob &J) {
        const WdGraph *g = J.g;
        // (codes: the f_atoms segment is not read; a lean graph has no planes -- the A planes stand in as the
        // segment's non-null base)
        R.fa = g->f_atoms_blk_x6 ? (const uint8_t *)g->f_atoms_blk_x6 : (const uint8_t *)(J.ws + J.L.Ab);
        R.kpa = g->ld_atoms; R.kcw = J.D.Fak / 32;
        R.kca = codes || J.D.atom ? 0 : R.kcw;
        R.eo = codes ? F(J, J.L.Eo) : (J.D.atom ? F(J, J.L.In3) + 2 * Hk : nullptr); R.Hk = Hk;
        R.ldeo = J.D.atom ? 3 * Hk : Hk;
        R.ag = (const uint8_t *)(J.ws + J.L.Ab); R.kp = Hk;
        R.wo = (const uint8_t *)(pk + (bn80 ? PL.WoX80 : PL.WoX)); R.bias = W(PL.bo);
        R.blocks = g->blocks;
        R.w_atoms = g->w_atoms; R.mol_start = g->mol_start; R.mol_size = g->mol_size; R.xn = g->degree_of_polym;
        R.agg = c->aggregation; R.norm = c->aggregation_norm; R.zero_vec = p->zero_vec;
        R.act = c->activation; R.slope = p->prelu; R.p_drop = c->dropout; R.seed = c->seed; R.layer = J.D.T;
        R.out = J.out; R.ncols = J.D.H; R.n_tiles = Hk / BNf;
        R.zosave = J.D.save ? F(J, J.L.Zo) : nullptr;
        // (debug variants 1a4: the W_o pre-activation into the free second ping-pong buffer, tools/debug_pairs.py)
        if (c->gemm_variant >= 100 && c->gemm_variant % 10 == 4 && J.D.T == 3)
            R.zosave = pairs ? F(J, J.L.Mp[1]) : F(J, J.L.Zb[1]);
        if (pairs && WD_WO_PAIRS) {
            R.apairs = (const uint8_t *)(J.ws + J.L.Ab); R.a_amax = slot(J, J.D.T - 1); R.a_nw = Hk / BNf; R.a_g = BNf;
            R.woh = (const uint8_t *)(pk + PL.WoH); R.wo_amax = (const uint32_t *)(pk + PL.wo_amax) + 64;
        }
    }, M, grid);
    if (grid > 0) {
        // one batch: single-chunk stages (55 KB, co-resident with other streams' layers); several: two
        if (pairs && WD_WO_PAIRS && n > 1)
            hipLaunchKernelGGL((wo_readout_kernel<80, 1, WD_MULTI, true>), dim3(grid), dim3(512), 0, st, M);
        else if (pairs && WD_WO_PAIRS)
            hipLaunchKernelGGL((wo_readout_kernel<80, 1, 1, true>), dim3(grid), dim3(512), 0, st, one_job(M));
        else if (bn80 && n > 1)
            hipLaunchKernelGGL((wo_readout_kernel<80, 2>), dim3(grid), dim3(64 * WoWaves<80>::WM * WoWaves<80>::WN), 0, st, M);
        else if (bn80)
            hipLaunchKernelGGL((wo_readout_kernel<80, 1, 1>), dim3(grid), dim3(64 * WoWaves<80>::WM * WoWaves<80>::WN), 0, st, one_job(M));
        else if (n == 1)
            hipLaunchKernelGGL((wo_readout_kernel<64, 1, 1>), dim3(grid), dim3(64 * WoWaves<64>::WM * WoWaves<64>::WN), 0, st, one_job(M));
        else
            hipLaunchKernelGGL((wo_readout_kernel<64, 1>), dim3(grid), dim3(64 * WoWaves<64>::WM * WoWaves<64>::WN), 0, st, M);
        WD_CHECK_LAUNCH("wo_readout");
    }
    return 0;
}

// the whole fused inference forward as one launch (small_fwd.hpp): one workgroup per molecule block
int small_forward(const WdGraph *g, const Dims &D, const WdParams *p, const WdConfig *c, const PackLayout &PL,
                  const char *pk, float *out, hipStream_t st) {
    if (D.nblk < 1) return 0;
    auto W = [&](size_t off) { return (const float *)(pk + off); };
    const bool bn80 = D.Hk % 80 == 0;
    SmallFwdP S{};
    S.blocks = g->blocks; S.codes = g->atom_codes; S.src_blk = g->bond_src_blk; S.tail = g->bond_tail;
    S.rev = g->b2revb;
    S.aell_idx = g->atom_ell_idx; S.aell_coef = g->atom_ell_coef;
    S.aptr = g->atom_gather.ptr; S.aidx = g->atom_gather.idx; S.acoef = g->atom_gather.coef;
    S.w_atoms = g->w_atoms; S.mol_start = g->mol_start; S.mol_size = g->mol_size; S.xn = g->degree_of_polym;
    S.wit = W(PL.WiT); S.woat = W(PL.WoaT);
    S.bi = p->b_i ? W(PL.bi) : nullptr; S.bh = p->b_h ? W(PL.bh) : nullptr; S.bo = W(PL.bo);
    S.wh = (const uint8_t *)(pk + PL.WhH); S.wh_amax = (const uint32_t *)(pk + PL.amax) + 64; S.whbr = fused_bn(D.Hk);
    S.wo = (const uint8_t *)(pk + (bn80 ? PL.WoX80 : PL.WoX)); S.wobr = bn80 ? 80 : 64; S.kcw = D.Fak / 32;
    S.Fa = D.Fa; S.Fb = D.Fb; S.T = D.T; S.undirected = D.undirected; S.agg = c->aggregation; S.norm = c->aggregation_norm;
    S.zero_vec = p->zero_vec; S.slope = p->prelu;
    S.out = out; S.ncols = D.H;
    WD_TRY(record_prof(c, 0, 0, st));
    host_with_act(c->activation, [&](auto act_c) {
        hipLaunchKernelGGL(small_forward_kernel<decltype(act_c)::value>, dim3(D.nblk), dim3(SF_THREADS), 0, st, S);
    });
    WD_CHECK_LAUNCH("small_forward");
    WD_TRY(record_prof(c, 0, 1, st));
    return 0;
}

}  // namespace

// ================================================================================================
// C-ABI
// ================================================================================================
int graph_build_prepare(const WdCompact *c, void *buffer, size_t bytes, int32_t flags, GraphBuildP &P, WdGraph &Gout);
int graph_build_launch(const GraphBuildP *P, int n, hipStream_t st);

extern "C" {

int wdmpnn_abi_version(void) { return WDMPNN_ABI_VERSION; }

int wdmpnn_self_check(int32_t *n_host_kernels, int32_t *n_device_kernels) {
    const SelfCheck &c = self_check_result();
    if (n_host_kernels) *n_host_kernels = c.n_host;
    if (n_device_kernels) *n_device_kernels = c.n_dev;
    return self_check_once();
}

// debug (tools/debug_pairs.py; not in the header): byte offsets in the forward workspace of inp, M_0 / M_1 pair
// tiles, A, the two scale-word slots and the two Z_t ping-pong buffers
int wdmpnn_debug_fwd_offsets(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *out) {
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    const FwdLayout L = fwd_layout(D, p->packed == nullptr);
    const PackLayout PL = pack_layout(D);
    const size_t v[15] = {L.Z.empty() ? 0 : L.Z[0], L.Mp[0], L.Mp[1], L.Ab, L.amax[0], L.amax[1], L.Zb[0], L.Zb[1],
                          L.total, (size_t)D.pairs, PL.WoH, PL.wo_amax, PL.WhH, PL.amax, L.Eo};
    memcpy(out, v, sizeof(v));
    return 0;
}

// experiment builds (WD_STAMPS): copy the layer kernel's phase stamps of the last launch to the host
int wdmpnn_debug_stamps(void *host, size_t bytes) {
#if WD_STAMPS
    if (hipDeviceSynchronize() != hipSuccess) return fail(WD_ERR_ARG, "sync");
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wd_stamps), std::min(bytes, sizeof(g_wd_stamps))) != hipSuccess)
        return fail(WD_ERR_ARG, "stamps copy");
    if (bytes > sizeof(g_wd_stamps) &&
        hipMemcpyFromSymbol((char *)host + sizeof(g_wd_stamps), HIP_SYMBOL(g_wd_lstamps),
                            std::min(bytes - sizeof(g_wd_stamps), sizeof(g_wd_lstamps))) != hipSuccess)
        return fail(WD_ERR_ARG, "loop stamps copy");
    const size_t eo = sizeof(g_wd_stamps) + sizeof(g_wd_lstamps);
    if (bytes > eo && hipMemcpyFromSymbol((char *)host + eo, HIP_SYMBOL(g_wd_estamps),
                                          std::min(bytes - eo, sizeof(g_wd_estamps))) != hipSuccess)
        return fail(WD_ERR_ARG, "embed stamps copy");
    return 0;
#else
    (void)host; (void)bytes;
    return fail(WD_ERR_UNSUPPORTED, "library built without WD_STAMPS");
#endif
}



const char *wdmpnn_last_error(void) { return g_err.c_str(); }

int wdmpnn_packed_params_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes) {
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (!bytes) return fail(WD_ERR_ARG, "null bytes");
    *bytes = pack_layout(D).total;
    return 0;
}

int wdmpnn_pack_params(const WdGraph *g, const WdParams *p, const WdConfig *c, void *packed, size_t bytes,
                       void *stream) {
    WD_KERNELS_OK();
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (!packed || bytes < pack_layout(D).total) return fail(WD_ERR_WORKSPACE, "packed buffer too small");
    return pack_params(D, p, (char *)packed, (hipStream_t)stream);
}

int wdmpnn_workspace_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes) {
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (!bytes) return fail(WD_ERR_ARG, "null bytes");
    *bytes = fwd_layout(D, p->packed == nullptr).total;
    return 0;
}

int wdmpnn_backward_workspace_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes) {
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (!bytes) return fail(WD_ERR_ARG, "null bytes");
    *bytes = bwd_layout(g, D).total;
    return 0;
}

int wdmpnn_forward(const WdGraph *g, const WdParams *p, const WdConfig *c, void *workspace, size_t workspace_bytes,
                   float *out, void *stream) {
    WD_KERNELS_OK();
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    const FwdLayout L = fwd_layout(D, p->packed == nullptr);
    if (!workspace || workspace_bytes < L.total)
        return fail(WD_ERR_WORKSPACE, "workspace too small: need %zu bytes, got %zu", L.total, workspace_bytes);
    if (!out) return fail(WD_ERR_ARG, "null out");
    const PackLayout PL = pack_layout(D);
    if (p->packed && p->packed_bytes < PL.total) return fail(WD_ERR_WORKSPACE, "packed params too small");
    hipStream_t st = (hipStream_t)stream;
    char *ws = (char *)workspace;
    auto F = [&](size_t off) { return (float *)(ws + off); };
    if (L.own_pack) WD_TRY(pack_params(D, p, ws + L.packed, st));
    const char *pk = L.own_pack ? ws + L.packed : (const char *)p->packed;
    auto W = [&](size_t off) { return (const float *)(pk + off); };
    const int Hk = D.Hk;

    // without plane copies of its A operand a split-plane GEMM splits in the kernel (gemm_x6_kernel)
    const bool split = !D.f32;
    const char *pkb = pk;

    if (D.small) return small_forward(g, D, p, c, PL, pk, out, st);
    if (D.blocked) {
        FusedJob J{g, D, L, ws, out};
        return fused_forward(&J, 1, p, c, PL, pk, st);
    }

    // L0: input layer (mpn.py:92-97)
    {
        const float *a = D.atom ? g->f_atoms : g->f_bonds;
        const int lda = D.atom ? g->ld_atoms : g->ld_bonds;
        const Epi e = epi_act(c->activation, p->prelu, W(PL.bi), nullptr, F(L.Z[0]), F(L.M[0]), Hk, c, 0);
        if (D.x6 && g->f_bonds_x6 && x6g_eligible(e))
            WD_TRY(gemm_x6g(g->f_bonds_x6, g->ld_bonds, D.Kink, nullptr, 0, 0, pkb + PL.WiX, D.Rp, Hk, e, st));
        else
            WD_TRY(gemm_nt(a, lda, D.Kink, nullptr, 0, 0, W(PL.Wi), D.Kink, D.Rp, Hk, e, st, split));
    }
    // L1..T-1: message passing (mpn.py:100-124): X_t = gather(M_{t-1}) [| bond features], then
    // M_t = act(inp + X_t W_h^T (+ b_h))
    int cur = 0;
    for (int t = 1; t < D.T; ++t) {
        const int prev = D.save ? t - 1 : cur;
        const int next = D.save ? t : 1 - cur;
        float *Xt = F(L.X[D.save ? t - 1 : 0]);
        float *Zt = D.save ? F(L.Z[t]) : nullptr;
        const Epi e = epi_act(c->activation, p->prelu, W(PL.bh), F(L.Z[0]), Zt, F(L.M[next]), Hk, c, t);
        const int32_t *sym = D.undirected ? g->b2revb : nullptr;
        if (t == 1) WD_TRY(record_prof(c, 0, 0, st));  // one pair around all the layers
        if (D.x6 && x6g_eligible(e)) {
            // X_t as plane tiles (+ fp32 for the weight gradient when training)
            WD_TRY(gather8(F(L.M[prev]), Hk, Hk, g->msg_gather, sym, D.save ? Xt : nullptr, D.ldx, ws + L.Xp, Hk, 0,
                           D.R, D.Rp, st));
            WD_TRY(gemm_x6g(ws + L.Xp, Hk, Hk, nullptr, 0, 0, pkb + PL.WhX, D.Rp, Hk, e, st));
        } else {
            WD_TRY(gather8(F(L.M[prev]), Hk, Hk, g->msg_gather, sym, Xt, D.ldx, nullptr, 0, 0, D.R, D.Rp, st));
            if (D.atom)
                WD_TRY(gather8(g->f_bonds, g->ld_bonds, D.Fbk, g->bond_feat_gather, nullptr, Xt + Hk, D.ldx, nullptr, 0,
                               0, D.R, D.Rp, st));
            WD_TRY(gemm_nt(Xt, D.ldx, D.ldx, nullptr, 0, 0, W(PL.Wh), D.ldx, D.Rp, Hk, e, st, split));
        }
        if (t == D.T - 1) WD_TRY(record_prof(c, 0, 1, st));
        cur = next;
    }
    const float *M_last = F(L.M[D.save ? D.T - 1 : cur]);
    // LT: atom hidden states (mpn.py:126-134): h = act([f_atoms | gather(M)] W_o^T + b_o)
    {
        const Epi e = epi_act(c->activation, p->prelu, W(PL.bo), nullptr, D.save ? F(L.Zo) : nullptr, F(L.h), Hk, c,
                              D.T);
        if (D.x6 && g->f_atoms_x6 && x6g_eligible(e)) {
            WD_TRY(gather8(M_last, Hk, Hk, g->atom_gather, nullptr, D.save ? F(L.A) : nullptr, Hk, ws + L.Ap, Hk, 0,
                           D.Va, D.Vap, st));
            WD_TRY(gemm_x6g(g->f_atoms_x6, g->ld_atoms, D.Fak, ws + L.Ap, Hk, Hk, pkb + PL.WoX, D.Vap, Hk, e, st));
        } else {
            WD_TRY(gather8(M_last, Hk, Hk, g->atom_gather, nullptr, F(L.A), Hk, nullptr, 0, 0, D.Va, D.Vap, st));
            WD_TRY(gemm_nt(g->f_atoms, g->ld_atoms, D.Fak, F(L.A), Hk, Hk, W(PL.Wo), D.Ko, D.Vap, Hk, e, st,
                           split));
        }
    }
    const float *hfin = F(L.h);
    int ldfin = Hk;
    // LT+1: atom descriptors layer (mpn.py:136-143): Linear + dropout, no activation
    if (D.desc) {
        WD_TRY(gemm_nt(F(L.h), Hk, Hk, g->atom_desc, D.dk, D.dk, W(PL.Wd), D.Kd, D.Vap, D.Hdk,
                       epi_act(WD_ACT_IDENTITY, nullptr, W(PL.bd), nullptr, D.save ? F(L.Zd) : nullptr, F(L.hd), D.Hdk,
                               c, D.T + 1),
                       st));
        hfin = F(L.hd);
        ldfin = D.Hdk;
    }
    // readout (mpn.py:145-171)
    if (D.B > 0) {
        hipLaunchKernelGGL(readout_kernel, dim3(D.B, (D.Hd + 4 * RO_QW - 1) / (4 * RO_QW)), dim3(RO_THREADS), 0, st,
                           readout_params(g, p, c, hfin, ldfin, D.Hd, out));
        WD_CHECK_LAUNCH("readout");
    }
    return 0;
}

int wdmpnn_forward_many(int32_t n, const WdGraph *graphs, const WdParams *p, const WdConfig *c,
                        void *const *workspaces, const size_t *workspace_bytes, float *const *outs, void *stream) {
    WD_KERNELS_OK();
    if (n < 0 || (n && (!graphs || !workspaces || !workspace_bytes || !outs))) return fail(WD_ERR_ARG, "forward_many: bad arrays");
    if (n == 0) return 0;
    if (!p || !c) return fail(WD_ERR_ARG, "null params/config");
    if (!p->packed) return fail(WD_ERR_ARG, "forward_many needs packed parameters (wdmpnn_pack_params)");
    if (c->save_for_backward) return fail(WD_ERR_UNSUPPORTED, "forward_many is inference only (save_for_backward = 0)");
    std::vector<FusedJob> jobs((size_t)n);
    for (int j = 0; j < n; ++j) {
        FusedJob &J = jobs[j];
        J.g = graphs + j;
        WD_TRY(get_dims(J.g, p, c, J.D));
        if (!J.D.blocked)
            return fail(WD_ERR_UNSUPPORTED, "forward_many: graph %d does not take the fused forward (molecule blocks, "
                                            "bond messages, no descriptors, depth >= 2)", j);
        J.L = fwd_layout(J.D, false);
        if (!workspaces[j] || workspace_bytes[j] < J.L.total)
            return fail(WD_ERR_WORKSPACE, "forward_many: workspace %d too small: need %zu bytes, got %zu", j, J.L.total,
                        workspace_bytes[j]);
        if (!outs[j]) return fail(WD_ERR_ARG, "forward_many: null out %d", j);
        J.ws = (char *)workspaces[j];
        J.out = outs[j];
    }
    const PackLayout PL = pack_layout(jobs[0].D);
    if (p->packed_bytes < PL.total) return fail(WD_ERR_WORKSPACE, "packed params too small");
    for (int j = 0; j < n; j += WD_MULTI)
        WD_TRY(fused_forward(jobs.data() + j, std::min(WD_MULTI, n - j), p, c, PL, (const char *)p->packed,
                             (hipStream_t)stream));
    return 0;
}

int wdmpnn_backward(const WdGraph *g, const WdParams *p, const WdConfig *c, const void *workspace,
                    size_t workspace_bytes, const float *dout, void *scratch, size_t scratch_bytes,
                    const WdGrads *grads, void *stream) {
    WD_KERNELS_OK();
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (!D.save) return fail(WD_ERR_ARG, "backward needs a forward run with save_for_backward=1");
    const FwdLayout L = fwd_layout(D, p->packed == nullptr);
    const BwdLayout Bl = bwd_layout(g, D);
    if (!workspace || workspace_bytes < L.total) return fail(WD_ERR_WORKSPACE, "forward workspace too small");
    if (!scratch || scratch_bytes < Bl.total)
        return fail(WD_ERR_WORKSPACE, "backward scratch too small: need %zu bytes, got %zu", Bl.total, scratch_bytes);
    if (!dout || !grads) return fail(WD_ERR_ARG, "null dout/grads");
    hipStream_t st = (hipStream_t)stream;
    char *ws = (char *)workspace;
    char *sc = (char *)scratch;
    auto F = [&](size_t off) { return (float *)(ws + off); };
    auto S = [&](size_t off) { return (float *)(sc + off); };
    const PackLayout PL = pack_layout(D);
    const char *pk = L.own_pack ? ws + L.packed : (const char *)p->packed;
    auto W = [&](size_t off) { return (const float *)(pk + off); };
    const int H = D.H, Hk = D.Hk;
    const bool prelu = c->activation == WD_ACT_PRELU;
    float *prelu_part = S(Bl.prelu);
    int prelu_used = 0;
    if (prelu && hipMemsetAsync(prelu_part, 0, Bl.prelu_floats * 4, st) != hipSuccess)
        return fail(WD_ERR_ARG, "memset failed");

    auto act_bwd = [&](ActBwd P) -> int {
        const size_t total = (size_t)P.rows_p * P.cols;
        if (total >= (size_t)1 << 31) return fail(WD_ERR_SHAPE, "act_bwd: %zu elements exceed the 32-bit index", total);
        auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
        const bool v4 = P.cols % 4 == 0 && P.ld % 4 == 0 && P.ldg % 4 == 0 && al(P.G) && al(P.out) &&
                        (!P.Z || al(P.Z)) && (!P.add_in || al(P.add_in)) && (!P.res_out || al(P.res_out));
        const int nb = ew_blocks(v4 ? total / 4 : total);
        if (P.words && (!v4 || (total / 4) % 256))
            return fail(WD_ERR_SHAPE, "act_bwd: scale words need 256-vector multiples (%zu elements)", total);
        if (prelu && P.Z) { P.prelu_part = prelu_part + prelu_used; prelu_used += nb; }
        if (v4) hipLaunchKernelGGL(act_bwd_kernel<4>, dim3(nb), dim3(256), 0, st, P);
        else hipLaunchKernelGGL(act_bwd_kernel<1>, dim3(nb), dim3(256), 0, st, P);
        WD_CHECK_LAUNCH("act_bwd");
        return 0;
    };
    auto base_bwd = [&](const float *Z, uint32_t layer, int act, int rows, int rows_p, int cols, float *out) {
        ActBwd P{};
        P.Z = Z; P.act = act; P.slope = p->prelu; P.p_drop = layer == 0 ? 0.f : c->dropout;  // (see epi_act)
        P.seed = c->seed; P.layer = layer;
        P.rows = rows; P.rows_p = rows_p; P.cols = cols; P.ld = cols; P.out = out;
        return P;
    };

    // readout backward -> dH [Vap][Hk or Hdk]; without descriptors fused with the W_o activation's backward
    // (readout_act_bwd_kernel: dZo straight from dout, no dH and no memset)
    const int ldH = D.desc ? D.Hdk : Hk;
    float *dH = S(Bl.dH);
    const int ro_wgs = (D.B + 1) * RO_ACT_Y;
    const bool ro_fused = !D.desc && Hk <= RO_ACT_MAXLD && (!prelu || prelu_used + ro_wgs <= (int)Bl.prelu_floats);
    if (ro_fused) {
        RoActBwd A{};
        A.Z = F(L.Zo); A.ld = Hk; A.act = c->activation; A.slope = p->prelu; A.p_drop = c->dropout;
        A.seed = c->seed; A.layer = D.T; A.out = S(Bl.dZo); A.rows = D.Va; A.rows_p = D.Vap;
        if (prelu) { A.prelu_part = prelu_part + prelu_used; prelu_used += ro_wgs; }
        hipLaunchKernelGGL(readout_act_bwd_kernel, dim3(D.B + 1, RO_ACT_Y), dim3(256), 0, st,
                           readout_params(g, p, c, nullptr, Hk, D.Hd, nullptr), dout, A);
        WD_CHECK_LAUNCH("readout_act_bwd");
    } else if (hipMemsetAsync(dH, 0, (size_t)D.Vap * ldH * 4, st) != hipSuccess) {
        return fail(WD_ERR_ARG, "memset failed");
    }
    if (D.B > 0 && !ro_fused) {
        hipLaunchKernelGGL(readout_bwd_kernel, dim3(D.B, (D.Hd + RO_BWD_COLS - 1) / RO_BWD_COLS), dim3(256), 0, st,
                           readout_params(g, p, c, nullptr, ldH, D.Hd, nullptr), dout, dH);
        WD_CHECK_LAUNCH("readout_bwd");
    }
    const float *dh = dH;
    if (D.desc) {  // hd = Zd * s (identity act)
        ActBwd P = base_bwd(F(L.Zd), D.T + 1, WD_ACT_IDENTITY, D.Va, D.Vap, D.Hdk, S(Bl.dZd));
        P.G = dH; P.ldg = D.Hdk;
        WD_TRY(act_bwd(P));
        Src dZ = make_src(D.Va, {seg_dense(S(Bl.dZd), D.Hdk, D.Hdk)});
        Src X = x_d(g, D, F(L.h));
        TnPlan tp = tn_plan(D.Hdk, X, D.Va);
        WD_TRY(gemm_tn(dZ, X, D.Hdk, D.Va, tp, S(Bl.slab), 0, st));
        WD_TRY(slab_reduce(tp, S(Bl.slab), D.Hd, {{0, 0, H}, {Hk, H, D.d}}, grads->W_d, D.Hd, grads->b_d,
                           X.s[2].kp0, st));
        // dh = dZd W_d[:, :H]
        WD_TRY(gemm_nt(S(Bl.dZd), D.Hdk, D.Hdk, nullptr, 0, 0, W(PL.WdT), D.Hdk, D.Vap, Hk,
                       epi_store(S(Bl.dHo), Hk), st, true));
        dh = S(Bl.dHo);
    }
    // the weight-gradient reductions, launched together at the end (slab_reduce_multi)
    SlabReduce red[SLAB_MAX];
    int nred = 0;
    // W_o layer
    {
        if (!ro_fused) {
            ActBwd P = base_bwd(F(L.Zo), D.T, c->activation, D.Va, D.Vap, Hk, S(Bl.dZo));
            P.G = dh; P.ldg = Hk;
            WD_TRY(act_bwd(P));
        }
        Src dZ = make_src(D.Va, {seg_dense(S(Bl.dZo), Hk, Hk)});
        Src X = x_o(g, D, F(L.A));
        TnPlan tp = tn_plan(Hk, X, D.Va);
        WD_TRY(gemm_tn(dZ, X, Hk, D.Va, tp, S(Bl.slab), 0, st));
        red[nred++] = slab_job(tp, S(Bl.slab), H, {{0, 0, D.Fa}, {D.Fak, D.Fa, H}}, grads->W_o, D.Fa + H, grads->b_o,
                               X.s[2].kp0);
        // dA = dZo W_o[:, Fa:] (dZo as plane tiles from the readout backward and this GEMM on LDS-DMA
        // staging measured no faster: 0.3734-0.3761 against 0.3729-0.3756 ms per training step, same box)
        WD_TRY(gemm_nt(S(Bl.dZo), Hk, Hk, nullptr, 0, 0, W(PL.WoT), Hk, D.Vap, Hk, epi_store(S(Bl.dA), Hk), st, true));
    }
    // gradient reaching M_{T-1} through the final aggregation, then the message layers
    float *dZbuf[2] = {S(Bl.dZ0), S(Bl.dZ1)};
    int cur = 0;
    {
        ActBwd P = base_bwd(F(L.Z[D.T - 1]), D.T - 1, c->activation, D.R, D.Rp, Hk, dZbuf[cur]);
        P.G = S(Bl.dA); P.ldg = Hk;
        P.ptr = g->atom_gather_t.ptr; P.idx = g->atom_gather_t.idx; P.coef = g->atom_gather_t.coef;
        if (D.T > 1) { P.res_out = S(Bl.dRes); P.res_init = 1; }
        WD_TRY(act_bwd(P));
    }
    const Src Xh0 = x_h(D, nullptr);
    const TnPlan tph = tn_plan(Hk, Xh0, D.R);
    uint32_t *y_words = (uint32_t *)S(Bl.words), *m_words = (uint32_t *)S(Bl.mwords);
    for (int t = D.T - 1; t >= 1 && D.blocked; --t) {
        // fused training forward: X_t = G M_{t-1} was never formed (the layer kernel computes G (M W_h^T)),
        // so the adjoint of the gather goes first: Y_t = S G^T dZ_t, dW_h (+)= Y_t^T M_{t-1} (M recomputed
        // from the saved Z_{t-1} while loading), db_h (+)= sum dZ_t, dM_{t-1} = Y_t W_h.
        float *dZt = dZbuf[cur];
        const int nxt = 1 - cur;
        float *Y = S(Bl.dX);
        {
            ActBwd Q{};
            Q.G = dZt; Q.ldg = Hk;
            Q.ptr = g->msg_gather_t.ptr; Q.idx = g->msg_gather_t.idx; Q.coef = g->msg_gather_t.coef;
            Q.rows = D.R; Q.rows_p = D.Rp; Q.cols = Hk; Q.ld = Hk; Q.out = D.undirected ? S(Bl.dMs) : Y;
            if (WD_BWD_H2 && !D.undirected) Q.words = y_words;
            WD_TRY(act_bwd(Q));
            if (D.undirected) {
                ActBwd U{};
                U.G = S(Bl.dMs); U.ldg = Hk; U.sym_rev = g->b2revb;
                U.rows = D.R; U.rows_p = D.Rp; U.cols = Hk; U.ld = Hk; U.out = Y;
                if (WD_BWD_H2) U.words = y_words;
                WD_TRY(act_bwd(U));
            }
        }
        // dZ_{t-1} = (Y_t W_h) * dropout * act'(Z_{t-1}), the residual sum of mpn.py:123 accumulated, in
        // the GEMM's epilogue (EPI_ACTBWD), which also publishes max |M_{t-1}| per tile for the weight
        // gradient below (so this GEMM goes first: neither reads what the other writes)
        Epi e{};
        e.kind = EPI_ACTBWD; e.Y = dZbuf[nxt]; e.ld = Hk; e.Z = F(L.Z[t - 1]); e.act = c->activation;
        e.slope = p->prelu; e.p_drop = t - 1 == 0 ? 0.f : c->dropout; e.seed = c->seed; e.layer = t - 1;
        e.rows_valid = D.R;
        if (t - 1 == 0) e.add_in = S(Bl.dRes);
        else { e.res_out = S(Bl.dRes); e.res_init = 0; }
        if (prelu) {
            const int tiles = (D.Rp / x6_bm(D.Rp)) * (Hk / 64);  // (gemm_x6_kernel's grid)
            if (prelu_used + tiles > (int)Bl.prelu_floats) return fail(WD_ERR_SHAPE, "PReLU partials overflow");
            e.prelu_part = prelu_part + prelu_used;
            prelu_used += tiles;
        }
        // (with Y_t as plane tiles written by the gather above and this GEMM on LDS-DMA staging, gemm_x6g: the
        // plane stores cost the gather 4-8 us, the GEMM gained 0-4.5 us; the in-kernel split is kept)
        if (WD_BWD_H2) e.amax = m_words;
        WD_TRY(gemm_nt(Y, Hk, Hk, nullptr, 0, 0, W(PL.WhT), Hk, D.Rp, Hk, e, st, true, WD_BWD_H2 ? y_words : nullptr,
                       Hk / 4, (const uint32_t *)W(PL.amax) + 64));
        // dW_h (+)= Y_t^T [M_{t-1} | 1], db_h (+)= sum dZ_t
        Seg m = seg_dense(F(L.Z[t - 1]), Hk, Hk);
        m.kind = SEG_ACT; m.act = c->activation; m.slope = p->prelu; m.p_drop = t - 1 == 0 ? 0.f : c->dropout;
        m.seed = c->seed; m.layer = t - 1;
        WD_TRY(gemm_tn(make_src(D.R, {seg_dense(Y, Hk, Hk)}), make_src(D.R, {m, seg_ones()}), Hk, D.R, tph,
                       S(Bl.slab_h), t != D.T - 1, st, dZt, WD_BWD_H2 ? y_words : nullptr, Hk / 4, m_words,
                       x6_bm(D.Rp), Hk / 64));
        cur = nxt;
    }
    for (int t = D.T - 1; t >= 1 && !D.blocked; --t) {
        float *dZt = dZbuf[cur];
        // dW_h, db_h (+)= dZ_t^T [X_t | 1]
        Src dZ = make_src(D.R, {seg_dense(dZt, Hk, Hk)});
        WD_TRY(gemm_tn(dZ, x_h(D, F(L.X[t - 1])), Hk, D.R, tph, S(Bl.slab_h), t != D.T - 1, st));
        // dX = dZ_t W_h[:, :H]
        WD_TRY(gemm_nt(dZt, Hk, Hk, nullptr, 0, 0, W(PL.WhT), Hk, D.Rp, Hk, epi_store(S(Bl.dX), Hk), st, true));
        // dM_{t-1} = gather^T(dX) (+ symmetrize), then through the activation of layer t-1
        const int nxt = 1 - cur;
        ActBwd P = base_bwd(F(L.Z[t - 1]), t - 1, c->activation, D.R, D.Rp, Hk, dZbuf[nxt]);
        if (D.undirected) {
            ActBwd Q{};
            Q.G = S(Bl.dX); Q.ldg = Hk;
            Q.ptr = g->msg_gather_t.ptr; Q.idx = g->msg_gather_t.idx; Q.coef = g->msg_gather_t.coef;
            Q.rows = D.R; Q.rows_p = D.Rp; Q.cols = Hk; Q.ld = Hk; Q.out = S(Bl.dMs);
            WD_TRY(act_bwd(Q));
            P.G = S(Bl.dMs); P.ldg = Hk; P.sym_rev = g->b2revb;
        } else {
            P.G = S(Bl.dX); P.ldg = Hk;
            P.ptr = g->msg_gather_t.ptr; P.idx = g->msg_gather_t.idx; P.coef = g->msg_gather_t.coef;
        }
        if (t - 1 == 0) P.add_in = S(Bl.dRes);
        else { P.res_out = S(Bl.dRes); P.res_init = 0; }
        WD_TRY(act_bwd(P));
        cur = nxt;
    }
    if (D.T > 1) {
        if (D.atom)
            red[nred++] = slab_job(tph, S(Bl.slab_h), H, {{0, 0, H}, {Hk, H, D.Fb}}, grads->W_h, H + D.Fb, grads->b_h,
                                   Xh0.s[1].kp0);
        else
            red[nred++] = slab_job(tph, S(Bl.slab_h), H, {{0, 0, H}}, grads->W_h, H, grads->b_h, Xh0.s[1].kp0);
    }
    // input layer: dW_i, db_i = dZ_0^T [f | 1]
    {
        Src dZ = make_src(D.R, {seg_dense(dZbuf[cur], Hk, Hk)});
        Src X = x_in(g, D);
        TnPlan tp = tn_plan(Hk, X, D.R);
        WD_TRY(gemm_tn(dZ, X, Hk, D.R, tp, S(Bl.slab_i), 0, st));
        red[nred++] = slab_job(tp, S(Bl.slab_i), H, {{0, 0, D.Kin}}, grads->W_i, D.Kin, grads->b_i, X.s[1].kp0);
    }
    // every weight gradient's split-K sum in one launch (three launches of ~4.8 us each before)
    WD_TRY(slab_reduce_multi(red, nred, st));
    if (prelu && grads->prelu) {
        hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, st, prelu_part, prelu_used, grads->prelu);
        WD_CHECK_LAUNCH("prelu sum");
    }
    return 0;
}

int wdmpnn_saved_layout(const WdGraph *g, const WdParams *p, const WdConfig *c, WdSaved *out) {
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (!out) return fail(WD_ERR_ARG, "null out");
    if (!D.save) return fail(WD_ERR_ARG, "saved_layout needs save_for_backward = 1");
    if (D.T > WDMPNN_MAX_SAVED_DEPTH) return fail(WD_ERR_UNSUPPORTED, "depth %d > %d", D.T, WDMPNN_MAX_SAVED_DEPTH);
    const FwdLayout L = fwd_layout(D, p->packed == nullptr);
    *out = WdSaved{};
    out->depth = D.T; out->rows = D.R; out->atom_rows = D.Va; out->ld = D.Hk;
    for (int t = 0; t < D.T; ++t) out->z[t] = L.Z[t];
    out->zo = L.Zo;
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

int wdmpnn_plane_bytes(int32_t rows, int32_t kp, size_t *bytes) {
    if (!bytes || rows < 0 || kp < 0) return fail(WD_ERR_ARG, "bad plane request");
    *bytes = (size_t)rows * kp * 6;
    return 0;
}

int wdmpnn_split_planes(const float *src, int32_t ld, int32_t rows, int32_t kp, void *dst, size_t dst_bytes,
                        void *stream) {
    WD_KERNELS_OK();
    if (rows == 0 || kp == 0) return 0;
    if (!src || !dst) return fail(WD_ERR_ARG, "null pointer");
    if (rows % 64 || kp % 32 || ld < kp || ld % 4 || !aligned16(src) || !aligned16(dst))
        return fail(WD_ERR_SHAPE, "split_planes: rows %% 64, kp %% 32, ld >= kp, ld %% 4 and 16-byte alignment "
                                  "required (rows %d kp %d ld %d)", rows, kp, ld);
    if (dst_bytes < (size_t)rows * kp * 6) return fail(WD_ERR_WORKSPACE, "plane buffer too small");
    hipLaunchKernelGGL(split_tiles_kernel<64>, dim3(ew_blocks((size_t)rows * kp / 8)), dim3(256), 0, (hipStream_t)stream,
                       src, ld, rows, kp, (uint8_t *)dst);
    WD_CHECK_LAUNCH("split_planes");
    return 0;
}

int wdmpnn_split_planes_rows(const float *src, int32_t ld, int32_t rows, int32_t kp, const int32_t *row_map,
                             int32_t out_rows, void *dst, size_t dst_bytes, void *stream) {
    WD_KERNELS_OK();
    if (out_rows == 0 || kp == 0) return 0;
    if (!src || !dst || !row_map) return fail(WD_ERR_ARG, "null pointer");
    if (out_rows % 64 || kp % 32 || ld < kp || ld % 4 || !aligned16(src) || !aligned16(dst))
        return fail(WD_ERR_SHAPE, "split_planes_rows: out_rows %% 64, kp %% 32, ld >= kp, ld %% 4 and 16-byte "
                                  "alignment required (out_rows %d kp %d ld %d)", out_rows, kp, ld);
    const size_t need = (size_t)out_rows * kp * 6;
    if (dst_bytes < need) return fail(WD_ERR_WORKSPACE, "plane buffer too small");
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(dst, 0, need, st) != hipSuccess) return fail(WD_ERR_ARG, "memset failed");
    if (rows > 0)
        hipLaunchKernelGGL(split_tiles_kernel<64>, dim3(ew_blocks((size_t)rows * kp / 8)), dim3(256), 0, st, src, ld, rows,
                           kp, (uint8_t *)dst, row_map);
    WD_CHECK_LAUNCH("split_planes_rows");
    return 0;
}

int wdmpnn_build_bond_features(const float *f_atoms, int32_t ld_atoms, int32_t atom_fdim, int32_t atom_rows,
                               const int32_t *b2a, const float *bond_tail, int32_t ld_tail, int32_t tail_dim,
                               int32_t rows, float *f_bonds, int32_t ld_bonds, void *stream) {
    WD_KERNELS_OK();
    if (rows == 0) return 0;
    if (!f_atoms || !b2a || !f_bonds || (tail_dim && !bond_tail)) return fail(WD_ERR_ARG, "null pointer");
    if (rows < 0 || atom_rows <= 0 || atom_fdim < 0 || tail_dim < 0 || atom_fdim > ld_atoms || tail_dim > ld_tail ||
        atom_fdim + tail_dim > ld_bonds)
        return fail(WD_ERR_SHAPE, "build_bond_features: need atom_fdim <= ld_atoms, tail_dim <= ld_tail, "
                                  "atom_fdim + tail_dim <= ld_bonds (got %d/%d, %d/%d, ld_bonds %d)",
                    atom_fdim, ld_atoms, tail_dim, ld_tail, ld_bonds);
    hipLaunchKernelGGL(build_bond_features_kernel, dim3(ew_blocks((size_t)rows * ld_bonds)), dim3(256), 0,
                       (hipStream_t)stream, f_atoms, ld_atoms, atom_fdim, atom_rows, b2a, bond_tail, ld_tail, tail_dim,
                       rows, f_bonds, ld_bonds);
    WD_CHECK_LAUNCH("build_bond_features");
    return 0;
}

int wdmpnn_index_select_rows(const float *src, int64_t n_src_rows, int64_t row_len, const int64_t *index,
                             int64_t n_index, float *out, void *stream) {
    WD_KERNELS_OK();
    if (n_index < 0 || row_len < 0 || n_src_rows < 0) return fail(WD_ERR_ARG, "negative size");
    if (n_index == 0 || row_len == 0) return 0;
    if (!src || !index || !out) return fail(WD_ERR_ARG, "null pointer");
    const size_t total = (size_t)n_index * row_len;
    hipLaunchKernelGGL(index_select_rows_kernel, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, src,
                       row_len, index, n_index, out);
    WD_CHECK_LAUNCH("index_select_rows");
    return 0;
}

int wdmpnn_graph_bytes(const WdCompact *c, size_t *bytes) {
    GraphLayout L;
    WD_TRY(graph_layout(c, L));
    if (!bytes) return fail(WD_ERR_ARG, "null bytes");
    *bytes = L.total;
    return 0;
}

int wdmpnn_build_graph(const WdCompact *c, void *buffer, size_t bytes, WdGraph *g, void *stream) {
    return wdmpnn_build_graph_ex(c, buffer, bytes, g, 0, stream);
}

int wdmpnn_build_graph_ex(const WdCompact *c, void *buffer, size_t bytes, WdGraph *g, int32_t flags, void *stream) {
    WD_KERNELS_OK();
    Multi<GraphBuildP> M{};
    if (!g) return fail(WD_ERR_ARG, "null graph");
    WD_TRY(graph_build_prepare(c, buffer, bytes, flags, M.p[0], *g));
    M.n = 1;
    M.t0[0] = 0;
    for (int j = 1; j <= WD_MULTI; ++j) M.t0[j] = c->n_blocks + 1;
    hipLaunchKernelGGL(graph_build_kernel, dim3(c->n_blocks + 1, M.p[0].lean ? 1 : GB_SLICES), dim3(256), 0,
                       (hipStream_t)stream, M);
    WD_CHECK_LAUNCH("graph_build");
    return 0;
}

}  // extern "C"

// the build parameters and the WdGraph of a compact batch in `buffer` (no launch)
int graph_build_prepare(const WdCompact *c, void *buffer, size_t bytes, int32_t flags, GraphBuildP &P, WdGraph &Gout) {
    if (flags & ~(WDMPNN_GRAPH_LEAN | WDMPNN_GRAPH_NO_PLANES))
        return fail(WD_ERR_ARG, "unknown graph build flags 0x%x", flags);
    const bool lean = flags & WDMPNN_GRAPH_LEAN, planes = !lean && !(flags & WDMPNN_GRAPH_NO_PLANES);
    GraphLayout L;
    WD_TRY(graph_layout(c, L));
    if (!buffer) return fail(WD_ERR_ARG, "null buffer");
    if (bytes < L.total) return fail(WD_ERR_WORKSPACE, "graph buffer too small: need %zu bytes, got %zu", L.total, bytes);
    if ((uintptr_t)buffer % 256) return fail(WD_ERR_ARG, "graph buffer must be 256-byte aligned");
    if (c->n_mols && (!c->mols || !c->xn)) return fail(WD_ERR_ARG, "null molecule arrays");
    if (!c->atoms || (c->n_bonds > 1 && !c->pairs) || (c->n_blocks && (!c->blocks || !c->block_nnz)))
        return fail(WD_ERR_ARG, "null compact arrays");
    char *base = (char *)buffer;
    auto F = [&](size_t o) { return (float *)(base + o); };
    auto I = [&](size_t o) { return (int32_t *)(base + o); };
    auto U = [&](size_t o) { return (uint8_t *)(base + o); };
    P = GraphBuildP{};
    P.c = *c;
    P.Fa = c->atom_fdim; P.Fb = c->bond_fdim; P.lda = L.lda; P.ldb = L.ldb; P.Vap = L.Vap; P.Rbp = L.Rbp;
    P.f_atoms = F(L.f_atoms); P.f_bonds = F(L.f_bonds);
    P.fa_x6 = planes ? U(L.fa_x6) : nullptr; P.fb_x6 = planes ? U(L.fb_x6) : nullptr;
    P.fa_blk_x6 = planes ? U(L.fa_blk_x6) : nullptr;
    P.w_atoms = F(L.w_atoms); P.xn = F(L.xn); P.mol_start = I(L.mol_start); P.mol_size = I(L.mol_size);
    P.b2revb = I(L.b2revb); P.blocks = I(L.blocks); P.bond_blk_row = I(L.bond_blk_row);
    P.atom_blk_row = I(L.atom_blk_row);
    P.bond_src_blk = U(L.bond_src_blk); P.bond_tail = (uint16_t *)(base + L.bond_tail);
    P.msg_ell_idx = U(L.msg_ell_idx); P.msg_ell_coef = F(L.msg_ell_coef);
    P.agg_ell_idx = U(L.agg_ell_idx); P.agg_ell_coef = F(L.agg_ell_coef);
    P.msg_ptr = I(L.csr[0][0]); P.msg_idx = I(L.csr[0][1]); P.msg_coef = F(L.csr[0][2]);
    P.agg_ptr = I(L.csr[1][0]); P.agg_idx = I(L.csr[1][1]); P.agg_coef = F(L.csr[1][2]);
    P.msgt_ptr = I(L.csr[2][0]); P.msgt_idx = I(L.csr[2][1]); P.msgt_coef = F(L.csr[2][2]);
    P.aggt_ptr = I(L.csr[3][0]); P.aggt_idx = I(L.csr[3][1]); P.aggt_coef = F(L.csr[3][2]);
    P.lean = lean;
    P.planes = planes;
    WdGraph G{};
    G.n_atoms = c->n_atoms; G.n_bonds = c->n_bonds; G.n_mols = c->n_mols;
    G.atom_fdim = c->atom_fdim; G.bond_fdim = c->bond_fdim; G.ld_atoms = L.lda; G.ld_bonds = L.ldb; G.bond_col0 = 0;
    G.f_atoms = P.f_atoms; G.f_bonds = P.f_bonds; G.w_atoms = P.w_atoms;
    G.mol_start = P.mol_start; G.mol_size = P.mol_size; G.degree_of_polym = P.xn;
    G.msg_gather = WdCsr{P.msg_ptr, P.msg_idx, P.msg_coef};
    G.atom_gather = WdCsr{P.agg_ptr, P.agg_idx, P.agg_coef};
    G.msg_gather_t = WdCsr{P.msgt_ptr, P.msgt_idx, P.msgt_coef};
    G.atom_gather_t = WdCsr{P.aggt_ptr, P.aggt_idx, P.aggt_coef};
    G.bond_feat_gather = WdCsr{nullptr, nullptr, nullptr};
    G.bond_feat_gather_t = WdCsr{nullptr, nullptr, nullptr};
    G.b2revb = P.b2revb;
    G.atom_desc = nullptr; G.desc_dim = 0; G.atom_messages = 0;
    G.f_atoms_x6 = P.fa_x6; G.f_bonds_x6 = P.fb_x6;
    G.n_blocks = c->n_blocks; G.blocks = P.blocks; G.bond_blk_row = P.bond_blk_row; G.f_atoms_blk_x6 = P.fa_blk_x6;
    G.msg_ell_idx = P.msg_ell_idx; G.msg_ell_coef = P.msg_ell_coef;
    G.atom_ell_idx = P.agg_ell_idx; G.atom_ell_coef = P.agg_ell_coef;
    G.atom_codes = c->atoms; G.bond_src_blk = P.bond_src_blk; G.bond_tail = P.bond_tail;
    if (lean) {  // what was not built is not handed out: a path that needs it fails in get_dims
        G.f_atoms = G.f_bonds = nullptr;
        G.f_atoms_x6 = G.f_bonds_x6 = G.f_atoms_blk_x6 = nullptr;
        G.msg_gather = G.msg_gather_t = WdCsr{nullptr, nullptr, nullptr};
        G.atom_gather_t = WdCsr{nullptr, nullptr, nullptr};
        G.msg_ell_idx = nullptr; G.msg_ell_coef = nullptr;
    }
    Gout = G;
    return 0;
}

// several prepared builds in one launch (the stream feed), chunks of WD_MULTI
int graph_build_launch(const GraphBuildP *P, int n, hipStream_t st) {
    for (int j0 = 0; j0 < n; j0 += WD_MULTI) {
        Multi<GraphBuildP> M{};
        M.n = std::min(WD_MULTI, n - j0);
        int t = 0;
        for (int j = 0; j < M.n; ++j) {
            M.p[j] = P[j0 + j];
            M.t0[j] = t;
            t += P[j0 + j].c.n_blocks + 1;
        }
        for (int j = M.n; j <= WD_MULTI; ++j) M.t0[j] = t;
        bool lean = true;
        for (int j = 0; j < M.n; ++j) lean = lean && M.p[j].lean;
        hipLaunchKernelGGL(graph_build_kernel, dim3(t, lean ? 1 : GB_SLICES), dim3(256), 0, st, M);
        WD_CHECK_LAUNCH("graph_build");
    }
    return 0;
}

extern "C" {

// ------------------------------------------------------------------------------------------------
// native streamed batches (feed.hpp)
// ------------------------------------------------------------------------------------------------
static int feed_graph_bound(int32_t kind, int32_t batch, int32_t fa, int32_t fb, size_t *bytes) {
    const FeedBounds f = feed_bounds(kind);
    WdCompact c{};
    c.n_mols = batch;
    c.n_atoms = batch * f.atoms_per_mol + 1;
    c.n_bonds = 2 * batch * f.pairs_per_mol + 1;
    c.n_blocks = batch;
    c.atom_fdim = fa; c.bond_fdim = fb;
    c.nnz_msg = (c.n_bonds - 1) * FEED_MAX_DEG;
    c.nnz_agg = c.n_bonds - 1;
    GraphLayout L;
    WD_TRY(graph_layout(&c, L));
    *bytes = L.total;
    return 0;
}

int wdmpnn_feed_slot_bytes(int32_t kind, int32_t batch, int32_t atom_fdim, int32_t bond_fdim, size_t *host_bytes,
                           size_t *device_bytes) {
    if (kind < 0 || kind > 2 || batch < 1 || !host_bytes || !device_bytes) return fail(WD_ERR_ARG, "feed: bad slot request");
    size_t g = 0;
    WD_TRY(feed_graph_bound(kind, batch, atom_fdim, bond_fdim, &g));
    *host_bytes = align256(feed_host_bytes(kind, batch));
    *device_bytes = *host_bytes + g;
    return 0;
}

int wdmpnn_feed_create(const WdFeedSpec *spec, void **feed) {
    WD_KERNELS_OK();
    if (!spec || !feed) return fail(WD_ERR_ARG, "feed: null argument");
    const WdFeedSpec &S = *spec;
    if (S.kind < 0 || S.kind > 2 || S.batch < 1 || S.n_batches < 0 || S.producers < 1 || S.slots < 2 ||
        S.target_blocks < 1 || (S.flags & ~(WDMPNN_GRAPH_LEAN | WDMPNN_GRAPH_NO_PLANES)) || !S.pinned || !S.device || ((uintptr_t)S.device & 255))
        return fail(WD_ERR_ARG, "feed: bad spec");
    Feed *F = new Feed();
    F->spec = S;
    F->R = S.slots;
    size_t hb = 0, db = 0;
    if (int rc = wdmpnn_feed_slot_bytes(S.kind, S.batch, S.atom_fdim, S.bond_fdim, &hb, &db)) {
        delete F;
        return rc;
    }
    F->host_bytes = hb; F->dev_bytes = db; F->graph_off = hb;
    F->slot.resize((size_t)F->R);
    // the feed stream at the highest priority: a graph build is a short, latency-bound launch (one
    // workgroup per molecule block); dispatched ahead of the queued forward workgroups it finishes while
    // the forward keeps the CUs busy, instead of waiting behind them
    int lo_pri = 0, hi_pri = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri);
    bool ok = hipStreamCreateWithPriority(&F->fs, hipStreamNonBlocking, hi_pri) == hipSuccess;
    for (int s = 0; s < F->R && ok; ++s) {
        Feed::Slot &Q = F->slot[(size_t)s];
        Q.turn = s;
        // (the two events host threads wait for are blocking-sync: a default event's hipEventSynchronize polls,
        // and the feeder, which runs several batches ahead, would hold a CPU busy for the whole stream -- one of
        // a rank's two CPUs when eight ranks share a 16-CPU quota)
        ok = hipEventCreateWithFlags(&Q.copy_done, hipEventDisableTiming | WD_FEED_EVENT_SYNC) == hipSuccess &&
             hipEventCreateWithFlags(&Q.ready, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&Q.released, hipEventDisableTiming | WD_FEED_EVENT_SYNC) == hipSuccess;
    }
    if (!ok) {
        delete F;
        return fail(WD_ERR_ARG, "feed: stream / event creation failed");
    }
    for (int t = 0; t < S.producers; ++t) F->threads.emplace_back(&Feed::producer, F, t);
    F->threads.emplace_back(&Feed::feeder, F);
    *feed = F;
    return 0;
}

int wdmpnn_feed_next(void *feed, void *stream, WdGraph *g, WdFeedBatch *info) {
    Feed *F = (Feed *)feed;
    if (!F || !g) return fail(WD_ERR_ARG, "feed_next: null argument");
    std::unique_lock<std::mutex> lk(F->mu);
    const int64_t i = F->handed;
    if (i >= F->spec.n_batches) return 1;
    Feed::Slot &S = F->slot[(size_t)(i % F->R)];
    F->cv.wait(lk, [&] { return !F->error.empty() || S.built == i; });
    if (!F->error.empty()) return fail(WD_ERR_ARG, "%s", F->error.c_str());
    if (hipStreamWaitEvent((hipStream_t)stream, S.ready, 0) != hipSuccess) return fail(WD_ERR_ARG, "feed_next: wait");
    *g = S.g;
    if (info) {
        *info = WdFeedBatch{};
        info->index = i;
        info->n_mols = S.counts[0]; info->n_atoms = S.counts[1]; info->n_bonds = S.counts[2];
        info->n_blocks = S.counts[3]; info->nnz_msg = S.counts[4];
        info->h2d_bytes = S.total;
    }
    F->handed = i + 1;
    if (WD_FEED_GROUP) F->cv.notify_all();  // (the feeder groups its builds while the consumer holds built batches)
    return 0;
}

int wdmpnn_feed_release(void *feed, void *stream) {
    Feed *F = (Feed *)feed;
    if (!F) return fail(WD_ERR_ARG, "feed_release: null feed");
    std::lock_guard<std::mutex> lk(F->mu);
    for (int64_t b = F->released_upto; b < F->handed; ++b)
        if (hipEventRecord(F->slot[(size_t)(b % F->R)].released, (hipStream_t)stream) != hipSuccess)
            return fail(WD_ERR_ARG, "feed_release: event");
    F->released_upto = F->handed;
    F->cv.notify_all();
    return 0;
}

// the workspace bound of one batch of the feed (the largest batch its generator makes)
static int feed_batch_workspace(const Feed *F, const WdParams *p, const WdConfig *c, size_t *bytes) {
    if (!p || !c || p->hidden <= 0 || c->depth < 2) return fail(WD_ERR_ARG, "feed forward: bad params / depth");
    const FeedBounds f = feed_bounds(F->spec.kind);
    Dims D{};
    D.H = p->hidden; D.Hk = rup(D.H, 64); D.T = c->depth;
    D.R = 2 * F->spec.batch * f.pairs_per_mol + 1; D.Rp = rup(D.R, 128);
    D.Va = F->spec.batch * f.atoms_per_mol + 1; D.Vap = rup(D.Va, 128);
    D.Fa = F->spec.atom_fdim; D.Fak = rup(D.Fa, 32); D.Fb = F->spec.bond_fdim; D.Fbk = rup(D.Fb, 32);
    D.Hd = D.H; D.Hdk = rup(D.Hd, 64); D.Kin = D.Fb; D.Kink = D.Fbk; D.ldx = D.Hk; D.Ko = D.Fak + D.Hk; D.Kd = D.Hk;
    D.x6 = true; D.blocked = true; D.nblk = F->spec.batch;  // (blocks hold whole molecules: <= batch)
    const size_t staged = fwd_layout(D, false).total;
    D.pairs = true;  // (the pair tiles too: whichever layout get_dims picks is covered)
    *bytes = align256(std::max(staged, fwd_layout(D, false).total));
    return 0;
}

int wdmpnn_feed_forward_workspace_bytes(void *feed, const WdParams *p, const WdConfig *c, int32_t k, size_t *bytes) {
    Feed *F = (Feed *)feed;
    if (!F || !bytes || k < 1) return fail(WD_ERR_ARG, "feed_forward_workspace_bytes: bad argument");
    size_t one = 0;
    WD_TRY(feed_batch_workspace(F, p, c, &one));
    *bytes = one * (size_t)k;
    return 0;
}

int wdmpnn_feed_forward(void *feed, int32_t k, const WdParams *p, const WdConfig *c, void *workspace,
                        size_t workspace_bytes, float *out, int64_t out_rows, void *stream, int32_t *got,
                        int64_t *rows, int64_t *edges, int64_t *h2d_bytes) {
    WD_KERNELS_OK();
    Feed *F = (Feed *)feed;
    if (!F || k < 1 || !p || !c || !workspace || !out || !got || !rows || !edges || !h2d_bytes)
        return fail(WD_ERR_ARG, "feed_forward: bad argument");
    if (!p->packed) return fail(WD_ERR_ARG, "feed_forward needs packed parameters (wdmpnn_pack_params)");
    if (c->save_for_backward) return fail(WD_ERR_UNSUPPORTED, "feed_forward is inference only");
    *got = 0; *rows = 0; *edges = 0; *h2d_bytes = 0;
    // at most R batches held unreleased (the feed builds batch i only after batch i - R is released)
    if (k > F->R) k = F->R;
    std::vector<WdGraph> gs;
    std::vector<void *> wsp;
    std::vector<size_t> wsb;
    std::vector<float *> outs;
    size_t used = 0;
    int64_t r = 0, e = 0;
    const int H = p->hidden;
    for (int j = 0; j < k; ++j) {
        WdGraph g{};
        WdFeedBatch info{};
        const int rc = wdmpnn_feed_next(feed, stream, &g, &info);
        if (rc == 1) break;
        if (rc) return rc;
        Dims D;
        WD_TRY(get_dims(&g, p, c, D));
        const size_t need = align256(fwd_layout(D, false).total);
        if (used + need > workspace_bytes) return fail(WD_ERR_WORKSPACE, "feed_forward: workspace too small");
        if (r + info.n_mols > out_rows) return fail(WD_ERR_WORKSPACE, "feed_forward: output too small");
        gs.push_back(g);
        wsp.push_back((char *)workspace + used);
        wsb.push_back(need);
        outs.push_back(out + (size_t)r * H);
        used += need;
        r += info.n_mols;
        e += info.n_bonds - 1;
        *h2d_bytes += (int64_t)info.h2d_bytes;
    }
    if (!gs.empty()) {
        WD_TRY(wdmpnn_forward_many((int32_t)gs.size(), gs.data(), p, c, wsp.data(), wsb.data(), outs.data(), stream));
        WD_TRY(wdmpnn_feed_release(feed, stream));
    }
    *got = (int32_t)gs.size();
    *rows = r;
    *edges = e;
    return 0;
}

int wdmpnn_feed_destroy(void *feed) {
    delete (Feed *)feed;
    return 0;
}

int wdmpnn_index_select_rows_backward(const float *grad, int64_t n_index, int64_t row_len, const int64_t *perm,
                                      const int64_t *ptr, int64_t n_src_rows, float *dsrc, void *stream) {
    WD_KERNELS_OK();
    if (n_index < 0 || row_len < 0 || n_src_rows < 0) return fail(WD_ERR_ARG, "negative size");
    if (n_src_rows == 0 || row_len == 0) return 0;
    if (!dsrc || !ptr || (n_index && (!grad || !perm))) return fail(WD_ERR_ARG, "null pointer");
    const size_t total = (size_t)n_src_rows * row_len;
    hipLaunchKernelGGL(index_select_rows_bwd_kernel, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, grad,
                       row_len, perm, ptr, n_src_rows, dsrc);
    WD_CHECK_LAUNCH("index_select_rows_backward");
    return 0;
}

// the encoder weights' packed copies as adam_kernel outputs (wdmpnn_adam_step_repack): the same
// destinations pack_params writes, element by element
struct RepackTarget {
    const float *param;
    int rows, cols;
    AdamOut out[6];
    int nout;
    uint32_t *amax;  // one word per 32 x 32 tile, or null
};
static AdamOut ao(void *dst, int kind, int ld, std::initializer_list<std::array<int, 3>> segs, int br = 0) {
    AdamOut o{};  // segs: {dst_col0, src_col0, K}
    o.dst = dst; o.kind = kind; o.ld = ld; o.br = br;
    for (const auto &g : segs) { o.dc0[o.nseg] = g[0]; o.sc0[o.nseg] = g[1]; o.K[o.nseg] = g[2]; ++o.nseg; }
    return o;
}

static int adam_launches(const WdAdamTensor *tensors, int n, const WdAdamHyper *h, hipStream_t st,
                         const RepackTarget *rt, int nrt, bool *found) {
    if (n < 0 || !h || (n && !tensors)) return fail(WD_ERR_ARG, "null or negative argument");
    if (h->step < 1) return fail(WD_ERR_ARG, "adam step must be >= 1");
    const double bc1 = 1.0 - std::pow((double)h->beta1, (double)h->step);
    const double bc2 = 1.0 - std::pow((double)h->beta2, (double)h->step);
    for (int s = 0; s < n; s += ADAM_MAX) {
        AdamLaunch A{};
        A.beta1 = h->beta1; A.beta2 = h->beta2; A.eps = h->eps; A.wd = h->weight_decay; A.lr = h->lr;
        A.step_size = (float)(h->lr / bc1); A.bc2_sqrt = (float)std::sqrt(bc2); A.decoupled = h->decoupled;
        int blocks = 0, nout = 0;
        for (int i = s; i < n && i < s + ADAM_MAX; ++i) {
            const WdAdamTensor &T = tensors[i];
            if (T.numel < 0) return fail(WD_ERR_ARG, "negative numel");
            if (T.numel == 0) continue;
            if (!T.param || !T.grad || !T.exp_avg || !T.exp_avg_sq) return fail(WD_ERR_ARG, "null tensor pointer");
            int64_t nb = (T.numel + ADAM_PER_BLOCK - 1) / ADAM_PER_BLOCK;
            for (int r = 0; r < nrt; ++r) {  // a repacked weight: tiles instead of element-wise blocks
                if (!rt[r].param || rt[r].param != T.param) continue;
                if (found[r]) return fail(WD_ERR_ARG, "adam_step_repack: a weight appears twice");
                if ((int64_t)rt[r].rows * rt[r].cols != T.numel)
                    return fail(WD_ERR_SHAPE, "adam_step_repack: weight size %lld, expected %d x %d", (long long)T.numel,
                                rt[r].rows, rt[r].cols);
                found[r] = true;
                AdamTileJob &J = A.tj[A.ntj++];
                J.t = A.n; J.rows = rt[r].rows; J.cols = rt[r].cols; J.tiles_c = (J.cols + ADAM_TILE - 1) / ADAM_TILE;
                J.blk0 = A.tile_blocks; J.amax = rt[r].amax;
                A.tile_blocks += ((J.rows + ADAM_TILE - 1) / ADAM_TILE) * J.tiles_c;
                J.o0 = nout;
                for (int o = 0; o < rt[r].nout; ++o) A.out[nout++] = rt[r].out[o];
                J.o1 = nout;
                nb = 0;
            }
            if (blocks + nb + A.tile_blocks > INT32_MAX / 2) return fail(WD_ERR_SHAPE, "adam launch too large");
            A.t[A.n] = T;
            A.blk0[A.n] = blocks;
            blocks += (int)nb;
            ++A.n;
        }
        if (!A.n) continue;
        A.blk0[A.n] = blocks;
        if (A.ntj) hipLaunchKernelGGL(adam_kernel<true>, dim3(A.tile_blocks + blocks), dim3(256), 0, st, A);
        else hipLaunchKernelGGL(adam_kernel<false>, dim3(blocks), dim3(256), 0, st, A);
        WD_CHECK_LAUNCH("adam");
    }
    return 0;
}

int wdmpnn_adam_step(const WdAdamTensor *tensors, int32_t n, const WdAdamHyper *h, void *stream) {
    WD_KERNELS_OK();
    return adam_launches(tensors, n, h, (hipStream_t)stream, nullptr, 0, nullptr);
}

int wdmpnn_adam_step_repack(const WdAdamTensor *tensors, int32_t n, const WdAdamHyper *h, const WdGraph *g,
                            const WdParams *p, const WdConfig *c, void *packed, size_t packed_bytes, void *stream) {
    WD_KERNELS_OK();
    Dims D;
    WD_TRY(get_dims(g, p, c, D));
    if (D.atom || D.desc) return fail(WD_ERR_UNSUPPORTED, "adam_step_repack: bond messages without descriptors only");
    const PackLayout L = pack_layout(D);
    if (!packed || packed_bytes < L.total) return fail(WD_ERR_WORKSPACE, "adam_step_repack: packed buffer too small");
    char *base = (char *)packed;
    auto F = [&](size_t off) { return (void *)(base + off); };
    const int H = D.H;
    const bool b80 = D.Hk % 80 == 0;
    uint32_t *wh_amax = (uint32_t *)(base + L.amax);
    RepackTarget rt[6] = {};
    // (pack_params' jobs, in its order: plain copy, transposes, plane tiles)
    rt[0] = {p->W_i, H, D.Kin, {}, 0, nullptr};
    rt[0].out[rt[0].nout++] = ao(F(L.Wi), AO_PLAIN, D.Kink, {{0, 0, D.Kin}});
    rt[0].out[rt[0].nout++] = ao(F(L.WiT), AO_TRANSPOSE, D.Hk, {{0, 0, D.Kin}});
    rt[0].out[rt[0].nout++] = ao(F(L.WiX), AO_PLANES, D.Kink, {{0, 0, D.Kin}}, 64);
    rt[1] = {p->b_i, 1, H, {}, 0, nullptr};
    rt[1].out[rt[1].nout++] = ao(F(L.bi), AO_PLAIN, D.Hk, {{0, 0, H}});
    rt[2] = {p->W_h, H, H, {}, 0, wh_amax + 65};
    rt[2].out[rt[2].nout++] = ao(F(L.Wh), AO_PLAIN, D.ldx, {{0, 0, H}});
    rt[2].out[rt[2].nout++] = ao(F(L.WhT), AO_TRANSPOSE, D.Hk, {{0, 0, H}});
    rt[2].out[rt[2].nout++] = ao(F(L.WhX), AO_PLANES, D.ldx, {{0, 0, H}}, 64);
    if (b80) rt[2].out[rt[2].nout++] = ao(F(L.WhX80), AO_PLANES, D.ldx, {{0, 0, H}}, 80);
    rt[3] = {p->b_h, 1, H, {}, 0, nullptr};
    rt[3].out[rt[3].nout++] = ao(F(L.bh), AO_PLAIN, D.Hk, {{0, 0, H}});
    rt[4] = {p->W_o, H, D.Fa + H, {}, 0, nullptr};
    rt[4].out[rt[4].nout++] = ao(F(L.Wo), AO_PLAIN, D.Ko, {{0, 0, D.Fa}, {D.Fak, D.Fa, H}});
    rt[4].out[rt[4].nout++] = ao(F(L.WoT), AO_TRANSPOSE, D.Hk, {{0, D.Fa, H}});
    rt[4].out[rt[4].nout++] = ao(F(L.WoaT), AO_TRANSPOSE, D.Hk, {{0, 0, D.Fa}});
    rt[4].out[rt[4].nout++] = ao(F(L.WoX), AO_PLANES, D.Ko, {{0, 0, D.Fa}, {D.Fak, D.Fa, H}}, 64);
    if (b80) rt[4].out[rt[4].nout++] = ao(F(L.WoX80), AO_PLANES, D.Ko, {{0, 0, D.Fa}, {D.Fak, D.Fa, H}}, 80);
    rt[5] = {p->b_o, 1, H, {}, 0, nullptr};
    rt[5].out[rt[5].nout++] = ao(F(L.bo), AO_PLAIN, D.Hk, {{0, 0, H}});
    bool found[6] = {};
    for (int r = 0; r < 6; ++r) found[r] = rt[r].param == nullptr;  // (bias-free layers: their packed zeros stay)
    hipStream_t st = (hipStream_t)stream;
    WD_TRY(adam_launches(tensors, n, h, st, rt, 6, found));
    for (int r = 0; r < 6; ++r)
        if (!found[r]) return fail(WD_ERR_ARG, "adam_step_repack: encoder weight %d is not among the tensors (its packed "
                                               "copies are stale now: pack before the next forward)", r);
    // W_h's fp16-pair tiles from the fresh plain copy, scaled by the max over adam_kernel's tile words
    const int nw = ((H + ADAM_TILE - 1) / ADAM_TILE) * ((H + ADAM_TILE - 1) / ADAM_TILE);
    hipLaunchKernelGGL(split_h2_kernel, dim3(ew_blocks((size_t)D.Hk * D.Hk / 8)), dim3(256), 0, st, (const float *)F(L.Wh),
                       D.ldx, D.Hk, D.Hk, fused_bn(D.Hk), (uint8_t *)F(L.WhH), wh_amax + 65, nw, wh_amax + 64);
    WD_CHECK_LAUNCH("adam_step_repack h2");
    return 0;
}

int wdmpnn_head_mse(const WdHead *h, void *stream) {
    WD_KERNELS_OK();
    if (!h) return fail(WD_ERR_ARG, "null head");
    if (h->B < 0 || h->F <= 0 || h->Hf <= 0 || h->T <= 0 || h->ld_x < h->F || h->ld_table < 2 * h->T)
        return fail(WD_ERR_SHAPE, "head: bad sizes");
    if (h->F > HEAD_MAX_F || h->Hf > HEAD_MAX_H || h->T > HEAD_MAX_T)
        return fail(WD_ERR_UNSUPPORTED, "head: F, Hf <= 4096 and T <= 64");
    if (h->act < 0 || h->act > WD_ACT_ELU || h->act == WD_ACT_PRELU) return fail(WD_ERR_UNSUPPORTED, "head activation");
    if (h->loss_kind != 0 && h->loss_kind != 1) return fail(WD_ERR_UNSUPPORTED, "head loss kind %d", h->loss_kind);
    if (!h->W1 || !h->W2 || !h->a || !h->dh || !h->dout || !h->lossrow || !h->dW1 || !h->dW2 || !h->loss ||
        (h->B && (!h->x || !h->table || !h->dx)))
        return fail(WD_ERR_ARG, "head: null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (h->B > 0) {
        hipLaunchKernelGGL(head_h_kernel, dim3(head_tiles(h->B, h->Hf, HEAD_H_TS)), dim3(256), 0, st, *h);
        WD_CHECK_LAUNCH("head_h");
        hipLaunchKernelGGL(head_rows_kernel, dim3((h->B + 3) / 4), dim3(256), 0, st, *h);
        WD_CHECK_LAUNCH("head_rows");
    }
    const long long rest = h->Hf + (long long)h->T * h->Hf + h->T + 1;
    const long long blocks = head_tiles(h->B, h->F, HEAD_H_TS) + head_tiles(h->Hf, h->F, HEAD_G_TS) + (rest + 255) / 256;
    hipLaunchKernelGGL(head_grads_kernel, dim3((unsigned)blocks), dim3(256), 0, st, *h);
    WD_CHECK_LAUNCH("head_grads");
    return 0;
}

int wdmpnn_scale(float *const *p, const int64_t *n, int32_t k, const float *s, void *stream) {
    WD_KERNELS_OK();
    if (k < 0 || k > 8 || !s || (k && (!p || !n))) return fail(WD_ERR_ARG, "scale: bad arguments");
    ScaleJobs J{};
    long long most = 0;
    for (int i = 0; i < k; ++i) {
        if (n[i] < 0 || (n[i] && !p[i])) return fail(WD_ERR_ARG, "scale: bad buffer");
        J.p[i] = p[i];
        J.n[i] = n[i];
        most = std::max<long long>(most, n[i]);
    }
    J.k = k;
    J.s = s;
    if (!most) return 0;
    hipLaunchKernelGGL(scale_kernel, dim3((unsigned)std::min<long long>((most + 255) / 256, 1024)), dim3(256), 0,
                       (hipStream_t)stream, J);
    WD_CHECK_LAUNCH("scale");
    return 0;
}

}  // extern "C"
