/*
 * wdmpnn.h — C-ABI of the MI355X-native wD-MPNN encoder (libwdmpnn.so, gfx950).
 *
 * Drop-in boundary.  The reference (ayildiri/polymer-chemprop, pure Python/PyTorch) has no FFI for
 * this path: the hot path is the nn.Module call chain
 *
 *     MoleculeModel.forward   chemprop/models/model.py:152-194
 *       -> MPN.forward        chemprop/models/mpn.py:210-289
 *         -> MPNEncoder.forward  chemprop/models/mpn.py:66-173        (replaced by wdmpnn_forward)
 *              index_select_ND   chemprop/nn_utils.py:50-67           (replaced by wdmpnn_index_select_rows
 *                                                                      and by the CSR gathers inside forward)
 *              BatchMolGraph     chemprop/features/featurization.py:742-875 (device layout = WdGraph)
 *         autograd backward of the above (train.py:79 loss.backward)  (replaced by wdmpnn_backward)
 *
 * The Python host package (polymer-chemprop_amd/chemprop_amd) keeps the reference's Python API and
 * binds these entry points with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every pointer in WdGraph / WdParams / WdGrads is a DEVICE pointer owned by the caller (the
 *    PyTorch caching allocator).  The library never allocates device memory.
 *  - Row 0 of every atom / bond array is the reference's zero pad row (featurization.py:767-781);
 *    n_atoms / n_bonds INCLUDE it, exactly like BatchMolGraph.n_atoms / n_bonds.
 *  - fp32 storage and fp32-accurate arithmetic, int32 indices.  The GEMMs run on MFMA with fp32
 *    accumulation over exact splits of the fp32 operands: fp16 hi / lo pairs with a power-of-two scale
 *    (three products per fp32 product, the message layers and the backward's W_h GEMMs) or three bf16
 *    planes (six products: W_o, W_i and the unblocked path).  Error against fp64 stays that of an fp32
 *    GEMM; WdConfig.gemm_variant 9 selects plain f32-in MFMA on the unblocked path.
 *  - Padding: f_atoms / f_bonds / atom_desc rows are allocated up to a multiple of 128 and their row
 *    stride covers the feature width rounded up to 32; padding is zero.  (The host packer,
 *    BatchMolGraph.device_graph, lays them out this way.)  Weights are the unpadded nn.Linear
 *    tensors; wdmpnn_pack_params builds the padded GEMM operands from them.
 *  - Return 0 on success, a negative WD_ERR_* code on argument errors, or -(hipError_t) on a HIP
 *    launch error; wdmpnn_last_error() then holds a message (thread-local).
 *  - All work is enqueued on `stream` (a hipStream_t; NULL = default stream); no host sync, no
 *    allocation, re-entrant per stream, no global mutable state besides the thread-local error.
 */
#ifndef WDMPNN_H
#define WDMPNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WDMPNN_ABI_VERSION 11
#define WDMPNN_ELL_WIDTH 8

enum WdActivation {     /* nn_utils.py:70-99 get_activation_function */
    WD_ACT_RELU = 0, WD_ACT_LEAKY_RELU = 1, WD_ACT_PRELU = 2, WD_ACT_TANH = 3,
    WD_ACT_SELU = 4, WD_ACT_ELU = 5, WD_ACT_IDENTITY = 6
};

enum WdAggregation {    /* mpn.py:158-163 */
    WD_AGG_MEAN = 0, WD_AGG_SUM = 1, WD_AGG_NORM = 2
};

enum WdError {
    WD_OK = 0, WD_ERR_ARG = -1000, WD_ERR_SHAPE = -1001, WD_ERR_WORKSPACE = -1002,
    WD_ERR_UNSUPPORTED = -1003
};

/* One row-gather list: row r of the gathered operand = sum_{e=ptr[r]}^{ptr[r+1]-1} coef[e] * src[idx[e]].
 * idx and coef must be readable (any value) for 8 entries past ptr[rows]: the gather kernels fetch the
 * first eight entries of a row unconditionally and discard the ones past its end. */
typedef struct WdCsr {
    const int32_t *ptr;   /* [rows + 1] */
    const int32_t *idx;   /* [ptr[rows]] source row ids */
    const float   *coef;  /* [ptr[rows]] coefficients, NULL = all ones */
} WdCsr;

/* Categorical codes of one atom / one bond pair (see "Compact graphs" below). */
typedef struct WdAtomCode {
    uint8_t col[8];         /* columns of f_atoms holding 1.0, ascending; 0xFF = unused slot     */
    float last;             /* f_atoms[atom_fdim - 1] (mass * 0.01)                              */
    float w;                /* w_atoms                                                           */
} WdAtomCode;
typedef struct WdBondPair {
    uint16_t a1, a2;        /* molecule-local atom ids: b1 = a1 -> a2, b2 = a2 -> a1             */
    uint16_t tail;          /* bond feature columns as bits (bit k = column atom_fdim + k)       */
    uint16_t reserved;
    float w12, w21;         /* w_bonds[b1], w_bonds[b2]                                          */
} WdBondPair;
/*
 * Device-resident packed BatchMolGraph (featurization.py:757-813) plus the gather lists derived
 * from it by the host packer (chemprop_amd/featurization.py, BatchMolGraph.device_graph()).
 */
typedef struct WdGraph {
    int32_t n_atoms;        /* V+1 (incl. pad row 0)                               */
    int32_t n_bonds;        /* E+1 (incl. pad row 0)                               */
    int32_t n_mols;         /* B = len(a_scope)                                    */
    int32_t atom_fdim;      /* Fa: columns of f_atoms actually used                */
    int32_t bond_fdim;      /* Fb: columns of f_bonds actually used (14 in atom-message mode) */
    int32_t ld_atoms;       /* row stride of f_atoms (floats)                      */
    int32_t ld_bonds;       /* row stride of f_bonds (floats)                      */
    int32_t bond_col0;      /* first used column of f_bonds (Fb_full - 14 in atom-message mode) */
    const float *f_atoms;   /* [n_atoms, ld_atoms]                                 */
    const float *f_bonds;   /* [n_bonds, ld_bonds]                                 */
    const float *w_atoms;   /* [n_atoms]  (featurization.py:778, pad weight 0)     */
    const int32_t *mol_start;  /* [B] a_scope[i][0]                                */
    const int32_t *mol_size;   /* [B] a_scope[i][1]                                */
    const float *degree_of_polym; /* [B]                                           */
    /* bond-message mode (mpn.py:110-120): X_b = sum_{j in in(b2a[b])} w_j M_j - M_{b2revb[b]} */
    WdCsr msg_gather;       /* rows = n_bonds (bond mode) or n_atoms (atom mode, a2a + pad-slot term) */
    WdCsr bond_feat_gather; /* atom mode only: rows = n_atoms, sum of f_bonds tails over a2b (mpn.py:106) */
    WdCsr atom_gather;      /* rows = n_atoms: final aggregate of mpn.py:126-131 (coef = edge weight) */
    const int32_t *b2revb;  /* [n_bonds] (undirected: mpn.py:101-102)                */
    /* transposed lists for the backward pass (gradient of the gathers) */
    WdCsr msg_gather_t;     /* rows = message rows: dM_j += sum coef * dX_row          */
    WdCsr bond_feat_gather_t; /* unused by the gradients (inputs need no grad); may be zero */
    WdCsr atom_gather_t;    /* rows = message rows: dM_j += coef * dA_atom              */
    /* atom_descriptors == 'descriptor' (mpn.py:136-143) */
    const float *atom_desc; /* [n_atoms, round32(desc_dim)] (row 0 zero pad) or NULL */
    int32_t desc_dim;
    int32_t atom_messages;  /* 1 = atom-message mode (mpn.py:47-53, 93-94, 104-108) */
    /* Optional bf16x3 plane tiles of f_atoms / f_bonds (wdmpnn_split_planes over all padded rows and
     * ld_atoms / ld_bonds columns), made once per packed graph: the exact split-plane form the bf16x6
     * GEMMs read.  NULL: those GEMMs split the fp32 features in the kernel instead. */
    const void *f_atoms_x6;
    const void *f_bonds_x6;
    /* Optional molecule blocks for the fused inference forward: consecutive molecules
     * grouped into blocks of <= 128 bond rows, <= 64 atom rows and <= 64 molecules, so that every gather
     * stays inside one block.  blocks[8 * k .. 8 * k + 5] = {bond_start, bond_count, atom_start, atom_count, mol_lo,
     * mol_hi} (natural row ids, half-open molecule range).  bond_blk_row[r] (r < rows of f_bonds) =
     * 128 * block + (r - bond_start) or -1; f_atoms_blk_x6 = plane tiles of f_atoms in the blocked atom
     * layout (row 64 * block + (a - atom_start), zero rows elsewhere).  n_blocks = 0: unavailable. */
    int32_t n_blocks;
    const int32_t *blocks;
    const int32_t *bond_blk_row;
    const void *f_atoms_blk_x6;
    /* Required with blocks: the first WDMPNN_ELL_WIDTH (W = 8) entries of every msg_gather / atom_gather
     * row in block-local ELL form, so that the fused kernels prefetch a row's list with independent
     * loads during the GEMM instead of a ptr -> idx chain after it.  *_ell_idx[W r + k] = idx - the
     * first row of the gathered kind in the row's block (bond_start for bond rows; atom_start in
     * atom-message mode, whose gathers read atom rows), uint8 < 128, *_ell_coef[W r + k] = coef; unused
     * slots coef 0 and a valid index; bit 7 of slot W - 1 set when the row has more than W entries (the
     * rest are read from the CSR lists).  Atom-message mode: msg_ell lists only the real a2a entries (the
     * pad slots' atom 0 is dropped; the fused path runs bias-free models only, whose pad messages are 0),
     * and the CSR rest of a longer row skips entries outside the block. */
    const uint8_t *msg_ell_idx;
    const float *msg_ell_coef;
    const uint8_t *atom_ell_idx;
    const float *atom_ell_coef;
    /* Optional categorical codes (compact graphs, wdmpnn_build_graph; NULL otherwise).  With blocks, the
     * fused forward then replaces the W_i GEMM and the f_atoms half of the W_o GEMM by sums of weight
     * columns (one-hot rows: f W^T = sum of the columns holding 1.0 + last * the last column):
     * atom_codes [n_atoms] natural rows; bond_src_blk [rows of f_bonds] = the block-local index of the
     * bond's source atom (b2a); bond_tail [rows of f_bonds] = its bond columns as bits. */
    const WdAtomCode *atom_codes;
    const uint8_t *bond_src_blk;
    const uint16_t *bond_tail;
    /* Optional, atom-message mode (ABI 8): per atom row the sum of its in-bonds' feature rows
     * (bond_feat_gather applied to f_bonds, mpn.py:105-106 summed over the slots: a function of the graph
     * alone) as bf16x3 plane tiles [rows of f_atoms][ld_bonds], made with the graph's other planes.  NULL:
     * the fused forward gathers it in one extra launch. */
    const void *atom_feat_sum_x6;
    /* Optional (ABI 9): the largest bond / atom row counts of any block (0 = unknown).  When every block
     * holds <= 32 of each (QM9-sized molecules) the fused inference forward runs as ONE launch, a
     * workgroup carrying its block from the input layer to the readout (small_fwd.hpp). */
    int32_t blk_max_bonds;
    int32_t blk_max_atoms;
} WdGraph;

/* nn.Module parameters of MPNEncoder (mpn.py:17-64); all device pointers, row-major like nn.Linear. */
typedef struct WdParams {
    int32_t hidden;         /* H = args.hidden_size                                */
    const float *W_i;       /* [H, Kin], Kin = bond_fdim (bond mode) or atom_fdim */
    const float *b_i;       /* [H] or NULL (args.bias)                             */
    const float *W_h;       /* [H, H] (bond mode) or [H, H + bond_fdim] (atom mode) */
    const float *b_h;       /* [H] or NULL                                         */
    const float *W_o;       /* [H, atom_fdim + H]                                  */
    const float *b_o;       /* [H] (always present, mpn.py:58)                     */
    const float *W_d;       /* [H+d, H+d] atom_descriptors_layer or NULL          */
    const float *b_d;       /* [H+d] or NULL                                       */
    const float *prelu;     /* [1] PReLU slope (device) when activation == PReLU   */
    const float *zero_vec;  /* [H] cached_zero_vector (mpn.py:44, 148-149)         */
    const void  *packed;    /* optional: output of wdmpnn_pack_params for these weights; NULL =
                               wdmpnn_forward packs into its own workspace (one extra launch)     */
    size_t packed_bytes;
} WdParams;

typedef struct WdConfig {
    int32_t depth;          /* args.depth (>= 1)                                   */
    int32_t undirected;     /* args.undirected                                     */
    int32_t activation;     /* WdActivation                                        */
    int32_t aggregation;    /* WdAggregation                                       */
    float   aggregation_norm;
    float   dropout;        /* args.dropout; 0 at eval                             */
    uint64_t seed;          /* dropout RNG stream (counter based, re-derivable in backward) */
    int32_t save_for_backward; /* 1: keep pre-activations + every message layer in the workspace */
    int32_t prof_slot;      /* first event pair used when prof_pool != NULL                      */
    void   *prof_pool;      /* optional WdEventPool: one event pair (pair prof_slot) is recorded around
                               the depth - 1 message-passing launches (the dominant kernel) of this
                               forward: before the first, after the last                          */
    int32_t gemm_variant;   /* 0 (default): fp32-accurate split GEMMs with the molecule-blocked
                               fused inference forward when WdGraph.blocks allow it: its message layers and
                               W_o read fp16 pair tiles their producers wrote (bond messages, hidden rounded
                               to 64 a multiple of 80), QM9-sized blocks take the one-launch forward;
                               9: f32-MFMA GEMMs on the unblocked path (precision A/B); 11: the fused
                               four-launch forward also for QM9-sized blocks (no one-launch forward);
                               12: as 11, the message layers staging M_{t-1} from fp32 Z_t rows through
                               registers (the round-5 default); 13: as 11, on pair tiles.            */
} WdConfig;

/* Gradients (device, caller-zeroed NOT required: every pointer is fully overwritten). NULL = skip. */
typedef struct WdGrads {
    float *W_i, *b_i, *W_h, *b_h, *W_o, *b_o, *W_d, *b_d, *prelu;
} WdGrads;

int wdmpnn_abi_version(void);
const char *wdmpnn_last_error(void);
/* Load-time kernel check (ABI 11): 0 when the library's gfx950 code object holds every kernel its host
 * code launches (a mismatched build would otherwise abort the process inside a HIP launch), else
 * WD_ERR_UNSUPPORTED with the missing kernel in wdmpnn_last_error().  Reads only the library file (no HIP
 * call, runs without a GPU); every compute entry point runs it once per process and fails the same way.
 * The counts (either pointer may be NULL): kernels the host registers, kernel descriptors in the code
 * object. */
int wdmpnn_self_check(int32_t *n_host_kernels, int32_t *n_device_kernels);

/* Padded / transposed copies of the weights for the GEMMs; depends only on the parameter values and
 * the encoder dimensions, so callers cache it per parameter version (chemprop_amd does). */
int wdmpnn_packed_params_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes);
int wdmpnn_pack_params(const WdGraph *g, const WdParams *p, const WdConfig *c, void *packed, size_t bytes,
                       void *stream);

/* Bytes of forward workspace (intermediates kept for backward when save_for_backward). */
int wdmpnn_workspace_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes);
/* Bytes of scratch for wdmpnn_backward. */
int wdmpnn_backward_workspace_bytes(const WdGraph *g, const WdParams *p, const WdConfig *c, size_t *bytes);

/* MPNEncoder.forward (mpn.py:66-173): out [n_mols, H (+desc_dim)]. */
int wdmpnn_forward(const WdGraph *g, const WdParams *p, const WdConfig *c,
                   void *workspace, size_t workspace_bytes, float *out, void *stream);

/* Several independent batches through the fused inference forward in one set of launches: the embed,
 * the depth - 1 message-passing layers and W_o + readout each run ONCE for up to 8 batches (their tiles
 * concatenated in one grid), instead of once per batch.  Replaces a loop of MPNEncoder.forward calls
 * over batches (the caller of chemprop/train/predict.py:30-40 issues one forward per batch) for batches
 * that are ready together; batch j's output equals wdmpnn_forward(graphs[j], ...) bitwise.
 * graphs[j]: each a molecule-blocked graph (WdGraph.blocks; compact-code or host-built), same feature
 * sizes; p->packed must hold the packed parameters (wdmpnn_pack_params); c->save_for_backward = 0;
 * workspaces[j] of wdmpnn_workspace_bytes(graphs[j], ...) bytes; outs[j] [n_mols_j, H].  Any n >= 0
 * (chunks of 8 per launch set). */
int wdmpnn_forward_many(int32_t n, const WdGraph *graphs, const WdParams *p, const WdConfig *c,
                        void *const *workspaces, const size_t *workspace_bytes, float *const *outs, void *stream);

/* Gradient of MPNEncoder.forward w.r.t. its parameters, given dout [n_mols, H (+desc_dim)] and the
 * workspace of a forward run with save_for_backward = 1 and identical g/p/c. */
int wdmpnn_backward(const WdGraph *g, const WdParams *p, const WdConfig *c,
                    const void *workspace, size_t workspace_bytes, const float *dout,
                    void *scratch, size_t scratch_bytes, const WdGrads *grads, void *stream);

/* Introspection of a save_for_backward forward's workspace (tests, debugging): byte offsets of the
 * saved fp32 pre-activations.  Z_t (t = 0 .. depth-1) = the input of the activation of message layer t
 * (t = 0: W_i, mpn.py:96-97; t >= 1: mpn.py:123), [rows][ld] in natural row order; zo = the W_o
 * pre-activation (mpn.py:133), [atom_rows][ld].  Padding rows / columns hold 0. */
#define WDMPNN_MAX_SAVED_DEPTH 32
typedef struct WdSaved {
    int32_t depth, rows, atom_rows, ld;
    size_t z[WDMPNN_MAX_SAVED_DEPTH];
    size_t zo;
} WdSaved;
int wdmpnn_saved_layout(const WdGraph *g, const WdParams *p, const WdConfig *c, WdSaved *out);

/* Measurement hook (bench.py): a pool of hipEvent pairs recorded by wdmpnn_forward around its
 * dominant launches (see WdConfig.prof_pool).  elapsed_ms synchronises on the events it reads. */
int wdmpnn_event_pool_create(int32_t n_pairs, void **pool);
int wdmpnn_event_pool_destroy(void *pool);
int wdmpnn_event_pool_elapsed_ms(void *pool, int32_t first, int32_t count, float *total_ms);

/* bf16x3 plane tiles of the first kp columns of an fp32 [rows, ld] matrix (rows % 64 == 0,
 * kp % 32 == 0, ld >= kp, ld % 4 == 0): the layout of WdGraph.f_atoms_x6 / f_bonds_x6.  The planes hold
 * every fp32 value exactly (x = h + m + l).  plane_bytes = rows * kp * 6. */
int wdmpnn_plane_bytes(int32_t rows, int32_t kp, size_t *bytes);
int wdmpnn_split_planes(const float *src, int32_t ld, int32_t rows, int32_t kp, void *dst, size_t dst_bytes,
                        void *stream);
/* The same with a row map: source row r goes to plane-tile row row_map[r] (skipped when < 0) of a
 * [out_rows, kp] plane-tile matrix whose other rows are zero-filled. */
int wdmpnn_split_planes_rows(const float *src, int32_t ld, int32_t rows, int32_t kp, const int32_t *row_map,
                             int32_t out_rows, void *dst, size_t dst_bytes, void *stream);

/* Device-side bond featurisation, replacing the host-side construction of every
 * f_bonds row as f_atoms[a1] + f_bond (featurization.py:467-468, 545-546, 616-617) and its H2D copy:
 * f_bonds[r][0 .. atom_fdim) = f_atoms[b2a[r]], f_bonds[r][atom_fdim .. + tail_dim) = bond_tail[r],
 * the rest of the ld_bonds columns 0, for r < rows.  b2a entries must index f_atoms rows
 * (< atom_rows); an out-of-range entry fills its row's atom part with NaN. */
int wdmpnn_build_bond_features(const float *f_atoms, int32_t ld_atoms, int32_t atom_fdim, int32_t atom_rows,
                               const int32_t *b2a, const float *bond_tail, int32_t ld_tail, int32_t tail_dim,
                               int32_t rows, float *f_bonds, int32_t ld_bonds, void *stream);

/* ------------------------------------------------------------------------------------------------
 * Compact graphs: categorical codes on the wire, the whole WdGraph built on the device
 * (SURVEY §8(f) row 2).
 *
 * The reference featurises every atom as six one-hot blocks + an aromatic bit + mass * 0.01
 * (featurization.py:190-211, 133 columns) and every bond as 14 binary columns (featurization.py:229-250);
 * each directed bond row is its source atom's row followed by the bond's (featurization.py:467-468,
 * 545-546, 616-617), and MolGraph appends bonds in pairs b1 = a1 -> a2, b2 = a2 -> a1 = b2revb[b1]
 * (featurization.py:469-480, 621-630), a2b[a] listing the bonds INTO a in creation order.  A batch in
 * that form travels as
 *   WdAtomCode [n_atoms]  the columns holding 1.0 (ascending, 0xFF = none) + the last column's value
 *                         (mass * 0.01) + the atom weight (w_atoms, featurization.py:507);
 *   WdBondPair [pairs]    molecule-local endpoints a1, a2, the 14 bond columns as a bit mask (bit k =
 *                         column atom_fdim + k) and the two directed weights (w_bonds, :628);
 *   mols [n_mols][4]      {atom_start, n_atoms, bond_start, n_bonds} (natural ids, pad row 0 included
 *                         in the numbering like BatchMolGraph.a_scope / b_scope) + xn [n_mols];
 *   blocks [n_blocks][8]  the molecule blocks of the fused forward (WdGraph.blocks) + block_nnz
 *                         [n_blocks][2] = {first msg_gather entry, first atom_gather entry} of the block;
 * about 14 bytes per directed edge, against ~450 for the fp32 rows + gather lists.  wdmpnn_build_graph
 * expands it on the device into every WdGraph array (fp32 feature rows, plane tiles, gather lists and
 * their transposes, ELL rows, block maps) with the same values and entry order as the host packer
 * (chemprop_amd.featurization.BatchMolGraph.device_graph): one launch.  Requires every molecule to fit
 * one block (<= 128 directed bonds, <= 64 atoms); atom_fdim <= 255 with the code's columns < atom_fdim - 1.
 * ------------------------------------------------------------------------------------------------ */
typedef struct WdCompact {
    int32_t n_mols, n_atoms, n_bonds, n_blocks;   /* n_atoms / n_bonds include the pad row        */
    int32_t atom_fdim, bond_fdim;                 /* 133 / 147 by default (bond_fdim - atom_fdim <= 16) */
    int32_t nnz_msg, nnz_agg;                     /* total entries of msg_gather / atom_gather    */
    const int32_t *mols;                          /* [n_mols][4]                                  */
    const float *xn;                              /* [n_mols] degree_of_polym                     */
    const WdAtomCode *atoms;                      /* [n_atoms], row 0 = pad (no columns, 0, 0)    */
    const WdBondPair *pairs;                      /* [(n_bonds - 1) / 2]                          */
    const int32_t *blocks;                        /* [n_blocks][8]                                */
    const int32_t *block_nnz;                     /* [n_blocks][2]                                */
} WdCompact;

/* Device bytes of the graph wdmpnn_build_graph writes (one buffer, caller-allocated). */
int wdmpnn_graph_bytes(const WdCompact *c, size_t *bytes);
/* Build the WdGraph of a compact batch into `buffer` (device, >= wdmpnn_graph_bytes, 256-byte aligned)
 * on `stream`; *g receives the struct (bond-message mode, blocks set, no descriptors) whose pointers
 * point into `buffer`.  All arrays of c are device pointers. */
int wdmpnn_build_graph(const WdCompact *c, void *buffer, size_t bytes, WdGraph *g, void *stream);
/* The same with flags.  WDMPNN_GRAPH_LEAN: skip the dense feature rows, their plane tiles, the bond
 * message gathers and the transposed gathers (most of the bytes written for a polymer batch); the graph
 * then serves only the fused inference forward (categorical codes) -- anything else returns
 * WD_ERR_UNSUPPORTED. */
#define WDMPNN_GRAPH_LEAN 1
/* WDMPNN_GRAPH_NO_PLANES: skip only the bf16 plane tiles of the feature rows (f_atoms_x6, f_bonds_x6,
 * f_atoms_blk_x6 stay NULL).  The fused forward and backward of a categorical-code graph never read them
 * (training streams); unblocked paths fall back to their register-split GEMMs. */
#define WDMPNN_GRAPH_NO_PLANES 2
int wdmpnn_build_graph_ex(const WdCompact *c, void *buffer, size_t bytes, WdGraph *g, int32_t flags, void *stream);

/* index_select_ND (nn_utils.py:50-67): out[i, :] = src[index[i], :], row_len floats per row.
 * Indices are int64 like the reference's LongTensor; out-of-range indices are an error checked by
 * the caller (the kernel clamps nothing and reads src[index]). */
int wdmpnn_index_select_rows(const float *src, int64_t n_src_rows, int64_t row_len,
                             const int64_t *index, int64_t n_index, float *out, void *stream);
/* Its gradient (the backward of nn_utils.py:64's index_select under autograd): dsrc[j, :] = sum of
 * grad[p, :] over the positions p with index[p] == j, in increasing p (deterministic, no atomics).
 * perm [n_index] = the positions sorted stably by index value, ptr [n_src_rows + 1] = the CSR bounds of
 * each source row in perm.  Every dsrc row is written (0 for rows never selected). */
int wdmpnn_index_select_rows_backward(const float *grad, int64_t n_index, int64_t row_len, const int64_t *perm,
                                      const int64_t *ptr, int64_t n_src_rows, float *dsrc, void *stream);

/* One Adam / AdamW optimizer step (torch.optim.Adam / AdamW semantics without amsgrad: the optimizer
 * step of train/train.py:84, built by utils.py:295-310) over n tensors in one launch per 16 tensors.
 * Replaces torch's multi-tensor / fused Adam kernels; per element: g += wd p (AdamW: p -= lr wd p),
 * m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, p -= lr / (1 - b1^step) * m / (sqrt(v) /
 * sqrt(1 - b2^step) + eps).  step is the 1-based step count after this update.  Every pointer is a
 * device pointer to contiguous fp32 data; tensors with numel 0 are skipped. */
typedef struct WdAdamTensor {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t numel;
} WdAdamTensor;
typedef struct WdAdamHyper {
    float lr, beta1, beta2, eps, weight_decay;
    int32_t step;         /* >= 1 */
    int32_t decoupled;    /* 1 = AdamW */
} WdAdamHyper;
int wdmpnn_adam_step(const WdAdamTensor *tensors, int32_t n, const WdAdamHyper *h, void *stream);
/* The same step, also rewriting the encoder's packed weights (wdmpnn_pack_params layout for g, p, c) from
 * the updated values: the copies the next training forward and backward read (padded plain, transposed,
 * bf16x3 plane tiles, W_h's fp16-pair tiles and scale) come out of the optimizer's own pass instead of a
 * pack before every forward (train.py:84 then mpn.py:66's next call).  tensors must hold p's W_i, b_i,
 * W_h, b_h, W_o and b_o (matched by param pointer, with their full sizes) and `packed` must hold a pack of
 * their previous values (its zero padding is kept); bond messages without descriptors only
 * (WD_ERR_UNSUPPORTED otherwise: pack after the plain step).  Afterwards `packed` equals a fresh
 * wdmpnn_pack_params of the updated weights bytewise except W_h's partial scale words (the per-workgroup
 * maxima before word 64, and the per-tile words after it, are the optimizer's, not pack_kernel's); the
 * folded word 64, the one every consumer reads, is equal. */
int wdmpnn_adam_step_repack(const WdAdamTensor *tensors, int32_t n, const WdAdamHyper *h, const WdGraph *g,
                            const WdParams *p, const WdConfig *c, void *packed, size_t packed_bytes, void *stream);

/* The training step's FFN head + masked MSE loss and their gradients in two launches (model.py:57-121
 * with ffn_num_layers = 2 and no dropout, train.py:55-74 with MSELoss): replaces the ~25 small torch ops
 * (and their host time) of ffn(emb), loss_func(preds, targets) * weights, .sum() / mask.sum() and their
 * autograd backward.  Row-major fp32 device arrays; w = target weight * data weight * mask per entry. */
typedef struct WdHead {
    const float *x; int32_t ld_x;          /* encoder output [B][ld_x], first F columns used        */
    int32_t B, F, Hf, T;                   /* rows, input width, hidden width, outputs (tasks)      */
    const float *W1, *b1, *W2, *b2;        /* nn.Linear(F, Hf), nn.Linear(Hf, T) (biases may be NULL) */
    const float *table; int32_t ld_table;  /* [B][ld_table]: targets [T], then weights w [T]        */
    float inv_n;                           /* 1 / mask.sum()                                        */
    int32_t act;                           /* WdActivation of the FFN (not PReLU)                   */
    float *a, *dh, *dout, *lossrow;        /* scratch [B][Hf], [B][Hf], [B][T], [B]                 */
    float *dx;                             /* [B][ld_x]: d loss / d x                               */
    float *dW1, *db1, *dW2, *db2;          /* parameter gradients (db1 / db2 NULL = skip)           */
    float *loss;                           /* [1]                                                   */
    int32_t loss_kind;                     /* 0: MSELoss (regression), 1: BCEWithLogitsLoss         */
                                           /* (classification: the FFN's logits, train.py:55-74 with */
                                           /* utils.py get_loss_func; sigmoid only at eval)           */
} WdHead;
int wdmpnn_head_mse(const WdHead *h, void *stream);
/* p_i[0 .. n_i) *= *s (device scalar) for k <= 8 buffers: the head's gradients times the loss's
 * incoming gradient in one launch. */
int wdmpnn_scale(float *const *p, const int64_t *n, int32_t k, const float *s, void *stream);

/* ------------------------------------------------------------------------------------------------
 * Native streamed batches (BASELINE.json configs[4]: millions of synthetic polymer graphs per rank,
 * never materialised).  Replaces chemprop's DataLoader + construct_molecule_batch + BatchMolGraph
 * (data.py:594-607, featurization.py:757-813) for the synthetic stream, and the per-batch
 * MPNEncoder.forward host work (mpn.py:77-90): generator threads stage compact batches into pinned
 * slots, a feed thread uploads them and builds each device graph (wdmpnn_build_graph_ex) on its own
 * stream, the caller's stream only waits on each graph's ready event.  Batch i is generated from
 * seed + i (mix the rank into the seed for disjoint shards) and handed out in order.
 * ------------------------------------------------------------------------------------------------ */
typedef struct WdFeedSpec {
    int32_t kind;           /* synthetic generator: 0 polymer, 1 QM9-like, 2 ZINC-like */
    int32_t batch;          /* graphs per batch */
    int64_t n_batches;
    uint64_t seed;          /* batch i: seed + i */
    int32_t producers;      /* generator threads (>= 1) */
    int32_t slots;          /* batches in flight: host and device slots (>= 2) */
    int32_t target_blocks;  /* molecule-block plan target (>= 1) */
    int32_t flags;          /* WDMPNN_GRAPH_LEAN: inference-only device graphs; WDMPNN_GRAPH_NO_PLANES */
    int32_t atom_fdim, bond_fdim;
    void *pinned;           /* caller-owned pinned host memory: slots x host slot bytes */
    void *device;           /* caller-owned device memory: slots x device slot bytes, 256-byte aligned */
} WdFeedSpec;
typedef struct WdFeedBatch {
    int64_t index;
    int32_t n_mols, n_atoms, n_bonds, n_blocks, nnz_msg, reserved;
    size_t h2d_bytes;       /* the staged image uploaded for this batch */
} WdFeedBatch;
int wdmpnn_feed_slot_bytes(int32_t kind, int32_t batch, int32_t atom_fdim, int32_t bond_fdim, size_t *host_bytes,
                           size_t *device_bytes);
int wdmpnn_feed_create(const WdFeedSpec *spec, void **feed);
/* The next batch: blocks until its graph has been enqueued, makes `stream` wait for it on the GPU and
 * returns its WdGraph (device pointers into the feed's slot, valid until released).  Returns 1 when the
 * stream is exhausted, 0 on success, < 0 on error (a producer's error included). */
int wdmpnn_feed_next(void *feed, void *stream, WdGraph *g, WdFeedBatch *info);
/* Every batch handed out so far is finished when `stream` reaches this point: their slots are reused
 * after it (the feed's own thread waits for that point before refilling a slot; the caller's thread
 * does not block, and no stream waits on `stream`). */
int wdmpnn_feed_release(void *feed, void *stream);
/* Workspace of wdmpnn_feed_forward for up to k batches of this feed. */
int wdmpnn_feed_forward_workspace_bytes(void *feed, const WdParams *p, const WdConfig *c, int32_t k, size_t *bytes);
/* Up to k next batches through the fused inference forward in one launch set (wdmpnn_forward_many),
 * then released: outputs [sum n_mols, H] into out (out_rows available), *got batches (0 = exhausted),
 * *rows output rows, *edges directed real edges, *h2d_bytes bytes uploaded for them. */
int wdmpnn_feed_forward(void *feed, int32_t k, const WdParams *p, const WdConfig *c, void *workspace,
                        size_t workspace_bytes, float *out, int64_t out_rows, void *stream, int32_t *got,
                        int64_t *rows, int64_t *edges, int64_t *h2d_bytes);
int wdmpnn_feed_destroy(void *feed);

#ifdef __cplusplus
}
#endif
#endif /* WDMPNN_H */
