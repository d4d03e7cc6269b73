// compact.hpp — host side of the compact graph format (include/wdmpnn.h "Compact graphs"): encoding a
// packed BatchMolGraph, decoding it back, the molecule-block plan, and a seeded generator of synthetic
// batches straight into compact form (the streamed workload of BASELINE.json configs[4]).
// Plain C++ (no Python); packer.cpp binds it.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "wdmpnn.h"

namespace compact {

struct Batch {
    int fa = 133, fb = 147;             // f_atoms / f_bonds widths (bond tail = fb - fa columns)
    std::vector<int32_t> mols;          // [B][4] {atom_start, n_atoms, bond_start, n_bonds}
    std::vector<float> xn;              // [B]
    std::vector<WdAtomCode> atoms;      // [V + 1], row 0 = pad
    std::vector<WdBondPair> pairs;      // [E / 2]
    int n_atoms() const { return (int)atoms.size(); }
    int n_bonds() const { return 1 + 2 * (int)pairs.size(); }
    int n_mols() const { return (int)xn.size(); }
};

inline WdAtomCode pad_atom() {
    WdAtomCode a;
    std::memset(a.col, 0xFF, 8);
    a.last = 0.f;
    a.w = 0.f;
    return a;
}

// ----------------------------------------------------------------------------------------------
// encode a packed batch (chemprop_amd BatchMolGraph arrays, the reference's offsets) -> compact;
// false (with a reason) when some row is not in the reference's categorical layout
// ----------------------------------------------------------------------------------------------
// tail rows are `row_w` floats wide: the bond columns are their last tail_w; when row_w > tail_w the
// rows are whole f_bonds rows and their first fa columns must equal the source atom's row (checked)
inline bool encode(int fa, int tail_w, int row_w, const float *f_atoms, const float *tail, const float *w_atoms,
                   const float *w_bonds, const int64_t *b2a, const int64_t *b2revb, const int64_t *deg,
                   const int64_t *in_idx, const int64_t *na, const int64_t *nb, const double *xn, int64_t B,
                   Batch &out, std::string &why) {
    if (fa < 2 || fa > 255 || tail_w < 0 || tail_w > 16 || (row_w != tail_w && row_w != fa + tail_w)) {
        why = "feature widths";
        return false;
    }
    const int t0 = row_w - tail_w;  // first bond column in a tail row
    out = Batch{};
    out.fa = fa;
    out.fb = fa + tail_w;
    int64_t V = 0, E = 0;
    for (int64_t i = 0; i < B; ++i) { V += na[i]; E += nb[i]; }
    out.atoms.resize((size_t)V + 1);
    out.atoms[0] = pad_atom();
    for (int64_t a = 1; a <= V; ++a) {
        const float *r = f_atoms + (size_t)a * fa;
        WdAtomCode c = pad_atom();
        int n = 0;
        for (int k0 = 0; k0 < fa - 1; k0 += 8) {  // skip all-zero groups of 8 columns (bit test, no float compare)
            const int k1 = std::min(k0 + 8, fa - 1);
            uint32_t any = 0;
            for (int k = k0; k < k1; ++k) { uint32_t u; std::memcpy(&u, r + k, 4); any |= u << 1; }  // ignores -0.0
            if (!any) continue;
            for (int k = k0; k < k1; ++k) {
                if (r[k] == 0.f) continue;
                if (r[k] != 1.f || n == 8) { why = "atom row not one-hot coded"; return false; }
                c.col[n++] = (uint8_t)k;
            }
        }
        c.last = r[fa - 1];
        c.w = w_atoms[a];
        out.atoms[(size_t)a] = c;
    }
    // pad rows must be the reference's zeros
    for (int k = 0; k < fa; ++k)
        if (f_atoms[k] != 0.f) { why = "pad atom row not zero"; return false; }
    std::vector<int64_t> iptr((size_t)V + 2, 0);
    for (int64_t a = 0; a <= V; ++a) iptr[(size_t)a + 1] = iptr[(size_t)a] + deg[a];
    out.mols.resize((size_t)B * 4);
    out.xn.resize((size_t)B);
    out.pairs.reserve((size_t)E / 2);
    int64_t ao = 1, bo = 1;
    for (int64_t i = 0; i < B; ++i) {
        out.mols[4 * i] = (int32_t)ao; out.mols[4 * i + 1] = (int32_t)na[i];
        out.mols[4 * i + 2] = (int32_t)bo; out.mols[4 * i + 3] = (int32_t)nb[i];
        out.xn[(size_t)i] = (float)xn[i];
        if (nb[i] % 2 || na[i] > 65535) { why = "molecule bonds not in pairs / too many atoms"; return false; }
        for (int64_t lb = 0; lb < nb[i]; lb += 2) {
            const int64_t b1 = bo + lb, b2 = b1 + 1;
            if (b2revb[b1] != b2 || b2revb[b2] != b1) { why = "b2revb not pairwise"; return false; }
            const int64_t a1 = b2a[b1] - ao, a2 = b2a[b2] - ao;
            if (a1 < 0 || a1 >= na[i] || a2 < 0 || a2 >= na[i]) { why = "b2a leaves its molecule"; return false; }
            WdBondPair q{};
            q.a1 = (uint16_t)a1; q.a2 = (uint16_t)a2;
            if (t0 && (std::memcmp(tail + (size_t)b1 * row_w, f_atoms + (size_t)b2a[b1] * fa, (size_t)fa * 4) ||
                       std::memcmp(tail + (size_t)b2 * row_w, f_atoms + (size_t)b2a[b2] * fa, (size_t)fa * 4))) {
                why = "bond rows do not start with their source atom row";
                return false;
            }
            for (int k = 0; k < tail_w; ++k) {
                const float v1 = tail[(size_t)b1 * row_w + t0 + k], v2 = tail[(size_t)b2 * row_w + t0 + k];
                if (v1 != v2 || (v1 != 0.f && v1 != 1.f)) { why = "bond columns not binary / not shared"; return false; }
                if (v1 == 1.f) q.tail |= (uint16_t)(1u << k);
            }
            q.w12 = w_bonds[b1]; q.w21 = w_bonds[b2];
            out.pairs.push_back(q);
        }
        // a2b = the bonds into each atom in creation order (featurization.py:471-476)
        for (int64_t la = 0; la < na[i]; ++la) {
            const int64_t a = ao + la;
            int64_t prev = -1, cnt = 0;
            for (int64_t e = iptr[(size_t)a]; e < iptr[(size_t)a + 1]; ++e) {
                const int64_t j = in_idx[e];
                if (j <= prev || j < bo || j >= bo + nb[i]) { why = "a2b not in creation order"; return false; }
                if (b2a[b2revb[j]] != a) { why = "a2b lists a bond not into its atom"; return false; }
                prev = j;
                ++cnt;
            }
            (void)cnt;
        }
        ao += na[i];
        bo += nb[i];
    }
    // every bond appears in exactly one a2b list (checked by count: sum(deg) == E)
    if (iptr[(size_t)V + 1] != E) { why = "a2b does not list every bond once"; return false; }
    if (deg[0] != 0) { why = "pad atom has bonds"; return false; }
    return true;
}

// ----------------------------------------------------------------------------------------------
// decode compact -> the arrays of the native pack() in tail mode (f_atoms [V+1][fa], bond tail
// [E+1][fb - fa], w_atoms, w_bonds, b2a, b2revb, deg, in_idx, n_atoms / n_bonds per molecule)
// ----------------------------------------------------------------------------------------------
struct Dense {
    std::vector<float> f_atoms, tail, w_atoms, w_bonds;
    std::vector<int64_t> b2a, b2revb, deg, in_idx, na, nb;
};

inline void decode(const Batch &c, Dense &d) {
    const int fa = c.fa, tw = c.fb - c.fa;
    const int64_t V1 = c.n_atoms(), E1 = c.n_bonds(), B = c.n_mols();
    d.f_atoms.assign((size_t)V1 * fa, 0.f);
    d.tail.assign((size_t)E1 * tw, 0.f);
    d.w_atoms.assign((size_t)V1, 0.f);
    d.w_bonds.assign((size_t)E1, 0.f);
    d.b2a.assign((size_t)E1, 0);
    d.b2revb.assign((size_t)E1, 0);
    d.deg.assign((size_t)V1, 0);
    d.na.resize((size_t)B);
    d.nb.resize((size_t)B);
    for (int64_t a = 1; a < V1; ++a) {
        const WdAtomCode &cd = c.atoms[(size_t)a];
        float *r = &d.f_atoms[(size_t)a * fa];
        for (int k = 0; k < 8; ++k)
            if (cd.col[k] != 0xFF) r[cd.col[k]] = 1.f;
        r[fa - 1] = cd.last;
        d.w_atoms[(size_t)a] = cd.w;
    }
    std::vector<int64_t> dst((size_t)E1, 0);
    for (int64_t i = 0; i < B; ++i) {
        const int64_t ao = c.mols[4 * i], bo = c.mols[4 * i + 2];
        d.na[(size_t)i] = c.mols[4 * i + 1];
        d.nb[(size_t)i] = c.mols[4 * i + 3];
        for (int64_t lb = 0; lb < c.mols[4 * i + 3]; lb += 2) {
            const WdBondPair &q = c.pairs[(size_t)((bo + lb - 1) / 2)];
            const int64_t b1 = bo + lb, b2 = b1 + 1;
            d.b2a[(size_t)b1] = ao + q.a1; d.b2a[(size_t)b2] = ao + q.a2;
            dst[(size_t)b1] = ao + q.a2; dst[(size_t)b2] = ao + q.a1;
            d.b2revb[(size_t)b1] = b2; d.b2revb[(size_t)b2] = b1;
            d.w_bonds[(size_t)b1] = q.w12; d.w_bonds[(size_t)b2] = q.w21;
            for (int k = 0; k < tw; ++k) {
                const float v = (float)((q.tail >> k) & 1);
                d.tail[(size_t)b1 * tw + k] = v;
                d.tail[(size_t)b2 * tw + k] = v;
            }
        }
    }
    for (int64_t b = 1; b < E1; ++b) ++d.deg[(size_t)dst[(size_t)b]];
    std::vector<int64_t> fill((size_t)V1 + 1, 0);
    for (int64_t a = 0; a < V1; ++a) fill[(size_t)a + 1] = fill[(size_t)a] + d.deg[(size_t)a];
    d.in_idx.assign((size_t)(E1 - 1), 0);
    for (int64_t b = 1; b < E1; ++b) d.in_idx[(size_t)fill[(size_t)dst[(size_t)b]]++] = b;
}

// ----------------------------------------------------------------------------------------------
// molecule blocks (the same greedy rule as BatchMolGraph.molecule_blocks) + per-block first entries
// of msg_gather / atom_gather (graph_build.hpp counts the same entries); false when a molecule
// exceeds a block
// ----------------------------------------------------------------------------------------------
constexpr int BLK_BONDS = 128, BLK_ATOMS = 64, BLK_MOLS = 64;

struct Plan {
    std::vector<int32_t> blocks;     // [nblk][8]
    std::vector<int32_t> block_nnz;  // [nblk][2]
    int64_t nnz_msg = 0, nnz_agg = 0;
    std::vector<int32_t> nz;         // scratch: nonzero in-weights per atom
    int n_blocks() const { return (int)(blocks.size() / 8); }
};

inline bool plan(const Batch &c, int target_blocks, Plan &p) {
    p.blocks.clear(); p.block_nnz.clear();  // (capacity kept: see generate)
    p.nnz_msg = p.nnz_agg = 0;
    const int64_t B = c.n_mols();
    int64_t big = 0, tot = 0;
    for (int64_t i = 0; i < B; ++i) {
        const int64_t bn = c.mols[4 * i + 3], an = c.mols[4 * i + 1];
        if (bn > BLK_BONDS || an > BLK_ATOMS) return false;
        big = std::max(big, bn);
        tot += bn;
    }
    const int64_t share = (tot + std::max(1, target_blocks) - 1) / std::max(1, target_blocks);
    const int64_t cap_b = std::min<int64_t>(BLK_BONDS, std::max(big, (share + 15) / 16 * 16));
    int32_t cur[8];
    bool have = false;
    for (int64_t i = 0; i < B; ++i) {
        const int32_t as = c.mols[4 * i], an = c.mols[4 * i + 1], bs = c.mols[4 * i + 2], bn = c.mols[4 * i + 3];
        if (have && cur[1] + bn <= cap_b && cur[3] + an <= BLK_ATOMS && i - cur[4] < BLK_MOLS) {
            cur[1] += bn; cur[3] += an; cur[5] = (int32_t)i + 1;
        } else {
            if (have) p.blocks.insert(p.blocks.end(), cur, cur + 8);
            const int32_t r[8] = {bs, bn, as, an, (int32_t)i, (int32_t)i + 1, 0, 0};
            std::memcpy(cur, r, sizeof r);
            have = true;
        }
    }
    if (have) p.blocks.insert(p.blocks.end(), cur, cur + 8);
    // entries: nz(a) = bonds into a with a nonzero weight; msg row a1 -> a2 (reverse weight w21):
    // nz(a1) - [w21 != 0] + [w21 != 1]; agg row a: nz(a)
    const int64_t V1 = c.n_atoms();
    p.nz.assign((size_t)V1, 0);
    std::vector<int32_t> &nz = p.nz;
    for (int64_t i = 0; i < B; ++i) {
        const int64_t ao = c.mols[4 * i], bo = c.mols[4 * i + 2];
        for (int64_t lb = 0; lb < c.mols[4 * i + 3]; lb += 2) {
            const WdBondPair &q = c.pairs[(size_t)((bo + lb - 1) / 2)];
            nz[(size_t)(ao + q.a2)] += q.w12 != 0.f;
            nz[(size_t)(ao + q.a1)] += q.w21 != 0.f;
        }
    }
    const int nblk = p.n_blocks();
    p.block_nnz.resize((size_t)nblk * 2);
    int64_t om = 0, oa = 0;
    for (int k = 0; k < nblk; ++k) {
        const int32_t *r = &p.blocks[(size_t)k * 8];
        p.block_nnz[(size_t)2 * k] = (int32_t)om;
        p.block_nnz[(size_t)2 * k + 1] = (int32_t)oa;
        for (int32_t mi = r[4]; mi < r[5]; ++mi) {
            const int64_t ao = c.mols[4 * mi], bo = c.mols[4 * mi + 2];
            for (int64_t lb = 0; lb < c.mols[4 * mi + 3]; lb += 2) {
                const WdBondPair &q = c.pairs[(size_t)((bo + lb - 1) / 2)];
                om += nz[(size_t)(ao + q.a1)] - (q.w21 != 0.f) + (q.w21 - 1.0f != 0.f);  // b1 = a1 -> a2
                om += nz[(size_t)(ao + q.a2)] - (q.w12 != 0.f) + (q.w12 - 1.0f != 0.f);  // b2 = a2 -> a1
            }
            for (int64_t la = 0; la < c.mols[4 * mi + 1]; ++la) oa += nz[(size_t)(ao + la)];
        }
    }
    p.nnz_msg = om;
    p.nnz_agg = oa;
    return true;
}

// ----------------------------------------------------------------------------------------------
// seeded synthetic batches (the distributions of chemprop_amd/synthetic.py, SURVEY §8(d), with this
// generator's own RNG: splitmix64)
// ----------------------------------------------------------------------------------------------
struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0xD1B54A32D192ED03ull) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double uniform(double lo, double hi) { return lo + (hi - lo) * uniform(); }
    int integers(int lo, int hi_incl) { return lo + (int)(uniform() * (double)(hi_incl - lo + 1)); }
};

// atom code laid out as atom_features (featurization.py:190-211) with the generator's choices
inline WdAtomCode gen_atom(Rng &r, int degree, float w) {
    static const int choices[6] = {100, 6, 5, 4, 5, 5};  // atomic_num, degree, charge, chiral, Hs, hybridization
    static const int anum[8] = {5, 6, 7, 8, 15, 16, 8, 5};
    WdAtomCode c = pad_atom();
    int off = 0, n = 0;
    for (int i = 0; i < 6; ++i) {
        int v;
        if (i == 0) v = anum[r.integers(0, 7)];
        else if (i == 1) v = std::min(degree, choices[1]);
        else v = r.integers(0, choices[i]);
        c.col[n++] = (uint8_t)(off + v);
        off += choices[i] + 1;
    }
    if (r.integers(0, 1)) c.col[n++] = (uint8_t)off;  // aromatic (column 131)
    c.last = (float)(r.uniform(10.0, 40.0) * 0.01);   // mass * 0.01 (column 132)
    c.w = w;
    return c;
}

// 14 bond columns (featurization.py:229-250): type one-hot 1..4, conjugated 5, ring 6, stereo 7..13
inline uint16_t gen_bond_tail(Rng &r) {
    uint16_t t = 0;
    t |= (uint16_t)(1u << (1 + r.integers(0, 3)));
    if (r.integers(0, 1)) t |= 1u << 5;
    if (r.integers(0, 1)) t |= 1u << 6;
    t |= (uint16_t)(1u << (7 + r.integers(0, 6)));
    return t;
}

// Edges of a molecule: a sorted, duplicate-free list of (a1 < a2) pairs (the iteration order of the
// std::set this replaced, so the generated batches are unchanged: no node allocations per edge).
using EdgeList = std::vector<std::pair<int, int>>;

inline void skeleton(Rng &r, int n, int offset, EdgeList &edges) {
    for (int i = 0; i + 1 < n; ++i) edges.push_back({offset + i, offset + i + 1});
    for (int k = 0; k < n / 5; ++k) {
        if (n < 4) break;
        const int i = r.integers(0, n - 4), j = r.integers(i + 3, n - 1);
        edges.push_back({offset + i, offset + j});
    }
}

inline void finish_edges(EdgeList &edges) {
    std::sort(edges.begin(), edges.end());
    edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
}

struct Rule { int a, b; float w12, w21; };

// one molecule appended to c (bonds: skeleton pairs in (a1 < a2) order, then rules in order); atom a
// gets weight w_first for a < n_first, else w_rest
inline void add_molecule(Batch &c, Rng &r, int n_atoms, const EdgeList &edges, const Rule *rules, int n_rules,
                         int n_first, float w_first, float w_rest, float xn) {
    const int32_t ao = (int32_t)c.atoms.size(), bo = c.n_bonds();
    int degree[64] = {};
    for (const auto &e : edges) { ++degree[e.first]; ++degree[e.second]; }
    for (int a = 0; a < n_atoms; ++a) c.atoms.push_back(gen_atom(r, degree[a], a < n_first ? w_first : w_rest));
    for (const auto &e : edges) {
        WdBondPair q{};
        q.a1 = (uint16_t)e.first; q.a2 = (uint16_t)e.second;
        q.tail = gen_bond_tail(r);
        q.w12 = 1.f; q.w21 = 1.f;
        c.pairs.push_back(q);
    }
    for (int k = 0; k < n_rules; ++k) {
        WdBondPair q{};
        q.a1 = (uint16_t)rules[k].a; q.a2 = (uint16_t)rules[k].b;
        q.tail = gen_bond_tail(r);
        q.w12 = rules[k].w12; q.w21 = rules[k].w21;
        c.pairs.push_back(q);
    }
    const int32_t nb = 2 * (int32_t)(edges.size() + n_rules);
    const int32_t row[4] = {ao, n_atoms, bo, nb};
    c.mols.insert(c.mols.end(), row, row + 4);
    c.xn.push_back(xn);
}

// kind: 0 = polymer (2 monomers x U{10..24} atoms, 10 stochastic rules incl. self loops, w ~ U[0.1, 0.5],
// Dirichlet(1, 1) fractions, degree_of_polym = 1 + log10(U[1, 1000])), 1 = QM9-like U{5..9} atoms,
// 2 = ZINC-like U{15..37} atoms (w = 1, Xn = 1)
inline void generate(int kind, int B, uint64_t seed, Batch &c) {
    // (c's vectors keep their capacity: a producer thread reuses one Batch, no allocation per batch)
    c.fa = 133; c.fb = 147;
    c.mols.clear(); c.xn.clear(); c.atoms.clear(); c.pairs.clear();
    const int amax = kind == 0 ? 48 : kind == 1 ? 9 : 37;
    c.atoms.reserve((size_t)B * amax + 1);
    c.pairs.reserve((size_t)B * (amax + amax / 5 + 10));
    c.mols.reserve((size_t)B * 4);
    c.xn.reserve((size_t)B);
    c.atoms.push_back(pad_atom());
    Rng r(seed);
    EdgeList edges;
    edges.reserve(64);
    for (int i = 0; i < B; ++i) {
        edges.clear();
        if (kind == 0) {
            const int na = r.integers(10, 24), nb = r.integers(10, 24);
            skeleton(r, na, 0, edges);
            skeleton(r, nb, na, edges);
            finish_edges(edges);
            int att[4];
            att[0] = r.integers(0, na - 1);
            do att[1] = r.integers(0, na - 1); while (att[1] == att[0]);
            att[2] = na + r.integers(0, nb - 1);
            do att[3] = na + r.integers(0, nb - 1); while (att[3] == att[2]);
            Rule rules[10];
            int nr = 0;
            for (int a = 0; a < 4; ++a)
                for (int b = a; b < 4; ++b) {
                    const float w12 = (float)r.uniform(0.1, 0.5);
                    const float w21 = (float)r.uniform(0.1, 0.5);
                    rules[nr++] = Rule{att[a], att[b], w12, w21};
                }
            const double f0 = r.uniform();
            const double xn = r.uniform(1.0, 1000.0);
            add_molecule(c, r, na + nb, edges, rules, nr, na, (float)f0, (float)(1.0 - f0),
                         (float)(1.0 + std::log10(xn)));
        } else {
            const int n = kind == 1 ? r.integers(5, 9) : r.integers(15, 37);
            skeleton(r, n, 0, edges);
            finish_edges(edges);
            add_molecule(c, r, n, edges, nullptr, 0, n, 1.f, 1.f, 1.f);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// staged upload image: mols | xn | atoms | pairs | blocks | block_nnz, each 256-byte aligned
// ----------------------------------------------------------------------------------------------
struct Staged {
    size_t off[6] = {0, 0, 0, 0, 0, 0}, total = 0;
};

inline size_t a256(size_t x) { return (x + 255) & ~size_t(255); }

inline Staged stage_layout(const Batch &c, const Plan &p) {
    Staged s;
    const size_t bytes[6] = {c.mols.size() * 4, c.xn.size() * 4, c.atoms.size() * sizeof(WdAtomCode),
                             c.pairs.size() * sizeof(WdBondPair), p.blocks.size() * 4, p.block_nnz.size() * 4};
    size_t o = 0;
    for (int k = 0; k < 6; ++k) { s.off[k] = o; o = a256(o + bytes[k]); }
    s.total = std::max<size_t>(o, 256);
    return s;
}

inline void stage_copy(const Batch &c, const Plan &p, const Staged &s, uint8_t *dst) {
    std::memcpy(dst + s.off[0], c.mols.data(), c.mols.size() * 4);
    std::memcpy(dst + s.off[1], c.xn.data(), c.xn.size() * 4);
    std::memcpy(dst + s.off[2], c.atoms.data(), c.atoms.size() * sizeof(WdAtomCode));
    std::memcpy(dst + s.off[3], c.pairs.data(), c.pairs.size() * sizeof(WdBondPair));
    std::memcpy(dst + s.off[4], p.blocks.data(), p.blocks.size() * 4);
    std::memcpy(dst + s.off[5], p.block_nnz.data(), p.block_nnz.size() * 4);
}

}  // namespace compact
