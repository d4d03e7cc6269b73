// packer.cpp — native batch packer for BatchMolGraph.
//
// Replaces the Python loops of the reference's BatchMolGraph.__init__ (featurization.py:757-813):
// the per-molecule MolGraph lists (f_atoms / f_bonds rows, w_atoms, w_bonds, a2b, b2a, b2revb,
// featurization.py:489-637 builds them as Python lists) are concatenated with the reference's
// offsets — row 0 of every atom / bond table is the zero pad (featurization.py:767-781), atom ids
// shift by 1 + atoms before the molecule, bond ids by 1 + bonds before it (:788-793) — straight into
// contiguous float32 / int64 buffers, reading the Python objects once.  The reference then builds
// torch tensors from nested lists (:805-811); that conversion is what costs the 77 ms per 64-polymer
// batch.  The CSR form of a2b (in_ptr from deg, in_idx in a2b slot order) replaces
// the padded a2b tensor, which the host rebuilds on demand (BatchMolGraph.a2b).
//
// CPython extension, no numpy headers: the outputs are bytearrays the caller views with
// np.frombuffer (no copy).  Rows may be lists / tuples of numbers or objects with the buffer
// protocol (a 2-D numpy table per molecule, or 1-D rows), float32/float64/int.  Single-threaded (it
// reads Python objects, so it holds the GIL); data parallelism comes from one packer per DataLoader
// worker / rank.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "compact.hpp"

namespace {

struct PyErrAlready {};  // a Python exception is set; unwind to the entry point

[[noreturn]] void fail(PyObject *type, const std::string &msg) {
    PyErr_SetString(type, msg.c_str());
    throw PyErrAlready{};
}

struct Ref {  // owned reference
    PyObject *p;
    explicit Ref(PyObject *o) : p(o) { if (!p) throw PyErrAlready{}; }
    ~Ref() { Py_XDECREF(p); }
    Ref(const Ref &) = delete;
    Ref &operator=(const Ref &) = delete;
};

inline double to_double(PyObject *o) {
    if (PyFloat_CheckExact(o)) return PyFloat_AS_DOUBLE(o);
    if (PyLong_CheckExact(o)) {
        const double v = PyLong_AsDouble(o);
        if (v == -1.0 && PyErr_Occurred()) throw PyErrAlready{};
        return v;
    }
    const double v = PyFloat_AsDouble(o);  // bool, numpy scalars, __float__
    if (v == -1.0 && PyErr_Occurred()) throw PyErrAlready{};
    return v;
}

inline int64_t to_int64(PyObject *o) {
    if (PyLong_CheckExact(o)) {
        const long long v = PyLong_AsLongLong(o);
        if (v == -1 && PyErr_Occurred()) throw PyErrAlready{};
        return v;
    }
    Ref i(PyNumber_Index(o));  // numpy integers
    const long long v = PyLong_AsLongLong(i.p);
    if (v == -1 && PyErr_Occurred()) throw PyErrAlready{};
    return v;
}

// copy n elements of a C-contiguous buffer (format f/d/e-less ints) converting to T
template <typename T>
void buffer_copy(const Py_buffer &b, Py_ssize_t n, T *dst, const char *what) {
    const char *f = b.format ? b.format : "B";
    if (*f == '<' || *f == '=' || *f == '@') ++f;
    const char *src = static_cast<const char *>(b.buf);
    switch (*f) {
    case 'f': for (Py_ssize_t i = 0; i < n; ++i) { float v; std::memcpy(&v, src + 4 * i, 4); dst[i] = (T)v; } break;
    case 'd': for (Py_ssize_t i = 0; i < n; ++i) { double v; std::memcpy(&v, src + 8 * i, 8); dst[i] = (T)v; } break;
    case 'q': case 'l':
        if (b.itemsize != 8) goto bad;
        for (Py_ssize_t i = 0; i < n; ++i) { int64_t v; std::memcpy(&v, src + 8 * i, 8); dst[i] = (T)v; } break;
    case 'i': for (Py_ssize_t i = 0; i < n; ++i) { int32_t v; std::memcpy(&v, src + 4 * i, 4); dst[i] = (T)v; } break;
    case 'B': case '?': for (Py_ssize_t i = 0; i < n; ++i) dst[i] = (T)(uint8_t)src[i]; break;
    case 'b': for (Py_ssize_t i = 0; i < n; ++i) dst[i] = (T)(int8_t)src[i]; break;
    default:
    bad:
        fail(PyExc_TypeError, std::string(what) + ": unsupported buffer element format '" + f + "'");
    }
}

struct Buf {  // a C-contiguous Py_buffer, released on scope exit
    Py_buffer b{};
    bool ok = false;
    Buf(PyObject *o) {
        if (PyObject_GetBuffer(o, &b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) == 0) ok = true;
        else PyErr_Clear();
    }
    ~Buf() { if (ok) PyBuffer_Release(&b); }
};

// `rows`: n_rows rows of `src_w` numbers; columns [col0, col0 + width) of each -> dst[r * width ..]
void fill_table(PyObject *rows, Py_ssize_t n_rows, Py_ssize_t src_w, Py_ssize_t col0, Py_ssize_t width, float *dst,
                const char *what) {
    if (n_rows == 0) return;
    if (!PyList_Check(rows) && !PyTuple_Check(rows) && PyObject_CheckBuffer(rows)) {
        Buf t(rows);
        if (t.ok) {
            if (t.b.ndim != 2 || t.b.shape[0] != n_rows || t.b.shape[1] != src_w)
                fail(PyExc_ValueError, std::string(what) + ": table shape does not match (rows, width)");
            if (col0 == 0 && width == src_w) {
                buffer_copy(t.b, n_rows * width, dst, what);
            } else {
                Py_buffer row = t.b;
                for (Py_ssize_t r = 0; r < n_rows; ++r) {
                    row.buf = static_cast<char *>(t.b.buf) + (r * src_w + col0) * t.b.itemsize;
                    buffer_copy(row, width, dst + r * width, what);
                }
            }
            return;
        }
    }
    Ref seq(PySequence_Fast(rows, what));
    if (PySequence_Fast_GET_SIZE(seq.p) != n_rows)
        fail(PyExc_ValueError, std::string(what) + ": row count differs from the graph's count");
    PyObject **items = PySequence_Fast_ITEMS(seq.p);
    for (Py_ssize_t r = 0; r < n_rows; ++r) {
        PyObject *row = items[r];
        float *d = dst + r * width;
        if (PyList_Check(row) || PyTuple_Check(row)) {
            const Py_ssize_t n = PyList_Check(row) ? PyList_GET_SIZE(row) : PyTuple_GET_SIZE(row);
            if (n != src_w) fail(PyExc_ValueError, std::string(what) + ": ragged feature rows");
            PyObject **it = PyList_Check(row) ? &PyList_GET_ITEM(row, 0) : &PyTuple_GET_ITEM(row, 0);
            for (Py_ssize_t k = 0; k < width; ++k) d[k] = (float)to_double(it[col0 + k]);
            continue;
        }
        Buf rb(row);
        if (rb.ok) {
            if (rb.b.ndim != 1 || rb.b.shape[0] != src_w)
                fail(PyExc_ValueError, std::string(what) + ": ragged feature rows");
            Py_buffer part = rb.b;
            part.buf = static_cast<char *>(rb.b.buf) + col0 * rb.b.itemsize;
            buffer_copy(part, width, d, what);
            continue;
        }
        Ref rs(PySequence_Fast(row, what));
        if (PySequence_Fast_GET_SIZE(rs.p) != src_w) fail(PyExc_ValueError, std::string(what) + ": ragged feature rows");
        PyObject **it = PySequence_Fast_ITEMS(rs.p);
        for (Py_ssize_t k = 0; k < width; ++k) d[k] = (float)to_double(it[col0 + k]);
    }
}

// The reference builds every bond row as f_atoms[source atom] + bond features (featurization.py:467-468,
// 545-546, 616-617).  Checks columns [0, fa_w) of the molecule's f_bonds rows against its packed
// f_atoms rows (float32 values), at the molecule-local source atom of each bond.
void check_bond_rows(PyObject *rows, Py_ssize_t n_rows, Py_ssize_t fa_w, const float *f_atoms_mol,
                     const int64_t *b2a_local) {
    std::vector<float> tmp((size_t)fa_w);
    for (Py_ssize_t r = 0; r < n_rows; ++r) {
        Ref seq(PySequence_GetItem(rows, r));
        // reuse fill_table on a one-row view: wrap the row in a 1-tuple
        Ref one(PyTuple_Pack(1, seq.p));
        const Py_ssize_t src_w = PyObject_Length(seq.p);
        if (src_w < fa_w) fail(PyExc_ValueError, "f_bonds rows are shorter than f_atoms rows");
        fill_table(one.p, 1, src_w, 0, fa_w, tmp.data(), "f_bonds");
        if (std::memcmp(tmp.data(), f_atoms_mol + b2a_local[r] * fa_w, (size_t)fa_w * 4) != 0)
            fail(PyExc_ValueError, "f_bonds[b][:atom_fdim] != f_atoms[b2a[b]]: the bond rows do not start with "
                                   "their source atom's features, so they cannot be rebuilt on the device");
    }
}

// a 1-D sequence of n numbers -> dst[i] = conv(x_i) + add
template <typename T>
void fill_vector(PyObject *v, Py_ssize_t n, T *dst, T add, const char *what) {
    if (n == 0) return;
    if (!PyList_Check(v) && !PyTuple_Check(v) && PyObject_CheckBuffer(v)) {
        Buf t(v);
        if (t.ok) {
            if (t.b.ndim != 1 || t.b.shape[0] != n)
                fail(PyExc_ValueError, std::string(what) + ": length differs from the graph's count");
            buffer_copy(t.b, n, dst, what);
            for (Py_ssize_t i = 0; i < n; ++i) dst[i] += add;
            return;
        }
    }
    Ref seq(PySequence_Fast(v, what));
    if (PySequence_Fast_GET_SIZE(seq.p) != n)
        fail(PyExc_ValueError, std::string(what) + ": length differs from the graph's count");
    PyObject **it = PySequence_Fast_ITEMS(seq.p);
    for (Py_ssize_t i = 0; i < n; ++i) {
        if constexpr (std::is_integral<T>::value) dst[i] = (T)to_int64(it[i]) + add;
        else dst[i] = (T)to_double(it[i]) + add;
    }
}

Py_ssize_t attr_int(PyObject *g, const char *name) {
    Ref a(PyObject_GetAttrString(g, name));
    return (Py_ssize_t)to_int64(a.p);
}

PyObject *new_bytes(Py_ssize_t n) {
    PyObject *b = PyByteArray_FromStringAndSize(nullptr, n);
    if (!b) throw PyErrAlready{};
    if (n) std::memset(PyByteArray_AS_STRING(b), 0, (size_t)n);
    return b;
}

// pack(mol_graphs, fa_w, fb_w[, tail_from[, check]]) -> (f_atoms, f_bonds, w_atoms, w_bonds, b2a, b2revb,
// deg, in_idx, n_atoms_per_mol, n_bonds_per_mol) as bytearrays (float32 [V+1][fa_w],
// float32 [E+1][fb_w - tail_from] (tail_from = 0: whole rows; = fa_w: only the bond-feature tail, the
// device rebuilds the rest from f_atoms, wdmpnn_build_bond_features; check = 1 verifies that the skipped
// columns equal the source atom's row),
// float32 [V+1], float32 [E+1], int64 [E+1] x 2, int64 [V+1], int64 [nnz], int64 [B] x 2)
PyObject *pack(PyObject *, PyObject *args) {
    PyObject *graphs_obj;
    Py_ssize_t fa_w, fb_w, tail_from = 0;
    int check = 0;
    if (!PyArg_ParseTuple(args, "Onn|np", &graphs_obj, &fa_w, &fb_w, &tail_from, &check)) return nullptr;
    if (tail_from < 0 || tail_from > fb_w || (tail_from != 0 && tail_from != fa_w)) {
        PyErr_SetString(PyExc_ValueError, "tail_from must be 0 or the f_atoms row width");
        return nullptr;
    }
    const Py_ssize_t fbo_w = fb_w - tail_from;  // f_bonds columns written
    PyObject *out[10] = {};
    try {
        Ref graphs(PySequence_Fast(graphs_obj, "mol_graphs must be a sequence"));
        const Py_ssize_t B = PySequence_Fast_GET_SIZE(graphs.p);
        PyObject **gs = PySequence_Fast_ITEMS(graphs.p);
        // pass 1: counts (featurization.py:784-786 read n_atoms / n_bonds), a2b sizes
        std::vector<int64_t> na(B), nb(B), nnz_of(B);
        int64_t V = 0, E = 0, nnz = 0;
        for (Py_ssize_t i = 0; i < B; ++i) {
            na[i] = attr_int(gs[i], "n_atoms");
            nb[i] = attr_int(gs[i], "n_bonds");
            if (na[i] < 0 || nb[i] < 0) fail(PyExc_ValueError, "negative n_atoms / n_bonds");
            Ref a2b(PyObject_GetAttrString(gs[i], "a2b"));
            Ref seq(PySequence_Fast(a2b.p, "a2b must be a sequence of sequences"));
            if (PySequence_Fast_GET_SIZE(seq.p) != na[i]) fail(PyExc_ValueError, "len(a2b) != n_atoms");
            int64_t c = 0;
            for (Py_ssize_t a = 0; a < na[i]; ++a) {
                const Py_ssize_t l = PyObject_Length(PySequence_Fast_GET_ITEM(seq.p, a));
                if (l < 0) throw PyErrAlready{};
                c += l;
            }
            nnz_of[i] = c;
            V += na[i]; E += nb[i]; nnz += c;
        }
        out[0] = new_bytes((V + 1) * fa_w * 4);
        out[1] = new_bytes((E + 1) * fbo_w * 4);
        out[2] = new_bytes((V + 1) * 4);
        out[3] = new_bytes((E + 1) * 4);
        out[4] = new_bytes((E + 1) * 8);
        out[5] = new_bytes((E + 1) * 8);
        out[6] = new_bytes((V + 1) * 8);
        out[7] = new_bytes(nnz * 8);
        out[8] = new_bytes(B * 8);
        out[9] = new_bytes(B * 8);
        float *f_atoms = reinterpret_cast<float *>(PyByteArray_AS_STRING(out[0]));
        float *f_bonds = reinterpret_cast<float *>(PyByteArray_AS_STRING(out[1]));
        float *w_atoms = reinterpret_cast<float *>(PyByteArray_AS_STRING(out[2]));
        float *w_bonds = reinterpret_cast<float *>(PyByteArray_AS_STRING(out[3]));
        int64_t *b2a = reinterpret_cast<int64_t *>(PyByteArray_AS_STRING(out[4]));
        int64_t *b2revb = reinterpret_cast<int64_t *>(PyByteArray_AS_STRING(out[5]));
        int64_t *deg = reinterpret_cast<int64_t *>(PyByteArray_AS_STRING(out[6]));
        int64_t *in_idx = reinterpret_cast<int64_t *>(PyByteArray_AS_STRING(out[7]));
        std::memcpy(PyByteArray_AS_STRING(out[8]), na.data(), B * 8);
        std::memcpy(PyByteArray_AS_STRING(out[9]), nb.data(), B * 8);
        // pass 2: rows at the reference's offsets (row 0 stays the zero pad)
        int64_t ao = 1, bo = 1, eo = 0;
        for (Py_ssize_t i = 0; i < B; ++i) {
            PyObject *g = gs[i];
            {
                Ref t(PyObject_GetAttrString(g, "f_atoms"));
                fill_table(t.p, na[i], fa_w, 0, fa_w, f_atoms + ao * fa_w, "f_atoms");
            }
            {
                Ref t(PyObject_GetAttrString(g, "f_bonds"));
                fill_table(t.p, nb[i], fb_w, tail_from, fbo_w, f_bonds + bo * fbo_w, "f_bonds");
            }
            {
                Ref t(PyObject_GetAttrString(g, "w_atoms"));
                fill_vector<float>(t.p, na[i], w_atoms + ao, 0.f, "w_atoms");
            }
            {
                Ref t(PyObject_GetAttrString(g, "w_bonds"));
                fill_vector<float>(t.p, nb[i], w_bonds + bo, 0.f, "w_bonds");
            }
            {
                Ref t(PyObject_GetAttrString(g, "b2a"));
                fill_vector<int64_t>(t.p, nb[i], b2a + bo, ao, "b2a");
            }
            if (tail_from && check) {
                std::vector<int64_t> local((size_t)nb[i]);
                for (int64_t r = 0; r < nb[i]; ++r) {
                    local[r] = b2a[bo + r] - ao;
                    if (local[r] < 0 || local[r] >= na[i]) fail(PyExc_ValueError, "b2a out of range");
                }
                Ref t(PyObject_GetAttrString(g, "f_bonds"));
                check_bond_rows(t.p, nb[i], fa_w, f_atoms + ao * fa_w, local.data());
            }
            {
                Ref t(PyObject_GetAttrString(g, "b2revb"));
                fill_vector<int64_t>(t.p, nb[i], b2revb + bo, bo, "b2revb");
            }
            {
                Ref a2b(PyObject_GetAttrString(g, "a2b"));
                Ref seq(PySequence_Fast(a2b.p, "a2b must be a sequence of sequences"));
                int64_t c = 0;
                for (Py_ssize_t a = 0; a < na[i]; ++a) {
                    PyObject *l = PySequence_Fast_GET_ITEM(seq.p, a);
                    const Py_ssize_t n = PyObject_Length(l);
                    if (n < 0) throw PyErrAlready{};
                    if (c + n > nnz_of[i]) fail(PyExc_ValueError, "a2b changed while packing");
                    deg[ao + a] = n;
                    fill_vector<int64_t>(l, n, in_idx + eo + c, bo, "a2b");
                    c += n;
                }
            }
            ao += na[i]; bo += nb[i]; eo += nnz_of[i];
        }
        PyObject *res = PyTuple_New(10);
        if (!res) throw PyErrAlready{};
        for (int k = 0; k < 10; ++k) PyTuple_SET_ITEM(res, k, out[k]);  // steals
        return res;
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    for (PyObject *o : out) Py_XDECREF(o);
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "pack failed");
    return nullptr;
}


// ---------------------------------------------------------------------------------------------
// Gather lists (the CSR forms of mpn.py:112-131 that the kernels consume), built natively.
// ---------------------------------------------------------------------------------------------
// A read-only typed view of a 1-D C-contiguous buffer argument.
template <typename T>
struct In {
    Py_buffer b{};
    const T *p = nullptr;
    Py_ssize_t n = 0;
    In(PyObject *o, const char *fmt, const char *what) {
        if (PyObject_GetBuffer(o, &b, PyBUF_C_CONTIGUOUS | PyBUF_FORMAT) != 0) throw PyErrAlready{};
        const char *f = b.format ? b.format : "B";
        if (*f == '<' || *f == '=' || *f == '@') ++f;
        bool ok = b.itemsize == (Py_ssize_t)sizeof(T);
        if (ok && fmt[0] == 'i') ok = *f == 'q' || *f == 'l' || *f == 'i';
        if (ok && fmt[0] == 'f') ok = *f == 'f';
        if (!ok) {
            PyBuffer_Release(&b);
            fail(PyExc_TypeError, std::string(what) + ": unexpected dtype");
        }
        p = static_cast<const T *>(b.buf);
        n = b.len / (Py_ssize_t)sizeof(T);
    }
    ~In() { PyBuffer_Release(&b); }
};

struct CsrOut {
    std::vector<int32_t> ptr, idx;
    std::vector<float> coef;
};

PyObject *csr_tuple(const CsrOut &c) {
    PyObject *t = PyTuple_New(3);
    if (!t) throw PyErrAlready{};
    auto put = [&](int k, const void *d, size_t bytes) {
        PyObject *b = PyByteArray_FromStringAndSize(static_cast<const char *>(d), (Py_ssize_t)bytes);
        if (!b) { Py_DECREF(t); throw PyErrAlready{}; }
        PyTuple_SET_ITEM(t, k, b);
    };
    put(0, c.ptr.data(), c.ptr.size() * 4);
    put(1, c.idx.data(), c.idx.size() * 4);
    put(2, c.coef.data(), c.coef.size() * 4);
    return t;
}

// stable counting-sort transpose: source row j lists (row r, coef) in entry order
CsrOut transpose(const CsrOut &c, int64_t n_src) {
    CsrOut t;
    t.ptr.assign((size_t)n_src + 1, 0);
    for (int32_t j : c.idx) {
        if (j < 0 || j >= n_src) fail(PyExc_ValueError, "gather index out of range");
        ++t.ptr[(size_t)j + 1];
    }
    for (int64_t j = 0; j < n_src; ++j) t.ptr[j + 1] += t.ptr[j];
    t.idx.resize(c.idx.size());
    t.coef.resize(c.idx.size());
    std::vector<int32_t> fill(t.ptr.begin(), t.ptr.end() - 1);
    const int64_t rows = (int64_t)c.ptr.size() - 1;
    for (int64_t r = 0; r < rows; ++r)
        for (int32_t e = c.ptr[r]; e < c.ptr[r + 1]; ++e) {
            const int32_t q = fill[c.idx[e]]++;
            t.idx[q] = (int32_t)r;
            t.coef[q] = c.coef[e];
        }
    return t;
}

// gathers(b2a, b2revb, w_bonds, deg, in_idx) -> (msg, agg, msg_t, agg_t), each (ptr, idx, coef)
// bytearrays (int32, int32, float32):
//   msg row b >= 1 (bond_message_gather, mpn.py:112-120): X_b = sum_{j in in(b2a[b])} w_j M_j - M_rev(b),
//     entries in a2b slot order, the reverse bond's coefficient w_rev - 1 (evaluated in double, then
//     rounded to float once) and dropped when 0; a reverse bond that is not among the in-bonds gets
//     its own -1 entry at the end of the row; row 0 (pad) is empty;
//   agg row a (atom_aggregate_gather, mpn.py:126-131): A_a = sum_{j in in(a)} w_j M_j (zero weights
//     dropped);
//   *_t: the transposes over the E + 1 source rows (the data-gradient gathers).
PyObject *gathers(PyObject *, PyObject *args) {
    PyObject *o_b2a, *o_rev, *o_w, *o_deg, *o_in;
    if (!PyArg_ParseTuple(args, "OOOOO", &o_b2a, &o_rev, &o_w, &o_deg, &o_in)) return nullptr;
    try {
        In<int64_t> b2a(o_b2a, "i", "b2a"), rev(o_rev, "i", "b2revb"), deg(o_deg, "i", "deg"), in(o_in, "i", "in_idx");
        In<float> w(o_w, "f", "w_bonds");
        const int64_t E1 = b2a.n, V1 = deg.n;
        if (rev.n != E1 || w.n != E1) fail(PyExc_ValueError, "b2a / b2revb / w_bonds lengths differ");
        std::vector<int64_t> iptr((size_t)V1 + 1, 0);
        for (int64_t a = 0; a < V1; ++a) iptr[a + 1] = iptr[a] + deg.p[a];
        if (iptr[V1] != in.n) fail(PyExc_ValueError, "sum(deg) != len(in_idx)");
        for (int64_t e = 0; e < in.n; ++e)
            if (in.p[e] < 0 || in.p[e] >= E1) fail(PyExc_ValueError, "in_idx out of range");
        CsrOut msg, agg;
        msg.ptr.reserve((size_t)E1 + 1);
        msg.ptr.push_back(0);
        if (E1 > 0) msg.ptr.push_back(0);  // row 0: pad bond, no entries
        for (int64_t b = 1; b < E1; ++b) {
            const int64_t a = b2a.p[b], r = rev.p[b];
            if (a < 0 || a >= V1 || r < 0 || r >= E1) fail(PyExc_ValueError, "b2a / b2revb out of range");
            bool has_rev = false;
            for (int64_t e = iptr[a]; e < iptr[a + 1]; ++e) {
                const int64_t j = in.p[e];
                double c = (double)w.p[j];
                if (j == r) { c -= 1.0; has_rev = true; }
                if (c != 0.0) { msg.idx.push_back((int32_t)j); msg.coef.push_back((float)c); }
            }
            if (!has_rev) { msg.idx.push_back((int32_t)r); msg.coef.push_back(-1.0f); }
            msg.ptr.push_back((int32_t)msg.idx.size());
        }
        agg.ptr.reserve((size_t)V1 + 1);
        agg.ptr.push_back(0);
        for (int64_t a = 0; a < V1; ++a) {
            for (int64_t e = iptr[a]; e < iptr[a + 1]; ++e) {
                const int64_t j = in.p[e];
                if (w.p[j] != 0.0f) { agg.idx.push_back((int32_t)j); agg.coef.push_back(w.p[j]); }
            }
            agg.ptr.push_back((int32_t)agg.idx.size());
        }
        const CsrOut msg_t = transpose(msg, E1), agg_t = transpose(agg, E1);
        PyObject *res = PyTuple_New(4);
        if (!res) throw PyErrAlready{};
        const CsrOut *all[4] = {&msg, &agg, &msg_t, &agg_t};
        for (int k = 0; k < 4; ++k) {
            PyObject *t;
            try { t = csr_tuple(*all[k]); } catch (...) { Py_DECREF(res); throw; }
            PyTuple_SET_ITEM(res, k, t);
        }
        return res;
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "gathers failed");
    return nullptr;
}

// ell(ptr, idx, coef, rows_p, row_base, width) -> (idx u8 [rows_p * width], coef f32 [rows_p * width]):
// the first `width` entries of every row in block-local form (idx - row_base[row], < 128), unused
// slots (0, 0), bit 7 of the last slot on rows with more entries (WdGraph.*_ell_*)
PyObject *ell(PyObject *, PyObject *args) {
    PyObject *o_ptr, *o_idx, *o_coef, *o_base;
    Py_ssize_t rows_p, width;
    if (!PyArg_ParseTuple(args, "OOOnOn", &o_ptr, &o_idx, &o_coef, &rows_p, &o_base, &width)) return nullptr;
    try {
        In<int32_t> ptr(o_ptr, "i", "ptr"), idx(o_idx, "i", "idx");
        In<float> coef(o_coef, "f", "coef");
        In<int64_t> base(o_base, "i", "row_base");
        const Py_ssize_t rows = ptr.n - 1;
        if (rows < 0 || rows > rows_p || base.n < rows || width < 1 || width > 64)
            fail(PyExc_ValueError, "ell: bad sizes");
        PyObject *oi = new_bytes(rows_p * width), *oc = nullptr;
        try { oc = new_bytes(rows_p * width * 4); } catch (...) { Py_DECREF(oi); throw; }
        uint8_t *di = reinterpret_cast<uint8_t *>(PyByteArray_AS_STRING(oi));
        float *dc = reinterpret_cast<float *>(PyByteArray_AS_STRING(oc));
        for (Py_ssize_t r = 0; r < rows; ++r) {
            const int32_t e0 = ptr.p[r], e1 = ptr.p[r + 1];
            for (int32_t e = e0; e < e1 && e - e0 < width; ++e) {
                const int64_t l = (int64_t)idx.p[e] - base.p[r];
                if (l < 0 || l >= 128) {
                    Py_DECREF(oi); Py_DECREF(oc);
                    fail(PyExc_ValueError, "ell_rows: an entry leaves its molecule block");
                }
                di[r * width + (e - e0)] = (uint8_t)l;
                dc[r * width + (e - e0)] = coef.p[e];
            }
            if (e1 - e0 > width) di[r * width + width - 1] |= 0x80;
        }
        PyObject *res = PyTuple_Pack(2, oi, oc);
        Py_DECREF(oi); Py_DECREF(oc);
        return res;
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "ell failed");
    return nullptr;
}

// ---------------------------------------------------------------------------------------------
// Compact graphs (compact.hpp, include/wdmpnn.h): encode / decode / plan / generate / stage
// ---------------------------------------------------------------------------------------------
PyObject *bytes_of(const void *d, size_t n) {
    PyObject *b = PyByteArray_FromStringAndSize(static_cast<const char *>(d), (Py_ssize_t)n);
    if (!b) throw PyErrAlready{};
    return b;
}

PyObject *batch_tuple(const compact::Batch &c) {
    PyObject *t = PyTuple_New(4);
    if (!t) throw PyErrAlready{};
    const void *d[4] = {c.mols.data(), c.xn.data(), c.atoms.data(), c.pairs.data()};
    const size_t n[4] = {c.mols.size() * 4, c.xn.size() * 4, c.atoms.size() * sizeof(WdAtomCode),
                         c.pairs.size() * sizeof(WdBondPair)};
    for (int k = 0; k < 4; ++k) {
        PyObject *b;
        try { b = bytes_of(d[k], n[k]); } catch (...) { Py_DECREF(t); throw; }
        PyTuple_SET_ITEM(t, k, b);
    }
    return t;
}

// (mols, xn, atoms, pairs) buffers -> Batch
void batch_from(PyObject *o_mols, PyObject *o_xn, PyObject *o_atoms, PyObject *o_pairs, int fa, int fb,
                compact::Batch &c) {
    Buf m(o_mols), x(o_xn), a(o_atoms), q(o_pairs);
    if (!m.ok || !x.ok || !a.ok || !q.ok) fail(PyExc_TypeError, "compact arrays must support the buffer protocol");
    if (m.b.len % 16 || x.b.len % 4 || a.b.len % (Py_ssize_t)sizeof(WdAtomCode) ||
        q.b.len % (Py_ssize_t)sizeof(WdBondPair) || m.b.len / 16 != x.b.len / 4 || a.b.len == 0)
        fail(PyExc_ValueError, "compact arrays have inconsistent sizes");
    c = compact::Batch{};
    c.fa = fa; c.fb = fb;
    c.mols.resize((size_t)m.b.len / 4);
    std::memcpy(c.mols.data(), m.b.buf, (size_t)m.b.len);
    c.xn.resize((size_t)x.b.len / 4);
    std::memcpy(c.xn.data(), x.b.buf, (size_t)x.b.len);
    c.atoms.resize((size_t)a.b.len / sizeof(WdAtomCode));
    std::memcpy(c.atoms.data(), a.b.buf, (size_t)a.b.len);
    c.pairs.resize((size_t)q.b.len / sizeof(WdBondPair));
    std::memcpy(c.pairs.data(), q.b.buf, (size_t)q.b.len);
    // structural checks (the device build trusts these)
    int64_t ao = 1, bo = 1;
    for (int i = 0; i < c.n_mols(); ++i) {
        const int32_t *r = &c.mols[(size_t)4 * i];
        if (r[0] != ao || r[2] != bo || r[1] < 0 || r[3] < 0 || r[3] % 2)
            fail(PyExc_ValueError, "compact molecules are not contiguous in the reference's numbering");
        for (int64_t lb = 0; lb < r[3]; lb += 2) {
            const WdBondPair &p = c.pairs[(size_t)((bo + lb - 1) / 2)];
            if (p.a1 >= r[1] || p.a2 >= r[1]) fail(PyExc_ValueError, "compact bond endpoint outside its molecule");
        }
        ao += r[1];
        bo += r[3];
    }
    if (ao != c.n_atoms() || bo != c.n_bonds()) fail(PyExc_ValueError, "compact molecules do not cover the tables");
}

// compact_encode(f_atoms, tail, w_atoms, w_bonds, b2a, b2revb, deg, in_idx, na, nb, xn(float64), fa, tail_w)
// -> (mols, xn, atoms, pairs) or (None, reason); tail = the bond columns [E+1][tail_w] or whole f_bonds rows
// [E+1][fa + tail_w] (then checked to start with their source atom's row)
PyObject *compact_encode(PyObject *, PyObject *args) {
    PyObject *o[11];
    int fa, tw;
    if (!PyArg_ParseTuple(args, "OOOOOOOOOOOii", &o[0], &o[1], &o[2], &o[3], &o[4], &o[5], &o[6], &o[7], &o[8], &o[9],
                          &o[10], &fa, &tw))
        return nullptr;
    try {
        In<float> f_atoms(o[0], "f", "f_atoms"), tail(o[1], "f", "tail"), w_atoms(o[2], "f", "w_atoms"),
            w_bonds(o[3], "f", "w_bonds");
        In<int64_t> b2a(o[4], "i", "b2a"), rev(o[5], "i", "b2revb"), deg(o[6], "i", "deg"), in(o[7], "i", "in_idx"),
            na(o[8], "i", "na"), nb(o[9], "i", "nb");
        Buf xb(o[10]);
        if (!xb.ok || xb.b.itemsize != 8) fail(PyExc_TypeError, "xn must be a float64 buffer");
        const int64_t B = na.n;
        if (nb.n != B || xb.b.len / 8 != B) fail(PyExc_ValueError, "per-molecule arrays differ in length");
        int64_t V = 0, E = 0;
        for (int64_t i = 0; i < B; ++i) { V += na.p[i]; E += nb.p[i]; }
        const int64_t row_w = E + 1 > 0 ? tail.n / (E + 1) : tw;
        if (f_atoms.n != (V + 1) * fa || tail.n != (E + 1) * row_w || w_atoms.n != V + 1 || w_bonds.n != E + 1 ||
            b2a.n != E + 1 || rev.n != E + 1 || deg.n != V + 1 || in.n != E)
            fail(PyExc_ValueError, "compact_encode: array sizes do not match the molecule counts");
        compact::Batch c;
        std::string why;
        if (!compact::encode(fa, tw, (int)row_w, f_atoms.p, tail.p, w_atoms.p, w_bonds.p, b2a.p, rev.p, deg.p, in.p, na.p, nb.p,
                             static_cast<const double *>(xb.b.buf), B, c, why)) {
            PyObject *s = PyUnicode_FromString(why.c_str());
            if (!s) throw PyErrAlready{};
            PyObject *r = PyTuple_Pack(2, Py_None, s);
            Py_DECREF(s);
            return r;
        }
        return batch_tuple(c);
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "compact_encode failed");
    return nullptr;
}

// compact_decode(mols, xn, atoms, pairs, fa, fb) -> pack()'s 10 outputs in tail mode
PyObject *compact_decode(PyObject *, PyObject *args) {
    PyObject *o[4];
    int fa, fb;
    if (!PyArg_ParseTuple(args, "OOOOii", &o[0], &o[1], &o[2], &o[3], &fa, &fb)) return nullptr;
    try {
        compact::Batch c;
        batch_from(o[0], o[1], o[2], o[3], fa, fb, c);
        compact::Dense d;
        compact::decode(c, d);
        PyObject *t = PyTuple_New(10);
        if (!t) throw PyErrAlready{};
        const void *ptr[10] = {d.f_atoms.data(), d.tail.data(), d.w_atoms.data(), d.w_bonds.data(), d.b2a.data(),
                               d.b2revb.data(), d.deg.data(), d.in_idx.data(), d.na.data(), d.nb.data()};
        const size_t n[10] = {d.f_atoms.size() * 4, d.tail.size() * 4, d.w_atoms.size() * 4, d.w_bonds.size() * 4,
                              d.b2a.size() * 8, d.b2revb.size() * 8, d.deg.size() * 8, d.in_idx.size() * 8,
                              d.na.size() * 8, d.nb.size() * 8};
        for (int k = 0; k < 10; ++k) {
            PyObject *b;
            try { b = bytes_of(ptr[k], n[k]); } catch (...) { Py_DECREF(t); throw; }
            PyTuple_SET_ITEM(t, k, b);
        }
        return t;
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "compact_decode failed");
    return nullptr;
}

// compact_generate(kind, B, seed) -> (mols, xn, atoms, pairs); kind 0 polymer, 1 qm9, 2 zinc
PyObject *compact_generate(PyObject *, PyObject *args) {
    int kind, B;
    unsigned long long seed;
    if (!PyArg_ParseTuple(args, "iiK", &kind, &B, &seed)) return nullptr;
    if (kind < 0 || kind > 2 || B < 0) {
        PyErr_SetString(PyExc_ValueError, "kind in {0, 1, 2}, B >= 0");
        return nullptr;
    }
    try {
        compact::Batch c;
        Py_BEGIN_ALLOW_THREADS
        compact::generate(kind, B, seed, c);
        Py_END_ALLOW_THREADS
        return batch_tuple(c);
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "compact_generate failed");
    return nullptr;
}

PyObject *stage_result(const compact::Batch &c, const compact::Plan &p, const compact::Staged &s, bool copied) {
    return Py_BuildValue("(O(iiiiLL)(nnnnnn)n)", copied ? Py_True : Py_False, c.n_mols(), c.n_atoms(), c.n_bonds(),
                         p.n_blocks(), (long long)p.nnz_msg, (long long)p.nnz_agg, (Py_ssize_t)s.off[0],
                         (Py_ssize_t)s.off[1], (Py_ssize_t)s.off[2], (Py_ssize_t)s.off[3], (Py_ssize_t)s.off[4],
                         (Py_ssize_t)s.off[5], (Py_ssize_t)s.total);
}

// compact_stage(mols, xn, atoms, pairs, fa, fb, target_blocks, dst_address, capacity)
// -> None (a molecule exceeds a block) | (copied, (n_mols, n_atoms, n_bonds, n_blocks, nnz_msg, nnz_agg),
//    offsets[6], total): the plan and the upload image written to dst (host memory, e.g. pinned) when it fits
PyObject *compact_stage(PyObject *, PyObject *args) {
    PyObject *o[4];
    int fa, fb, target;
    unsigned long long dst;
    Py_ssize_t cap;
    if (!PyArg_ParseTuple(args, "OOOOiiiKn", &o[0], &o[1], &o[2], &o[3], &fa, &fb, &target, &dst, &cap)) return nullptr;
    try {
        compact::Batch c;
        batch_from(o[0], o[1], o[2], o[3], fa, fb, c);
        compact::Plan p;
        if (!compact::plan(c, target, p)) Py_RETURN_NONE;
        const compact::Staged s = compact::stage_layout(c, p);
        const bool fits = dst && (Py_ssize_t)s.total <= cap;
        if (fits) compact::stage_copy(c, p, s, reinterpret_cast<uint8_t *>(dst));
        return stage_result(c, p, s, fits);
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "compact_stage failed");
    return nullptr;
}

// generate_stage(kind, B, seed, target_blocks, dst_address, capacity) -> as compact_stage, plus the
// generated (mols, xn, atoms, pairs) when keep is set; generation, plan and copy run without the GIL
// (the streaming producer thread, bench.py / chemprop_amd.stream)
PyObject *generate_stage(PyObject *, PyObject *args) {
    int kind, B, target, keep = 0;
    unsigned long long seed, dst;
    Py_ssize_t cap;
    if (!PyArg_ParseTuple(args, "iiKiKn|p", &kind, &B, &seed, &target, &dst, &cap, &keep)) return nullptr;
    if (kind < 0 || kind > 2 || B < 0) {
        PyErr_SetString(PyExc_ValueError, "kind in {0, 1, 2}, B >= 0");
        return nullptr;
    }
    try {
        compact::Batch c;
        compact::Plan p;
        compact::Staged s;
        bool ok = false, fits = false;
        Py_BEGIN_ALLOW_THREADS
        compact::generate(kind, B, seed, c);
        ok = compact::plan(c, target, p);
        if (ok) {
            s = compact::stage_layout(c, p);
            fits = dst && (Py_ssize_t)s.total <= cap;
            if (fits) compact::stage_copy(c, p, s, reinterpret_cast<uint8_t *>(dst));
        }
        Py_END_ALLOW_THREADS
        if (!ok) Py_RETURN_NONE;
        PyObject *r = stage_result(c, p, s, fits);
        if (!r || !keep) return r;
        PyObject *arrays;
        try { arrays = batch_tuple(c); } catch (...) { Py_DECREF(r); throw; }
        PyObject *both = PyTuple_Pack(2, r, arrays);
        Py_DECREF(r);
        Py_DECREF(arrays);
        return both;
    } catch (const PyErrAlready &) {
    } catch (const std::exception &e) {
        PyErr_SetString(PyExc_RuntimeError, e.what());
    }
    if (!PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "generate_stage failed");
    return nullptr;
}

PyMethodDef methods[] = {
    {"pack", pack, METH_VARARGS,
     "pack(mol_graphs, fa_w, fb_w, tail_from=0, check=False) -> 10 bytearrays: the concatenated BatchMolGraph tables "
     "(featurization.py:757-813)"},
    {"gathers", gathers, METH_VARARGS,
     "gathers(b2a, b2revb, w_bonds, deg, in_idx) -> (msg, agg, msg_t, agg_t) CSR gather lists (mpn.py:112-131)"},
    {"ell", ell, METH_VARARGS, "ell(ptr, idx, coef, rows_p, row_base, width) -> block-local ELL rows"},
    {"compact_encode", compact_encode, METH_VARARGS,
     "compact_encode(f_atoms, tail, w_atoms, w_bonds, b2a, b2revb, deg, in_idx, na, nb, xn, fa, tail_w) -> "
     "(mols, xn, atoms, pairs) | (None, reason)"},
    {"compact_decode", compact_decode, METH_VARARGS,
     "compact_decode(mols, xn, atoms, pairs, fa, fb) -> pack()'s outputs in tail mode"},
    {"compact_generate", compact_generate, METH_VARARGS, "compact_generate(kind, B, seed) -> (mols, xn, atoms, pairs)"},
    {"compact_stage", compact_stage, METH_VARARGS,
     "compact_stage(mols, xn, atoms, pairs, fa, fb, target_blocks, dst, capacity) -> plan + upload image"},
    {"generate_stage", generate_stage, METH_VARARGS,
     "generate_stage(kind, B, seed, target_blocks, dst, capacity[, keep]) -> generated batch's plan + upload image"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_wdpack", "native BatchMolGraph packer", -1, methods,
                      nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__wdpack(void) { return PyModule_Create(&module); }
