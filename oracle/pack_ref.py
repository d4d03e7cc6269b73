"""Test infrastructure (CPU checker, never imported by chemprop_amd): a numpy restatement of the
reference's BatchMolGraph concatenation (featurization.py:757-813) — pad row 0 in every table
(:767-781), atom ids offset by 1 + atoms before the molecule, bond ids by 1 + bonds before it
(:788-793), a2b padded with 0 to max(1, max in-degree) (:802-809).  The native packer
(csrc/packer.cpp) is checked against it on random inputs; both are checked against the arrays the
real reference produced (tests/golden, test_oracle_golden.py)."""
import numpy as np


def pack(mol_graphs):
    na = np.array([g.n_atoms for g in mol_graphs], np.int64)
    nb = np.array([g.n_bonds for g in mol_graphs], np.int64)
    a_off = 1 + np.concatenate([[0], np.cumsum(na)[:-1]]).astype(np.int64)
    b_off = 1 + np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64)
    fa_w = next(len(g.f_atoms[0]) for g in mol_graphs if g.n_atoms)
    fb_w = next((len(g.f_bonds[0]) for g in mol_graphs if g.n_bonds), 0)

    def stack(name, width, dtype):
        parts = [np.asarray(getattr(g, name), dtype).reshape(-1, width) for g in mol_graphs]
        return np.concatenate([np.zeros((1, width), dtype)] + parts)

    a2b_rows = [[0]]
    for g, bo in zip(mol_graphs, b_off):
        a2b_rows += [[int(b) + int(bo) for b in l] for l in g.a2b]
    max_nb = max(1, max(len(r) for r in a2b_rows[1:]) if len(a2b_rows) > 1 else 0)
    a2b_rows[0] = []
    a2b = np.array([r + [0] * (max_nb - len(r)) for r in a2b_rows], np.int64)
    return dict(
        f_atoms=stack('f_atoms', fa_w, np.float32),
        f_bonds=stack('f_bonds', fb_w, np.float32),
        w_atoms=np.concatenate([[0.0]] + [np.asarray(g.w_atoms, np.float64) for g in mol_graphs]).astype(np.float32),
        w_bonds=np.concatenate([[0.0]] + [np.asarray(g.w_bonds, np.float64) for g in mol_graphs]).astype(np.float32),
        b2a=np.concatenate([[0]] + [np.asarray(g.b2a, np.int64).reshape(-1) + o for g, o in zip(mol_graphs, a_off)]),
        b2revb=np.concatenate([[0]] + [np.asarray(g.b2revb, np.int64).reshape(-1) + o for g, o in zip(mol_graphs, b_off)]),
        a2b=a2b,
        a_scope=[(int(s), int(n)) for s, n in zip(a_off, na)],
        b_scope=[(int(s), int(n)) for s, n in zip(b_off, nb)],
        max_num_bonds=max_nb,
    )


# ---------------------------------------------------------------------------------------------
# Gather lists (mpn.py:112-131 as row gathers), numpy restatements of the native packer's
# ``gathers`` / ``ell`` (csrc/packer.cpp), checked bit for bit in tests/test_native_packer.py.
# ---------------------------------------------------------------------------------------------
def _from_rows(row_of_entry, idx, coef, n_rows):
    order = np.argsort(row_of_entry, kind='stable')
    ptr = np.zeros(n_rows + 1, np.int64)
    np.cumsum(np.bincount(row_of_entry, minlength=n_rows), out=ptr[1:])
    return ptr.astype(np.int32), idx[order].astype(np.int32), coef[order].astype(np.float32)


def _entries_of_in(in_ptr, in_idx, deg, atoms):
    counts = deg[atoms]
    rows = np.repeat(np.arange(len(atoms), dtype=np.int64), counts)
    starts = np.repeat(in_ptr[atoms], counts)
    slot = np.arange(len(rows), dtype=np.int64) - np.repeat(np.cumsum(counts) - counts, counts)
    return rows, in_idx[starts + slot]


def bond_message_gather(b2a, rev, w, deg, in_idx):
    """X_b = sum_{j in in(b2a[b])} w_j M_j - M_rev(b) (mpn.py:112-120): the reverse bond's coefficient
    becomes w_rev - 1 (dropped when 0), or an explicit -1 entry when it is not an in-bond."""
    E1 = len(b2a)
    in_ptr = np.concatenate([[0], np.cumsum(deg)])
    bonds = np.arange(1, E1, dtype=np.int64)
    rows, j = _entries_of_in(in_ptr, in_idx, deg, b2a[bonds])
    rows = bonds[rows]
    coef = w[j].astype(np.float64)
    is_rev = j == rev[rows]
    coef[is_rev] -= 1.0
    has_rev = np.zeros(E1, bool)
    has_rev[rows[is_rev]] = True
    missing = bonds[~has_rev[bonds]]
    rows = np.concatenate([rows, missing])
    j = np.concatenate([j, rev[missing]])
    coef = np.concatenate([coef, -np.ones(len(missing))])
    keep = coef != 0.0
    return _from_rows(rows[keep], j[keep], coef[keep], E1)


def atom_aggregate_gather(w, deg, in_idx):
    """A_a = sum_{j in in(a)} w_j M_j (mpn.py:126-131), zero weights dropped."""
    V1 = len(deg)
    in_ptr = np.concatenate([[0], np.cumsum(deg)])
    rows, j = _entries_of_in(in_ptr, in_idx, deg, np.arange(V1, dtype=np.int64))
    coef = w[j]
    keep = coef != 0.0
    return _from_rows(rows[keep], j[keep], coef[keep], V1)


def transpose(ptr, idx, coef, n_src):
    rows = np.repeat(np.arange(len(ptr) - 1, dtype=np.int64), np.diff(ptr))
    return _from_rows(idx.astype(np.int64), rows, coef, n_src)


def ell_rows(ptr, idx, coef, rows_p, base, width):
    n = len(ptr) - 1
    eidx = np.zeros((rows_p, width), np.uint8)
    ecoef = np.zeros((rows_p, width), np.float32)
    cnt = np.diff(ptr)
    row = np.repeat(np.arange(n), cnt)
    slot = np.arange(len(row)) - np.repeat(ptr[:-1], cnt)
    keep = slot < width
    local = idx[:len(row)].astype(np.int64) - base[row]
    eidx[row[keep], slot[keep]] = local[keep].astype(np.uint8)
    ecoef[row[keep], slot[keep]] = coef[:len(row)][keep]
    eidx[:n, width - 1] |= np.where(cnt > width, 0x80, 0).astype(np.uint8)
    return eidx.reshape(-1), ecoef.reshape(-1)
