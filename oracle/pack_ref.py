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
