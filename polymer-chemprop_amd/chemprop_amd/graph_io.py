"""Pre-featurised MolGraph tables on disk (one ``.npz``, no pickles): the dataset form the training entry
point reads when SMILES featurisation (RDKit) is not available.  One record per CSV row, each holding
the attributes ``BatchMolGraph`` reads from a reference ``MolGraph`` (featurization.py:761-800):
f_atoms, f_bonds, w_atoms, w_bonds, a2b, b2a, b2revb, degree_of_polym.

Layout (concatenated over the records, int64 offsets): ``n_atoms`` / ``n_bonds`` / ``degree_of_polym``
per record; ``f_atoms`` [sum V][atom_fdim], ``w_atoms``; ``f_bonds`` [sum E][bond_fdim], ``w_bonds``,
``b2a`` / ``b2revb`` (molecule-local); ``a2b_len`` per atom + ``a2b`` (molecule-local bond ids).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from .synthetic import SynthMolGraph


def save_graphs(path: str, graphs: Sequence) -> None:
    na = np.array([g.n_atoms for g in graphs], np.int64)
    nb = np.array([g.n_bonds for g in graphs], np.int64)
    fa_w = next((len(g.f_atoms[0]) for g in graphs if g.n_atoms), 0)
    fb_w = next((len(g.f_bonds[0]) for g in graphs if g.n_bonds), 0)

    def cat(rows, width, dtype=np.float32):
        arr = [np.asarray(r, dtype).reshape(-1, width) for r in rows if len(r)]
        return np.concatenate(arr) if arr else np.zeros((0, width), dtype)

    a2b_len = np.array([len(x) for g in graphs for x in g.a2b], np.int64)
    a2b = np.array([j for g in graphs for x in g.a2b for j in x], np.int64)
    np.savez_compressed(
        path, n_atoms=na, n_bonds=nb,
        degree_of_polym=np.array([g.degree_of_polym for g in graphs], np.float64),
        f_atoms=cat([g.f_atoms for g in graphs], fa_w), f_bonds=cat([g.f_bonds for g in graphs], fb_w),
        w_atoms=np.concatenate([np.asarray(g.w_atoms, np.float32) for g in graphs] or [np.zeros(0, np.float32)]),
        w_bonds=np.concatenate([np.asarray(g.w_bonds, np.float32) for g in graphs] or [np.zeros(0, np.float32)]),
        b2a=np.concatenate([np.asarray(g.b2a, np.int64) for g in graphs] or [np.zeros(0, np.int64)]),
        b2revb=np.concatenate([np.asarray(g.b2revb, np.int64) for g in graphs] or [np.zeros(0, np.int64)]),
        a2b_len=a2b_len, a2b=a2b)


def load_graphs(path: str) -> List[SynthMolGraph]:
    d = np.load(path, allow_pickle=False)
    na, nb = d['n_atoms'], d['n_bonds']
    ao = np.concatenate([[0], np.cumsum(na)])
    bo = np.concatenate([[0], np.cumsum(nb)])
    lens = d['a2b_len']
    lo = np.concatenate([[0], np.cumsum(lens)])
    f_atoms, f_bonds = d['f_atoms'], d['f_bonds']
    out = []
    for i in range(len(na)):
        a0, a1, b0, b1 = int(ao[i]), int(ao[i + 1]), int(bo[i]), int(bo[i + 1])
        a2b = [d['a2b'][lo[a]:lo[a + 1]].tolist() for a in range(a0, a1)]
        out.append(SynthMolGraph(f_atoms[a0:a1], f_bonds[b0:b1], d['w_atoms'][a0:a1], d['w_bonds'][b0:b1], a2b,
                                 d['b2a'][b0:b1], d['b2revb'][b0:b1], float(d['degree_of_polym'][i])))
    return out
