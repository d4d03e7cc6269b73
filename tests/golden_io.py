"""Load the committed golden fixtures (tests/golden/*.npz, made by tools/make_goldens.py from the
real reference) into chemprop_amd objects."""
from __future__ import annotations

import glob
import json
import os
import types

import numpy as np
import torch

from chemprop_amd import synthetic
from chemprop_amd.featurization import BatchMolGraph

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def golden_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, '*.npz')))


def normwise(a, b):
    """max|a-b| / max|b| (the parity metric of SURVEY.md §8(c))."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = max(float(np.abs(b).max()) if b.size else 0.0, 1e-30)
    return float(np.abs(a - b).max()) / den if b.size else 0.0


def _mols(z, prefix):
    na, nb = z[f'{prefix}n_atoms'], z[f'{prefix}n_bonds']
    fa, fb = z[f'{prefix}f_atoms'], z[f'{prefix}f_bonds']
    wa, wb = z[f'{prefix}w_atoms'], z[f'{prefix}w_bonds']
    b2a, rev = z[f'{prefix}b2a'], z[f'{prefix}b2revb']
    a2b_len, a2b_idx = z[f'{prefix}a2b_len'], z[f'{prefix}a2b_idx']
    dp = z[f'{prefix}degree_of_polym']
    mols, ao, bo, lo, io = [], 0, 0, 0, 0
    for k in range(len(na)):
        n, m = int(na[k]), int(nb[k])
        a2b = []
        for a in range(n):
            L = int(a2b_len[lo + a])
            a2b.append([int(x) for x in a2b_idx[io:io + L]])
            io += L
        lo += n
        g = synthetic.SynthMolGraph(fa[ao:ao + n].tolist(), fb[bo:bo + m].tolist(), wa[ao:ao + n].tolist(),
                                    wb[bo:bo + m].tolist(), a2b, b2a[bo:bo + m].tolist(), rev[bo:bo + m].tolist(),
                                    float(dp[k]))
        mols.append(g)
        ao += n
        bo += m
    return mols


def load(name):
    z = np.load(os.path.join(GOLDEN_DIR, f'{name}.npz'), allow_pickle=False)
    cfg = json.loads(str(z['config']))
    args = types.SimpleNamespace(**cfg)
    args.device = torch.device('cpu')
    seed = int(z['param_seed'])
    n_slots = int(z['n_slots'])
    mol_lists = [_mols(z, f's{s}_mol_') for s in range(n_slots)]
    graphs = [BatchMolGraph(m) for m in mol_lists]
    packed = [{k: z[f's{s}_{k}'] for k in ('a2b', 'b2a', 'b2revb', 'a_scope', 'b_scope', 'max_num_bonds')}
              for s in range(n_slots)]
    names = json.loads(str(z['param_names']))
    grads = {k[len('grad/'):]: z[k] for k in z.files if k.startswith('grad/')}
    desc = None
    if 'descriptors' in z.files:
        d = z['descriptors']
        desc, o = [], 0
        for g in mol_lists[0]:
            desc.append(d[o:o + g.n_atoms])
            o += g.n_atoms
    features = [f for f in z['features']] if 'features' in z.files else None
    return types.SimpleNamespace(name=name, args=args, seed=seed, level=str(z['level']), mol_lists=mol_lists,
                                 graphs=graphs, packed=packed, param_names=names, output=z['output'],
                                 R=z['R'] if 'R' in z.files else None, grads=grads, desc=desc, features=features)


def param_value(name, shape, seed):
    return torch.from_numpy(synthetic.synthetic_parameter(name, shape, seed))
