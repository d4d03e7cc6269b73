"""Golden vectors for the host-side plumbing of the training entry point (chemprop_amd.cli, .polymer),
produced by the REAL reference functions loaded from /root/reference (build container only):

* parse_polymer_rules (featurization.py:335-364) on polymer rule strings -> polymer_info, degree;
* split_data(split_type='random') (data/utils.py:392-549) on row indices -> train / val / test;
* StandardScaler (data/scaler.py:6-63) fit / transform / inverse_transform with missing targets;
* NoamLR (nn_utils.py:115-194) learning-rate sequences, including steps_per_epoch = 0.

Writes tests/golden/host_plumbing.json.  Run: PYTHONDONTWRITEBYTECODE=1 python tools/make_host_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ref_loader  # noqa: E402

STRINGS = [
    '[*:1]c1cc(F)c([*:2])cc1F.[*:3]c1c(O)cc(O)c([*:4])c1O|0.5|0.5|<1-3:0.25:0.25<1-4:0.25:0.25<2-3:0.25:0.25'
    '<2-4:0.25:0.25<1-2:0.25:0.25<3-4:0.25:0.25<1-1:0.25:0.25<2-2:0.25:0.25<3-3:0.25:0.25<4-4:0.25:0.25~100',
    'CC([*:1])C.c1cnccc1CC[*:2]|0.2|0.8|<1-2:1:1',
    '[*:1]CC[*:2].[*:3]c1ccc([*:4])cc1|0.75|0.25|<1-3:0.5:0.5<2-4:0.5:0.5~3.5',
    '[*:1]C(=O)O[*:2]|1|<1-2:0.5:0.5<1-1:0.5:0.5<2-2:0.5:0.5~1',
    '[*:1]C[*:2].[*:3]N[*:4]|0.4|0.6|<1-3:0.3:0.7<2-4:0.7:0.3~1000',
    'CCO|1|',
]


def load_utils(ref):
    """chemprop/data/utils.py and scaler.py under stub parents (its other imports are not used by the
    random split)."""
    data_pkg = types.ModuleType('chemprop.data')
    data_pkg.__path__ = []
    sys.modules['chemprop.data'] = data_pkg
    dd = types.ModuleType('chemprop.data.data')
    dd.MoleculeDatapoint = object
    dd.MoleculeDataset = list  # split_data wraps index lists: a plain list keeps them
    sys.modules['chemprop.data.data'] = dd
    sc = types.ModuleType('chemprop.data.scaffold')
    sc.log_scaffold_stats = sc.scaffold_split = None
    sys.modules['chemprop.data.scaffold'] = sc
    sys.modules['chemprop.args'].PredictArgs = object
    feats = sys.modules['chemprop.features']
    feats.load_features = feats.load_valid_atom_or_bond_features = None
    utils = ref_loader._load('chemprop.data.utils', 'chemprop/data/utils.py')
    scaler = ref_loader._load('chemprop.data.scaler', 'chemprop/data/scaler.py')
    return utils, scaler


def main():
    ref = ref_loader.load_reference()
    utils, scaler_mod = load_utils(ref)
    out = {'polymer_rules': [], 'split': [], 'scaler': [], 'noam': []}
    for s in STRINGS:
        rules = s.split('<')[1:]
        if not rules:
            continue
        info, deg = ref.featurization.parse_polymer_rules(list(rules))
        out['polymer_rules'].append({'string': s, 'rules': rules, 'info': [list(x) for x in info], 'degree': float(deg)})
    for n, sizes, seed in ((10, (0.8, 0.1, 0.1), 0), (10, (0.8, 0.1, 0.1), 3), (37, (0.7, 0.15, 0.15), 1),
                           (200, (0.8, 0.1, 0.1), 0), (5, (0.6, 0.2, 0.2), 7), (10, (0.7, 0.2, 0.1), 0)):
        try:
            tr, va, te = utils.split_data(list(range(n)), split_type='random', sizes=sizes, seed=seed)
        except ValueError:  # sum(sizes) != 1 in floating point (0.7 + 0.2 + 0.1): the reference refuses
            out['split'].append({'n': n, 'sizes': sizes, 'seed': seed, 'raises': True})
            continue
        out['split'].append({'n': n, 'sizes': sizes, 'seed': seed, 'train': list(tr), 'val': list(va), 'test': list(te)})
    rng = np.random.default_rng(0)
    for rows, tasks in ((8, 1), (10, 3)):
        X = rng.standard_normal((rows, tasks)).round(6).tolist()
        X[1][0] = None
        if tasks > 1:
            X[2][1] = None
            for r in X:
                r[2] = 1.5 if r[2] is not None else None  # constant column: std 0 -> 1
        sc = scaler_mod.StandardScaler(replace_nan_token=None).fit(X)
        out['scaler'].append({'X': X, 'means': sc.means.tolist(), 'stds': sc.stds.tolist(),
                              'transform': [[None if v is None else float(v) for v in r] for r in sc.transform(X).tolist()],
                              'inverse': sc.inverse_transform([[0.5] * tasks, [-1.0] * tasks]).tolist()})
    for warm, total, spe in ((2.0, 30, 1), (2.0, 5, 4), (0.5, 3, 10), (2.0, 30, 0)):
        opt = torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))], lr=1e-4)
        with np.errstate(all='ignore'):
            sch = ref.nn_utils.NoamLR(opt, warmup_epochs=[warm], total_epochs=[total], steps_per_epoch=spe,
                                      init_lr=[1e-4], max_lr=[1e-3], final_lr=[1e-4])
            lrs = []
            for _ in range(max(1, total * spe) + 3):
                sch.step()
                lrs.append(float(opt.param_groups[0]['lr']))
        out['noam'].append({'warmup_epochs': warm, 'total_epochs': total, 'steps_per_epoch': spe, 'lrs': lrs})
    path = os.path.join(ROOT, 'tests', 'golden', 'host_plumbing.json')
    with open(path, 'w') as f:
        json.dump(out, f, indent=1)
    print('wrote', path, {k: len(v) for k, v in out.items()})


if __name__ == '__main__':
    main()
