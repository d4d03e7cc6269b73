"""A 10-row polymer CSV in the wD-MPNN input format (README.md:13-22) + its pre-featurised graphs, the
workload of BASELINE.json configs[0] (``chemprop_train --polymer`` regression on a 10-row polymer CSV).

Monomer pairs with two attachment points each, monomer fractions, the 10 stochastic rules between the 4
attachment points (incl. self loops) with random weights (the reference's sum-to-1 check never fires,
featurization.py:362), and a degree of polymerisation; graphs from ``chemprop_amd.polymer.synthetic_polymer_graph`` (structure from the string,
synthetic atom / bond features: RDKit is not available).  Targets: a smooth function of the fractions
and Xn plus noise (seeded).  Writes tests/data/polymer10.csv and tests/data/polymer10_graphs.npz.
"""
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
from chemprop_amd.graph_io import save_graphs  # noqa: E402
from chemprop_amd.polymer import synthetic_polymer_graph  # noqa: E402

A = ['[*:1]c1cc(F)c([*:2])cc1F', '[*:1]c1ccc2c(c1)sc1cc([*:2])ccc12', '[*:1]c1cc2ccc3cc([*:2])cc4ccc(c1)c2c34',
     '[*:1]c1ccc([*:2])c2nsnc12', '[*:1]c1cc(Cl)c([*:2])s1']
B = ['[*:3]c1c(O)cc(O)c([*:4])c1O', '[*:3]c1ccc([*:4])cc1', '[*:3]c1ccc2cc([*:4])ccc2c1', '[*:3]C#C[*:4]',
     '[*:3]c1cnc([*:4])cn1']


def rules(p, rng):
    """10 rules over the attachment points 1..4 (i <= j) with random symmetric weights."""
    out = []
    for i in range(1, 5):
        for j in range(i, 5):
            w = round(float(rng.uniform(0.05, 0.5)), 3)
            out.append(f'{i}-{j}:{w}:{w}')
    return '<' + '<'.join(out)


def main():
    rng = np.random.default_rng(2022)
    rows, graphs = [], []
    for k in range(10):
        fa = round(float(rng.choice([0.25, 0.5, 0.75])), 2)
        xn = float(rng.choice([1, 10, 100, 1000]))
        s = f'{A[k % 5]}.{B[(3 * k) % 5]}|{fa}|{round(1 - fa, 2)}|{rules(k, rng)}~{xn:g}'
        y = 1.5 * fa - 0.3 * np.log10(xn) + 0.1 * rng.standard_normal()
        rows.append([s, f'{y:.6f}'])
        graphs.append(synthetic_polymer_graph(s, seed=k))
    out = os.path.join(ROOT, 'tests', 'data')
    with open(os.path.join(out, 'polymer10.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['poly_chemprop_input', 'EA vs SHE (eV)'])
        w.writerows(rows)
    save_graphs(os.path.join(out, 'polymer10_graphs.npz'), graphs)
    print('wrote', len(rows), 'rows')


if __name__ == '__main__':
    main()
