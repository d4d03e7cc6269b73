"""Polymer input strings (the wD-MPNN input format, README.md:13-22) without RDKit.

``SMILES|f1|f2|...|<i-j:w_ij:w_ji<...~Xn``: monomer SMILES joined by '.', one fraction per monomer,
then the stochastic edge rules between attachment points ``[*:i]`` and an optional degree of
polymerisation.  Restated here (host-side plumbing, no GPU):

* ``split_polymer_string``  data.py:695-703 (``make_mols`` polymer branch) + rdkit.py:31-35 (fragment
  count check of ``make_polymer_mol``);
* ``parse_polymer_rules``    featurization.py:335-364, quirks included: the weight check never fires
  (``np.isclose(...) is False`` is always False) and the last rule string loses its ``~Xn`` suffix in
  place, as in the reference;
* ``fragment_attachments`` / ``count_heavy_atoms``: the ``[*:k]`` attachment labels and heavy-atom
  counts read from the SMILES text (RDKit reads them from the molecule: featurization.py:286-323);
* ``synthetic_polymer_graph``: a MolGraph-shaped graph for a polymer string whose fragment sizes,
  attachment points, monomer fractions (w_atoms, featurization.py:507), rule edges with their weights
  (featurization.py:575-633) and degree of polymerisation follow the string; atom and bond features
  are synthetic (``chemprop_amd.synthetic``), since RDKit featurisation is out of scope here.
"""
from __future__ import annotations

import math
import re
from collections import Counter
from typing import List, Tuple

import numpy as np

from . import synthetic


def split_polymer_string(s: str) -> Tuple[str, List[str], List[str]]:
    """(monomer SMILES, fragment weights, rule strings) as data.py:698-703 splits them; raises the
    ValueError of rdkit.py:31-35 when the fragment and weight counts differ."""
    smiles = s.split('|')[0]
    weights = s.split('|')[1:-1]
    rules = s.split('<')[1:]
    n_frag = len(smiles.split('.'))
    if len(weights) != n_frag:
        raise ValueError(f'number of input monomers/fragments ({n_frag}) does not match number of '
                         f'input number of weights ({len(weights)})')
    return smiles, weights, rules


def parse_polymer_rules(rules: List[str]):
    """featurization.py:335-364: ([(idx1, idx2, w12, w21), ...], 1 + log10(Xn)).  Mutates ``rules[-1]``
    like the reference (drops ``~Xn``)."""
    polymer_info = []
    counter = Counter()
    if '~' in rules[-1]:
        Xn = float(rules[-1].split('~')[1])
        rules[-1] = rules[-1].split('~')[0]
    else:
        Xn = 1.
    for rule in rules:
        if rule == "":
            continue
        if len(rule.split(':')) != 3:
            raise ValueError(f'incorrect format for input information "{rule}"')
        idx1, idx2 = rule.split(':')[0].split('-')
        w12 = float(rule.split(':')[1])
        w21 = float(rule.split(':')[2])
        polymer_info.append((idx1, idx2, w12, w21))
        counter[idx1] += float(w21)
        counter[idx2] += float(w12)
    for k, v in counter.items():
        if np.isclose(v, 1.0) is False:  # never true (np.bool_ is not False): the reference's check is inert
            raise ValueError(f'sum of weights of incoming stochastic edges should be 1 -- found {v} for [*:{k}]')
    return polymer_info, 1. + np.log10(Xn)


_ATTACH = re.compile(r'\[\*:(\d+)\]')
# organic-subset atoms outside brackets (two-letter symbols first), bracket atoms, aromatic atoms
_ATOM = re.compile(r'\[[^\]]*\]|Br|Cl|[BCNOPSFI]|[bcnops]')


def fragment_attachments(smiles: str) -> List[List[str]]:
    """The attachment labels ``[*:k]`` of every monomer (fragment) of a polymer SMILES, in text order."""
    return [_ATTACH.findall(frag) for frag in smiles.split('.')]


def count_heavy_atoms(fragment: str) -> int:
    """Heavy atoms of one fragment's SMILES, wildcards ``*`` / ``[*:k]`` excluded (the R groups that
    ``remove_wildcard_atoms`` drops, featurization.py:325-331)."""
    n = 0
    for tok in _ATOM.findall(fragment):
        if tok.startswith('[') and tok[1:2] == '*':
            continue
        n += 1
    return n


def synthetic_polymer_graph(s: str, seed: int) -> synthetic.SynthMolGraph:
    """A MolGraph-shaped graph of polymer string ``s`` (see the module docstring)."""
    smiles, weights, rules = split_polymer_string(s)
    info, degree_of_polym = parse_polymer_rules(list(rules))
    frags = smiles.split('.')
    attach = fragment_attachments(smiles)
    rng = np.random.default_rng(seed)
    sizes = [max(1, count_heavy_atoms(f)) for f in frags]
    offsets = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(int)
    pairs = set()
    for off, n in zip(offsets, sizes):
        pairs |= synthetic._skeleton(rng, int(n), int(off))
    # attachment atom of label k: a distinct atom of the fragment that carries [*:k]
    where = {}
    for f, (off, n, labels) in enumerate(zip(offsets, sizes, attach)):
        picks = rng.choice(n, size=min(n, len(labels)), replace=False) if labels else []
        for lab, a in zip(labels, picks):
            where[lab] = int(off + a)
        for lab in labels[len(picks):]:  # more labels than atoms: share atoms
            where[lab] = int(off + rng.integers(0, n))
    rule_pairs = []
    for idx1, idx2, w12, w21 in info:
        if idx1 not in where or idx2 not in where:
            raise ValueError(f'cannot find atom attached to [*:{idx1 if idx1 not in where else idx2}]')
        rule_pairs.append((where[idx1], where[idx2], float(w12), float(w21)))
    w_atoms = [float(w) for w, n in zip(weights, sizes) for _ in range(n)]
    return synthetic._build(rng, int(sum(sizes)), pairs, rule_pairs, w_atoms, float(degree_of_polym))


def degree_from_xn(xn: float) -> float:
    """featurization.py:364: degree_of_polym = 1 + log10(Xn)."""
    return 1.0 + math.log10(xn)
