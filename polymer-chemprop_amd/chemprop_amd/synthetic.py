"""Seeded synthetic featurised graphs with the shape of the reference's MolGraph.

RDKit is not available in this image, so SMILES -> graph featurisation cannot run.  The hot path
consumes *featurised* graphs, so benchmarks and parity tests use graphs built here.  Each object is
duck-typed to the attributes ``BatchMolGraph.__init__`` reads from a reference ``MolGraph``
(``chemprop/features/featurization.py:761-800``): ``f_atoms, f_bonds, w_atoms, w_bonds, a2b, b2a,
b2revb, n_atoms, n_bonds, degree_of_polym, overwrite_default_atom_features,
overwrite_default_bond_features``.

Bond enumeration follows ``MolGraph.__init__``:

* intra-monomer bonds in ``(a1 < a2)`` pair order (``featurization.py:530-560``): bond ``b1 = a1->a2``
  goes to ``a2b[a2]``, ``b2 = a2->a1`` to ``a2b[a1]``, ``f_bonds[b1] = f_atoms[a1] + f_bond``;
* then one directed pair per polymer rule ``(r1, r2, w12, w21)`` in rule order
  (``featurization.py:576-633``), weights ``[w12, w21]``.  A rule ``i-i`` yields a self-loop pair
  (``a1 == a2``), as the reference does.

Generator parameters follow SURVEY.md §8(d): polymer = 2 monomers x U{10..24} heavy atoms (chain +
floor(n/5) ring closures), 2 attachment atoms per monomer, 10 stochastic rules (all i<=j pairs of the
4 attachment points, incl. self loops) with w ~ U[0.1, 0.5], monomer fractions ~ Dirichlet(1, 1),
Xn ~ U[1, 1000] -> degree_of_polym = 1 + log10(Xn) (``featurization.py:340-364``).
"""
from __future__ import annotations

import math
from typing import List, Optional

import numpy as np

# Feature sizes of the reference's default featurisation (featurization.py:19-45).
ATOM_FEATURE_CHOICES = (100, 6, 5, 4, 5, 5)  # atomic_num, degree, charge, chiral, num_Hs, hybridization
ATOM_FDIM = sum(c + 1 for c in ATOM_FEATURE_CHOICES) + 2  # 133
BOND_FDIM_ONLY = 14
BOND_FDIM = ATOM_FDIM + BOND_FDIM_ONLY  # 147


class SynthMolGraph:
    """A featurised graph with the public attributes of the reference ``MolGraph``."""

    def __init__(self, f_atoms, f_bonds, w_atoms, w_bonds, a2b, b2a, b2revb, degree_of_polym=1.0):
        self.f_atoms = f_atoms
        self.f_bonds = f_bonds
        self.w_atoms = w_atoms
        self.w_bonds = w_bonds
        self.a2b = a2b
        self.b2a = b2a
        self.b2revb = b2revb
        self.n_atoms = len(f_atoms)
        self.n_bonds = len(f_bonds)
        self.degree_of_polym = degree_of_polym
        self.overwrite_default_atom_features = False
        self.overwrite_default_bond_features = False
        self.is_polymer = degree_of_polym != 1.0


def _atom_feature(rng: np.random.Generator, degree: int) -> List[float]:
    """One atom vector laid out as ``atom_features`` (featurization.py:190-211)."""
    vec: List[float] = []
    for i, n in enumerate(ATOM_FEATURE_CHOICES):
        onehot = [0.0] * (n + 1)
        if i == 0:
            onehot[int(rng.choice([5, 6, 7, 8, 15, 16, 8, 5]))] = 1.0  # C, N, O, F, S, Cl-ish
        elif i == 1:
            onehot[min(degree, n)] = 1.0
        else:
            onehot[int(rng.integers(0, n + 1))] = 1.0
        vec.extend(onehot)
    vec.append(float(rng.integers(0, 2)))              # aromatic
    vec.append(float(rng.uniform(10.0, 40.0)) * 0.01)  # mass * 0.01
    return vec


def _bond_feature(rng: np.random.Generator) -> List[float]:
    """One bond vector laid out as ``bond_features`` (featurization.py:229-250)."""
    fb = [0.0] * BOND_FDIM_ONLY
    fb[1 + int(rng.integers(0, 4))] = 1.0  # bond type
    fb[5] = float(rng.integers(0, 2))      # conjugated
    fb[6] = float(rng.integers(0, 2))      # in ring
    fb[7 + int(rng.integers(0, 7))] = 1.0  # stereo one-hot (6 + unk)
    return fb


def _skeleton(rng: np.random.Generator, n: int, offset: int = 0):
    """Chain plus floor(n/5) ring closures, as (a1 < a2) undirected pairs."""
    edges = {(offset + i, offset + i + 1) for i in range(n - 1)}
    for _ in range(n // 5):
        if n < 4:
            break
        i = int(rng.integers(0, n - 3))
        j = int(rng.integers(i + 3, n))
        edges.add((offset + i, offset + j))
    return edges


def _build(rng, n_atoms, undirected_pairs, rule_pairs, w_atoms, xn_degree, star_degree=None):
    degree = [0] * n_atoms
    for a1, a2 in undirected_pairs:
        degree[a1] += 1
        degree[a2] += 1
    f_atoms = [_atom_feature(rng, d) for d in degree]
    f_bonds, w_bonds, b2a, b2revb = [], [], [], []
    a2b: List[List[int]] = [[] for _ in range(n_atoms)]
    n_bonds = 0

    def add(a1, a2, w12, w21):
        nonlocal n_bonds
        fb = _bond_feature(rng)
        f_bonds.append(f_atoms[a1] + fb)
        f_bonds.append(f_atoms[a2] + fb)
        b1, b2 = n_bonds, n_bonds + 1
        a2b[a2].append(b1)
        b2a.append(a1)
        a2b[a1].append(b2)
        b2a.append(a2)
        b2revb.append(b2)
        b2revb.append(b1)
        w_bonds.extend([w12, w21])
        n_bonds += 2

    for a1, a2 in sorted(undirected_pairs):  # (a1 < a2) enumeration order of MolGraph
        add(a1, a2, 1.0, 1.0)
    for a1, a2, w12, w21 in rule_pairs:
        add(a1, a2, w12, w21)
    return SynthMolGraph(f_atoms, f_bonds, list(w_atoms), w_bonds, a2b, b2a, b2revb, xn_degree)


def polymer_graph(rng: np.random.Generator, min_atoms: int = 10, max_atoms: int = 24) -> SynthMolGraph:
    """A 2-monomer stochastic copolymer graph (SURVEY.md §8(d) 'Polymer')."""
    na = int(rng.integers(min_atoms, max_atoms + 1))
    nb = int(rng.integers(min_atoms, max_atoms + 1))
    pairs = _skeleton(rng, na, 0) | _skeleton(rng, nb, na)
    # attachment atoms: 2 distinct per monomer -> R1, R2 on A; R3, R4 on B
    ra = rng.choice(na, size=2, replace=False)
    rb = rng.choice(nb, size=2, replace=False) + na
    attach = [int(ra[0]), int(ra[1]), int(rb[0]), int(rb[1])]
    rules = []
    for i in range(4):
        for j in range(i, 4):
            rules.append((attach[i], attach[j], float(rng.uniform(0.1, 0.5)), float(rng.uniform(0.1, 0.5))))
    frac = rng.dirichlet([1.0, 1.0])
    w_atoms = [float(frac[0])] * na + [float(frac[1])] * nb
    xn = float(rng.uniform(1.0, 1000.0))
    return _build(rng, na + nb, pairs, rules, w_atoms, 1.0 + math.log10(xn))


def molecule_graph(rng: np.random.Generator, min_atoms: int, max_atoms: int) -> SynthMolGraph:
    """A plain (non-polymer) molecule: unit weights, degree_of_polym 1 (QM9-like / ZINC-like)."""
    n = int(rng.integers(min_atoms, max_atoms + 1))
    pairs = _skeleton(rng, n, 0)
    return _build(rng, n, pairs, [], [1.0] * n, 1.0)


def star_graph(rng: np.random.Generator, n_leaves: int) -> SynthMolGraph:
    """A hub with ``n_leaves`` neighbours: in-degree far above one wavefront (edge case)."""
    pairs = {(0, i) for i in range(1, n_leaves + 1)}
    return _build(rng, n_leaves + 1, pairs, [], [1.0] * (n_leaves + 1), 1.0)


def single_atom_graph(rng: np.random.Generator) -> SynthMolGraph:
    return _build(rng, 1, set(), [], [1.0], 1.0)


def empty_graph() -> SynthMolGraph:
    return SynthMolGraph([], [], [], [], [], [], [], 1.0)


def make_batch(kind: str, batch_size: int, seed: int) -> List[SynthMolGraph]:
    """``kind`` in {'polymer', 'qm9', 'zinc'}: the workloads of BASELINE.json ``configs``."""
    rng = np.random.default_rng(seed)
    if kind == 'polymer':
        return [polymer_graph(rng) for _ in range(batch_size)]
    if kind == 'qm9':
        return [molecule_graph(rng, 5, 9) for _ in range(batch_size)]
    if kind == 'zinc':
        return [molecule_graph(rng, 15, 37) for _ in range(batch_size)]
    raise ValueError(f'unknown synthetic kind {kind!r}')


def edge_case_batch(seed: int, star_leaves: int = 70) -> List[SynthMolGraph]:
    """Empty molecule, single atom, a hub of degree > 64, and two polymers."""
    rng = np.random.default_rng(seed)
    return [polymer_graph(rng, 4, 6), empty_graph(), single_atom_graph(rng),
            star_graph(rng, star_leaves), polymer_graph(rng, 3, 5)]


def synthetic_parameter(name: str, shape, seed: int) -> np.ndarray:
    """Deterministic values for one parameter, keyed by its state_dict name (golden fixtures).

    >=2-D tensors get xavier-normal scale (the reference's ``initialize_weights``,
    ``nn_utils.py:102-112``); 1-D tensors (biases, PReLU slope, ``cached_zero_vector``) get
    U(-0.5, 0.5) instead of the reference's zeros so that the bias / PReLU / empty-molecule
    paths are exercised by the goldens.
    """
    import zlib
    rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
    shape = tuple(int(s) for s in shape)
    if len(shape) >= 2:
        fan_out, fan_in = shape[0], int(np.prod(shape[1:]))
        std = math.sqrt(2.0 / (fan_in + fan_out))
        return (rng.standard_normal(shape) * std).astype(np.float32)
    return rng.uniform(-0.5, 0.5, size=shape).astype(np.float32)


def fill_parameters(module, seed: int) -> None:
    """Overwrite every parameter of ``module`` with :func:`synthetic_parameter` values."""
    import torch
    with torch.no_grad():
        for name, p in module.named_parameters():
            p.copy_(torch.from_numpy(synthetic_parameter(name, p.shape, seed)))


def random_descriptors(graphs: List[SynthMolGraph], size: int, seed: int) -> List[np.ndarray]:
    """Per-molecule atom descriptor arrays for ``--atom_descriptors descriptor`` (mpn.py:77-79)."""
    rng = np.random.default_rng(seed)
    return [rng.standard_normal((g.n_atoms, size)).astype(np.float32) for g in graphs]
