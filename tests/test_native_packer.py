"""CPU: the native BatchMolGraph packer (csrc/packer.cpp) against the numpy
restatement of featurization.py:757-813 (oracle/pack_ref.py) — bit-exact tables and indices — on
list inputs (the reference MolGraph's own representation), numpy inputs, and malformed inputs.
The reference's own packed arrays pin both (test_oracle_golden.py::test_packing_matches_reference)."""
import copy

import numpy as np
import pytest
import torch

from chemprop_amd import synthetic
from chemprop_amd.featurization import BatchMolGraph
from oracle import pack_ref

BATCHES = {
    'polymer': lambda: synthetic.make_batch('polymer', 16, 3),
    'qm9': lambda: synthetic.make_batch('qm9', 32, 4),
    'edge': lambda: synthetic.edge_case_batch(6),
    'zinc': lambda: synthetic.make_batch('zinc', 8, 5),
}


def check(g, ref):
    np.testing.assert_array_equal(g.f_atoms.numpy(), ref['f_atoms'])
    np.testing.assert_array_equal(g.f_bonds.numpy(), ref['f_bonds'])
    np.testing.assert_array_equal(g.w_atoms.numpy(), ref['w_atoms'])
    np.testing.assert_array_equal(g.w_bonds.numpy(), ref['w_bonds'])
    np.testing.assert_array_equal(g.b2a.numpy(), ref['b2a'])
    np.testing.assert_array_equal(g.b2revb.numpy(), ref['b2revb'])
    np.testing.assert_array_equal(g.a2b.numpy(), ref['a2b'])
    assert g.a_scope == ref['a_scope'] and g.b_scope == ref['b_scope']
    assert g.max_num_bonds == ref['max_num_bonds']


@pytest.mark.parametrize('kind', sorted(BATCHES))
def test_native_packer_matches_restatement(kind):
    mgs = BATCHES[kind]()
    check(BatchMolGraph(mgs), pack_ref.pack(mgs))


def test_native_packer_accepts_numpy_and_tuple_inputs():
    mgs = synthetic.make_batch('polymer', 6, 11)
    ref = pack_ref.pack(mgs)
    alt = []
    for i, g in enumerate(mgs):
        h = copy.copy(g)
        if i % 3 == 0:    # whole tables as numpy (float64 / int32)
            h.f_atoms = np.asarray(g.f_atoms, np.float64)
            h.f_bonds = np.asarray(g.f_bonds, np.float32)
            h.b2a = np.asarray(g.b2a, np.int32)
            h.b2revb = np.asarray(g.b2revb, np.int64)
            h.w_bonds = np.asarray(g.w_bonds, np.float64)
            h.a2b = [np.asarray(l, np.int64) for l in g.a2b]
        elif i % 3 == 1:  # tuples of numpy scalars, rows as 1-D arrays
            h.f_atoms = tuple(tuple(np.float32(x) for x in r) for r in g.f_atoms)
            h.f_bonds = [np.asarray(r, np.float64) for r in g.f_bonds]
            h.a2b = tuple(tuple(np.int64(b) for b in l) for l in g.a2b)
            h.w_atoms = tuple(np.float64(w) for w in g.w_atoms)
        alt.append(h)
    check(BatchMolGraph(alt), ref)


def test_native_packer_rejects_malformed_graphs():
    mgs = synthetic.make_batch('qm9', 3, 2)
    bad = copy.copy(mgs[1])
    bad.f_atoms = [list(r) for r in mgs[1].f_atoms]
    bad.f_atoms[2] = bad.f_atoms[2][:-1]
    with pytest.raises(ValueError, match='ragged'):
        BatchMolGraph([mgs[0], bad])
    bad = copy.copy(mgs[1])
    bad.a2b = list(mgs[1].a2b)[:-1]
    with pytest.raises(ValueError, match='a2b'):
        BatchMolGraph([mgs[0], bad])
    bad = copy.copy(mgs[1])
    bad.w_bonds = ['x'] * mgs[1].n_bonds
    with pytest.raises(TypeError):
        BatchMolGraph([bad])
    bad = copy.copy(mgs[1])
    bad.b2a = list(mgs[1].b2a) + [0]
    with pytest.raises(ValueError, match='b2a'):
        BatchMolGraph([bad])


@pytest.mark.parametrize('kind', sorted(BATCHES))
def test_bond_tail_mode_rebuilds_the_same_f_bonds(kind):
    """device_bond_features keeps only the bond-feature tail of f_bonds on the host (the device rebuilds
    f_atoms[b2a] ‖ tail); the host view assembled from it equals the full packing bit for bit."""
    mgs = BATCHES[kind]()
    full = BatchMolGraph(mgs)
    tail = BatchMolGraph(mgs, device_bond_features=True, check_bond_features=True)
    fa_w = full.f_atoms.shape[1]
    np.testing.assert_array_equal(tail._np['bond_tail'], full.f_bonds.numpy()[:, fa_w:])
    np.testing.assert_array_equal(tail.f_bonds.numpy(), full.f_bonds.numpy())
    for a, b in zip(tail.get_components(), full.get_components()):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b)
        else:
            assert a == b


def test_bond_tail_check_rejects_rows_that_are_not_atom_plus_bond():
    mgs = synthetic.make_batch('qm9', 3, 8)
    bad = copy.copy(mgs[1])
    bad.f_bonds = [list(r) for r in mgs[1].f_bonds]
    bad.f_bonds[0][3] += 1.0  # atom part of bond 0 no longer equals f_atoms[b2a[0]]
    with pytest.raises(ValueError, match='source atom'):
        BatchMolGraph([mgs[0], bad], device_bond_features=True, check_bond_features=True)
    BatchMolGraph([mgs[0], bad], device_bond_features=True)  # unchecked: the caller vouches for the layout
    # numpy tables work in tail mode too
    h = copy.copy(mgs[2])
    h.f_bonds = np.asarray(mgs[2].f_bonds, np.float64)
    t = BatchMolGraph([h], device_bond_features=True, check_bond_features=True)
    np.testing.assert_array_equal(t.f_bonds.numpy(), BatchMolGraph([mgs[2]]).f_bonds.numpy())


@pytest.mark.parametrize('kind', sorted(BATCHES))
def test_native_gather_lists_match_restatement(kind):
    """csrc/packer.cpp ``gathers`` / ``ell`` against the numpy restatements (oracle/pack_ref.py): the
    same entries in the same order, bit for bit, including the transposes and the ELL rows."""
    from chemprop_amd.featurization import ELLW, ell_rows
    g = BatchMolGraph(BATCHES[kind]())
    b2a, rev, w = g._np['b2a'], g._np['b2revb'], g._np['w_bonds']
    ref_msg = pack_ref.bond_message_gather(b2a, rev, w, g._deg, g._in_idx)
    ref_agg = pack_ref.atom_aggregate_gather(w, g._deg, g._in_idx)
    msg, agg, msg_t, agg_t = g._native_gathers()
    for got, ref in ((msg, ref_msg), (agg, ref_agg),
                     (msg_t, pack_ref.transpose(*ref_msg, g.n_bonds)), (agg_t, pack_ref.transpose(*ref_agg, g.n_bonds))):
        for a, b in zip((got.ptr, got.idx, got.coef), ref):
            np.testing.assert_array_equal(a, b)
    g2 = BatchMolGraph(BATCHES[kind]() if kind != 'edge' else synthetic.edge_case_batch(3, star_leaves=40))
    blocks = g2.molecule_blocks()
    blk_b = np.full(g2.n_bonds, -1)
    for k, (bs, bn) in enumerate(blocks[:, :2]):
        blk_b[bs:bs + bn] = k
    bstart = np.append(blocks[:, 0], 0).astype(np.int64)
    m2 = g2.bond_message_gather()
    for W in (ELLW, 3):
        a = ell_rows(m2, m2.rows + 5, bstart[blk_b], W)
        b = pack_ref.ell_rows(m2.ptr, m2.idx, m2.coef, m2.rows + 5, bstart[blk_b], W)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
