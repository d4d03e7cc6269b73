"""CPU: the CSR gather lists that the HIP kernels consume reproduce the reference's padded gathers
(mpn.py:104-131) exactly in exact arithmetic, and their transposes are the adjoint gathers used by
the backward pass."""
import numpy as np
import pytest
import torch

import golden_io
from chemprop_amd import synthetic
from chemprop_amd.featurization import BatchMolGraph
from oracle.mpn_ref import index_select_ND

GRAPHS = {
    'polymer': lambda: synthetic.make_batch('polymer', 8, 1),
    'qm9': lambda: synthetic.make_batch('qm9', 16, 2),
    'edge': lambda: synthetic.edge_case_batch(3),
    'zinc': lambda: synthetic.make_batch('zinc', 4, 4),
}


def rand(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape)


@pytest.mark.parametrize('kind', sorted(GRAPHS))
def test_bond_message_gather_matches_padded_formula(kind):
    g = BatchMolGraph(GRAPHS[kind]())
    H = 7
    M = rand((g.n_bonds, H), 0)
    Mt = torch.from_numpy(M)
    a_msg = (index_select_ND(Mt, g.a2b) * index_select_ND(g.w_bonds.double(), g.a2b)[..., None]).sum(dim=1)
    X_ref = (a_msg[g.b2a] - Mt[g.b2revb]).numpy()
    X = g.bond_message_gather().apply(M)
    # coefficients are float32 (w_rev - 1 is rounded once): float32-level agreement; row 0 = pad, unused
    np.testing.assert_allclose(X[1:], X_ref[1:], rtol=1e-6, atol=1e-6 * np.abs(X_ref).max())


@pytest.mark.parametrize('kind', sorted(GRAPHS))
def test_atom_aggregate_gather(kind):
    g = BatchMolGraph(GRAPHS[kind]())
    M = rand((g.n_bonds, 5), 1)
    Mt = torch.from_numpy(M)
    A_ref = (index_select_ND(Mt, g.a2b) * index_select_ND(g.w_bonds.double(), g.a2b)[..., None]).sum(dim=1).numpy()
    np.testing.assert_allclose(g.atom_aggregate_gather(False).apply(M), A_ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('kind', ['polymer', 'qm9', 'edge'])
def test_atom_message_mode_gathers(kind):
    g = BatchMolGraph(GRAPHS[kind]())
    if g.n_atoms > g.n_bonds:
        pytest.skip('atom-message readout indexes w_bonds with atom ids (reference would raise)')
    M = rand((g.n_atoms, 6), 2)
    Mt = torch.from_numpy(M)
    a2a = g.get_a2a()
    msg, feat = g.atom_message_gather()
    np.testing.assert_allclose(msg.apply(M), index_select_ND(Mt, a2a).sum(dim=1).numpy(), rtol=1e-12, atol=1e-12)
    fb = g.f_bonds[:, -14:].double()
    np.testing.assert_allclose(feat.apply(fb.numpy()), index_select_ND(fb, g.a2b).sum(dim=1).numpy(), atol=1e-12)
    A_ref = (index_select_ND(Mt, a2a) * index_select_ND(g.w_bonds.double(), a2a)[..., None]).sum(dim=1).numpy()
    np.testing.assert_allclose(g.atom_aggregate_gather(True).apply(M), A_ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('kind', sorted(GRAPHS))
def test_transposes_are_adjoint(kind):
    g = BatchMolGraph(GRAPHS[kind]())
    for csr, n_src in ((g.bond_message_gather(), g.n_bonds), (g.atom_aggregate_gather(False), g.n_bonds)):
        S = rand((n_src, 3), 3)
        Y = rand((csr.rows, 3), 4)
        lhs = float((csr.apply(S) * Y).sum())
        rhs = float((S * csr.transpose(n_src).apply(Y)).sum())
        assert abs(lhs - rhs) <= 1e-9 * max(1.0, abs(lhs))


def test_empty_molecule_and_hub_degree():
    g = BatchMolGraph(synthetic.edge_case_batch(5, star_leaves=70))
    assert g.max_num_bonds >= 70
    assert (0 in [n for _, n in g.a_scope])
    csr = g.bond_message_gather()
    assert csr.ptr[-1] == len(csr.idx) and np.all(np.diff(csr.ptr) >= 0)


def test_get_b2b_matches_reference_definition():
    g = BatchMolGraph(synthetic.make_batch('polymer', 3, 7))
    b2b = g.get_b2b()
    ref = g.a2b[g.b2a] * (g.a2b[g.b2a] != g.b2revb.unsqueeze(1)).long()
    assert torch.equal(b2b, ref)


@pytest.mark.parametrize('kind', sorted(GRAPHS))
def test_molecule_blocks_cover_molecules_and_contain_their_gathers(kind):
    """WdGraph.blocks (fused forward): consecutive whole molecules, capacity limits respected, every
    bond / atom row in exactly one block, and every gather entry of a row inside the row's block."""
    from chemprop_amd.featurization import BLK_ATOMS, BLK_BONDS
    g = BatchMolGraph(GRAPHS[kind]() if kind != 'edge' else synthetic.edge_case_batch(3, star_leaves=40))
    blocks = g.molecule_blocks()
    assert blocks is not None
    assert blocks[0, 4] == 0 and blocks[-1, 5] == len(g.a_scope)
    assert np.all(blocks[1:, 4] == blocks[:-1, 5])
    assert np.all(blocks[:, 1] <= BLK_BONDS) and np.all(blocks[:, 3] <= BLK_ATOMS)
    for k, (bs, bn, as_, an, ml, mh, _, _) in enumerate(blocks):
        assert bn == sum(n for _, n in g.b_scope[ml:mh]) and an == sum(n for _, n in g.a_scope[ml:mh])
    blk_b = np.full(g.n_bonds, -1)
    for k, (bs, bn) in enumerate(blocks[:, :2]):
        blk_b[bs:bs + bn] = k
    assert np.all(blk_b[1:] >= 0)  # every real bond row in a block
    csr = g.bond_message_gather()
    row = np.repeat(np.arange(csr.rows), np.diff(csr.ptr))
    assert np.array_equal(blk_b[row], blk_b[csr.idx])


def test_molecule_blocks_refuse_an_oversized_molecule():
    g = BatchMolGraph(synthetic.edge_case_batch(5, star_leaves=130))  # 131 atoms > BLK_ATOMS
    assert g.molecule_blocks() is None


@pytest.mark.parametrize('kind', sorted(GRAPHS))
def test_ell_rows_restate_the_gather_lists(kind):
    """The block-local ELL rows (WdGraph.*_ell_*) hold the first ELLW CSR entries of every row (unused
    slots weight 0, bit 7 of the last slot marks longer rows): applying them plus the CSR tail equals
    the CSR."""
    from chemprop_amd.featurization import ELLW, ell_rows
    g = BatchMolGraph(GRAPHS[kind]() if kind != 'edge' else synthetic.edge_case_batch(3, star_leaves=40))
    blocks = g.molecule_blocks()
    bstart = np.zeros(len(blocks) + 1, np.int64)
    bstart[:-1] = blocks[:, 0]
    blk_b = np.full(g.n_bonds, -1)
    for k, (bs, bn) in enumerate(blocks[:, :2]):
        blk_b[bs:bs + bn] = k
    csr = g.bond_message_gather()
    for W in (ELLW, 8, 2):  # the shipped width, and narrow ones so that the tail path is exercised
        check_ell(csr, blk_b, bstart, *ell_rows(csr, csr.rows, bstart[blk_b], W), W)


def check_ell(csr, blk_b, bstart, idx, coef, W):
    idx, coef = idx.reshape(-1, W), coef.reshape(-1, W)
    S = rand((csr.rows, 4), 9)
    out = np.zeros((csr.rows, 4))
    for r in range(1, csr.rows):
        base = bstart[blk_b[r]]
        for k in range(W):
            out[r] += coef[r, k] * S[base + (idx[r, k] & 0x7f)]
        assert bool(idx[r, W - 1] & 0x80) == (csr.ptr[r + 1] - csr.ptr[r] > W)
        for e in range(csr.ptr[r] + W, csr.ptr[r + 1]):
            out[r] += csr.coef[e] * S[csr.idx[e]]
    np.testing.assert_allclose(out[1:], csr.apply(S)[1:], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize('name', golden_io.golden_names())
def test_golden_graphs_gather_lists_consistent(name):
    case = golden_io.load(name)
    for g in case.graphs:
        csr = g.bond_message_gather()
        assert csr.rows == g.n_bonds
        assert np.all(csr.idx >= 0) and np.all(csr.idx < g.n_bonds)


def test_molecule_blocks_cap_the_molecule_count():
    """Empty molecules take no rows; a block still holds at most BLK_MOLS molecules (the readout
    stages one scope per molecule)."""
    from chemprop_amd.featurization import BLK_MOLS
    rng = np.random.default_rng(3)
    mols = [synthetic.empty_graph() for _ in range(150)] + [synthetic.polymer_graph(rng, 3, 5)]
    g = BatchMolGraph(mols)
    blocks = g.molecule_blocks()
    assert blocks is not None and np.all(blocks[:, 5] - blocks[:, 4] <= BLK_MOLS) and len(blocks) >= 3
