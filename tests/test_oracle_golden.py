"""CPU: pin the oracle (oracle/mpn_ref.py) and the host packing against the REAL reference's outputs
stored in tests/golden/ (tools/make_goldens.py), and check that chemprop_amd modules have the
reference's parameter names (state_dict compatibility)."""
import numpy as np
import pytest
import torch

import golden_io
from chemprop_amd import synthetic
from chemprop_amd.featurization import get_atom_fdim, get_bond_fdim
from chemprop_amd.model import MoleculeModel
from chemprop_amd.mpn import MPNEncoder
from oracle import mpn_ref

NAMES = golden_io.golden_names()
TOL = 1e-5  # max|out - ref| <= 1e-5 * max|ref| per tensor


def build_module(case):
    a = case.args
    if case.level == 'encoder':
        return MPNEncoder(a, get_atom_fdim(), get_bond_fdim(atom_messages=a.atom_messages))
    return MoleculeModel(a)


def oracle_run(case, module):
    p = {n: t.detach().clone().requires_grad_(t.requires_grad) for n, t in module.named_parameters()}
    if case.level == 'encoder':
        out = mpn_ref.encoder_forward(p, case.graphs[0], case.args, case.desc)
    else:
        out = mpn_ref.model_forward(p, case.graphs, case.args, case.features)
    return p, out


def test_goldens_present():
    assert len(NAMES) >= 10


@pytest.mark.parametrize('name', NAMES)
def test_packing_matches_reference(name):
    case = golden_io.load(name)
    for g, ref in zip(case.graphs, case.packed):
        assert g.max_num_bonds == int(ref['max_num_bonds'])
        np.testing.assert_array_equal(g.a2b.numpy(), ref['a2b'])
        np.testing.assert_array_equal(g.b2a.numpy(), ref['b2a'])
        np.testing.assert_array_equal(g.b2revb.numpy(), ref['b2revb'])
        np.testing.assert_array_equal(np.array(g.a_scope, np.int64).reshape(-1, 2), ref['a_scope'])
        np.testing.assert_array_equal(np.array(g.b_scope, np.int64).reshape(-1, 2), ref['b_scope'])


@pytest.mark.parametrize('name', NAMES)
def test_parameter_names_match_reference(name):
    case = golden_io.load(name)
    module = build_module(case)
    assert [n for n, _ in module.named_parameters()] == case.param_names


@pytest.mark.parametrize('name', NAMES)
def test_oracle_matches_reference(name):
    case = golden_io.load(name)
    module = build_module(case)
    synthetic.fill_parameters(module, case.seed)
    module.eval()
    p, out = oracle_run(case, module)
    assert out.shape == case.output.shape
    assert golden_io.normwise(out.detach().numpy(), case.output) <= TOL
    if case.R is not None:
        (out * torch.from_numpy(case.R)).sum().backward()
        for n, g in case.grads.items():
            assert p[n].grad is not None, n
            err = golden_io.normwise(p[n].grad.numpy(), g)
            assert err <= TOL, (n, err)
