"""GPU: the HIP path (libwdmpnn.so through chemprop_amd) against the reference goldens and the oracle.

Parity bar (north_star): fp32, max|out - ref| <= 1e-5 * max|ref| per tensor, for the
encoder output and every parameter gradient.
"""
import numpy as np
import pytest
import torch

import golden_io
from chemprop_amd import TrainArgs, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim
from chemprop_amd.model import MoleculeModel
from chemprop_amd.mpn import MPNEncoder
from chemprop_amd.nn_utils import index_select_ND
from oracle import mpn_ref

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = torch.device('cuda:0')


def loaded_libs():
    with open('/proc/self/maps') as f:
        return f.read()


def test_native_library_is_the_code_that_runs():
    enc = MPNEncoder(TrainArgs(hidden_size=32), get_atom_fdim(), get_bond_fdim()).to(DEV)
    enc(BatchMolGraph(synthetic.make_batch('polymer', 2, 0)))
    torch.cuda.synchronize()
    assert 'libwdmpnn.so' in loaded_libs()


def run_case(case, grads=True):
    a = case.args
    a.device = DEV
    if case.level == 'encoder':
        m = MPNEncoder(a, get_atom_fdim(), get_bond_fdim(atom_messages=a.atom_messages))
    else:
        m = MoleculeModel(a)
    synthetic.fill_parameters(m, case.seed)
    m = m.to(DEV).eval()
    out = m(case.graphs[0], case.desc) if case.level == 'encoder' else m(case.graphs, case.features)
    g = {}
    if grads and case.R is not None:
        (out * torch.from_numpy(case.R).to(DEV)).sum().backward()
        g = {n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters() if p.grad is not None}
    return out.detach().cpu().numpy(), g


@pytest.mark.parametrize('name', golden_io.golden_names())
def test_golden_forward_and_gradients(name):
    case = golden_io.load(name)
    out, grads = run_case(case)
    assert out.shape == case.output.shape
    err = golden_io.normwise(out, case.output)
    assert err <= TOL, err
    for n, ref in case.grads.items():
        assert n in grads, f'missing gradient {n}'
        e = golden_io.normwise(grads[n], ref)
        assert e <= TOL, (n, e)


def _oracle_vs_hip(graphs, args, seed, desc=None):
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=args.atom_messages))
    synthetic.fill_parameters(enc, seed)
    p = {n: t.detach().clone().requires_grad_(t.requires_grad) for n, t in enc.named_parameters()}
    ref = mpn_ref.encoder_forward(p, graphs, args, desc)
    enc = enc.to(DEV)
    out = enc(graphs, desc)
    R = torch.randn(ref.shape, generator=torch.Generator().manual_seed(seed))
    (ref * R).sum().backward()
    (out * R.to(DEV)).sum().backward()
    res = {'output': golden_io.normwise(out.detach().cpu().numpy(), ref.detach().numpy())}
    for n, t in enc.named_parameters():
        if t.grad is not None:
            res[n] = golden_io.normwise(t.grad.cpu().numpy(), p[n].grad.numpy())
    return res


@pytest.mark.parametrize('kind,b,hidden,depth,extra', [
    ('polymer', 64, 300, 3, {}),                                   # the benchmark configuration
    ('polymer', 128, 300, 3, dict(bias=True)),
    ('qm9', 64, 300, 3, dict(activation='ELU')),
    ('zinc', 64, 512, 5, {}),
    ('polymer', 32, 96, 4, dict(undirected=True, aggregation='sum')),
    ('polymer', 32, 64, 3, dict(atom_messages=True, bias=True)),
    ('polymer', 16, 70, 3, dict(activation='PReLU', bias=True, aggregation='norm')),
])
def test_random_graphs_vs_oracle(kind, b, hidden, depth, extra):
    args = TrainArgs(hidden_size=hidden, depth=depth, **extra)
    graphs = BatchMolGraph(synthetic.make_batch(kind, b, 100 + b))
    res = _oracle_vs_hip(graphs, args, seed=b)
    bad = {k: v for k, v in res.items() if v > TOL}
    assert not bad, bad


def test_edge_cases_hub_degree_empty_single_atom():
    args = TrainArgs(hidden_size=64, depth=3, bias=True)
    graphs = BatchMolGraph(synthetic.edge_case_batch(9, star_leaves=130))
    res = _oracle_vs_hip(graphs, args, seed=5)
    assert all(v <= TOL for v in res.values()), res


def test_atom_descriptors_layer():
    args = TrainArgs(hidden_size=48, atom_descriptors='descriptor', atom_descriptors_size=12)
    mols = synthetic.make_batch('polymer', 8, 3)
    desc = synthetic.random_descriptors(mols, 12, 3)
    res = _oracle_vs_hip(BatchMolGraph(mols), args, seed=3, desc=desc)
    assert all(v <= TOL for v in res.values()), res


def test_block_diagonal_independence_at_full_size():
    """Size-independent property at 4x the bench batch: encoding a batch equals encoding its halves."""
    args = TrainArgs(hidden_size=300, depth=3, device=DEV)
    mols = synthetic.make_batch('polymer', 256, 77)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 1)
    enc = enc.to(DEV).eval()
    with torch.no_grad():
        full = enc(BatchMolGraph(mols))
        a = enc(BatchMolGraph(mols[:100]))
        b = enc(BatchMolGraph(mols[100:]))
        perm = list(reversed(mols))
        rev = enc(BatchMolGraph(perm))
    both = torch.cat([a, b])
    assert golden_io.normwise(full.cpu().numpy(), both.cpu().numpy()) <= 1e-6
    assert golden_io.normwise(rev.flip(0).cpu().numpy(), full.cpu().numpy()) <= 1e-6


def test_repeat_runs_are_bitwise_deterministic():
    args = TrainArgs(hidden_size=300, depth=3)
    g = BatchMolGraph(synthetic.make_batch('polymer', 64, 5))
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 2)
    enc = enc.to(DEV)
    outs, grads = [], []
    for _ in range(2):
        enc.zero_grad()
        out = enc(g)
        out.square().sum().backward()
        outs.append(out.detach().cpu())
        grads.append(enc.W_h.weight.grad.detach().cpu().clone())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(grads[0], grads[1])


def test_dropout_training_mode():
    args = TrainArgs(hidden_size=64, depth=3, dropout=0.3)
    g = BatchMolGraph(synthetic.make_batch('polymer', 16, 6))
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 4)
    enc = enc.to(DEV)
    enc.eval()
    with torch.no_grad():
        e1, e2 = enc(g), enc(g)
    assert torch.equal(e1, e2)
    enc.train()
    t1 = enc(g)
    t2 = enc(g)
    assert not torch.equal(t1, t2)  # fresh mask per call
    assert torch.isfinite(t1).all()
    t1.sum().backward()
    assert all(torch.isfinite(p.grad).all() for p in enc.parameters() if p.grad is not None)


def test_index_select_nd():
    src = torch.randn(50, 7, device=DEV)
    idx = torch.randint(0, 50, (13, 4), device=DEV)
    out = index_select_ND(src, idx)
    assert torch.equal(out, src[idx])
    with pytest.raises(IndexError):
        index_select_ND(src, torch.tensor([[50]], device=DEV))
