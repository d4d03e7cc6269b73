"""wdmpnn_forward_many (MPNEncoder.forward_many): several independent batches through the fused
inference forward in one set of launches.  Each batch's output equals its own MPNEncoder.forward
bitwise (same kernels, same arithmetic, only the grid is shared), across batch kinds and sizes, more
than one launch group (> 8 batches), host-built and device-built graphs, undirected messages and a
bias; the oracle checks one of them."""
import pytest
import torch

import golden_io
from chemprop_amd import TrainArgs, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim
from chemprop_amd.mpn import MPNEncoder

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _enc(**kw):
    args = TrainArgs(**kw)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 4)
    return enc.to(DEV).eval(), args


@pytest.mark.parametrize('kw', [dict(hidden_size=300, depth=3), dict(hidden_size=64, depth=4, bias=True, undirected=True),
                                dict(hidden_size=512, depth=2, activation='tanh', aggregation='sum')])
def test_forward_many_equals_single_calls(kw):
    enc, _ = _enc(**kw)
    graphs = [BatchMolGraph(synthetic.make_batch(kind, b, 60 + i), device_bond_features=True)
              for i, (kind, b) in enumerate([('polymer', 64), ('qm9', 64), ('polymer', 7), ('zinc', 32), ('qm9', 1),
                                             ('polymer', 64), ('qm9', 64), ('qm9', 64), ('polymer', 16), ('zinc', 8)])]
    graphs.append(BatchMolGraph(synthetic.make_batch('polymer', 9, 5), compact=False))  # host-built graph
    with torch.no_grad():
        one = [enc(g) for g in graphs]
        many = enc.forward_many(graphs)
        again = enc.forward_many(graphs)  # cached plan
    torch.cuda.synchronize()
    assert len(many) == len(graphs)
    for a, b, c in zip(one, many, again):
        assert a.shape == b.shape and torch.equal(a, b) and torch.equal(b, c)


def test_forward_many_matches_oracle_and_handles_edge_cases():
    from oracle import mpn_ref
    enc, args = _enc(hidden_size=96, depth=3, bias=True)
    p = {n: t.detach().cpu().clone() for n, t in enc.named_parameters()}
    mols = synthetic.edge_case_batch(3, star_leaves=20)
    graphs = [BatchMolGraph(mols), BatchMolGraph(synthetic.make_batch('polymer', 12, 8))]
    with torch.no_grad():
        outs = enc.forward_many(graphs)
    for g, o in zip(graphs, outs):
        ref = mpn_ref.encoder_forward(p, g, args)
        assert golden_io.normwise(o.cpu().numpy(), ref.numpy()) <= 1e-5
    assert enc.forward_many([]) == []


def test_forward_many_with_gradients_takes_the_one_batch_path():
    enc, _ = _enc(hidden_size=32, depth=3)
    enc.train()
    graphs = [BatchMolGraph(synthetic.make_batch('qm9', 8, s)) for s in range(3)]
    outs = enc.forward_many(graphs)
    assert all(o.requires_grad for o in outs)
    sum(o.sum() for o in outs).backward()
    assert enc.W_h.weight.grad is not None


def test_full_block_plan_gives_the_same_outputs():
    """block_target=1 (forward_many's throughput layout: small batches in full molecule blocks) changes
    only the block plan: outputs equal the default plan's within fp32 rounding (the pair-operand layers
    scale each block's fp16 operands by that block's maxima, so the roundings differ with the blocking;
    the register-staged layers, gemm_variant 12, are bitwise independent of it), and forward_many on such
    graphs equals the single calls bitwise."""
    enc, _ = _enc(hidden_size=300, depth=3)
    mols = [synthetic.make_batch('qm9', 64, 900 + i) for i in range(6)]
    sliced = [BatchMolGraph(m, device_bond_features=True) for m in mols]
    full = [BatchMolGraph(m, device_bond_features=True, block_target=1) for m in mols]
    assert full[0].molecule_blocks().shape[0] < sliced[0].molecule_blocks().shape[0]
    with torch.no_grad():
        a = [enc(g) for g in sliced]
        b = [enc(g) for g in full]
        c = enc.forward_many(full)
        enc._gemm_variant = 12
        a12 = [enc(g) for g in sliced]
        b12 = [enc(g) for g in full]
        enc._gemm_variant = 0
    torch.cuda.synchronize()
    for x, y, z in zip(a, b, c):
        assert golden_io.normwise(x.cpu().numpy(), y.cpu().numpy()) <= 2e-6 and torch.equal(y, z)
    for x, y in zip(a12, b12):
        assert torch.equal(x, y)


def test_prepare_caches_plans_and_keeps_outputs():
    """MPNEncoder.prepare (host-side setup: device graphs registered on the given streams, call plans cached)
    changes no result: forwards after it equal an unprepared encoder's bitwise, on the current stream and on a
    prepared side stream, and the plans are in place before the first forward."""
    enc, _ = _enc(hidden_size=300, depth=3)
    ref, _ = _enc(hidden_size=300, depth=3)
    graphs = [BatchMolGraph(synthetic.make_batch(kind, b, 70 + i), device_bond_features=True)
              for i, (kind, b) in enumerate([('polymer', 16), ('qm9', 64), ('polymer', 5)])]
    side = torch.cuda.Stream(DEV)
    enc.prepare(graphs, [side])
    assert all(len(g.device_graph(DEV, False, get_bond_fdim()).encoder_plans) == 1 for g in graphs)
    with torch.no_grad():
        a = [enc(g) for g in graphs]
        with torch.cuda.stream(side):
            b = [enc(g) for g in graphs]
        c = [ref(g) for g in graphs]
    torch.cuda.synchronize()
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, y) and torch.equal(x, z)
