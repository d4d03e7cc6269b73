"""Compact graphs (include/wdmpnn.h "Compact graphs"): categorical codes on the wire,
every device array built on the GPU by ``wdmpnn_build_graph``.

CPU: the native encoder / decoder round-trips the packed BatchMolGraph bit for bit, the block plan and
entry offsets equal the host packer's, the generator is deterministic and yields reference-shaped
MolGraph tables, and non-categorical inputs are refused (host path).
GPU: the device-built WdGraph equals the host-built one array by array (bitwise), and the encoder on
it equals the host path bitwise and the oracle at 1e-5.
"""
import ctypes

import numpy as np
import pytest
import torch

import golden_io
from chemprop_amd import TrainArgs, _native, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim, _packer

KINDS = {'polymer': 0, 'qm9': 1, 'zinc': 2}


def batches():
    return [('polymer', synthetic.make_batch('polymer', 64, 3)), ('qm9', synthetic.make_batch('qm9', 40, 4)),
            ('zinc', synthetic.make_batch('zinc', 24, 5)), ('edge', synthetic.edge_case_batch(9, star_leaves=20)),
            ('polymer_small', synthetic.make_batch('polymer', 3, 11))]


@pytest.mark.parametrize('case', range(5))
@pytest.mark.parametrize('tail_mode', [False, True])
def test_encode_decode_roundtrip(case, tail_mode):
    name, mols = batches()[case]
    g = BatchMolGraph(mols, device_bond_features=tail_mode)
    assert g._compact is not None, g._compact_why
    h = BatchMolGraph.from_compact(*g._compact)
    for attr in ('f_atoms', 'f_bonds', 'w_atoms', 'w_bonds', 'b2a', 'b2revb', 'a2b'):
        a, b = getattr(g, attr).numpy(), getattr(h, attr).numpy()
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b), attr
    assert (g.n_atoms, g.n_bonds, g.a_scope, g.b_scope, g.max_num_bonds) == \
        (h.n_atoms, h.n_bonds, h.a_scope, h.b_scope, h.max_num_bonds)
    assert np.array_equal(np.float32(g.degree_of_polym), np.float32(h.degree_of_polym))


@pytest.mark.parametrize('case', range(5))
def test_plan_matches_host_blocks_and_entries(case):
    """compact_stage's molecule blocks = BatchMolGraph.molecule_blocks(); its per-block first entries and
    totals = the host packer's gather lists (csrc/packer.cpp ``gathers``)."""
    name, mols = batches()[case]
    g = BatchMolGraph(mols)
    host = np.zeros(1 << 20, np.uint8)
    info = _packer().compact_stage(*g._compact, 133, 147, 64, host.ctypes.data, host.nbytes)
    copied, (n_mols, n_atoms, n_bonds, n_blocks, nnz_msg, nnz_agg), off, total = info
    assert copied and (n_mols, n_atoms, n_bonds) == (len(mols), g.n_atoms, g.n_bonds)
    blocks = g.molecule_blocks()
    assert n_blocks == len(blocks)
    assert np.array_equal(host[off[4]:off[4] + blocks.nbytes].view(np.int32).reshape(-1, 8), blocks)
    msg, agg = g.bond_message_gather(), g.atom_aggregate_gather()
    assert (nnz_msg, nnz_agg) == (len(msg.idx), len(agg.idx))
    nnz = host[off[5]:off[5] + 8 * n_blocks].view(np.int32).reshape(-1, 2)
    assert np.array_equal(nnz[:, 0], msg.ptr[blocks[:, 0]]) and np.array_equal(nnz[:, 1], agg.ptr[blocks[:, 2]])


def test_stage_refuses_molecules_larger_than_a_block():
    g = BatchMolGraph(synthetic.edge_case_batch(9, star_leaves=130))
    assert g._compact is not None
    assert _packer().compact_stage(*g._compact, 133, 147, 64, 0, 0) is None


def test_encode_refuses_non_categorical_rows():
    mols = synthetic.make_batch('polymer', 4, 1)
    mols[1].f_atoms[2][5] = 0.5  # not one-hot
    assert BatchMolGraph(mols)._compact is None
    mols = synthetic.make_batch('polymer', 4, 1)
    mols[2].f_bonds[3][140] = 2.0  # bond column not binary
    assert BatchMolGraph(mols)._compact is None
    mols = synthetic.make_batch('polymer', 4, 1)
    mols[0].f_bonds[0][0] = 1.0 - mols[0].f_bonds[0][0]  # bond row does not start with its atom row
    g = BatchMolGraph(mols)
    assert g._compact is None and 'source atom' in g._compact_why
    assert BatchMolGraph(synthetic.make_batch('qm9', 4, 1), compact=False)._compact is None


@pytest.mark.parametrize('kind', list(KINDS))
def test_generator_deterministic_and_reference_shaped(kind):
    a = _packer().compact_generate(KINDS[kind], 32, 7)
    b = _packer().compact_generate(KINDS[kind], 32, 7)
    c = _packer().compact_generate(KINDS[kind], 32, 8)
    assert all(bytes(x) == bytes(y) for x, y in zip(a, b)) and bytes(a[2]) != bytes(c[2])
    g = BatchMolGraph.from_compact(*a)
    na = np.array([n for _, n in g.a_scope])
    lo, hi = {'polymer': (20, 48), 'qm9': (5, 9), 'zinc': (15, 37)}[kind]
    assert na.min() >= lo and na.max() <= hi
    fa = g.f_atoms.numpy()[1:]
    # atom_features layout (featurization.py:190-211): one 1 in each of the six one-hot blocks
    starts = np.cumsum([0, 101, 7, 6, 5, 6, 6])
    for s, e in zip(starts[:-1], starts[1:]):
        assert np.array_equal(fa[:, s:e].sum(1), np.ones(len(fa)))
    assert set(np.unique(fa[:, 131])) <= {0.0, 1.0} and (fa[:, 132] >= 0.1).all() and (fa[:, 132] <= 0.4).all()
    fb = g.f_bonds.numpy()
    assert np.array_equal(fb[1:, :133], fa[g.b2a.numpy()[1:] - 1])
    rev = g.b2revb.numpy()
    assert np.array_equal(rev[rev[1:]], np.arange(1, g.n_bonds))
    if kind == 'polymer':  # 10 rules per graph, weights in [0.1, 0.5], fractions summing to 1 per graph
        w = g.w_bonds.numpy()[1:]
        assert ((w == 1.0) | ((w >= 0.1) & (w <= 0.5))).sum() == len(w)
        assert (w < 1.0).sum() == 20 * 32
        xn = np.array(g.degree_of_polym)
        assert (xn >= 1.0).all() and (xn <= 4.0).all()
    # the decoded tables pack back into the same compact codes
    h = BatchMolGraph(_as_molgraphs(g))
    assert all(bytes(x) == bytes(y) for x, y in zip(h._compact, a))


def _as_molgraphs(g):
    """Per-molecule MolGraph-like objects from a batch's tables (inverse of BatchMolGraph)."""
    out = []
    fa, fb = g.f_atoms.numpy(), g.f_bonds.numpy()
    wa, wb, b2a, rev = g.w_atoms.numpy(), g.w_bonds.numpy(), g.b2a.numpy(), g.b2revb.numpy()
    a2b = g.a2b.numpy()
    deg = (a2b != 0).sum(1)
    for (a0, na), (b0, nb), xn in zip(g.a_scope, g.b_scope, g.degree_of_polym):
        m = synthetic.SynthMolGraph(fa[a0:a0 + na].tolist(), fb[b0:b0 + nb].tolist(), wa[a0:a0 + na].tolist(),
                                    wb[b0:b0 + nb].tolist(),
                                    [[int(j) - b0 for j in a2b[a, :deg[a]]] for a in range(a0, a0 + na)],
                                    (b2a[b0:b0 + nb] - a0).tolist(), (rev[b0:b0 + nb] - b0).tolist(), xn)
        out.append(m)
    return out


# ------------------------------------------------------------------------------------------------ GPU
DEV = torch.device('cuda:0')


def _read(dg, ptr, nbytes):
    for t in [dg.buffer] + list(dg.views.values()):
        base, size = t.data_ptr(), t.numel() * t.element_size()
        if base <= ptr and ptr + nbytes <= base + size:
            flat = t.view(torch.uint8) if t.dim() == 1 and t.dtype == torch.uint8 else t.reshape(-1).view(torch.uint8)
            return flat[ptr - base:ptr - base + nbytes].cpu().numpy()
    raise AssertionError('pointer outside the graph buffers')


def _arrays(dg):
    s = dg.struct
    V1, E1, B, nblk = s.n_atoms, s.n_bonds, s.n_mols, s.n_blocks
    Vap, Rbp = -(-V1 // 128) * 128, -(-E1 // 128) * 128
    lda, ldb = s.ld_atoms, s.ld_bonds
    out = {'f_atoms': (s.f_atoms, Vap * lda * 4), 'f_bonds': (s.f_bonds, Rbp * ldb * 4),
           'f_atoms_x6': (s.f_atoms_x6, Vap * lda * 6), 'f_bonds_x6': (s.f_bonds_x6, Rbp * ldb * 6),
           'f_atoms_blk_x6': (s.f_atoms_blk_x6, nblk * 64 * lda * 6), 'w_atoms': (s.w_atoms, V1 * 4),
           'mol_start': (s.mol_start, B * 4), 'mol_size': (s.mol_size, B * 4), 'xn': (s.degree_of_polym, B * 4),
           'b2revb': (s.b2revb, E1 * 4), 'blocks': (s.blocks, nblk * 32), 'bond_blk_row': (s.bond_blk_row, Rbp * 4),
           'msg_ell_idx': (s.msg_ell_idx, Rbp * 8), 'msg_ell_coef': (s.msg_ell_coef, Rbp * 32),
           'atom_ell_idx': (s.atom_ell_idx, Vap * 8), 'atom_ell_coef': (s.atom_ell_coef, Vap * 32)}
    for name, csr, rows in (('msg', s.msg_gather, E1), ('agg', s.atom_gather, V1), ('msg_t', s.msg_gather_t, E1),
                            ('agg_t', s.atom_gather_t, E1)):
        ptr = _read(dg, csr.ptr, (rows + 1) * 4).view(np.int32)
        nnz = int(ptr[-1]) + 8
        out[name + '_ptr'] = (csr.ptr, (rows + 1) * 4)
        out[name + '_idx'] = (csr.idx, nnz * 4)
        out[name + '_coef'] = (csr.coef, nnz * 4)
    return {k: _read(dg, p, n) for k, (p, n) in out.items()}


@pytest.mark.gpu
@pytest.mark.parametrize('case', range(5))
@pytest.mark.parametrize('tail_mode', [False, True])
def test_device_built_graph_equals_host_built(case, tail_mode):
    name, mols = batches()[case]
    g_dev = BatchMolGraph(mols, device_bond_features=tail_mode)
    g_host = BatchMolGraph(mols, device_bond_features=tail_mode, compact=False)
    d_dev, d_host = g_dev.device_graph(DEV, False, get_bond_fdim()), g_host.device_graph(DEV, False, get_bond_fdim())
    assert d_dev.built_on_device and not d_host.built_on_device
    # compact upload: ~14 B per edge on polymers (the bench workload, <= 16), more per edge on small molecules
    # (per-molecule records and blocks), + the 256-byte alignment of six arrays
    assert d_dev.h2d_bytes <= (16 if name.startswith('polymer') else 24) * (g_dev.n_bonds - 1) + 6 * 256
    for f in ('n_atoms', 'n_bonds', 'n_mols', 'atom_fdim', 'bond_fdim', 'ld_atoms', 'ld_bonds', 'n_blocks'):
        assert getattr(d_dev.struct, f) == getattr(d_host.struct, f), f
    a, b = _arrays(d_dev), _arrays(d_host)
    bad = [k for k in a if not np.array_equal(a[k], b[k])]
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize('kind,b,hidden,depth,extra', [
    ('polymer', 64, 300, 3, {}),
    ('qm9', 64, 300, 3, dict(bias=True, activation='ELU')),
    ('zinc', 128, 512, 5, dict(aggregation='sum')),
    ('polymer', 16, 96, 4, dict(undirected=True, activation='tanh', aggregation='norm')),
])
def test_generated_batches_forward_and_backward_vs_oracle(kind, b, hidden, depth, extra):
    """Natively generated batches (the streamed workload's generator): device-built graph, inference
    (blocked) and training (unblocked, backward) paths against the fp32 oracle on the decoded tables."""
    from chemprop_amd.mpn import MPNEncoder
    from oracle import mpn_ref
    args = TrainArgs(hidden_size=hidden, depth=depth, **extra)
    g = BatchMolGraph.from_compact(*_packer().compact_generate(KINDS[kind], b, 31 + b))
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 6)
    p = {n: t.detach().clone() for n, t in enc.named_parameters()}
    enc = enc.to(DEV)
    with torch.no_grad():
        out = enc.eval()(g)
    assert g.device_graph(DEV, False, get_bond_fdim()).built_on_device
    ref = mpn_ref.encoder_forward(p, g, args)
    assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= 1e-5
    out_t = enc(g)
    assert golden_io.normwise(out_t.detach().cpu().numpy(), ref.numpy()) <= 1e-5
    out_t.square().sum().backward()
    assert all(torch.isfinite(q.grad).all() for q in enc.parameters() if q.grad is not None)


@pytest.mark.gpu
def test_compact_and_host_paths_agree():
    """Compact (device-built) vs host-packed graph, inference and training (both run the fused
    molecule-blocked kernels): the compact graph's input layer and W_o atom half are sums of weight
    columns (embed_kernel) instead of GEMMs over the one-hot rows, so only rounding differs (outputs
    and gradients within 1e-5 normwise, the parity bar)."""
    from chemprop_amd.mpn import MPNEncoder
    mols = synthetic.make_batch('polymer', 64, 13)
    args = TrainArgs(hidden_size=300, depth=3)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 2)
    enc = enc.to(DEV)
    outs = []
    for compact in (True, False):
        g = BatchMolGraph(mols, compact=compact)
        with torch.no_grad():
            o1 = enc.eval()(g)
        enc.zero_grad()
        o2 = enc.train()(g)
        o2.square().sum().backward()
        outs.append([o1.cpu(), o2.detach().cpu()] + [q.grad.cpu().clone() for q in enc.parameters() if q.grad is not None])
    (a, *ra), (b, *rb) = outs
    assert len(ra) == len(rb)
    for x, y in zip(ra, rb):
        assert golden_io.normwise(x.numpy(), y.numpy()) <= 1e-5
    assert golden_io.normwise(a.numpy(), b.numpy()) <= 1e-6
