"""GPU: the HIP path (libwdmpnn.so through chemprop_amd) against the reference goldens and the oracle.

Parity bar (north_star): fp32, max|out - ref| <= 1e-5 * max|ref| per tensor, for
every output and every parameter gradient:
  * vs the reference goldens (outputs and gradients, grad-enabled and no-grad forward paths);
  * on the large random batches: outputs vs the fp32 oracle, gradients vs an fp64 evaluation of the
    same op sequence that shares the HIP forward's kink decisions (``_oracle_vs_hip``).
"""
import numpy as np
import pytest
import torch

import golden_io
from chemprop_amd import TrainArgs, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim
from chemprop_amd.model import MoleculeModel
from chemprop_amd.mpn import MPNEncoder
from chemprop_amd.mpn import saved_preactivations as mpn_saved_preactivations
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


def run_case(case, grads=True, no_grad=False):
    a = case.args
    a.device = DEV
    if case.level == 'encoder':
        m = MPNEncoder(a, get_atom_fdim(), get_bond_fdim(atom_messages=a.atom_messages))
    else:
        m = MoleculeModel(a)
    synthetic.fill_parameters(m, case.seed)
    m = m.to(DEV).eval()
    with torch.set_grad_enabled(not no_grad):
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
    # the same golden through the inference call (no autograd: the molecule-blocked fused kernels
    # wherever the batch allows them, the benchmark's path)
    out_ng, _ = run_case(case, grads=False, no_grad=True)
    err = golden_io.normwise(out_ng, case.output)
    assert err <= TOL, ('no-grad path', err)


def _oracle_vs_hip(graphs, args, seed, desc=None, row_scale=None):
    """Errors of the HIP training path (forward + backward) against the oracle.  The output must meet
    1e-5 normwise vs the fp32 oracle (the reference's own arithmetic).  Parameter gradients must meet
    1e-5 normwise vs an fp64 evaluation of the same op sequence that takes the branch of every kinked
    activation (ReLU, LeakyReLU, PReLU, SELU) from the HIP forward's own saved pre-activations
    (mpn.saved_preactivations): a pre-activation within rounding of 0 lands on either side of the
    kink depending on summation order, and at B >= 64 those sub-ulp flips move the reference's own fp32
    weight gradients by up to ~3e-4 from fp64; sharing the decisions leaves only the arithmetic to
    compare."""
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=args.atom_messages))
    synthetic.fill_parameters(enc, seed)
    R = torch.randn((len(graphs.a_scope), args.hidden_size + (args.atom_descriptors_size if desc else 0)),
                    generator=torch.Generator().manual_seed(seed))
    if row_scale is not None:  # per-molecule magnitudes of the output gradient
        R = R * row_scale[:, None]
    cpu_params = {n: t.detach().clone() for n, t in enc.named_parameters()}
    trainable = {n for n, t in enc.named_parameters() if t.requires_grad}
    enc = enc.to(DEV)
    out = enc(graphs, desc)
    saved = mpn_saved_preactivations(out)
    masks = {'Z': [z.cpu() > 0 for z in saved['Z']], 'Zo': saved['Zo'].cpu() > 0}
    (out * R.to(DEV)).sum().backward()
    hip = {'output': out.detach().cpu().numpy()}
    hip.update({n: t.grad.cpu().numpy() for n, t in enc.named_parameters() if t.grad is not None})
    with torch.no_grad():
        ref32 = mpn_ref.encoder_forward(cpu_params, graphs, args, desc).numpy()
    p = {n: t.to(torch.float64).requires_grad_(n in trainable) for n, t in cpu_params.items()}
    out64 = mpn_ref.encoder_forward(p, graphs, args, desc, dtype=torch.float64, masks=masks)
    (out64 * R.to(torch.float64)).sum().backward()
    ref64 = {n: p[n].grad.numpy() for n in p if p[n].grad is not None}
    res = {'output': (golden_io.normwise(hip['output'], ref32), TOL)}
    for k, r64 in ref64.items():
        assert k in hip, f'missing {k}'
        res[k] = (golden_io.normwise(hip[k], r64), TOL)
    return res


def _check(res):
    bad = {k: v for k, v in res.items() if not v[0] <= v[1]}
    assert not bad, bad


@pytest.mark.parametrize('kind,b,hidden,depth,extra', [
    ('polymer', 64, 300, 3, {}),                                   # the benchmark configuration
    ('polymer', 64, 300, 3, dict(activation='LeakyReLU')),
    ('polymer', 64, 300, 3, dict(activation='tanh', bias=True)),
    ('polymer', 128, 300, 3, dict(bias=True)),
    ('polymer', 128, 300, 3, dict(bias=True, activation='SELU')),
    ('qm9', 64, 300, 3, dict(activation='ELU')),
    ('zinc', 64, 512, 5, {}),
    ('polymer', 32, 96, 4, dict(undirected=True, aggregation='sum')),
    ('polymer', 32, 64, 3, dict(atom_messages=True, bias=True)),
    ('polymer', 16, 70, 3, dict(activation='PReLU', bias=True, aggregation='norm')),
    ('polymer', 8, 1100, 2, dict(activation='ELU')),                 # hidden > 1024 (readout backward chunks)
    ('polymer', 6, 2400, 3, dict(bias=True)),                        # the reference hyperopt's largest hidden
    ('polymer', 3, 2850, 2, {}),  # Hk 2880: 72 embed scale words per block (> 64, folded by lane_word)
])
def test_random_graphs_vs_oracle(kind, b, hidden, depth, extra):
    args = TrainArgs(hidden_size=hidden, depth=depth, **extra)
    graphs = BatchMolGraph(synthetic.make_batch(kind, b, 100 + b))
    _check(_oracle_vs_hip(graphs, args, seed=b))


def _scale_mass(g, factor):
    """Multiply a molecule's mass feature (the last atom column, featurization.py:210) by ``factor``, in
    f_atoms and in the f_atoms half of its f_bonds rows: its messages grow by about that much."""
    for row in g.f_atoms:
        row[-1] *= factor
    fa = len(g.f_atoms[0])
    for b, row in enumerate(g.f_bonds):
        row[fa - 1] = g.f_atoms[g.b2a[b]][-1]
    return g


@pytest.mark.parametrize('activation', ['ReLU', 'LeakyReLU'])
def test_per_molecule_accuracy_in_mixed_magnitude_blocks(activation):
    """The fused layers scale their fp16-pair operand per (molecule block, column tile) from the block's max
    (planes.hpp h2).  Molecules whose messages are 10^2 - 10^4 x smaller than a block-mate's must still meet
    1e-5 against the fp64 oracle relative to their OWN row maximum (per-element pair error <= max(2^-22 |x s|,
    2^-25) in scaled units: no loss until a row is ~2^-18 of the block max).  Full molecule blocks
    (block_target=1) so that the scaled and unscaled molecules share blocks."""
    rng_mols = synthetic.make_batch('qm9', 24, 61)
    for i, f in ((2, 1e2), (9, 1e4), (17, 1e3)):
        _scale_mass(rng_mols[i], f)
    g = BatchMolGraph(rng_mols, block_target=1)
    assert g.device_graph(DEV, False, get_bond_fdim()).struct.n_blocks < 24  # molecules do share blocks
    args = TrainArgs(hidden_size=300, depth=3, activation=activation)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 8)
    p = {n: t.detach().to(torch.float64) for n, t in enc.named_parameters()}
    enc = enc.to(DEV).eval()
    with torch.no_grad():
        out = enc(g).cpu().double()
        ref = mpn_ref.encoder_forward(p, g, args, dtype=torch.float64)
    mx = ref.abs().max(dim=1).values
    assert float(mx.max() / mx.min()) > 100  # the magnitudes really are mixed
    err = (out - ref).abs().max(dim=1).values / mx
    assert float(err.max()) <= TOL, err.tolist()


@pytest.mark.parametrize('activation,depth', [('ReLU', 5), ('LeakyReLU', 4)])
def test_gradients_with_wide_dynamic_range(activation, depth):
    """The backward's W_h GEMMs run on fp16 pairs scaled per group of Y_t (256 float4) and per 128 x 64 tile
    of M_{t-1} (gemm_x6.hpp): entries far below their group's max keep an absolute error near 2^-22 of it.
    Output gradients spanning 10^-4 .. 10^4 across molecules, messages 10^2 - 10^3 x larger in three
    molecules, deep T: every weight gradient must still meet 1e-5 normwise against the fp64 evaluation
    (the weight gradients are sums over all rows, where those absolute errors stay below the sum's own
    fp32 rounding)."""
    mols = synthetic.make_batch('polymer', 24, 71)
    for i, f in ((3, 1e2), (11, 1e3), (19, 3e2)):
        _scale_mass(mols[i], f)
    g = BatchMolGraph(mols)
    scale = torch.tensor([10.0 ** ((7 * i) % 9 - 4) for i in range(24)])
    assert float(scale.max() / scale.min()) >= 1e8
    args = TrainArgs(hidden_size=300, depth=depth, activation=activation, bias=True)
    _check(_oracle_vs_hip(g, args, seed=71, row_scale=scale))


def test_edge_cases_hub_degree_empty_single_atom():
    args = TrainArgs(hidden_size=64, depth=3, bias=True)
    graphs = BatchMolGraph(synthetic.edge_case_batch(9, star_leaves=130))
    _check(_oracle_vs_hip(graphs, args, seed=5))


def test_atom_descriptors_layer():
    args = TrainArgs(hidden_size=48, atom_descriptors='descriptor', atom_descriptors_size=12)
    mols = synthetic.make_batch('polymer', 8, 3)
    desc = synthetic.random_descriptors(mols, 12, 3)
    _check(_oracle_vs_hip(BatchMolGraph(mols), args, seed=3, desc=desc))


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


def test_batches_in_flight_on_streams_match_serial():
    """bench.py's --streams: independent batches round-robin over HIP streams, the first call on a
    side stream (the weight pack happens there, other streams wait on its event)."""
    args = TrainArgs(hidden_size=300, depth=3)
    graphs = [BatchMolGraph(synthetic.make_batch('polymer', 64, 40 + i), device_bond_features=True)
              for i in range(6)]
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 4)
    enc = enc.to(DEV).eval()
    streams = [torch.cuda.Stream(DEV) for _ in range(3)]
    with torch.no_grad():
        outs = [None] * len(graphs)
        for i, g in enumerate(graphs):
            with torch.cuda.stream(streams[i % 3]):
                outs[i] = enc(g)
        torch.cuda.synchronize(DEV)
        serial = [enc(g) for g in graphs]
    for a, b in zip(outs, serial):
        assert torch.equal(a.cpu(), b.cpu())


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
    torch.manual_seed(7)
    r1 = enc(g)
    torch.manual_seed(7)
    r2 = enc(g)
    assert torch.equal(r1, r2)  # torch.manual_seed reproduces the masks
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


@pytest.mark.parametrize('n_src,shape,row', [(50, (13, 4), (7,)), (300, (2185, 9), (300,)), (5, (0,), (3,)),
                                             (40, (64,), (2, 3))])
def test_index_select_nd_backward_deterministic(n_src, shape, row):
    """The HIP transposed gather (wdmpnn_index_select_rows_backward) equals the fp64 scatter-add of the
    reference's autograd, rows never selected get 0, and two runs agree bit for bit."""
    g = torch.Generator().manual_seed(n_src)
    src = torch.randn((n_src,) + row, generator=g)
    idx = torch.randint(0, n_src, shape, generator=g)
    R = torch.randn(tuple(shape) + row, generator=g)
    ref = torch.zeros((n_src,) + row, dtype=torch.float64)
    ref.index_add_(0, idx.reshape(-1), R.double().reshape((-1,) + row))
    grads = []
    for _ in range(2):
        s = src.to(DEV).requires_grad_(True)
        (index_select_ND(s, idx.to(DEV)) * R.to(DEV)).sum().backward()
        grads.append(s.grad.cpu())
    assert torch.equal(grads[0], grads[1])
    err = (grads[0].double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)
    assert float(err) <= 1e-6


@pytest.mark.parametrize('variant', [0, 9])
def test_gemm_paths_agree(variant):
    """Both GEMM families (WdConfig.gemm_variant 0: bf16x6 split planes; 9: f32 MFMA) compute the
    forward within the parity bar, blocked inference and unblocked training forward alike."""
    args = TrainArgs(hidden_size=300, depth=3, bias=True)
    g = BatchMolGraph(synthetic.make_batch('polymer', 48, 9))
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 8)
    p = {n: t.detach().clone() for n, t in enc.named_parameters()}
    ref = mpn_ref.encoder_forward(p, g, args)
    enc = enc.to(DEV).eval()
    enc._gemm_variant = variant
    with torch.no_grad():
        out = enc(g)
    assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL
    out = enc(g)  # grad enabled: unblocked kernels
    assert golden_io.normwise(out.detach().cpu().numpy(), ref.numpy()) <= TOL


@pytest.mark.parametrize('kind,b,hidden,depth,extra', [
    ('polymer', 64, 300, 3, {}),                                        # bench config: 80-column tiles
    ('polymer', 64, 300, 3, dict(activation='tanh', bias=True, aggregation='sum')),
    ('polymer', 32, 300, 4, dict(undirected=True, activation='ELU', aggregation='norm')),
    ('zinc', 64, 512, 5, dict(activation='LeakyReLU')),                 # 64-column tiles
    ('qm9', 96, 128, 3, dict(activation='SELU', bias=True)),           # many molecules per block
    ('polymer', 16, 70, 2, dict(activation='PReLU', bias=True)),       # Hk = 128, T = 2 (single layer)
    ('qm9', 64, 300, 3, {}),                                            # bench secondary (configs[1] shape)
    ('polymer', 128, 300, 3, {}),                                       # configs[2] batch size
    ('zinc', 512, 512, 5, {}),                                          # bench secondary (configs[3] shape)
])
def test_blocked_fused_forward(kind, b, hidden, depth, extra):
    """The molecule-blocked fused inference forward (WdConfig.gemm_variant 0, no grad) matches the
    fp32 oracle at 1e-5 normwise."""
    args = TrainArgs(hidden_size=hidden, depth=depth, **extra)
    g = BatchMolGraph(synthetic.make_batch(kind, b, 400 + b))
    assert g.molecule_blocks() is not None
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 12)
    p = {n: t.detach().clone() for n, t in enc.named_parameters()}
    ref = mpn_ref.encoder_forward(p, g, args)
    enc = enc.to(DEV).eval()
    enc._gemm_variant = 0
    with torch.no_grad():
        out = enc(g)
    assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL


@pytest.mark.parametrize('kind,b,hidden,depth,extra', [
    ('polymer', 64, 300, 3, {}),                                         # the benchmark: Hk 320, 80-column tiles
    ('polymer', 64, 300, 4, dict(activation='LeakyReLU', bias=True)),   # two pair hand-offs between layers
    ('polymer', 32, 300, 3, dict(undirected=True, activation='tanh')),
    ('polymer', 24, 600, 3, dict(activation='SELU', aggregation='sum')),  # Hk 640: 8 layer tiles, 20 embed words
    ('polymer', 16, 300, 2, dict(activation='PReLU', bias=True)),       # T = 2: the embed's pairs feed the last layer
    ('qm9', 96, 300, 3, dict(activation='ELU')),                        # many molecules per block
    ('polymer', 8, 1600, 3, {}),                                         # Hk 1600: 50 chunks, 50 embed words
])
def test_pair_operand_layers_vs_register_staged(kind, b, hidden, depth, extra):
    """The message layers reading M_{t-1} as fp16 pair tiles written by their producer (the embed, the
    previous layer; per-tile scales, one shared scale per block in the GEMM, gemm_x6.hpp h2_mainloop_pairs; the
    default path, WdConfig.gemm_variant 13 forces them also for QM9-sized blocks) meet the fp32 oracle at 1e-5
    and agree with the register-staged layers (variant 12) to fp32 rounding; both runs bitwise reproducible."""
    args = TrainArgs(hidden_size=hidden, depth=depth, **extra)
    kw = dict(block_target=1) if kind == 'qm9' else {}  # (QM9: full blocks, past the one-launch forward's 32 rows)
    g = BatchMolGraph(synthetic.make_batch(kind, b, 500 + b), device_bond_features=True, **kw)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 14)
    p = {n: t.detach().clone() for n, t in enc.named_parameters()}
    ref = mpn_ref.encoder_forward(p, g, args)
    enc = enc.to(DEV).eval()
    with torch.no_grad():
        enc._gemm_variant = 13
        pairs = enc(g)
        pairs2 = enc(g)
        enc._gemm_variant = 12
        staged = enc(g)
        enc._gemm_variant = 0
    torch.cuda.synchronize()
    assert torch.equal(pairs, pairs2)
    assert golden_io.normwise(pairs.cpu().numpy(), ref.numpy()) <= TOL
    assert golden_io.normwise(staged.cpu().numpy(), ref.numpy()) <= TOL
    assert golden_io.normwise(pairs.cpu().numpy(), staged.cpu().numpy()) <= 2e-6


def _runs_blocked(enc, g):
    """True when the native forward of ``enc`` on ``g`` takes the molecule-blocked fused path: its
    workspace (fwd_layout) differs from the same graph's with the blocks withheld."""
    import ctypes
    from chemprop_amd import _native
    dg = g.device_graph(DEV, enc.atom_messages, enc.bond_fdim)
    gs = enc._graph_struct(dg)
    cfg = enc._config(False)
    params = tuple(t.detach().float() if t is not None else None for t in enc._param_tuple())
    pstruct, _ = enc._packed_params(gs, cfg, params, DEV)
    sizes = []
    for nb in (gs.n_blocks, 0):
        g2 = _native.WdGraph.from_buffer_copy(gs)
        g2.n_blocks = nb
        n = ctypes.c_size_t()
        _native.check(_native.lib().wdmpnn_workspace_bytes(ctypes.byref(g2), ctypes.byref(pstruct), ctypes.byref(cfg),
                                                           ctypes.byref(n)), 'workspace')
        sizes.append(n.value)
    return sizes[0] != sizes[1]


@pytest.mark.parametrize('kind,b,hidden,depth,extra', [
    ('polymer', 64, 300, 3, {}),                                        # the bench's atom_messages secondary
    ('qm9', 32, 64, 2, dict(activation='tanh')),
    ('zinc', 24, 128, 4, dict(activation='PReLU')),
    ('polymer', 8, 96, 3, dict(activation='ELU', aggregation='sum')),
])
def test_blocked_atom_messages_forward(kind, b, hidden, depth, extra):
    """atom_messages=True without biases runs the molecule-blocked fused layers (a2a neighbour sums in the
    layer epilogue, the bond-feature half of W_h folded into the residual) and matches the fp32 oracle at
    1e-5 normwise; with a bias the same batch falls back to the unblocked path, also at 1e-5."""
    for bias in (False, True):
        args = TrainArgs(hidden_size=hidden, depth=depth, atom_messages=True, bias=bias, **extra)
        g = BatchMolGraph(synthetic.make_batch(kind, b, 900 + b))
        enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=True))
        synthetic.fill_parameters(enc, 21)
        p = {n: t.detach().clone() for n, t in enc.named_parameters()}
        ref = mpn_ref.encoder_forward(p, g, args)
        enc = enc.to(DEV).eval()
        assert _runs_blocked(enc, g) == (not bias)
        with torch.no_grad():
            out = enc(g)
        assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL
        if not bias:  # the same forward with the per-atom bond-feature sums gathered in the forward instead
            dg = g.device_graph(DEV, True, enc.bond_fdim)
            assert dg.struct.atom_feat_sum_x6
            dg.struct.atom_feat_sum_x6 = 0
            dg.encoder_structs.clear()
            dg.encoder_plans.clear()
            with torch.no_grad():
                out2 = enc(g)
            assert torch.equal(out, out2)


def test_blocked_atom_messages_edge_cases():
    """atom_messages=True on the edge-case batch (empty and single-atom molecules, a hub that still fits a
    block) and on a 130-leaf hub that exceeds a block (unblocked fallback): fp32 oracle at 1e-5."""
    args = TrainArgs(hidden_size=64, depth=3, atom_messages=True)
    for leaves in (20, 130):
        g = BatchMolGraph(synthetic.edge_case_batch(9, star_leaves=leaves))
        enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=True))
        synthetic.fill_parameters(enc, 5)
        p = {n: t.detach().clone() for n, t in enc.named_parameters()}
        ref = mpn_ref.encoder_forward(p, g, args)
        enc = enc.to(DEV).eval()
        assert _runs_blocked(enc, g) == (leaves == 20)
        with torch.no_grad():
            out = enc(g)
        assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL


def test_blocked_forward_edge_cases_and_fallback():
    """Empty / single-atom molecules in blocks, and a 130-leaf hub molecule that exceeds a block (the
    forward falls back to the unblocked plane-tile path)."""
    args = TrainArgs(hidden_size=64, depth=3, bias=True)
    rng = np.random.default_rng(4)
    many_empty = [synthetic.empty_graph() for _ in range(150)] + [synthetic.polymer_graph(rng, 3, 5)] + \
        [synthetic.empty_graph() for _ in range(70)]  # blocks capped at BLK_MOLS molecules
    for mols in (synthetic.edge_case_batch(9, star_leaves=20), synthetic.edge_case_batch(9, star_leaves=130),
                 many_empty):
        g = BatchMolGraph(mols)
        enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
        synthetic.fill_parameters(enc, 5)
        p = {n: t.detach().clone() for n, t in enc.named_parameters()}
        ref = mpn_ref.encoder_forward(p, g, args)
        enc = enc.to(DEV).eval()
        enc._gemm_variant = 0
        with torch.no_grad():
            out = enc(g)
        assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL


@pytest.mark.parametrize('kind,b,extra', [('polymer', 64, {}), ('qm9', 32, dict(bias=True)),
                                          ('edge', 9, dict(activation='ELU')),
                                          ('polymer', 8, dict(atom_messages=True, hidden_size=64))])
def test_device_bond_features(kind, b, extra):
    """f_bonds rebuilt on the device from f_atoms + bond tail + b2a
    (wdmpnn_build_bond_features) equals the host-packed f_bonds bit for bit, and the encoder's output
    (forward and gradients) is bitwise identical to the host-featurised graph's."""
    mols = synthetic.make_batch(kind, b, 77) if kind != 'edge' else synthetic.edge_case_batch(b, star_leaves=30)
    g_host = BatchMolGraph(mols, compact=False)
    g_dev = BatchMolGraph(mols, device_bond_features=True, check_bond_features=True, compact=False)
    am = bool(extra.get('atom_messages'))
    fdim = get_bond_fdim(atom_messages=am)
    d_host = g_host.device_graph(DEV, am, fdim)
    d_dev = g_dev.device_graph(DEV, am, fdim)
    assert d_dev.h2d_bytes <= d_host.h2d_bytes if am else d_dev.h2d_bytes < d_host.h2d_bytes
    if not am:
        assert torch.equal(d_dev.views['f_bonds'].view(torch.uint8).reshape(-1)[:d_host.views['f_bonds'].numel()],
                           d_host.views['f_bonds'])
    args = TrainArgs(**{'hidden_size': 128, 'depth': 3, **extra})
    outs = []
    for g in (g_host, g_dev):
        torch.manual_seed(0)
        enc = MPNEncoder(args, get_atom_fdim(), fdim)
        synthetic.fill_parameters(enc, 3)
        enc = enc.to(DEV)
        out = enc(g)
        out.square().sum().backward()
        outs.append((out.detach().cpu(), [p.grad.detach().cpu() for p in enc.parameters() if p.grad is not None]))
        with torch.no_grad():
            outs[-1] += (enc.eval()(g).cpu(),)
    (o1, g1, e1), (o2, g2, e2) = outs
    assert torch.equal(o1, o2) and torch.equal(e1, e2)
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))


@pytest.mark.parametrize('extra', [dict(), dict(activation='PReLU', bias=True)])
def test_dropout_masks_agree_across_paths(extra):
    """Training-mode dropout (counter-hash masks on each W_h update and on W_o, none on the input
    layer's message = act(input), mpn.py:97/124/134): the grad-enabled forward (unblocked kernels)
    and the no-grad forward (molecule-blocked fused kernels) drop the same elements."""
    args = TrainArgs(hidden_size=96, depth=3, dropout=0.25, **extra)
    g = BatchMolGraph(synthetic.make_batch('polymer', 32, 21))
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 8)
    enc = enc.to(DEV).train()
    torch.manual_seed(123)
    with torch.no_grad():
        a = enc(g)
    torch.manual_seed(123)
    b = enc(g)
    assert golden_io.normwise(a.cpu().numpy(), b.detach().cpu().numpy()) <= TOL


def test_training_step_fused_adam_and_pinned_targets():
    """train_step on the GPU (pinned target table, the HIP Adam from build_optimizer) agrees with the
    same steps through torch's plain per-parameter Adam (the reference's optimizer)."""
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=64, depth=3, device=DEV)
    g = BatchMolGraph(synthetic.make_batch('polymer', 16, 9), device_bond_features=True)
    targets = [[0.1 * i - 0.5, None if i % 5 == 0 else float(i % 3)] for i in range(16)]
    args.num_tasks = 2
    models, opts = [], []
    for fused in (True, False):
        torch.manual_seed(0)
        m = MoleculeModel(args)
        initialize_weights(m)
        m = m.to(DEV)
        opt = build_optimizer(m, 1e-3) if fused else torch.optim.Adam(m.parameters(), lr=1e-3, foreach=False)
        assert type(opt).__name__ == ('HipAdam' if fused else 'Adam')
        models.append(m)
        opts.append(opt)
    for _ in range(3):
        losses = [train_step(m, [g], targets, get_loss_func('regression'), o) for m, o in zip(models, opts)]
        assert abs(float(losses[0]) - float(losses[1])) <= 1e-6 * max(1.0, abs(float(losses[1])))
    for (n, a), b in zip(models[0].named_parameters(), models[1].parameters()):
        d = float((a - b).detach().abs().max())
        assert d <= 1e-6, (n, d)


@pytest.mark.parametrize('act,bias', [('ReLU', False), ('PReLU', True), ('tanh', True)])
def test_direct_training_step_equals_autograd_step(act, bias):
    """train_step's direct path (no autograd engine: the encoder's training forward, the fused head's
    gradients and the native backward written straight into .grad) gives the autograd path's losses,
    gradients and parameters bitwise, over several steps (gradients overwritten, never accumulated), with
    and without a GradBucket."""
    from chemprop_amd.dp import GradBucket
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=48, depth=3, device=DEV, activation=act, bias=bias)
    graphs = [BatchMolGraph(synthetic.make_batch('polymer', 12, 30 + i), device_bond_features=True) for i in range(3)]
    targets = [[[0.3 * j - 1.0 + i] for j in range(12)] for i in range(3)]
    for use_bucket in (False, True):
        res = []
        for direct in (True, False):
            torch.manual_seed(0)
            m = MoleculeModel(args)
            initialize_weights(m)
            m = m.to(DEV)
            bucket = GradBucket(m) if use_bucket else None
            opt = build_optimizer(m, 1e-3)
            losses = [float(train_step(m, [g], t, get_loss_func('regression'), opt, bucket=bucket, direct=direct))
                      for _ in range(2) for g, t in zip(graphs, targets)]
            res.append((losses, [q.detach().clone() for q in m.parameters()],
                        [q.grad.clone() for q in m.parameters() if q.requires_grad]))
        assert res[0][0] == res[1][0]
        assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))
        assert all(torch.equal(a, b) for a, b in zip(res[0][2], res[1][2]))


def test_classification_steps_take_the_fused_direct_path():
    """A classification MoleculeModel (BCEWithLogitsLoss on the FFN's logits, train.py:55-74) trains
    through the fused head and the direct step: the same losses and parameters bitwise as the fused head
    under autograd, and within 1e-5 of the torch ops (fused_head=False) over four steps."""
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import _fusable_head, build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=48, depth=3, device=DEV, dataset_type='classification')
    args.num_tasks = 2
    graphs = [BatchMolGraph(synthetic.make_batch('polymer', 12, 60 + i), device_bond_features=True) for i in range(2)]
    rng = np.random.default_rng(3)
    targets = [[[None if rng.random() < 0.15 else float(rng.random() < 0.5) for _ in range(2)] for _ in range(12)]
               for _ in range(2)]
    lf = get_loss_func('classification')
    res = []
    for mode in ('direct', 'autograd', 'torch'):
        torch.manual_seed(0)
        m = MoleculeModel(args)
        initialize_weights(m)
        m = m.to(DEV)
        assert _fusable_head(m, lf, 'classification') is not None
        opt = build_optimizer(m, 1e-3)
        losses = [float(train_step(m, [g], t, lf, opt, dataset_type='classification', direct=mode == 'direct',
                                   fused_head=mode != 'torch'))
                  for _ in range(2) for g, t in zip(graphs, targets)]
        res.append((losses, [q.detach().clone() for q in m.parameters()]))
    assert res[0][0] == res[1][0]
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))
    for a, b in zip(res[0][0], res[2][0]):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (a, b)
    for a, b in zip(res[0][1], res[2][1]):
        assert golden_io.normwise(a.cpu().numpy(), b.cpu().numpy()) <= 1e-4


def test_direct_steps_without_host_sync_read_each_steps_targets():
    """The direct step's head kernel reads its loss table in place from a ring of 4 coherent mapped host
    buffers.  Ten steps with ten different target sets and NO host sync between them (the losses stay on
    the device until the end) give bitwise the losses and parameters of the copy path (autograd step,
    targets copied to the device): every rewritten ring slot is seen by the kernel that reads it."""
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=48, depth=3, device=DEV)
    g = BatchMolGraph(synthetic.make_batch('polymer', 12, 40), device_bond_features=True)
    targets = [[[0.25 * j - 2.0 + 0.7 * i] for j in range(12)] for i in range(10)]
    res = []
    for direct in (True, False):
        torch.manual_seed(0)
        m = MoleculeModel(args)
        initialize_weights(m)
        m = m.to(DEV)
        opt = build_optimizer(m, 1e-3)
        losses = [train_step(m, [g], t, get_loss_func('regression'), opt, direct=direct) for t in targets]
        torch.cuda.synchronize()
        res.append(([float(x) for x in losses], [q.detach().clone() for q in m.parameters()]))
    assert len(set(res[0][0])) == 10
    assert res[0][0] == res[1][0]
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


@pytest.mark.parametrize('hidden', [48, 300])
def test_adam_repack_rewrites_the_training_pack_bytewise(hidden):
    """The direct step's packed weights are rewritten by HipAdam's own pass (wdmpnn_adam_step_repack): after
    every step the persistent training pack is bytewise a fresh wdmpnn_pack_params of the updated weights
    (plain, transposed, bf16x3 tiles of 64 and 80 rows, W_h's fp16 pairs and scale word), only the first
    forward packs, and the losses and parameters are bitwise those of steps that pack before every forward."""
    import ctypes
    from chemprop_amd import _native
    from chemprop_amd import train as T
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=hidden, depth=3, device=DEV)
    graphs = [BatchMolGraph(synthetic.make_batch('polymer', 12, 50 + i), device_bond_features=True) for i in range(2)]
    targets = [[[0.3 * j - 1.0 + i] for j in range(12)] for i in range(2)]
    res = []
    try:
        for repack in (True, False):
            T.ADAM_REPACK = repack
            torch.manual_seed(0)
            m = MoleculeModel(args)
            initialize_weights(m)
            m = m.to(DEV)
            enc = m.encoder.encoder[0]
            opt = build_optimizer(m, 1e-3)
            packs = []
            real = enc._packed_params
            enc._packed_params = lambda *a, **k: (packs.append(1), real(*a, **k))[1]
            losses = []
            for step in range(4):
                g, t = graphs[step % 2], targets[step % 2]
                losses.append(float(train_step(m, [g], t, get_loss_func('regression'), opt)))
                if repack:
                    tp = enc._train_pack
                    gs, cfg, p = tp['gs'], tp['cfg'], tp['p']
                    fresh = torch.zeros_like(tp['buf'])
                    _native.check(_native.lib().wdmpnn_pack_params(ctypes.byref(gs), ctypes.byref(p), ctypes.byref(cfg),
                                                                   fresh.data_ptr(), fresh.numel(),
                                                                   _native.current_stream(DEV)), 'pack')
                    torch.cuda.synchronize()
                    # bytewise equal except W_h's partial scale words (pack_kernel's 64 per-workgroup maxima
                    # in a fresh pack, adam_kernel's per-workgroup maxima after a repack): one 256-byte aligned
                    # run of 65 + nw words whose word 64, the folded scale the layers read, is equal
                    diff = (fresh != tp['buf']).nonzero().flatten().cpu()
                    if diff.numel():
                        start = int(diff[0]) // 256 * 256
                        nw = (-(-hidden // 32)) ** 2
                        assert int(diff[-1]) < start + 4 * (65 + nw), (step, fresh.numel(), diff[:16].tolist(),
                                                                       diff[-16:].tolist(), diff.numel())
                        assert torch.equal(fresh[start + 256:start + 260], tp['buf'][start + 256:start + 260])
            del enc._packed_params
            res.append((losses, [q.detach().clone() for q in m.parameters()], len(packs)))
    finally:
        T.ADAM_REPACK = True
    assert res[0][2] == 1 and res[1][2] == 4
    assert res[0][0] == res[1][0]
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


@pytest.mark.parametrize('kind', ['adam', 'adamw'])
def test_hip_adam_matches_torch_adam(kind):
    """HipAdam (one wdmpnn_adam_step launch) vs torch's single-tensor Adam / AdamW over 6 steps: weight
    decay, an lr changed between steps (what NoamLR does), a parameter without gradient, more than 16
    tensors (two launches) and a state_dict round trip; every parameter and moment within 1e-6."""
    from chemprop_amd.train import HipAdam
    gen = torch.Generator().manual_seed(5)
    shapes = [(300, 147), (300,), (1,), (7, 3), (1025,)] + [(13 + k,) for k in range(14)]
    base = [torch.randn(s, generator=gen) for s in shapes]
    ref = [torch.nn.Parameter(t.clone()) for t in base]
    hip = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    cls = torch.optim.AdamW if kind == 'adamw' else torch.optim.Adam
    o_ref = cls(ref, lr=1e-2, weight_decay=0.05, foreach=False)
    o_hip = HipAdam(hip, lr=1e-2, weight_decay=0.05, decoupled=kind == 'adamw')
    for step in range(6):
        grads = [torch.randn(s, generator=gen) for s in shapes]
        for k, (a, b, g) in enumerate(zip(ref, hip, grads)):
            a.grad = None if k == 3 else g.clone()
            b.grad = None if k == 3 else g.clone().to(DEV)
        for o in (o_ref, o_hip):
            o.param_groups[0]['lr'] = 1e-2 / (1 + step)
        o_ref.step()
        o_hip.step()
        if step == 2:
            sd = o_hip.state_dict()
            o_hip = HipAdam(hip, lr=1e-2, weight_decay=0.05, decoupled=kind == 'adamw')
            o_hip.load_state_dict(sd)
    for k, (a, b) in enumerate(zip(ref, hip)):
        d = float((a.detach() - b.detach().cpu()).abs().max())
        assert d <= 1e-6 * max(1.0, float(a.detach().abs().max())), (k, d)
        if k != 3:
            for name in ('exp_avg', 'exp_avg_sq'):
                x, y = o_ref.state[a][name], o_hip.state[b][name].cpu()
                assert float((x - y).abs().max()) <= 1e-6 * max(1.0, float(x.abs().max())), (k, name)
    assert 3 not in [i for i, b in enumerate(hip) if b in o_hip.state]


def test_hip_adam_parameter_without_gradient_on_some_steps():
    """torch's Adam keeps a step count per parameter: a parameter whose gradient is None on some steps
    (a layer used only under some conditions) lags behind; HipAdam groups its launches by step count and
    matches torch on every parameter and moment."""
    from chemprop_amd.train import HipAdam
    gen = torch.Generator().manual_seed(9)
    shapes = [(64, 33), (17,), (5, 5)]
    base = [torch.randn(s, generator=gen) for s in shapes]
    ref = [torch.nn.Parameter(t.clone()) for t in base]
    hip = [torch.nn.Parameter(t.clone().to(DEV)) for t in base]
    o_ref = torch.optim.Adam(ref, lr=1e-2, foreach=False)
    o_hip = HipAdam(hip, lr=1e-2)
    for step in range(7):
        for k, (a, b, s) in enumerate(zip(ref, hip, shapes)):
            g = torch.randn(s, generator=gen)
            skip = (k == 1 and step in (1, 2, 5)) or (k == 2 and step == 0)
            a.grad = None if skip else g.clone()
            b.grad = None if skip else g.clone().to(DEV)
        o_ref.step()
        o_hip.step()
    for a, b in zip(ref, hip):
        assert float((a.detach() - b.detach().cpu()).abs().max()) <= 1e-6 * max(1.0, float(a.detach().abs().max()))
        assert int(o_ref.state[a]['step']) == int(o_hip.state[b]['step'])
        for name in ('exp_avg', 'exp_avg_sq'):
            x, y = o_ref.state[a][name], o_hip.state[b][name].cpu()
            assert float((x - y).abs().max()) <= 1e-6 * max(1.0, float(x.abs().max()))


@pytest.mark.parametrize('b,tasks,act,features,dataset', [(128, 1, 'ReLU', 0, 'regression'),
                                                           (16, 2, 'tanh', 0, 'regression'),
                                                           (33, 3, 'ELU', 5, 'regression'),
                                                           (8, 1, 'LeakyReLU', 0, 'regression'),
                                                           (20, 2, 'SELU', 0, 'regression'),
                                                           (128, 1, 'ReLU', 0, 'classification'),
                                                           (33, 3, 'tanh', 5, 'classification')])
def test_fused_head_loss_matches_torch(b, tasks, act, features, dataset):
    """The fused FFN head + masked loss (wdmpnn_head_mse: the train step's default path; MSE for regression,
    BCE on the logits for classification) gives the torch head's loss and every gradient (head, encoder)
    within 1e-5; missing targets, target and data weights, several tasks, extra molecule features, and a
    scaled incoming gradient."""
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import _fusable_head, batch_loss, get_loss_func, head_loss
    args = TrainArgs(hidden_size=96, depth=3, activation=act, ffn_hidden_size=80, device=DEV,
                     dataset_type=dataset)
    args.num_tasks = tasks
    if features:
        args.use_input_features, args.features_size = True, features
    g = BatchMolGraph(synthetic.make_batch('polymer', b, 31 + b), device_bond_features=True)
    rng = np.random.default_rng(b)
    value = (lambda: float(rng.normal())) if dataset == 'regression' else (lambda: float(rng.random() < 0.4))
    targets = [[None if rng.random() < 0.2 else value() for _ in range(tasks)] for _ in range(b)]
    tw = list(rng.uniform(0.5, 1.5, tasks))
    dw = list(rng.uniform(0.5, 1.5, b))
    feats = [rng.normal(size=features).astype(np.float32) for _ in range(b)] if features else None
    torch.manual_seed(0)
    m = MoleculeModel(args)
    initialize_weights(m)
    m = m.to(DEV).train()
    lf = get_loss_func(dataset)
    head = _fusable_head(m, lf, dataset)
    assert head is not None
    res = []
    for fused in (True, False):
        m.zero_grad(set_to_none=True)
        if fused:
            loss = head_loss(m.encoder([g], feats), head, targets, tw, dw)
        else:
            loss = batch_loss(m([g], feats), targets, lf, dataset, tw, dw)
        (loss * 0.75).backward()
        res.append((float(loss), {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}))
    (l0, g0), (l1, g1) = res
    assert abs(l0 - l1) <= 1e-6 * max(1.0, abs(l1))
    assert g0.keys() == g1.keys()
    for n in g1:
        assert golden_io.normwise(g0[n].cpu().numpy(), g1[n].cpu().numpy()) <= TOL, n


def test_inference_plan_cache_follows_config_and_weights():
    """The cached inference call (MPNEncoder._infer: per-graph plan + packed weights) picks up a changed
    aggregation and in-place weight updates, and agrees with the
    autograd path of the same encoder."""
    args = TrainArgs(hidden_size=48, depth=3, bias=True)
    g = BatchMolGraph(synthetic.make_batch('polymer', 8, 77))
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 3)
    cpu = {n: t.detach().clone() for n, t in enc.named_parameters()}
    enc = enc.to(DEV).eval()
    for agg in ('mean', 'sum', 'norm', 'mean'):
        enc.aggregation = agg
        args.aggregation = agg
        with torch.no_grad():
            out = enc(g)
            again = enc(g)
        ref = mpn_ref.encoder_forward(cpu, g, args)
        assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL, agg
        assert torch.equal(out, again)
        assert len(g.device_graph(DEV, False, get_bond_fdim()).encoder_plans) <= 3
    with torch.no_grad():
        enc.W_h.weight.mul_(0.5)  # in-place: bumps the version counter
        cpu['W_h.weight'].mul_(0.5)
        out = enc(g)
    ref = mpn_ref.encoder_forward(cpu, g, args)
    assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= TOL
    grad_path = enc(g)  # grad enabled: the autograd.Function path
    assert golden_io.normwise(grad_path.detach().cpu().numpy(), ref.numpy()) <= TOL


def test_backward_after_the_batch_graph_is_dropped():
    """The graph may be dropped between forward and backward (a temporary BatchMolGraph inside the call):
    the autograd context keeps its device buffers alive, so the gradients equal those of a run that
    keeps the graph (regression: the context held only raw pointers)."""
    mols = synthetic.make_batch('polymer', 16, 0)
    args = TrainArgs(hidden_size=64, depth=3)
    grads = []
    for keep in (True, False):
        enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
        synthetic.fill_parameters(enc, 1)
        enc = enc.to(DEV)
        g = BatchMolGraph(mols)
        out = enc(g) if keep else enc(BatchMolGraph(mols))
        if not keep:
            del g
        junk = [torch.randn(1 << 20, device=DEV) for _ in range(8)]  # reuse any freed device memory
        out.square().sum().backward()
        del junk
        grads.append([p.grad.cpu() for p in enc.parameters() if p.grad is not None])
    assert all(torch.equal(a, b) for a, b in zip(*grads))


def _small_batch(seed):
    """QM9-sized molecules plus an empty molecule, a single atom and a molecule with 9 atoms in one
    ring-closed chain: every block <= 32 bond rows / atoms (the one-launch forward's domain)."""
    rng = np.random.default_rng(seed)
    mols = synthetic.make_batch('qm9', 40, seed)
    mols[5:5] = [synthetic.empty_graph(), synthetic.single_atom_graph(rng)]
    return mols


@pytest.mark.parametrize('act,bias,agg', [('ReLU', False, 'mean'), ('LeakyReLU', True, 'sum'), ('PReLU', True, 'norm'),
                                          ('tanh', False, 'mean'), ('SELU', True, 'mean'), ('ELU', False, 'sum')])
def test_one_launch_small_block_forward_is_bitwise_the_four_launch_forward(act, bias, agg):
    """QM9-sized blocks run the whole inference forward as ONE launch (small_fwd.hpp).  It must give
    torch.equal outputs to the four-launch fused forward with register-staged layers (WdConfig.gemm_variant
    12: the same arithmetic in the same order) for every activation, with and without biases, every
    aggregation, on the default block plan (about one molecule per block) and on blocks of two to three
    molecules (block_target=20: <= 32 rows), and match the fp32 oracle at 1e-5, as must the four-launch
    forward on fp16 pair tiles (variant 13: per-tile scales, a different but fp32-accurate rounding)."""
    args = TrainArgs(hidden_size=300, depth=3, activation=act, bias=bias, aggregation=agg)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, 13)
    p = {n: t.detach().clone() for n, t in enc.named_parameters()}
    enc = enc.to(DEV).eval()
    for target in (None, 20):
        mols = _small_batch(21)
        g = BatchMolGraph(mols, device_bond_features=True) if target is None else \
            BatchMolGraph(mols, device_bond_features=True, block_target=target)
        dg = g.device_graph(DEV, False, get_bond_fdim())
        assert 0 < dg.struct.blk_max_bonds <= 32 and dg.struct.blk_max_atoms <= 32
        assert target is None or dg.struct.n_blocks <= 24  # several molecules per block
        with torch.no_grad():
            one = enc(g)
            enc._gemm_variant = 12
            four = enc(g)
            enc._gemm_variant = 13
            four_pairs = enc(g)
            enc._gemm_variant = 0
        torch.cuda.synchronize()
        assert torch.equal(one, four), (target, float((one - four).abs().max()))
        with torch.no_grad():
            ref = mpn_ref.encoder_forward(p, g, args)
        assert golden_io.normwise(one.cpu().numpy(), ref.numpy()) <= TOL
        assert golden_io.normwise(four_pairs.cpu().numpy(), ref.numpy()) <= TOL
