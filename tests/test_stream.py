"""Streamed synthetic batches (chemprop_amd.stream, BASELINE.json configs[4]): generation + staging on
producer threads, H2D + device graph build on a feed stream, overlapped with the encoder on the
compute stream.  Every batch is a full polymer batch; sampled batches are checked against the oracle
on their decoded tables, the whole stream against a second pass (bitwise), and the training step on
streamed batches against the same step on host-packed copies."""
import numpy as np
import pytest
import torch

import golden_io
from chemprop_amd import TrainArgs, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim
from chemprop_amd.mpn import MPNEncoder
from chemprop_amd.stream import StreamedBatches, stage_capacity

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda:0')


def _encoder(hidden=300, depth=3, seed=3, **kw):
    enc = MPNEncoder(TrainArgs(hidden_size=hidden, depth=depth, **kw), get_atom_fdim(), get_bond_fdim())
    synthetic.fill_parameters(enc, seed)
    return enc.to(DEV).eval()


def test_stream_60_batches_vs_oracle_and_replay():
    from oracle import mpn_ref
    enc = _encoder()
    p = {n: t.detach().cpu().clone() for n, t in enc.named_parameters()}
    args = TrainArgs(hidden_size=300, depth=3)
    outs, checked = [], 0
    with torch.no_grad():
        for i, g in enumerate(StreamedBatches('polymer', 64, 60, seed=11, device=DEV, keep_host=True, producers=3)):
            out = enc(g)
            outs.append(out)
            assert g.device_graph(DEV, False, get_bond_fdim()).built_on_device
            if i % 10 == 3:  # sampled batches against the oracle on the decoded reference tables
                ref = mpn_ref.encoder_forward(p, g, args)
                assert golden_io.normwise(out.cpu().numpy(), ref.numpy()) <= 1e-5
                checked += 1
        torch.cuda.synchronize()
        again = [enc(g) for g in StreamedBatches('polymer', 64, 60, seed=11, device=DEV, producers=1, slots=3)]
    assert checked == 6
    assert all(torch.equal(a, b) for a, b in zip(outs, again))  # same seeds, any producer count: same batches
    assert not torch.equal(outs[0], outs[1])


def test_lean_graphs_give_the_same_forward_and_refuse_training():
    """Inference-only device graphs (upload_compact lean: no feature rows, planes or transposed gathers)
    give bitwise the full graphs' fused forward; a training forward or an unblocked path on one raises
    instead of reading the missing arrays."""
    enc = _encoder()
    with torch.no_grad():
        full = [enc(g) for g in StreamedBatches('polymer', 64, 6, seed=21, device=DEV)]
        lean = [enc(g) for g in StreamedBatches('polymer', 64, 6, seed=21, device=DEV, lean=True)]
    assert all(torch.equal(a, b) for a, b in zip(full, lean))
    g = next(iter(StreamedBatches('polymer', 16, 1, seed=4, device=DEV, lean=True)))
    assert g.device_graph(DEV, False, get_bond_fdim()).lean
    with pytest.raises(NotImplementedError):
        enc.train()(g)  # grad enabled: the training forward needs the feature rows for its backward
    enc.eval()
    enc._gemm_variant = 9  # the unblocked f32 path
    with torch.no_grad(), pytest.raises(NotImplementedError):
        enc(g)


def test_streams_of_two_ranks_are_disjoint():
    a = next(iter(StreamedBatches('polymer', 8, 1, seed=5, device=DEV, rank=0, keep_host=True)))
    b = next(iter(StreamedBatches('polymer', 8, 1, seed=5, device=DEV, rank=1, keep_host=True)))
    assert bytes(a._compact[2]) != bytes(b._compact[2])


@pytest.mark.parametrize('kind', ['qm9', 'zinc'])
def test_stream_other_kinds_fit_their_slots(kind):
    enc = _encoder(hidden=64)
    n = 0
    with torch.no_grad():
        for g in StreamedBatches(kind, 128, 5, seed=2, device=DEV):
            assert torch.isfinite(enc(g)).all()
            n += 1
    assert n == 5 and stage_capacity(kind, 128) > 0


def test_training_on_streamed_batches_matches_host_packed():
    """train_step on streamed (device-built) batches = the same steps on BatchMolGraphs packed on the host
    from the decoded tables (compact=False): the same losses and parameters up to the rounding of the
    compact input layer (sums of weight columns instead of a GEMM over one-hot rows)."""
    from chemprop_amd.model import MoleculeModel
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=96, depth=3, device=DEV)
    stream = list(StreamedBatches('polymer', 32, 4, seed=9, device=DEV, keep_host=True))
    host = [BatchMolGraph(_molgraphs(g), compact=False) for g in stream]
    rng = np.random.default_rng(0)
    targets = [[[float(x)] for x in rng.standard_normal(32)] for _ in stream]
    res = []
    for batches in (stream, host):
        torch.manual_seed(0)
        m = MoleculeModel(args)
        initialize_weights(m)
        m = m.to(DEV)
        opt = build_optimizer(m, 1e-3)
        losses = [float(train_step(m, [g], t, get_loss_func('regression'), opt)) for g, t in zip(batches, targets)]
        res.append((losses, [q.detach().cpu() for q in m.parameters()]))
    np.testing.assert_allclose(res[0][0], res[1][0], rtol=1e-5)
    for a, b in zip(res[0][1], res[1][1]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def test_wide_hidden_runs_fused_on_lean_streamed_graphs():
    """hidden 2850 (Hk 2880: 72 scale words per molecule block, more than one per lane): the streamed lean
    graphs -- which only the molecule-blocked fused forward can encode -- give the oracle's output, and
    NativeFeed.encode gives the per-batch forwards bitwise."""
    from chemprop_amd.stream import NativeFeed
    from oracle import mpn_ref
    enc = _encoder(hidden=2850, depth=2, seed=4)
    p = {n: t.detach().cpu().clone() for n, t in enc.named_parameters()}
    with torch.no_grad():
        full = list(StreamedBatches('polymer', 8, 3, seed=31, device=DEV, keep_host=True))
        ref = [enc(g) for g in full]
        lean = [enc(g) for g in StreamedBatches('polymer', 8, 3, seed=31, device=DEV, lean=True)]
        feed = torch.cat([out.clone() for out, *_ in
                          NativeFeed('polymer', 8, 3, seed=31, device=DEV, producers=2, lean=True).encode(enc, k=2)])
        torch.cuda.synchronize()
        want = mpn_ref.encoder_forward(p, full[0], TrainArgs(hidden_size=2850, depth=2))
    assert golden_io.normwise(ref[0].cpu().numpy(), want.numpy()) <= 1e-5
    assert all(torch.equal(a, b) for a, b in zip(ref, lean))
    assert torch.equal(feed, torch.cat(ref))


def _molgraphs(g):
    from test_compact import _as_molgraphs
    return _as_molgraphs(g)


# ---------------------------------------------------------------- native feed (wdmpnn_feed_*)
def test_native_feed_reproduces_the_python_stream():
    """Same seeds -> the same batches in the same order as StreamedBatches (generation, staging, upload
    and device build now on native threads): bitwise equal encoder outputs, any producer / slot count."""
    from chemprop_amd.stream import NativeFeed
    enc = _encoder()
    with torch.no_grad():
        ref = [enc(g) for g in StreamedBatches('polymer', 64, 20, seed=17, device=DEV, rank=1, lean=True)]
        for producers, slots in ((4, None), (1, 3), (7, 16)):
            got = []
            for g in NativeFeed('polymer', 64, 20, seed=17, device=DEV, rank=1, producers=producers, slots=slots,
                                lean=True):
                got.append(enc(g))
            torch.cuda.synchronize()
            assert len(got) == len(ref)
            assert all(torch.equal(a, b) for a, b in zip(ref, got)), (producers, slots)


def test_native_feed_encode_equals_per_batch_forward():
    """NativeFeed.encode (wdmpnn_feed_forward: k batches per launch set, slots reused across calls) gives
    the per-batch forwards' outputs bitwise, for a k that does not divide the batch count."""
    from chemprop_amd.stream import NativeFeed
    enc = _encoder(hidden=96, depth=3, bias=True)
    with torch.no_grad():
        ref = torch.cat([enc(g) for g in StreamedBatches('qm9', 32, 23, seed=3, device=DEV)])
        outs, n, edges = [], 0, 0
        for out, got, e, _ in NativeFeed('qm9', 32, 23, seed=3, device=DEV, producers=3, slots=6, lean=True).encode(enc, k=5):
            outs.append(out.clone())
            n += got
            edges += e
    assert n == 23 and edges > 0
    assert torch.equal(torch.cat(outs), ref)


def test_native_feed_training_matches_python_stream():
    from chemprop_amd.model import MoleculeModel
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.stream import NativeFeed
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=64, depth=3, device=DEV)
    rng = np.random.default_rng(1)
    targets = [[[float(x)] for x in rng.standard_normal(16)] for _ in range(6)]
    res = []
    for make in (lambda: StreamedBatches('polymer', 16, 6, seed=5, device=DEV),
                 lambda: NativeFeed('polymer', 16, 6, seed=5, device=DEV, slots=4),
                 lambda: NativeFeed('polymer', 16, 6, seed=5, device=DEV, slots=4, planes=False)):
        torch.manual_seed(0)
        m = MoleculeModel(args)
        initialize_weights(m)
        m = m.to(DEV)
        opt = build_optimizer(m, 1e-3)
        losses = [float(train_step(m, [g], t, get_loss_func('regression'), opt)) for g, t in zip(make(), targets)]
        res.append((losses, [q.detach().cpu() for q in m.parameters()]))
    for r in res[1:]:  # (the third: graphs without plane tiles, WDMPNN_GRAPH_NO_PLANES)
        assert res[0][0] == r[0]
        assert all(torch.equal(a, b) for a, b in zip(res[0][1], r[1]))


def test_native_feed_bad_spec_raises():
    from chemprop_amd.stream import NativeFeed
    with pytest.raises(ValueError):
        NativeFeed('protein', 8, 1, seed=0, device=DEV)
    f = NativeFeed('qm9', 8, 0, seed=0, device=DEV)
    assert list(f) == []


def test_native_feed_released_batch_raises_and_close_is_safe():
    """A NativeFeed batch used after the next one was requested raises (its slot may hold another batch);
    a feed dropped or closed before or during iteration stops its threads (context manager, close twice,
    garbage collection)."""
    import gc
    from chemprop_amd.stream import NativeFeed
    enc = _encoder(hidden=64)
    with torch.no_grad(), NativeFeed('polymer', 8, 4, seed=2, device=DEV, slots=4) as f:
        it = iter(f)
        g1 = next(it)
        out1 = enc(g1)
        g2 = next(it)
        with pytest.raises(RuntimeError, match='released'):
            enc(g1)
        assert enc(g2).shape == out1.shape
    f.close()  # idempotent
    NativeFeed('polymer', 8, 50, seed=2, device=DEV, slots=4)  # dropped unread
    gc.collect()
    torch.cuda.synchronize()
