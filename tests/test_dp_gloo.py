"""CPU, world size 2 over gloo: the data-parallel layer (chemprop_amd/dp.py) used by multi-GPU training
(SURVEY.md §8(e)).  Ranks start from rank 0's parameters, train on disjoint shards, average
gradients with one all-reduce of the flat bucket, and must end with identical parameters equal to
a single-process run that averages the two shards' gradients."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import dp_worker
from chemprop_amd import dp
from chemprop_amd.train import batch_loss, get_loss_func


def free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_is_disjoint_and_covering():
    items = list(range(23))
    parts = [dp.shard(items, r, 4) for r in range(4)]
    assert sorted(x for p in parts for x in p) == items
    assert all(len(set(a) & set(b)) == 0 for i, a in enumerate(parts) for b in parts[i + 1:])


def test_two_rank_gradient_allreduce_matches_single_process(tmp_path):
    out = str(tmp_path / 'dp.pt')
    mp.spawn(dp_worker.run, args=(2, free_port(), out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    p0, p1 = res['params']
    assert torch.equal(p0, p1), 'ranks diverged'
    # single-process reference: rank 0's init, each step averages the two shards' gradients
    torch.manual_seed(100)
    model = dp_worker.TinyModel()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    lf = get_loss_func('regression')
    shards = [dp.shard([dp_worker.data(s) for s in range(6)], r, 2) for r in range(2)]
    for step in range(2):
        grads = []
        for r in range(2):
            model.zero_grad()
            x, y = shards[r][step]
            batch_loss(model(x), y, lf).backward()
            grads.append([p.grad.clone() for p in model.parameters()])
        for p, g0, g1 in zip(model.parameters(), *grads):
            p.grad = (g0 + g1) / 2
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    assert torch.allclose(p0, ref, atol=1e-6, rtol=1e-5)
    assert res['nbytes'] == 4 * sum(p.numel() for p in model.parameters())


def test_two_segment_allreduce_averages_every_gradient(tmp_path):
    """GradBucket's early segment (the ``ffn`` head, launched by start_early while the encoder backward
    would still run) and the rest: every gradient ends as the mean over the ranks."""
    out = str(tmp_path / 'seg.pt')
    mp.spawn(dp_worker.run_segments, args=(2, free_port(), out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    assert res['head_first'] and res['early_launched'] == 1
    assert res['n_early'] == 16 * 2 + 2
    for k, g in enumerate(res['grads']):
        assert torch.equal(g, torch.full_like(g, 10 * k + 1.5)), k


def test_ranks_on_different_step_paths_issue_the_same_collectives(tmp_path):
    """One rank calls start_early (direct step), the other does not (autograd path): each still issues two
    all-reduces (head segment, then the rest) and every gradient is the mean (no count / size mismatch)."""
    out = str(tmp_path / 'mixed.pt')
    mp.spawn(dp_worker.run_mixed_paths, args=(2, free_port(), out), nprocs=2, join=True)
    res = torch.load(out, weights_only=False)
    assert [r['works'] for r in res] == [2, 2]
    for r in res:
        for k, g in enumerate(r['grads']):
            assert torch.equal(g, torch.full_like(g, 10 * k + 1.5)), k


@pytest.mark.gpu
def test_two_rank_molecule_model_on_gpu_matches_single_process(tmp_path):
    """World size 2 on cuda:0 (gloo): the real MoleculeModel with the HIP encoder (its autograd.Function
    returns fresh gradient tensors that must land in the GradBucket views), fused Adam, two DP steps on
    disjoint shards = one process taking the same steps on the averaged gradients."""
    from chemprop_amd import TrainArgs
    from chemprop_amd.featurization import BatchMolGraph
    from chemprop_amd.model import MoleculeModel
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer
    out = str(tmp_path / 'dp_gpu.pt')
    mp.spawn(dp_worker.run_gpu, args=(2, free_port(), out), nprocs=2, join=True)
    p0, p1 = torch.load(out, weights_only=True)['params']
    assert torch.equal(p0, p1), 'ranks diverged'
    dev = torch.device('cuda:0')
    torch.manual_seed(200)  # rank 0's init (broadcast)
    model = MoleculeModel(TrainArgs(hidden_size=64, depth=3, device=dev))
    initialize_weights(model)
    model = model.to(dev)
    opt = build_optimizer(model, 1e-3)
    lf = get_loss_func('regression')
    shards = [dp.shard([dp_worker.gpu_data(s) for s in range(4)], r, 2) for r in range(2)]
    for step in range(2):
        grads = []
        for r in range(2):
            model.zero_grad()
            mols, y = shards[r][step]
            batch_loss(model([BatchMolGraph(mols)]), y, lf).backward()
            grads.append([p.grad.clone() for p in model.parameters() if p.requires_grad])
        for p, g0, g1 in zip([q for q in model.parameters() if q.requires_grad], *grads):
            p.grad = (g0 + g1) / 2
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    names, off, bad = [n for n, _ in model.named_parameters()], 0, {}
    for n, p in zip(names, model.parameters()):
        d = float((p0[off:off + p.numel()] - ref[off:off + p.numel()]).abs().max()) if p.numel() else 0.0
        if d > 1e-6:
            bad[n] = d
        off += p.numel()
    assert not bad, bad
