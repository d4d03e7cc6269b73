"""Worker functions for the world-size-2 gloo tests (spawned processes import this module)."""
import os
import sys

import torch
import torch.distributed as dist
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]

from chemprop_amd import dp  # noqa: E402
from chemprop_amd.train import get_loss_func, train_step  # noqa: E402


class TinyModel(nn.Module):
    """Stand-in for MoleculeModel with the same forward signature (CPU, gloo tests only)."""

    def __init__(self):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(6, 16), nn.ReLU(), nn.Linear(16, 2))

    def forward(self, batch, features_batch=None):
        return self.net(batch)


def data(seed, n=8):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 6, generator=g)
    y = [[float(v) if (i + j) % 5 else None for j, v in enumerate(row)] for i, row in enumerate(torch.randn(n, 2, generator=g))]
    return x, y


def run(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    env = dp.init_distributed('gloo')
    torch.manual_seed(100 + rank)  # deliberately different init per rank
    model = TinyModel()
    dp.broadcast_parameters(model)
    bucket = dp.GradBucket(model)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    batches = dp.shard([data(s) for s in range(6)], env.rank, env.world_size)
    loss_func = get_loss_func('regression')
    for x, y in batches[:2]:
        train_step(model, x, y, loss_func, opt, bucket=bucket)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save({'params': [g for g in gathered], 'nbytes': bucket.nbytes}, out_path)
    dist.barrier()
    dist.destroy_process_group()


class HeadModel(nn.Module):
    """An encoder part and an ``ffn`` head: GradBucket's default early segment is the head."""

    def __init__(self):
        super().__init__()
        self.enc = nn.Linear(6, 16)
        self.ffn = nn.Sequential(nn.ReLU(), nn.Linear(16, 2))


def run_segments(rank, world, port, out_path):
    """Rank-dependent gradients all-reduced in two segments (start_early: the head, then the rest)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dp.init_distributed('gloo')
    torch.manual_seed(0)
    model = HeadModel()
    bucket = dp.GradBucket(model)
    for k, p in enumerate(model.parameters()):
        p.grad.copy_(torch.full_like(p, float(10 * k + rank + 1)))
    bucket.start_early()
    n_early_launched = len(bucket._works)
    bucket.start_allreduce()
    bucket.finish_allreduce()
    if rank == 0:
        torch.save({'grads': [p.grad.clone() for p in model.parameters()], 'n_early': bucket.n_early,
                    'early_launched': n_early_launched, 'head_first': bucket.params[0] is model.ffn[1].weight},
                   out_path)
    dist.barrier()
    dist.destroy_process_group()


def run_mixed_paths(rank, world, port, out_path):
    """Rank 0 takes the direct step's order (start_early, then start_allreduce), rank 1 the autograd
    path's (start_allreduce only): both must issue the same two collectives and average every gradient."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dp.init_distributed('gloo')
    torch.manual_seed(0)
    model = HeadModel()
    bucket = dp.GradBucket(model)
    for k, p in enumerate(model.parameters()):
        p.grad.copy_(torch.full_like(p, float(10 * k + rank + 1)))
    if rank == 0:
        bucket.start_early()
    bucket.start_allreduce()
    n_works = len(bucket._works)
    bucket.finish_allreduce()
    res = [None] * world
    dist.all_gather_object(res, {'works': n_works, 'grads': [p.grad.clone() for p in model.parameters()]})
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


def run_gpu(rank, world, port, out_path):
    """Two ranks on cuda:0 (gloo process group): MoleculeModel with the HIP encoder, DP training with the
    flat GradBucket all-reduce, fused Adam, on disjoint synthetic polymer shards."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from chemprop_amd import TrainArgs, synthetic
    from chemprop_amd.featurization import BatchMolGraph
    from chemprop_amd.model import MoleculeModel
    from chemprop_amd.nn_utils import initialize_weights
    from chemprop_amd.train import build_optimizer
    env = dp.init_distributed('gloo')
    dev = torch.device('cuda:0')
    args = TrainArgs(hidden_size=64, depth=3, device=dev)
    torch.manual_seed(200 + rank)  # deliberately different init per rank: the broadcast must fix it
    model = MoleculeModel(args)
    initialize_weights(model)
    model = model.to(dev)
    dp.broadcast_parameters(model)
    bucket = dp.GradBucket(model)
    opt = build_optimizer(model, 1e-3)
    shards = dp.shard([gpu_data(s) for s in range(4)], env.rank, env.world_size)
    loss_func = get_loss_func('regression')
    for mols, y in shards:
        train_step(model, [BatchMolGraph(mols)], y, loss_func, opt, bucket=bucket)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save({'params': gathered}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def gpu_data(seed, n=16):
    from chemprop_amd import synthetic
    g = torch.Generator().manual_seed(seed)
    y = [[float(v)] for v in torch.randn(n, generator=g)]
    return synthetic.make_batch('polymer', n, 300 + seed), y
