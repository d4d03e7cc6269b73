"""Host-side cost of one training step (bench.py training workload): per-phase host enqueue times
(no synchronisation inside the step) and a cProfile of 50 steps."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402
from chemprop_amd.model import MoleculeModel  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402
from chemprop_amd.train import batch_loss, build_optimizer, get_loss_func, train_step  # noqa: E402

dev = torch.device('cuda:0')
args = TrainArgs(hidden_size=300, depth=3, device=dev)
torch.manual_seed(0)
model = MoleculeModel(args)
initialize_weights(model)
model = model.to(dev)
opt = build_optimizer(model, 1e-4)
lf = get_loss_func('regression')
rng = torch.Generator().manual_seed(0)
batches = []
for i in range(4):
    g = BatchMolGraph(synthetic.make_batch('polymer', 128, 7000 + i), device_bond_features=True)
    g.device_graph(dev, False, get_bond_fdim())
    batches.append(([g], torch.randn(128, 1, generator=rng).tolist()))
for i in range(20):
    train_step(model, *batches[i % 4], lf, opt)
torch.cuda.synchronize()

ph = {k: 0.0 for k in ('zero_grad', 'forward', 'loss', 'backward', 'step')}
N = 100
t_all = time.perf_counter()
for i in range(N):
    mb, tb = batches[i % 4]
    t0 = time.perf_counter()
    model.train()
    model.zero_grad()
    t1 = time.perf_counter()
    preds = model(mb, None)
    t2 = time.perf_counter()
    loss = batch_loss(preds, tb, lf)
    t3 = time.perf_counter()
    loss.backward()
    t4 = time.perf_counter()
    opt.step()
    t5 = time.perf_counter()
    ph['zero_grad'] += t1 - t0; ph['forward'] += t2 - t1; ph['loss'] += t3 - t2
    ph['backward'] += t4 - t3; ph['step'] += t5 - t4
torch.cuda.synchronize()
wall = time.perf_counter() - t_all
print({k: round(v / N * 1e6, 1) for k, v in ph.items()}, 'host us/step; wall', round(wall / N * 1e6, 1), 'us/step')

pr = cProfile.Profile()
pr.enable()
for i in range(50):
    train_step(model, *batches[i % 4], lf, opt)
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats('tottime').print_stats(30)
pstats.Stats(pr).sort_stats('cumulative').print_stats(40)
