"""Where the streamed training step's extra time goes: per-step host time of train_step (enqueue only),
of the feed's hand-out (next()), and the synchronised wall time per step, resident (4 cycled graphs)
against streamed (NativeFeed, a new graph every step).  python tools/train_stream_host.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402
from chemprop_amd.model import MoleculeModel  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402
from chemprop_amd.stream import NativeFeed  # noqa: E402
from chemprop_amd.train import build_optimizer, get_loss_func, train_step  # noqa: E402

dev = torch.device('cuda:0')
B, STEPS = 128, int(os.environ.get('STEPS', '400'))
torch.manual_seed(0)
model = MoleculeModel(TrainArgs(hidden_size=300, depth=3, device=dev))
initialize_weights(model)
model = model.to(dev)
opt = build_optimizer(model, 1e-4)
loss = get_loss_func('regression')
rng = torch.Generator().manual_seed(0)
targets = [torch.randn(B, 1, generator=rng).tolist() for _ in range(8)]
res = {}

graphs = []
for i in range(4):
    g = BatchMolGraph(synthetic.make_batch('polymer', B, 7000 + i), device_bond_features=True)
    g.device_graph(dev, False, get_bond_fdim())
    graphs.append(g)
for i in range(20):
    train_step(model, [graphs[i % 4]], targets[i % 8], loss, opt)
torch.cuda.synchronize()
host = 0.0
t0 = time.perf_counter()
for i in range(STEPS):
    h = time.perf_counter()
    train_step(model, [graphs[i % 4]], targets[i % 8], loss, opt)
    host += time.perf_counter() - h
torch.cuda.synchronize()
res['resident'] = {'ms_per_step': (time.perf_counter() - t0) / STEPS * 1e3, 'host_train_step_ms': host / STEPS * 1e3}
# pure host cost: the GPU drained before each step, so nothing in the step waits on it
host = 0.0
for i in range(100):
    torch.cuda.synchronize()
    h = time.perf_counter()
    train_step(model, [graphs[i % 4]], targets[i % 8], loss, opt)
    host += time.perf_counter() - h
torch.cuda.synchronize()
res['resident']['host_idle_gpu_ms'] = host / 100 * 1e3

for planes in (False,):
    for i, g in enumerate(NativeFeed('polymer', B, 20, seed=77, device=dev, planes=planes)):
        train_step(model, [g], targets[i % 8], loss, opt)
    torch.cuda.synchronize()
    host = nxt = 0.0
    it = iter(NativeFeed('polymer', B, STEPS + 100, seed=4048, device=dev, planes=planes))
    t0 = time.perf_counter()
    for i in range(STEPS):
        h = time.perf_counter()
        g = next(it)
        n = time.perf_counter()
        train_step(model, [g], targets[i % 8], loss, opt)
        host += time.perf_counter() - n
        nxt += n - h
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    hi = ni = 0.0
    for i in range(100):
        torch.cuda.synchronize()
        h = time.perf_counter()
        g = next(it)
        n = time.perf_counter()
        train_step(model, [g], targets[i % 8], loss, opt)
        hi += time.perf_counter() - n
        ni += n - h
    torch.cuda.synchronize()
    try:
        next(it)
    except StopIteration:
        pass
    res[f'streamed_planes{int(planes)}'] = {'ms_per_step': dt / STEPS * 1e3, 'host_train_step_ms': host / STEPS * 1e3,
                                            'host_next_ms': nxt / STEPS * 1e3, 'host_idle_gpu_ms': hi / 100 * 1e3,
                                            'next_idle_gpu_ms': ni / 100 * 1e3}
# variants of the streamed loop: one producer thread; slots for every batch (no slot reuse: the feed runs
# ahead freely)
for tag, kw in (('slots_all', dict(slots=STEPS + 2)),):
    it = iter(NativeFeed('polymer', B, STEPS, seed=4048, device=dev, planes=False, **kw))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, g in enumerate(it):
        train_step(model, [g], targets[i % 8], loss, opt)
    torch.cuda.synchronize()
    res[tag] = {'ms_per_step': (time.perf_counter() - t0) / STEPS * 1e3}
# the same streamed graphs, all built before the timed loop (slots for every batch: nothing of the feed
# runs while the steps do)
N2 = 200
it = iter(NativeFeed('polymer', B, N2, seed=4048, device=dev, planes=False, slots=N2 + 2))
pre = [next(it) for _ in range(N2)]
torch.cuda.synchronize()
t0 = time.perf_counter()
for i, g in enumerate(pre):
    train_step(model, [g], targets[i % 8], loss, opt)
torch.cuda.synchronize()
res['prebuilt_streamed'] = {'ms_per_step': (time.perf_counter() - t0) / N2 * 1e3}
t0 = time.perf_counter()
for i in range(N2):
    train_step(model, [pre[i % 4]], targets[i % 8], loss, opt)
torch.cuda.synchronize()
res['prebuilt_4_cycled'] = {'ms_per_step': (time.perf_counter() - t0) / N2 * 1e3}
del pre
try:
    next(it)
except StopIteration:
    pass
print(json.dumps(res))
