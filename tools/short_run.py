"""Where a short timed region (the driver's bench.py --steps 20 --warmup 5) loses against a long one: the
bench's headline loop (8 resident polymer B=64 batches, 3 streams) timed for K steps after W warm-up steps,
repeated; per configuration the median us/step, the host enqueue time of the K steps (loop end before
the sync).  'fresh' builds new graphs and a new encoder before each repeat (the GPU idles meanwhile, as
in bench.py between packing and timing); 'spin' keeps the GPU busy ~0.1 s right before the warm-up;
'cpu' spins the host only."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

import bench  # noqa: E402
from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402

dev = torch.device('cuda:0')


def setup():
    graphs = [BatchMolGraph(synthetic.make_batch('polymer', 64, 1000 + i), device_bond_features=True) for i in range(8)]
    for g in graphs:
        g.device_graph(dev, False, get_bond_fdim())
    enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
    return graphs, enc


streams = bench.bench_streams(dev, 3)


def run(graphs, enc, k, w, nstreams=3, pre=None, trace=False):
    ss = streams[:nstreams]
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]

    def step(i):
        with torch.cuda.stream(ss[i % len(ss)]):
            enc(graphs[i % len(graphs)])
            if trace:
                evs[i + 1].record()
    with torch.no_grad():
        step(0)
        torch.cuda.synchronize()
        if pre == 'spin':
            torch.cuda._sleep(int(2e8))
        elif pre == 'gc':
            import gc
            gc.collect()
        elif pre == 'cpu':
            t = time.perf_counter() + 0.1
            while time.perf_counter() < t:
                pass
        for i in range(1, w):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if trace:
            evs[0].record()
        hs = []
        for i in range(k):
            step(i)
            hs.append(time.perf_counter())
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    ends = [evs[0].elapsed_time(e) * 1e3 for e in evs[1:]] if trace else None
    if trace:
        ends = (ends, [(b - a) * 1e6 for a, b in zip([t0] + hs[:-1], hs)])
    return (t2 - t0) / k * 1e6, (t1 - t0) / k * 1e6, ends


for label, k, w, fresh, pre in (('20/5 fresh', 20, 5, True, None), ('20/5 fresh spin', 20, 5, True, 'spin'),
                                ('20/5 fresh cpu', 20, 5, True, 'cpu'), ('20/5 fresh gc', 20, 5, True, 'gc'), ('20/5 warm', 20, 5, False, None),
                                ('200/20 fresh', 200, 20, True, None), ('20/5 warm 1 strm', 20, 5, False, None)):
    walls, hosts = [], []
    g, e = setup()
    for rep in range(5):
        if fresh and rep:
            g, e = setup()
        wall, host, _ = run(g, e, k, w, 1 if '1 strm' in label else 3, pre)
        walls.append(wall)
        hosts.append(host)
    print(f'{label:18s} wall {statistics.median(walls):6.1f} us/step (min {min(walls):6.1f})  host enqueue '
          f'{statistics.median(hosts):6.1f} us/step', flush=True)
g, e = setup()
for pre in (None, 'gc'):
    wall, host, ends = run(g, e, 20, 5, 3, pre, trace=True)
    print(f'trace pre={pre}: wall {wall:.1f} host {host:.1f}; forward ends (us after the first launch): '
          + ' '.join(f'{x:.0f}' for x in ends[0]), flush=True)
    print('   host us per step: ' + ' '.join(f'{x:.0f}' for x in ends[1]), flush=True)
    wall, host, ends = run(g, e, 20, 5, 3, pre, trace=True)
    print(f'   again (warm) wall {wall:.1f} host {host:.1f}; host us per step: ' + ' '.join(f'{x:.0f}' for x in ends[1]),
          flush=True)
    g, e = setup()
