"""QM9-like B=64 forwards (depth 3, hidden 300; 8 resident batches) with 1..6 batches in flight on as many
HIP streams: us per forward (the secondary workload's shape; its stream count is bench.default_streams)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

import bench  # noqa: E402
from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402

dev = torch.device('cuda:0')
kind = sys.argv[1] if len(sys.argv) > 1 else 'qm9'
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
graphs = [BatchMolGraph(synthetic.make_batch(kind, 64, 5000 + i), device_bond_features=True) for i in range(8)]
for g in graphs:
    g.device_graph(dev, False, get_bond_fdim())
ss = bench.bench_streams(dev, 6)
with torch.no_grad():
    for n in range(1, 7):
        best = None
        for rep in range(3):
            for i in range(24):
                torch.cuda.set_stream(ss[i % n])
                enc(graphs[i % 8])
            torch.cuda.set_stream(ss[0])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(400):
                torch.cuda.set_stream(ss[i % n])
                enc(graphs[i % 8])
            torch.cuda.set_stream(ss[0])
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 400 * 1e6
            best = dt if best is None else min(best, dt)
        print(f'{kind}: {n} in flight: {best:.1f} us per forward', flush=True)
