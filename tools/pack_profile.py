"""Host-side profile of BatchMolGraph packing + device_graph() (GPU box): cProfile of 40 batches of the
bench workload (device bond features), top functions by own time."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402

dev = torch.device('cuda:0')
mols = [synthetic.make_batch('polymer', 64, 4242 + i) for i in range(8)]


def run(n):
    for i in range(n):
        g = BatchMolGraph(mols[i % 8], device_bond_features=True)
        g.device_graph(dev, False, get_bond_fdim())
    torch.cuda.synchronize()


run(10)
t0 = time.perf_counter()
run(40)
print(f'pack + device_graph: {(time.perf_counter() - t0) / 40 * 1e3:.3f} ms per batch', flush=True)
cProfile.run('run(40)', '/tmp/pack.prof')
pstats.Stats('/tmp/pack.prof').sort_stats('tottime').print_stats(25)
