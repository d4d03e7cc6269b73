"""Single-stream QM9-shaped forward time against the molecule-block plan (BatchMolGraph.block_target)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402

dev = torch.device('cuda:0')
enc = MPNEncoder(TrainArgs(hidden_size=300, depth=3, device=dev), get_atom_fdim(), get_bond_fdim())
initialize_weights(enc)
enc = enc.to(dev).eval()
for target in [int(x) for x in os.environ.get('TARGETS', '64 32 16 8 1 64').split()]:
    gs = [BatchMolGraph(synthetic.make_batch('qm9', 64, 5000 + i), device_bond_features=True, block_target=target)
          for i in range(8)]
    with torch.no_grad():
        for g in gs:
            enc(g)
        torch.cuda.synchronize()
        n = 400
        t0 = time.perf_counter()
        for i in range(n):
            enc(gs[i % 8])
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
    print(f'block_target {target:3d}: blocks {gs[0].molecule_blocks().shape[0]:3d}  {dt * 1e6:6.1f} us per forward (one in flight)')
