"""QM9-shaped batches (B=64, ~900 edges): forward time per batch for several block plans
(BatchMolGraph(block_target=...)), one and two batches in flight.  python tools/block_target_sweep.py"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch
from chemprop_amd import TrainArgs, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim
import bench
dev = torch.device('cuda:0')
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
for kind, B in (('qm9', 64), ('polymer', 64), ('zinc', 512)):
    mols = [synthetic.make_batch(kind, B, 5000 + i) for i in range(8)]
    for tgt in (64, 32, 16, 8):
        gs = [BatchMolGraph(m, device_bond_features=True, block_target=tgt) for m in mols]
        for g in gs:
            g.device_graph(dev, False, get_bond_fdim())
        ss = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
        res = []
        with torch.no_grad():
            for ns in (1, 2):
                for i in range(20):
                    enc(gs[i % 8])
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                n = 200 if kind != 'zinc' else 30
                for i in range(n):
                    with torch.cuda.stream(ss[i % ns]):
                        enc(gs[i % 8])
                torch.cuda.synchronize()
                res.append((time.perf_counter() - t0) / n * 1e6)
        print(f'{kind:8s} block_target {tgt:3d}: blocks {gs[0].molecule_blocks().shape[0]:4d}  one in flight {res[0]:7.1f} us  two {res[1]:7.1f} us', flush=True)
