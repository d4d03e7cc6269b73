"""A/B the GEMM tile variants (WdConfig.gemm_variant) on the bench workload, interleaved in one
process (cdna_hip_programming.md §5.4 rule 24).  GPU only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402

dev = torch.device('cuda:0')
VARIANTS = [int(v) for v in os.environ.get('VARIANTS', '9 10 11 12').split()]
for kind, b, H, T in (('polymer', 64, 300, 3), ('polymer', 128, 300, 3), ('zinc', 512, 512, 5)):
    g = BatchMolGraph(synthetic.make_batch(kind, b, 3))
    g.device_graph(dev)
    torch.manual_seed(0)
    enc = MPNEncoder(TrainArgs(hidden_size=H, depth=T), 133, 147)
    initialize_weights(enc)
    enc = enc.to(dev).eval()
    res = {v: [] for v in VARIANTS}
    with torch.no_grad():
        for rnd in range(5):
            for v in res:
                enc._gemm_variant = v
                for _ in range(5):
                    enc(g)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(50):
                    enc(g)
                torch.cuda.synchronize()
                res[v].append((time.perf_counter() - t0) / 50 * 1e6)
    print(kind, b, H, T, {v: f'{min(x):.1f}/{sorted(x)[2]:.1f} us' for v, x in res.items()}, flush=True)
