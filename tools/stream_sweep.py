"""Streamed-workload sweep (configs[4]): NativeFeed throughput by producer threads -- generation + upload +
device build alone (graphs taken and released, no forward) and with the fused forward (encode, k per
launch set).  python tools/stream_sweep.py [graphs]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs  # noqa: E402
from chemprop_amd.stream import NativeFeed  # noqa: E402
import bench  # noqa: E402

dev = torch.device('cuda:0')
graphs = int(sys.argv[1]) if len(sys.argv) > 1 else 64000
n = graphs // 64
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
with torch.no_grad():
    for _ in NativeFeed('polymer', 64, 32, seed=1, device=dev, lean=True).encode(enc, 8):
        pass
for producers in [int(x) for x in (sys.argv[2].split(',') if len(sys.argv) > 2 else '2,4,8,12,16'.split(','))]:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e = 0
    for g in NativeFeed('polymer', 64, n, seed=5, device=dev, producers=producers, lean=True, slots=32):
        e += g.n_bonds - 1
    torch.cuda.synchronize()
    t_feed = time.perf_counter() - t0
    for k in ((8,) if len(sys.argv) > 2 else (4, 8)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e2 = 0
        with torch.no_grad():
            for out, got, ed, _ in NativeFeed('polymer', 64, n, seed=5, device=dev, producers=producers, lean=True,
                                              slots=4 * k).encode(enc, k):
                e2 += ed
        torch.cuda.synchronize()
        t_enc = time.perf_counter() - t0
        print(f'producers {producers:2d} k {k}: feed only {e / t_feed / 1e6:7.1f} M edges/s '
              f'({t_feed / n * 1e6:6.1f} us/batch)  encode {e2 / t_enc / 1e6:7.1f} M edges/s '
              f'({t_enc / n * 1e6:6.1f} us/batch)', flush=True)
