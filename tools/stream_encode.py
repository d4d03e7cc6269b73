"""The streamed inference workload alone (NativeFeed.encode), for profiling: python tools/stream_encode.py
[graphs] [producers] [k]"""
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
producers = int(sys.argv[2]) if len(sys.argv) > 2 else 12
k = int(sys.argv[3]) if len(sys.argv) > 3 else 8
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
for rep in range(int(os.environ.get('REPS', '2'))):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e = 0
    with torch.no_grad():
        nb = int(os.environ.get('FIRST', graphs // 64)) if rep == 0 else graphs // 64
        for out, got, ed, _ in NativeFeed('polymer', 64, nb, seed=5 + rep, device=dev, producers=producers,
                                          lean=True, slots=4 * k).encode(enc, k):
            e += ed
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f'rep {rep} producers {producers} k {k}: {e / dt / 1e6:.1f} M edges/s ({dt / nb * 1e6:.1f} us/batch, {nb} batches)',
          flush=True)
