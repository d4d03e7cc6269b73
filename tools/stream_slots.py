"""Streamed inference (configs[4]) by feed slots: NativeFeed.encode throughput with k = 8 batches per launch
set and 12 producer threads, after the bench's warm-up.  python tools/stream_slots.py [graphs] [slots,...]"""
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
graphs = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
slots = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else '32,64,128').split(',')]
n = graphs // 64
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
with torch.no_grad():
    for _ in NativeFeed('polymer', 64, 1024, seed=99, device=dev, producers=12, lean=True, slots=32).encode(enc, 8):
        pass
    for rep in range(2):
        for s in slots:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e = 0
            for out, got, ed, _ in NativeFeed('polymer', 64, n, seed=2024, device=dev, producers=12, lean=True,
                                              slots=s).encode(enc, 8):
                e += ed
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f'slots {s:4d}: {e / dt / 1e6:7.1f} M edges/s ({n / dt * 64 / 1e6:.2f} M graphs/s)', flush=True)
