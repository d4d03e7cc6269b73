"""Host cost of a graph's FIRST inference forward against a repeat (GPU only).  The GPU is held busy
by torch.cuda._sleep so that every figure is pure host enqueue time.  Cases, per graph:
  first     a fresh graph (device_graph() already built) on the current stream
  new_strm  the same graph on a stream it has not run on yet
  repeat    the same (graph, stream) again
and the pieces of the first call (DeviceGraph.use_on, the encoder's plan, the packed-weight stream check)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402

dev = torch.device('cuda:0')
N = 16
torch.manual_seed(0)
enc = MPNEncoder(TrainArgs(hidden_size=300, depth=3), 133, 147)
initialize_weights(enc)
enc = enc.to(dev).eval()
graphs = [BatchMolGraph(synthetic.make_batch('polymer', 64, 100 + i), device_bond_features=True) for i in range(N)]
for g in graphs:
    g.device_graph(dev, False, get_bond_fdim())
s2 = torch.cuda.Stream(dev)
with torch.no_grad():
    enc(graphs[0])
    with torch.cuda.stream(s2):
        enc(graphs[0])
    torch.cuda.synchronize()
    torch.cuda._sleep(int(3e9))

    def t(fn):
        t0 = time.perf_counter()
        fn()
        return (time.perf_counter() - t0) * 1e6

    first, new_strm, repeat = [], [], []
    for g in graphs[1:]:
        first.append(t(lambda: enc(g)))
        repeat.append(t(lambda: enc(g)))

        def other():
            with torch.cuda.stream(s2):
                enc(g)
        new_strm.append(t(other))
    torch.cuda.synchronize()


def med(x):
    return sorted(x)[len(x) // 2]


print(f'first {med(first):.1f} us  new_stream {med(new_strm):.1f} us  repeat {med(repeat):.1f} us  '
      f'(medians over {N - 1} graphs; stream context manager included in new_stream)', flush=True)
