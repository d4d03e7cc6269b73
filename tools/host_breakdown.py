"""Host enqueue cost of the inference forward, piece by piece (GPU only; the GPU is held busy by
torch.cuda._sleep so every figure is host time).  Median us per call over REPS calls."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, _native, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402

REPS = 200
dev = torch.device('cuda:0')
torch.manual_seed(0)
enc = MPNEncoder(TrainArgs(hidden_size=300, depth=3), 133, 147)
initialize_weights(enc)
enc = enc.to(dev).eval()
KIND = sys.argv[1] if len(sys.argv) > 1 else 'polymer'
g = BatchMolGraph(synthetic.make_batch(KIND, 64, 3), device_bond_features=True)
dg = g.device_graph(dev, False, get_bond_fdim())
L = _native.lib()
res = {}


def timeit(name, fn):
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    res[name] = ts[len(ts) // 2] * 1e6


with torch.no_grad():
    for _ in range(10):
        enc(g)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(4e9))
    stream = torch.cuda.current_stream(dev)
    timeit('enc(g) total', lambda: enc(g))
    timeit('torch.cuda.current_stream', lambda: torch.cuda.current_stream(dev))
    timeit('_native.current_stream (raw id)', lambda: _native.current_stream(dev))
    timeit('g.device_graph lookup', lambda: g.device_graph(dev, False, 147))
    timeit('dg.use_on (seen stream)', lambda: dg.use_on(stream))
    timeit('enc._param_tuple', enc._param_tuple)
    params = enc._param_tuple()
    gs = enc._graph_struct(dg)
    cfg = enc._config(False)
    timeit('enc._packed_params (hit)', lambda: enc._packed_params(gs, cfg, params, dev, stream=stream))
    timeit('torch.empty ws', lambda: torch.empty(30 << 20, dtype=torch.uint8, device=dev))
    timeit('torch.empty out', lambda: torch.empty((64, 300), dtype=torch.float32, device=dev))
    pstruct, _ = enc._packed_params(gs, cfg, params, dev, stream=stream)
    nbytes = ctypes.c_size_t()
    L.wdmpnn_workspace_bytes(ctypes.byref(gs), ctypes.byref(pstruct), ctypes.byref(cfg), ctypes.byref(nbytes))
    ws = torch.empty(nbytes.value, dtype=torch.uint8, device=dev)
    out = torch.empty((gs.n_mols, 300), device=dev)
    args = (ctypes.byref(gs), ctypes.byref(pstruct), ctypes.byref(cfg), ws.data_ptr(), nbytes.value, out.data_ptr(),
            stream.cuda_stream)
    timeit('native wdmpnn_forward', lambda: L.wdmpnn_forward(*args))
    timeit('native wdmpnn_workspace_bytes', lambda: L.wdmpnn_workspace_bytes(
        ctypes.byref(gs), ctypes.byref(pstruct), ctypes.byref(cfg), ctypes.byref(nbytes)))
    timeit('ctypes no-op (wdmpnn_last_error)', lambda: L.wdmpnn_last_error())
    s2 = torch.cuda.Stream(dev)

    def ctx():
        with torch.cuda.stream(s2):
            pass
    timeit('with torch.cuda.stream(s): pass', ctx)
    timeit('torch.cuda.set_stream x2', lambda: (torch.cuda.set_stream(s2), torch.cuda.set_stream(stream)))

    def ctx_fwd():
        with torch.cuda.stream(s2):
            enc(g)
    timeit('with stream: enc(g)', ctx_fwd)
    ev = torch.cuda.Event()
    timeit('event.record', lambda: ev.record(stream))
    torch.cuda.synchronize()
print(f'# {KIND} B=64')
for k, v in res.items():
    print(f'{k:40s} {v:7.2f} us', flush=True)
