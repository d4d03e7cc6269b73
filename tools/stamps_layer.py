"""Phase timeline of the fused message-passing layer kernel (experiment build with WD_STAMPS=1, selected
with WDMPNN_LIB): one polymer B=64 forward (depth 3: the first layer, then the last), per workgroup
s_memrealtime stamps (100 MHz, chip-wide) at: 0 start, 1 params + scale loaded, 2 GEMM done (wave 0),
3 all waves past the GEMM, 4 epilogue: residual issued, 5 atom sums done, 6 end.
    WDMPNN_LIB=exp/libwdmpnn_stamps.so python tools/stamps_layer.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

import bench  # noqa: E402
from chemprop_amd import TrainArgs, _native, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim  # noqa: E402

dev = torch.device('cuda:0')
kind = sys.argv[1] if len(sys.argv) > 1 else 'polymer'
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
enc._gemm_variant = int(os.environ.get('WD_VARIANT', '0'))  # (13: pair operands)
g = BatchMolGraph(synthetic.make_batch(kind, 64, 1000), device_bond_features=True)
g.device_graph(dev, False, get_bond_fdim())
L = _native.lib()
L.wdmpnn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(8192 * 16, dtype=np.uint64)
names = ['params', 'gemm(w0)', 'gemm(all)', 'acc+resid', 'atom sums', 'X+store']
with torch.no_grad():
    for _ in range(30):
        enc(g)
    for rep in range(3):
        torch.cuda.synchronize()
        enc(g)
        torch.cuda.synchronize()
        _native.check(L.wdmpnn_debug_stamps(buf.ctypes.data, buf.nbytes), 'stamps')
        q = buf.reshape(8192, 16).astype(np.int64)
        for layer, off in (('first', 0), ('last', 8)):
            t = q[:, off:off + 7]
            nwg = int((t[:, 0] > 0).sum())
            t = t[:nwg]
            t0 = t[:, 0].min()
            rel = (t - t0) * 10  # ns
            dur = np.diff(t, axis=1) * 10
            print(f'rep {rep} {layer}: {nwg} WGs, span {rel[:, 6].max() / 1e3:.2f} us; start spread '
                  f'p50 {np.median(rel[:, 0]) / 1e3:.2f} max {rel[:, 0].max() / 1e3:.2f} us; end p10/p50/max '
                  f'{np.percentile(rel[:, 6], 10) / 1e3:.2f}/{np.median(rel[:, 6]) / 1e3:.2f}/{rel[:, 6].max() / 1e3:.2f} us')
            print('   phase p50 (us): ' + '  '.join(f'{n} {np.median(dur[:, k]) / 1e3:.2f}' for k, n in enumerate(names)))
            print('   phase p90 (us): ' + '  '.join(f'{n} {np.percentile(dur[:, k], 90) / 1e3:.2f}' for k, n in enumerate(names)))
        buf[:] = 0

# per-chunk loop stamps of the last launch (the last layer): consumer wave 0 (0 before its B wait, 1 after,
# 2 after the barrier, 3 after its MFMAs) and producer wave 4 (4 before a store, 5 after it), shader clock
buf2 = np.zeros(8192 * 16 + 512 * 16 * 8, dtype=np.uint64)
with torch.no_grad():
    torch.cuda.synchronize()
    enc(g)
    torch.cuda.synchronize()
    _native.check(L.wdmpnn_debug_stamps(buf2.ctypes.data, buf2.nbytes), 'stamps')
ls = buf2[8192 * 16:].reshape(512, 16, 8).astype(np.int64)[:256]
print('chunk  Bwait  barrier  mfma(w0)  period | prod store  (cycles, median over WGs)')
for kc in range(10):
    c = ls[:, kc]
    nxt = ls[:, kc + 1, 0] if kc < 9 else c[:, 3]
    print(f'{kc:5d} {np.median(c[:, 1] - c[:, 0]):6.0f} {np.median(c[:, 2] - c[:, 1]):8.0f} '
          f'{np.median(c[:, 3] - c[:, 2]):9.0f} {np.median(nxt - c[:, 0]):7.0f} | '
          f'{np.median(c[:, 5] - c[:, 4]) if kc < 9 else 0:10.0f}')
