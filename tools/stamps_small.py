"""Phase timeline of the one-launch small-block forward (small_fwd.hpp; experiment build with WD_STAMPS=1,
selected with WDMPNN_LIB): one QM9-like B=64 forward (depth 3), per workgroup s_memrealtime stamps (100 MHz):
0 start, 1 graph staged, 2 Ea, 3 inp, layer 1: 4 operand staged, 5 GEMM (wave 0), 6 atom sums, 7 Z;
layer 2: 8-11; 12 A image, 13 W_o GEMM (wave 0), 14 h, 15 readout done.
    WDMPNN_LIB=exp/libwdmpnn_stamps.so python tools/stamps_small.py"""
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
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
g = BatchMolGraph(synthetic.make_batch('qm9', 64, 5000), device_bond_features=True)
g.device_graph(dev, False, get_bond_fdim())
L = _native.lib()
L.wdmpnn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(8192 * 16, dtype=np.uint64)
names = ['graph', 'Ea', 'inp', 'stage1', 'gemm1', 'gather1', 'Z1', 'stage2', 'gemm2', 'gather2', 'Z2', 'A img',
         'Wo gemm', 'h', 'readout']
with torch.no_grad():
    for _ in range(30):
        enc(g)
    for rep in range(3):
        torch.cuda.synchronize()
        enc(g)
        torch.cuda.synchronize()
        _native.check(L.wdmpnn_debug_stamps(buf.ctypes.data, buf.nbytes), 'stamps')
        q = buf.reshape(8192, 16).astype(np.int64)
        nwg = int((q[:, 0] > 0).sum())
        t = q[:nwg]
        rel = (t - t[:, 0].min()) * 10
        dur = np.diff(t, axis=1) * 10
        print(f'rep {rep}: {nwg} WGs, span {rel[:, 15].max() / 1e3:.2f} us, start spread max {rel[:, 0].max() / 1e3:.2f} us')
        print('   phase p50 (us): ' + '  '.join(f'{n} {np.median(dur[:, k]) / 1e3:.2f}' for k, n in enumerate(names)))
        print('   phase max (us): ' + '  '.join(f'{n} {dur[:, k].max() / 1e3:.2f}' for k, n in enumerate(names)))
        buf[:] = 0
