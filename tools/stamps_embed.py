"""Phase timeline of the pair-path embed kernel (experiment build with WD_STAMPS=1, selected with WDMPNN_LIB):
one polymer B=64 forward (WD_EMBED_EO_LAST 0), per workgroup s_memrealtime stamps (100 MHz) at: 0 start,
2 loads issued + Eo done, 3 the W_i tile in LDS, 4 Ea done, 5 inp rows stored, 6 tile max published, 7 M_0
pair tiles stored.  (Round 6's log, profiles/round6_stamps_embed.log, also had a stamp 1 after the W_o tile.)
    WDMPNN_LIB=exp/libwdmpnn_est.so python tools/stamps_embed.py"""
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
g = BatchMolGraph(synthetic.make_batch('polymer', 64, 1000), device_bond_features=True)
g.device_graph(dev, False, get_bond_fdim())
L = _native.lib()
L.wdmpnn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
n_main, n_loop = 8192 * 16, 512 * 16 * 8
buf = np.zeros(n_main + n_loop + 8192 * 8, dtype=np.uint64)
names = ['loads+Eo', 'Wi tile', 'Ea', 'inp rows', 'max', 'pairs']
with torch.no_grad():
    for _ in range(30):
        enc(g)
    for rep in range(3):
        torch.cuda.synchronize()
        enc(g)
        torch.cuda.synchronize()
        _native.check(L.wdmpnn_debug_stamps(buf.ctypes.data, buf.nbytes), 'stamps')
        t = buf[n_main + n_loop:].reshape(8192, 8).astype(np.int64)[:, [0, 2, 3, 4, 5, 6, 7]]
        nwg = int((t[:, 0] > 0).sum())
        t = t[:nwg]
        rel = (t - t[:, 0].min()) * 10  # ns
        dur = np.diff(t, axis=1) * 10
        print(f'rep {rep}: {nwg} WGs, span {rel[:, 6].max() / 1e3:.2f} us; start p50 {np.median(rel[:, 0]) / 1e3:.2f} '
              f'max {rel[:, 0].max() / 1e3:.2f} us; end p10/p50/max {np.percentile(rel[:, 6], 10) / 1e3:.2f}/'
              f'{np.median(rel[:, 6]) / 1e3:.2f}/{rel[:, 6].max() / 1e3:.2f} us')
        print('   phase p50 (us): ' + '  '.join(f'{n} {np.median(dur[:, k]) / 1e3:.2f}' for k, n in enumerate(names)))
        print('   phase p90 (us): ' + '  '.join(f'{n} {np.percentile(dur[:, k], 90) / 1e3:.2f}' for k, n in enumerate(names)))
        buf[:] = 0
