"""Per-wave phase times of the DMA layer kernel's chunk loop (experiment build with s_memtime stamps in
x6_mainloop; WDMPNN_LIB = that build): python tools/stamps_dma.py"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch
from chemprop_amd import TrainArgs, _native, synthetic
from chemprop_amd.featurization import BatchMolGraph, get_bond_fdim
import bench
dev = torch.device('cuda:0')
enc = bench.make_encoder(TrainArgs(hidden_size=300, depth=3, device=dev), dev)
g = BatchMolGraph(synthetic.make_batch('polymer', 64, 1000), device_bond_features=True)
g.device_graph(dev, False, get_bond_fdim())
L = _native.lib()
L.wdmpnn_debug_loop.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(4096 * 64, dtype=np.uint64)
with torch.no_grad():
    for _ in range(20): enc(g)
    for rep in range(2):
        torch.cuda.synchronize(); enc(g); torch.cuda.synchronize()
        L.wdmpnn_debug_loop(buf.ctypes.data, buf.nbytes)
        q = buf.reshape(4096, 8, 8)[:256].astype(np.int64)
        for w in range(8):
            print(f'rep {rep} wave {w}: loop {np.median(q[:,w,0]):7.0f} vmcnt+lgkm wait {np.median(q[:,w,1]):6.0f} '
                  f'barrier {np.median(q[:,w,2]):6.0f} dma-issue {np.median(q[:,w,3]):6.0f} compute {np.median(q[:,w,4]):7.0f} '
                  f'(a_rows median {np.median(q[:,w,5]):.0f})')
