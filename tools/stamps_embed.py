"""Per-workgroup phase times of embed_kernel (experiment build with -DWD_EMBED_STAMP; WDMPNN_LIB = that
build): python tools/stamps_embed.py.  Phases (shader clocks): loads + W_o staging, Eo, W_i staging + Ea,
bond rows + stores drained; plus the wall-clock (100 MHz) spread of workgroup starts / ends."""
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
L.wdmpnn_debug_embed.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(4096 * 8, dtype=np.uint64)
with torch.no_grad():
    for _ in range(20): enc(g)
    for rep in range(3):
        torch.cuda.synchronize(); enc(g); torch.cuda.synchronize()
        L.wdmpnn_debug_embed(buf.ctypes.data, buf.nbytes)
        q = buf.reshape(4096, 8).astype(np.int64)
        n = int((q[:, 6] > 0).sum())
        q = q[:n]
        ph = np.diff(q[:, 0:5], axis=1)
        tot = q[:, 4] - q[:, 0]
        ws, we = q[:, 5] - q[:, 5].min(), q[:, 6] - q[:, 5].min()
        print(f'rep {rep}: {n} workgroups; median cycles loads {np.median(ph[:,0]):.0f} Eo {np.median(ph[:,1]):.0f} '
              f'Wi+Ea {np.median(ph[:,2]):.0f} bonds+drain {np.median(ph[:,3]):.0f} total {np.median(tot):.0f} (p90 {np.percentile(tot,90):.0f}); '
              f'wall start spread {ws.max()/100:.2f} us, last end {we.max()/100:.2f} us, median wg {np.median(we-ws)/100:.2f} us; '
              f'CUs {len(set(q[:,7].tolist()))}')
        # bond phase
        print(f'   start quantiles (us) {np.percentile(ws,[10,50,90,100])/100}; end quantiles {np.percentile(we,[10,50,90,100])/100}')
