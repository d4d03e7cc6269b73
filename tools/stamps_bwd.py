"""Per-chunk timeline of a backward GEMM in the training step (experiment build with WD_STAMPS=1 and
WD_STAMP_GEMM=1: gemm_x6_kernel, the last launch = dZ_0 = Y_1 W_h; =2: gemm_tn_x6_kernel with a SEG_ACT
operand, the last launch = dW_h of layer 1).  Wave 0 of each workgroup stamps the shader clock at: 0 step
start (prefetch issue), 1 after the chunk's MFMAs are issued, 2 after the next chunk is staged (its loads
waited for, split, written to LDS), 3 after the barrier.
    WDMPNN_LIB=exp/libwdmpnn_stg1.so python tools/stamps_bwd.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

import bench  # noqa: E402
from chemprop_amd import _native  # noqa: E402

dev = torch.device('cuda:0')
bench.training_workload(dev, steps=3)
torch.cuda.synchronize()
L = _native.lib()
L.wdmpnn_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(8192 * 16 + 512 * 16 * 8, dtype=np.uint64)
_native.check(L.wdmpnn_debug_stamps(buf.ctypes.data, buf.nbytes), 'stamps')
ls = buf[8192 * 16:].reshape(512, 16, 8).astype(np.int64)
live = ls[:, 0, 0] > 0
ls = ls[live]
print(f'{live.sum()} workgroups stamped (first 512)')
print('chunk  mfma-issue  stage-next  barrier  period   (cycles, median / p90 over WGs)')
for kc in range(15):
    c = ls[:, kc]
    ok = c[:, 3] > 0
    if not ok.any():
        break
    c = c[ok]
    nxt = ls[ok, kc + 1, 0]
    per = np.where(nxt > c[:, 0], nxt - c[:, 0], 0)
    f = lambda x: f'{np.median(x):6.0f}/{np.percentile(x, 90):6.0f}'
    print(f'{kc:5d}  {f(c[:, 1] - c[:, 0])}  {f(c[:, 2] - c[:, 1])}  {f(c[:, 3] - c[:, 2])}  {f(per)}')
