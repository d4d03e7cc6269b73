"""Stage-by-stage check of the pair-operand forward (round 6) against the register-staged one, on one GPU.

Runs the fused inference forward stopped after each stage (WdConfig.gemm_variant 1ab: a = 1 pair layers, 2
register-staged layers; b = stage) and decodes the intermediate buffers of the encoder's workspace
(wdmpnn_debug_fwd_offsets): M_0 pairs vs act(inp), M_1 pairs vs act(Z_1) of the staged path, A pairs vs
the staged path's bf16x3 A planes, then the outputs.
    python tools/debug_pairs.py [kind] [batch] [hidden]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import torch  # noqa: E402

from chemprop_amd import TrainArgs, _native, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from oracle import mpn_ref  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else 'polymer'
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
H = int(sys.argv[3]) if len(sys.argv) > 3 else 300
dev = torch.device('cuda:0')
args = TrainArgs(hidden_size=H, depth=3)
g = BatchMolGraph(synthetic.make_batch(kind, B, 464), device_bond_features=True)
enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
synthetic.fill_parameters(enc, 12)
p = {n: t.detach().clone() for n, t in enc.named_parameters()}
ref = mpn_ref.encoder_forward(p, g, args).numpy()
enc = enc.to(dev).eval()
L = _native.lib()
L.wdmpnn_debug_fwd_offsets.argtypes = [ctypes.c_void_p] * 4
blocks = np.array(g.molecule_blocks(), np.int64)
Hk = -(-H // 64) * 64
nch = Hk // 32
EPB = int(os.environ.get('WD_EMBED_PAIR_BN', '32'))  # the embed's pair tile width (wdmpnn.hip EPB)


def run(v):
    enc._gemm_variant = v
    with torch.no_grad():
        out = enc(g)
    torch.cuda.synchronize()
    dg = g.device_graph(dev, False, get_bond_fdim())
    gs = enc._graph_struct(dg)
    cfg = enc._config(False)
    cfg.gemm_variant = v
    params = tuple(t.detach().float() if t is not None else None for t in enc._param_tuple())
    pstruct, _ = enc._packed_params(gs, cfg, params, dev)
    offs = (ctypes.c_size_t * 15)()
    _native.check(L.wdmpnn_debug_fwd_offsets(ctypes.addressof(gs), ctypes.addressof(pstruct), ctypes.addressof(cfg),
                                             ctypes.addressof(offs)), 'offsets')
    ws = enc._ws_by_stream[_native.current_stream(dev)].cpu().numpy()
    assert gs.n_blocks == len(blocks), (gs.n_blocks, len(blocks))
    pk = enc._pack_cache[1].cpu().numpy()
    return out.cpu().numpy(), ws, list(offs) + [pk]


def f32(ws, off, n):
    return ws[off:off + 4 * n].view(np.float32)


def words(ws, off, per):
    return ws[off:off + 4 * len(blocks) * per].view(np.uint32).reshape(len(blocks), per)


def scale(w):
    se = np.clip(268 - (w.astype(np.int64) >> 23), 1, 253)
    return np.ldexp(1.0, se - 127)


def pairs(ws, off, rows, wds, G):
    """decode [nblk][Hk/32][2][rows][32 halves] pair tiles -> [nblk][rows][Hk] float64"""
    t = ws[off:off + len(blocks) * nch * 2 * rows * 64].view(np.float16).reshape(len(blocks), nch, 2, rows, 32)
    v = (t[:, :, 0].astype(np.float64) + t[:, :, 1].astype(np.float64))  # [nblk][nch][rows][32]
    v = v.transpose(0, 2, 1, 3).reshape(len(blocks), rows, Hk)
    s = scale(wds)[:, np.arange(Hk) // G]  # [nblk][Hk]
    return v / s[:, None, :]


def planes(ws, off, rows):
    t = ws[off:off + len(blocks) * nch * 3 * rows * 64].view(np.uint16).reshape(len(blocks), nch, 3, rows, 32)
    f = (t.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return f.sum(axis=2).transpose(0, 2, 1, 3).reshape(len(blocks), rows, Hk)


def err(a, b, mask_rows):
    d, m = [], []
    for k, (bs, bn, as_, an, *_) in enumerate(blocks):
        r = mask_rows(k)
        d.append(np.abs(a[k, :r] - b[k, :r]).max(initial=0.0))
        m.append(np.abs(b[k, :r]).max(initial=0.0))
    return max(d) / max(max(m), 1e-30), int(np.argmax(d))


relu = lambda x: np.maximum(x, 0)  # noqa: E731
o, ws, off = run(111)
print('offsets', off)
inp = f32(ws, off[0], (len(ws) - off[0]) // 4)
R = lambda k: blocks[k][1]  # noqa: E731
inp_blk = np.zeros((len(blocks), 128, Hk))
for k, (bs, bn, *_) in enumerate(blocks):
    inp_blk[k, :bn] = inp[bs * Hk:(bs + bn) * Hk].reshape(bn, Hk)
w0 = words(ws, off[4], Hk // EPB)
m0 = pairs(ws, off[1], 128, w0, EPB)
print('M0 pairs vs act(inp): rel err %.3e (block %d)' % err(m0, relu(inp_blk), R))
print('   embed words block 0:', [hex(x) for x in w0[0]])

o, ws, off = run(112)
w1 = words(ws, off[5], Hk // 80)
m1 = pairs(ws, off[2], 128, w1, 80)
o2, ws2, off2 = run(122)
z1 = f32(ws2, off2[7], len(ws2) // 4 - off2[7] // 4)
z1_blk = np.zeros((len(blocks), 128, Hk))
for k, (bs, bn, *_) in enumerate(blocks):
    z1_blk[k, :bn] = z1[bs * Hk:(bs + bn) * Hk].reshape(bn, Hk)
print('M1 pairs vs act(Z1) staged: rel err %.3e (block %d)' % err(m1, relu(z1_blk), R))
print('   layer-1 words block 0:', [hex(x) for x in w1[0]])

o, ws, off = run(113)
wa = words(ws, off[4], Hk // 80)
a_p = pairs(ws, off[3], 64, wa, 80)
o2, ws2, off2 = run(123)
a_s = planes(ws2, off2[3], 64)
print('A pairs vs A planes staged: rel err %.3e (block %d)' % err(a_p, a_s, lambda k: blocks[k][3]))

# W_o's fp16 pair tiles and scale word against W_o[:, Fa:]
pk = off[15]
Fa = get_atom_fdim()
wo = p['W_o.weight'].double().numpy()[:, Fa:]
wmax = pk[off[11]:off[11] + 4 * 65].view(np.uint32)
print('W_o words: folded', hex(wmax[64]), 'max of 64', hex(wmax[:64].max()), 'true', hex(np.abs(wo).astype(np.float32).view(np.uint32).max()))
t = pk[off[10]:off[10] + Hk * Hk * 4].view(np.float16).reshape(Hk // 80, nch, 2, 80, 32).astype(np.float64)
woh = (t[:, :, 0] + t[:, :, 1]).transpose(0, 2, 1, 3).reshape(Hk, Hk) / scale(np.array([wmax[64]]))[0]
print('W_o pairs vs W_o[:, Fa:]: max abs err %.3e (max %.3e)' % (np.abs(woh[:H, :H] - wo).max(), np.abs(wo).max()))
o, ws, off = run(114)
zo_p = f32(ws, off[2], (len(ws) - off[2]) // 4)
o2, ws2, off2 = run(124)
zo_s = f32(ws2, off2[7], (len(ws2) - off2[7]) // 4)
na = g.n_atoms
d = np.abs(zo_p[Hk:na * Hk] - zo_s[Hk:na * Hk])
print('W_o pre-activation pairs vs staged: max abs %.3e of max %.3e; worst row %d col %d' % (
    d.max(), np.abs(zo_s[Hk:na * Hk]).max(), (np.argmax(d) // Hk) + 1, np.argmax(d) % Hk))
rows = np.abs(zo_p[Hk:na * Hk] - zo_s[Hk:na * Hk]).reshape(-1, Hk).max(axis=1)
print('   rows with error > 1e-3:', int((rows > 1e-3).sum()), 'of', na - 1, ' cols:', sorted(set((np.argwhere(d.reshape(-1, Hk) > 1e-3)[:, 1] // 16).tolist()))[:20])
# where: by the row's 16-row group in its block (the MFMA wave), and Eo of the two paths
row_blk = np.zeros(na, np.int64)
for k, (bs, bn, as_, an, *_) in enumerate(blocks):
    row_blk[as_:as_ + an] = np.arange(an)
bad = rows > 1e-3
for w in range(4):
    sel = (row_blk[1:na] // 16) == w
    print('   rows of wave %d: %d, bad %d' % (w, int(sel.sum()), int((bad & sel).sum())))
# expected pre-activation from the decoded A pairs (this run's Ab) and W_o, per chunk contribution
wa4 = words(ws, off[4], Hk // 80)
a_p4 = pairs(ws, off[3], 64, wa4, 80)
Wfull = np.zeros((Hk, Hk))
Wfull[:H, :H] = wo
bias_o = p['W_o.bias'].double().numpy()
eo_all = f32(ws, off[14], (len(ws) - off[14]) // 4)[:na * Hk].reshape(na, Hk).astype(np.float64)
for k, (bs, bn, as_, an, *_) in enumerate(blocks[:3]):
    A = a_p4[k, :an]
    exp = A @ Wfull.T + eo_all[as_:as_ + an]
    exp[:, :H] += bias_o
    got = zo_p[as_ * Hk:(as_ + an) * Hk].reshape(an, Hk).astype(np.float64)
    dif = got - exp
    print('block %d (%d atoms): max |got-exp| per row group:' % (k, an), [float(np.abs(dif[r:r + 16]).max(initial=0)) for r in range(0, an, 16)])
    for r in (0, 17, 33):
        if r >= an:
            continue
        contrib = np.stack([A[r, 32 * c:32 * c + 32] @ Wfull[:, 32 * c:32 * c + 32].T for c in range(nch)])  # [nch][Hk]
        # least-squares weights of the chunk contributions that explain the row's error
        coef, *_ = np.linalg.lstsq(contrib.T, dif[r], rcond=None)
        print('   row %d err %.3e, chunk weights %s' % (r, np.abs(dif[r]).max(), np.round(coef, 3).tolist()))
eo_p = f32(ws, off[14], (len(ws) - off[14]) // 4)[:na * Hk]
eo_s = f32(ws2, off2[14], (len(ws2) - off2[14]) // 4)[:na * Hk]
print('Eo pairs path vs staged path: max abs %.3e' % np.abs(eo_p[Hk:] - eo_s[Hk:]).max())
o, _, _ = run(110)
o2, _, _ = run(120)
n = lambda a, b: float(np.abs(a - b).max() / np.abs(b).max())  # noqa: E731
print('outputs: pairs vs oracle %.3e, staged vs oracle %.3e, pairs vs staged %.3e' % (n(o, ref), n(o2, ref), n(o, o2)))
