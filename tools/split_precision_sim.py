"""CPU emulation of the split-operand GEMM schemes, judged like tools/x6_precision.py (encoder output,
max|out - ref64| / max|ref64|), without a GPU.

The fp64 oracle (oracle/mpn_ref.py) runs with its W_h / W_o linears replaced by an emulation of
  f32    an fp32 GEMM (operands rounded to fp32, fp32 accumulation),
  x6     bf16x3 planes, products hh hm mh hl lh mm (the kernels' gemm_x6.hpp scheme),
  h2     fp16 hi + lo with a per-tensor power-of-two scale (max |x| s in [2^14, 2^15)), products hh hl lh,
  h2w    the weights scaled, the activations not (s = 1),
  h2n    neither scaled,
each product term a separate fp32-accumulated matmul.  Test infrastructure: imports the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402
from oracle import mpn_ref  # noqa: E402


def bf16(x):
    return x.to(torch.float32).to(torch.bfloat16).to(torch.float64)


def f16(x):
    return x.to(torch.float32).to(torch.float16).to(torch.float64)


def planes_x6(x):
    x = x.to(torch.float32).to(torch.float64)
    h = bf16(x)
    m = bf16(x - h)
    return h, m, bf16(x - h - m)


def pow2_scale(x, scaled):
    if not scaled:
        return 1.0
    mx = float(x.abs().max())
    return 1.0 if mx == 0 else 2.0 ** (14 - np.floor(np.log2(mx)))


def planes_h2(x, scaled):
    x = x.to(torch.float32).to(torch.float64)
    s = pow2_scale(x, scaled)
    xs = x * s
    h = f16(xs)
    return h / s, f16(xs - h) / s


def mm32(a, b):
    return (a.to(torch.float32) @ b.to(torch.float32).T).to(torch.float64)


def make_linear(mode):
    def lin(p, name, x):
        w = p[f'{name}.weight']
        b = p.get(f'{name}.bias')
        if name not in ('W_h', 'W_o') or mode == 'f64':
            y = x @ w.T
        elif mode == 'f32':
            y = mm32(x, w)
        elif mode == 'x6':
            A, B = planes_x6(x), planes_x6(w)
            y = sum(mm32(A[i], B[j]) for i, j in ((0, 0), (0, 1), (1, 0), (0, 2), (2, 0), (1, 1)))
        else:
            A, B = planes_h2(x, mode == 'h2'), planes_h2(w, mode in ('h2', 'h2w'))
            y = sum(mm32(A[i], B[j]) for i, j in ((0, 0), (0, 1), (1, 0)))
        return y if b is None else y + b
    return lin


def nw(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-300))


def main():
    orig = mpn_ref._linear
    cases = (('polymer', 64, 300, 3, {}), ('polymer', 64, 300, 3, dict(activation='tanh', bias=True)),
             ('polymer', 128, 300, 3, dict(bias=True, activation='SELU')),
             ('qm9', 64, 300, 3, dict(activation='ELU')), ('zinc', 64, 512, 5, {}),
             ('polymer', 16, 2400, 3, {}))
    for kind, b, H, T, extra in cases:
        for wscale in (1.0, 1e-3, 1e-5):
            args = TrainArgs(hidden_size=H, depth=T, **extra)
            g = BatchMolGraph(synthetic.make_batch(kind, b, 11))
            torch.manual_seed(0)
            enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=args.atom_messages))
            initialize_weights(enc)
            p = {n: t.detach().clone().to(torch.float64) for n, t in enc.named_parameters()}
            p['W_i.weight'] = p['W_i.weight'] * wscale  # small activations: the unscaled fp16 range test
            res = {}
            try:
                mpn_ref._linear = make_linear('f64')
                with torch.no_grad():
                    ref = mpn_ref.encoder_forward(p, g, args, dtype=torch.float64)
                for mode in ('f32', 'x6', 'h2', 'h2w', 'h2n'):
                    mpn_ref._linear = make_linear(mode)
                    with torch.no_grad():
                        res[mode] = nw(mpn_ref.encoder_forward(p, g, args, dtype=torch.float64), ref)
            finally:
                mpn_ref._linear = orig
            print(kind, b, H, T, extra, f'W_i x{wscale:g}', ' '.join(f'{k}={v:.2e}' for k, v in res.items()),
                  flush=True)


if __name__ == '__main__':
    main()
