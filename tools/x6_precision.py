"""Accuracy of the GEMM paths against an fp64 evaluation of the reference op sequence (GPU only).

For each configuration, prints max|out - ref64| / max|ref64| of the encoder output for
  ref32  the fp32 oracle (the reference's own arithmetic, CPU),
  f32    the HIP path with the f32-MFMA GEMM (WdConfig.gemm_variant 9),
  x6     the default HIP path: bf16x6 split-plane GEMMs (gemm_variant 0; molecule-blocked when the
         batch allows it, operands split in the kernel in atom-message mode),
so the split GEMM can be judged against the fp32 arithmetic it replaces."""
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

dev = torch.device('cuda:0')


def nw(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


for kind, b, H, T, extra in (('polymer', 64, 300, 3, {}), ('polymer', 64, 300, 3, dict(activation='tanh', bias=True)),
                             ('polymer', 128, 300, 3, dict(bias=True, activation='SELU')),
                             ('qm9', 64, 300, 3, dict(activation='ELU')), ('zinc', 128, 512, 5, {}),
                             ('polymer', 32, 64, 3, dict(atom_messages=True, bias=True))):
    args = TrainArgs(hidden_size=H, depth=T, **extra)
    g = BatchMolGraph(synthetic.make_batch(kind, b, 11))
    torch.manual_seed(0)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=args.atom_messages))
    initialize_weights(enc)
    refs = {}
    for dt in (torch.float32, torch.float64):
        p = {n: t.detach().clone().to(dt) for n, t in enc.named_parameters()}
        with torch.no_grad():
            refs[dt] = mpn_ref.encoder_forward(p, g, args, dtype=dt).numpy()
    enc = enc.to(dev).eval()
    res = {'ref32': nw(refs[torch.float32], refs[torch.float64])}
    for name, v in (('f32', 9), ('x6', 0)):
        enc._gemm_variant = v
        with torch.no_grad():
            res[name] = nw(enc(g).cpu().numpy(), refs[torch.float64])
    print(kind, b, H, T, extra, ' '.join(f'{k}={v:.2e}' for k, v in res.items()), flush=True)
