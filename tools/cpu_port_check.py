"""the CPU baseline (oracle/mpn_ref.py, the op-for-op restatement bench.py times on the GPU
host) must time within +-10 % of the REAL reference forward on the same batch.  Build container only
(needs /root/reference): both run here, interleaved, on one polymer B=64 batch (depth 3, hidden 300,
eval, no_grad), at 8 threads and 1 thread; median of repeated forwards.

    PYTHONDONTWRITEBYTECODE=1 python tools/cpu_port_check.py > profiles/round2_cpu_port_check.txt
"""
import os
import platform
import statistics
import sys
import time
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, 'polymer-chemprop_amd')]

import torch  # noqa: E402

from chemprop_amd import TrainArgs, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph  # noqa: E402
from oracle import mpn_ref  # noqa: E402
from ref_loader import load_reference  # noqa: E402


def cpu_model():
    with open('/proc/cpuinfo') as f:
        for line in f:
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    return platform.processor()


def main():
    ref = load_reference()
    mols = synthetic.make_batch('polymer', 64, 1000)
    args = TrainArgs(hidden_size=300, depth=3, device=torch.device('cpu'))
    torch.manual_seed(0)
    refargs = types.SimpleNamespace(**{**args.__dict__, 'device': torch.device('cpu')})
    enc = ref.mpn.MPNEncoder(refargs, 133, 147).eval()
    p = {n: t.detach() for n, t in enc.named_parameters()}
    g_ref = ref.featurization.BatchMolGraph(mols)
    g_port = BatchMolGraph(mols, compact=False)
    print(f'# CPU: {cpu_model()}, {os.cpu_count()} logical CPUs; torch {torch.__version__}; '
          f'MKL {torch.backends.mkl.is_available()}; batch E={g_port.n_bonds - 1} V={g_port.n_atoms - 1}')
    for threads in (8, 1):
        torch.set_num_threads(threads)
        tr, tp = [], []
        with torch.no_grad():
            a, b = enc(g_ref), mpn_ref.encoder_forward(p, g_port, args)
            assert float((a - b).abs().max() / a.abs().max()) < 1e-5
            n = 30 if threads > 1 else 20
            for _ in range(n):
                t0 = time.perf_counter(); enc(g_ref); tr.append(time.perf_counter() - t0)
                t0 = time.perf_counter(); mpn_ref.encoder_forward(p, g_port, args); tp.append(time.perf_counter() - t0)
        mr, mp = statistics.median(tr), statistics.median(tp)
        print(f'threads={threads}: reference {mr * 1e3:.2f} ms, port {mp * 1e3:.2f} ms, port/reference = '
              f'{mp / mr:.3f} ({"within" if abs(mp / mr - 1) <= 0.10 else "OUTSIDE"} +-10 %), '
              f'reference {(g_port.n_bonds - 1) / mr:.0f} edges/s')


if __name__ == '__main__':
    main()
