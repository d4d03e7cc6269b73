#!/usr/bin/env python3
"""Benchmark: edges/sec of the wD-MPNN encoder forward (MPNEncoder.forward, mpn.py:66-173) on
synthetic polymer batches of 64 graphs, depth 3, hidden 300 (BASELINE.json metric), inputs packed
and resident in HBM before the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One process per GPU.  Every rank encodes its own disjoint synthetic batches (seed = base + rank):
the path shards as independent graphs with no data-path collective (weak scaling); the only
collectives are the barrier and the max-over-ranks of the elapsed time.

Rank 0 prints ONE JSON line (stdout).  Diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'polymer-chemprop_amd'))
sys.path.insert(0, ROOT)


def _pin_cpus(argv):
    """--cpus N: restrict this process to N CPUs of its affinity set (rank r of a node takes the r-th
    disjoint slice) before torch or the HIP runtime start any thread, so that one GPU can measure what a
    rank gets when eight ranks share a 16-CPU quota (N = 2).  Every later thread (torch's, the HIP
    runtime's, the native feed's producers and feeder) inherits the set, and the producer cap
    (chemprop_amd.stream.producer_cap) reads it.  Returns the CPU list, or None without the option."""
    n = 0
    for i, x in enumerate(argv):
        if x == '--cpus' and i + 1 < len(argv):
            n = int(argv[i + 1])
        elif x.startswith('--cpus='):
            n = int(x.split('=', 1)[1])
    if n <= 0:
        return None
    allowed = sorted(os.sched_getaffinity(0))
    r = int(os.environ.get('LOCAL_RANK', '0'))
    pick = allowed[(r * n) % len(allowed):][:n]
    if len(pick) < n:
        pick = allowed[:n]
    os.sched_setaffinity(0, pick)
    os.environ['OMP_NUM_THREADS'] = str(n)
    return pick


PINNED_CPUS = _pin_cpus(sys.argv)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from chemprop_amd import TrainArgs, _native, synthetic  # noqa: E402
from chemprop_amd.featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim  # noqa: E402
from chemprop_amd.mpn import MPNEncoder  # noqa: E402
from chemprop_amd.nn_utils import initialize_weights  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 / fp16 (the layer issues 3 fp16 products per fp32 product, W_o 6 bf16)
HBM_PEAK_GBS = 8000.0
PMC_TRAFFIC = "round6_pmc_traffic.json"  # per-kernel HBM bytes per launch (tools/pmc_summary.py)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_encoder(args, device):
    torch.manual_seed(0)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim())
    initialize_weights(enc)  # model.py:39 semantics: xavier_normal_ weights, zero biases
    return enc.to(device).eval()


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _usable_cores(fallback):
    from chemprop_amd.stream import usable_cores
    return usable_cores(fallback)


def cpu_baseline(args, graph, seconds):
    """The oracle (op-for-op restatement of the reference forward, oracle/mpn_ref.py) on the GPU box's
    host cores: median over ~``seconds`` of forwards with torch's thread count set to the cores this
    process may run on (its affinity set), then a shorter 1-thread sample.  Fidelity to the real
    reference (profiles/round2_cpu_port_check.txt, 8-CPU build container): at 1 thread the port takes
    1.09-1.14x the reference's time; at 8 threads 0.86-0.96x, i.e. the port can be up to ~14 % faster
    than the reference there, which understates the GPU's speed-up over the real reference."""
    from oracle import mpn_ref
    enc = make_encoder(args, torch.device('cpu'))
    p = {n: t.detach() for n, t in enc.named_parameters()}

    def sample(secs, min_n):
        times = []
        t_end = time.perf_counter() + secs
        with torch.no_grad():
            mpn_ref.encoder_forward(p, graph, args)  # warm-up
            while len(times) < min_n or time.perf_counter() < t_end:
                t0 = time.perf_counter()
                mpn_ref.encoder_forward(p, graph, args)
                times.append(time.perf_counter() - t0)
        return statistics.median(times), len(times)

    prev = torch.get_num_threads()
    cores, affinity, quota = _usable_cores(prev)
    torch.set_num_threads(cores)
    med, n = sample(seconds, 5)
    torch.set_num_threads(1)
    med1, n1 = sample(seconds / 3, 3)
    torch.set_num_threads(prev)
    E = graph.n_bonds - 1
    return {'value': E / med, 'unit': 'edges/s', 'cores': cores, 'kind': 'port',
            'sample': f'{n} forwards of one polymer B={len(graph.a_scope)} batch (E={E} directed edges), median '
                      f'{med * 1e3:.2f} ms at {cores} threads (the CPUs this process may use: affinity set, capped by '
                      f'the cgroup CPU quota), eval/no_grad',
            'single_thread': {'value': E / med1, 'ms': med1 * 1e3, 'forwards': n1},
            'host': {'cpu_model': _cpu_model(), 'logical_cpus': os.cpu_count(), 'affinity_cpus': affinity,
                     'cgroup_cpu_quota': quota,
                     'torch_default_threads': prev, 'torch': torch.__version__,
                     'mkl': bool(torch.backends.mkl.is_available()),
                     'mkldnn': bool(torch.backends.mkldnn.is_available())}}


def pmc_traffic(prefix):
    """HBM bytes per launch of the kernels named prefix* (mean over their variants), from the PMC
    summary tools/pmc.sh + tools/pmc_summary.py committed for this build (counters need their own
    rocprofv3 pass, so the bench cannot collect them while it times)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', PMC_TRAFFIC)
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    v = [x['traffic_bytes'] for k, x in d.items() if k.startswith(prefix)]
    if not v:
        return None, None
    return sum(v) / len(v), f'profiles/{PMC_TRAFFIC}: {d.get("_note", "")}'


ROCPROF_STATS = "round6_bench_b64_kernel_stats.csv"  # rocprofv3 --kernel-trace --stats of the headline, one stream


def rocprof_alone(prefix):
    """(mean launch us of the kernels named ``prefix``* -- their variants weighted by calls --, source) from the
    committed rocprofv3 kernel-stats summary of the headline workload with one batch in flight: the
    dominant kernel's time alone on the GPU, next to the events' in-flight figure the bench measures."""
    import csv
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', ROCPROF_STATS)
    try:
        rows = list(csv.DictReader(open(path)))
    except OSError:
        return None, None
    calls = tot = 0
    for r in rows:
        name = r['Name'].replace('void ', '').replace('wd::', '')
        if name.startswith(prefix):
            calls += int(r['Calls'])
            tot += float(r['TotalDurationNs'])
    if not calls:
        return None, None
    return tot / calls / 1e3, f'profiles/{ROCPROF_STATS} ({calls} launches)'


def forward_roofline(graphs, a, t_fwd):
    """Whole-forward fractions per SURVEY §8(d): algorithmic bytes (fp32, each logical tensor read or
    written once, gathers at unique size, int32 indices) and FLOPs of mpn.py:92-171 for the average
    timed batch, over the measured time per forward, against 8 TB/s HBM and 157.3 TF/s fp32 MFMA."""
    s, H, T = 4.0, a.hidden, a.depth
    Fa, Fb = get_atom_fdim(), get_bond_fdim()
    n = len(graphs)
    E = sum(g.n_bonds - 1 for g in graphs) / n
    V = sum(g.n_atoms - 1 for g in graphs) / n
    B = sum(len(g.a_scope) for g in graphs) / n
    byt = (s * (E * Fb + Fb * H + E * H)
           + (T - 1) * (s * (3 * E * H + 2 * V * H + H * H + E) + 4 * (4 * E + V + 1))
           + s * (E * H + E + V * H) + 4 * (E + V + 1)
           + s * (V * Fa + 2 * V * H + (Fa + H) * H + H)
           + s * (V * H + V + B * H + B) + 4 * (B + 1))
    flops = 2 * E * Fb * H + (T - 1) * 2 * E * H * H + 2 * V * (Fa + H) * H
    t_hbm, t_mfma = byt / (HBM_PEAK_GBS * 1e9), flops / (FP32_MFMA_PEAK_TFLOPS * 1e12)
    return {'algorithmic_bytes': byt, 'algorithmic_flops': flops, 'us_per_forward': t_fwd * 1e6,
            'hbm_frac': t_hbm / t_fwd, 'mfma_fp32_frac': t_mfma / t_fwd,
            'combined_frac': max(t_hbm, t_mfma) / t_fwd,
            'note': 'SURVEY 8(d) formulas; combined = max(bytes/8 TB/s, flops/157.3 TF/s) / measured time'}


def device_identity(device):
    """This rank's GPU as the HIP runtime reports it (ordinal, PCI domain:bus:device, UUID, name): the
    bench line lists every rank's, so a multi-GPU line shows how many distinct devices ran it."""
    p = torch.cuda.get_device_properties(device)
    pci = f'{getattr(p, "pci_domain_id", 0):04x}:{getattr(p, "pci_bus_id", 0):02x}:{getattr(p, "pci_device_id", 0):02x}'
    return {'ordinal': device.index, 'pci': pci, 'uuid': str(getattr(p, 'uuid', '')), 'name': p.name,
            'visible_devices': torch.cuda.device_count()}


def default_streams(edges_per_batch):
    """Batches in flight per GPU for a batch size: three (one per HIP stream) while a batch's launches
    leave CUs idle in their ramps, barriers and epilogues (polymer-sized batches: 2 / 3 / 4 in flight
    measured 155-158 / 172-173 / 173-175 M edges/s on one box, profiles/round3_streams_ab.txt), four for
    QM9-sized batches (each forward one launch of ~64 workgroups: four fill the chip), one for
    large batches whose grids fill the chip on their own (ZINC-sized B = 512: two streams measured 50.5 vs
    52.6 M edges/s, BENCH_r02.json).  Every step is still one full, independent batch."""
    if edges_per_batch < 2048:  # QM9-sized (~900 edges): the one-launch small-block forward (64 workgroups a
        return 4                # batch): 1 / 2 / 3 / 4 in flight 36.9 / 18.4 / 12.4 / 9.8 us per forward, 5-6
                                # (past the 4 hardware queues) 12-15 (profiles/round5_qm9_streams.txt)
    return 3 if edges_per_batch < 16384 else 1


_STREAMS = []


def bench_streams(device, n):
    """n streams for batches in flight: the current stream + extra HIP streams shared by every workload of
    the run.  The HIP runtime binds streams to a handful of hardware queues (GPU_MAX_HW_QUEUES = 4 on the
    box); streams created after the native feed's own stream came to share a queue with a busy one, and
    two QM9-sized batches in flight took 75 instead of 27 us per forward (same box, profiles/round3_*)"""
    while len(_STREAMS) < n - 1:
        _STREAMS.append(torch.cuda.Stream(device))
    return [torch.cuda.current_stream(device)] + _STREAMS[:n - 1]


def secondary_workload(device, kind, batch, depth, hidden, steps, warmup=10, n_batches=8, streams=None, many=8):
    """Other BASELINE.json configs' shapes (configs[1]: QM9-like molecules, batch 64, depth 3, hidden
    300; configs[3]: ZINC-like molecules, batch 512, depth 5, hidden 512), timed like the headline:
    resident graphs, eval forward, synchronised wall time over ``steps`` forwards, with ``streams``
    independent batches in flight (as the headline) and with one; and ``many`` batches per call on one
    stream (MPNEncoder.forward_many: one set of launches for all of them)."""
    enc = make_encoder(TrainArgs(hidden_size=hidden, depth=depth, device=device), device)
    graphs = [BatchMolGraph(synthetic.make_batch(kind, batch, 5000 + i), device_bond_features=True)
              for i in range(n_batches)]
    for g in graphs:
        g.device_graph(device, False, get_bond_fdim())
    if streams is None:
        streams = default_streams(sum(g.n_bonds - 1 for g in graphs) / len(graphs))
    ss = bench_streams(device, streams)  # (streams created here instead, after the feed's: 23.9 vs 19.5 us, round 6)
    enc.prepare(graphs, ss)  # (resident inputs registered on the streams and their plans cached, as main())

    prev_stream = torch.cuda.current_stream(device)

    def timed(n_streams):
        def fwd(i):
            if n_streams == 1:
                return enc(graphs[i % len(graphs)])
            torch.cuda.set_stream(ss[i % n_streams])  # (see main(): step)
            return enc(graphs[i % len(graphs)])
        for i in range(warmup):
            fwd(i)
        torch.cuda.set_stream(prev_stream)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for i in range(steps):
            fwd(i)
        torch.cuda.set_stream(prev_stream)
        torch.cuda.synchronize(device)
        return time.perf_counter() - t0

    # forward_many packs its batches into full molecule blocks (block_target=1): its launches have enough
    # workgroups without cutting each small batch into slivers (featurization.BatchMolGraph)
    graphs_many = [BatchMolGraph(synthetic.make_batch(kind, batch, 5000 + i), device_bond_features=True,
                                 block_target=1) for i in range(n_batches)]
    for g in graphs_many:
        g.device_graph(device, False, get_bond_fdim())

    def timed_many(k):
        # k batches per call on one stream (wdmpnn_forward_many: one set of launches for the k batches)
        sets = [[graphs_many[(i * k + j) % len(graphs_many)] for j in range(k)] for i in range(len(graphs_many))]
        for i in range(warmup):
            enc.forward_many(sets[i % len(sets)])
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for i in range(steps // k):
            enc.forward_many(sets[i % len(sets)])
        torch.cuda.synchronize(device)
        return time.perf_counter() - t0, sum(g.n_bonds - 1 for i in range(steps // k) for g in sets[i % len(sets)])

    with torch.no_grad():
        enc(graphs[0])  # weights packed once, on the default stream
        torch.cuda.synchronize(device)
        dt = timed(len(ss))
        dt1 = timed(1) if len(ss) > 1 else dt
        dtm, Em = timed_many(many)
    E = sum(graphs[i % len(graphs)].n_bonds - 1 for i in range(steps))
    return {'workload': f'{kind}-like synthetic batches of {batch} molecules, depth {depth}, hidden {hidden}',
            'value': E / dt, 'unit': 'edges/s', 'ms_per_step': dt / steps * 1e3, 'steps': steps,
            'avg_edges': E / steps, 'streams': len(ss),
            'single_stream': {'value': E / dt1, 'ms_per_step': dt1 / steps * 1e3},
            'forward_many': {'value': Em / dtm, 'ms_per_step': dtm / (steps // many * many) * 1e3,
                             'batches_per_call': many,
                             'note': 'one stream; MPNEncoder.forward_many: embed, layers and W_o + readout '
                                     'launched once per call for all its batches, packed in full molecule blocks '
                                     '(BatchMolGraph(block_target=1))'}}


def atom_messages_workload(device, steps=50, warmup=5):
    """The reference's ``atom_messages`` mode (mpn.py:47-53, 93-94, 104-108, 126-128) on the bench's polymer
    batches (B = 64, depth 3, hidden 300, the reference's default bias=False): the molecule-blocked fused
    layers over atom rows (a2a neighbour sums in the layer epilogue), eval forward, one in flight."""
    args = TrainArgs(hidden_size=300, depth=3, device=device, atom_messages=True)
    torch.manual_seed(0)
    enc = MPNEncoder(args, get_atom_fdim(), get_bond_fdim(atom_messages=True))
    initialize_weights(enc)
    enc = enc.to(device).eval()
    graphs = [BatchMolGraph(synthetic.make_batch('polymer', 64, 6000 + i)) for i in range(4)]
    with torch.no_grad():
        for i in range(warmup):
            enc(graphs[i % 4])
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for i in range(steps):
            enc(graphs[i % 4])
        torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    E = sum(graphs[i % 4].n_bonds - 1 for i in range(steps))
    return {'workload': 'atom_messages=True (mpn.py:47-53): polymer batches of 64, depth 3, hidden 300, '
                        'molecule-blocked fused atom-row layers', 'value': E / dt, 'unit': 'edges/s',
            'ms_per_step': dt / steps * 1e3,
            'steps': steps}


def training_workload(device, batch=128, steps=100, warmup=10):
    """BASELINE.json configs[2] shape (copolymer batches of 128 with weighted edges, full training
    step): MoleculeModel (encoder + FFN, regression, one task) forward + loss + backward (the
    deterministic HIP backward) + Adam step per batch, resident graphs, synchronised wall time."""
    from chemprop_amd.model import MoleculeModel
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=300, depth=3, device=device)
    torch.manual_seed(0)
    model = MoleculeModel(args)
    initialize_weights(model)
    model = model.to(device)
    opt = build_optimizer(model, 1e-4)
    loss_func = get_loss_func('regression')
    rng = torch.Generator().manual_seed(0)
    batches = []
    for i in range(4):
        g = BatchMolGraph(synthetic.make_batch('polymer', batch, 7000 + i), device_bond_features=True)
        g.device_graph(device, False, get_bond_fdim())
        batches.append(([g], torch.randn(batch, 1, generator=rng).tolist()))
    for i in range(warmup):
        train_step(model, *batches[i % 4], loss_func, opt)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for i in range(steps):
        train_step(model, *batches[i % 4], loss_func, opt)
    torch.cuda.synchronize(device)
    dt = time.perf_counter() - t0
    E = sum(batches[i % 4][0][0].n_bonds - 1 for i in range(steps))
    # training roofline: the encoder's algorithmic forward FLOPs (SURVEY §8(d) formula, mpn.py:92-171) x 3
    # (each GEMM's backward = two GEMMs of the same size: data and weight gradients), per step
    import types
    fwd = forward_roofline([batches[i][0][0] for i in range(4)], types.SimpleNamespace(hidden=300, depth=3), dt / steps)
    flops = 3.0 * fwd['algorithmic_flops']
    return {'workload': f'training step: MoleculeModel on synthetic polymer batches of {batch}, depth 3, hidden 300, '
                        'MSE + Adam (forward, backward, optimizer step)',
            'value': E / dt, 'unit': 'edges/s', 'ms_per_step': dt / steps * 1e3, 'graphs_per_s': batch * steps / dt,
            'steps': steps,
            'roofline': {'flops_per_step': flops, 'achieved_tflops': flops / (dt / steps) / 1e12,
                         'mfma_fp32_frac': flops / (dt / steps) / (FP32_MFMA_PEAK_TFLOPS * 1e12),
                         'note': 'encoder forward FLOPs x 3 per step over the measured step time, against the '
                                 'fp32 dense MFMA peak (the FFN head, loss and optimizer are not counted)'}}


def streamed_workload(device, args, rank, world, graphs_per_rank, batch=64, producers=4, barrier=None, k=8):
    """BASELINE.json configs[4]: synthetic polymer graphs streamed per rank (10 M over 8 GPUs = 1.25 M per
    rank by default: weak scaling), generated on the fly by native producer threads, staged in compact
    form (~14 B per edge), uploaded and expanded on the GPU by the native feed thread (wdmpnn_feed_*,
    chemprop_amd.stream.NativeFeed) while earlier batches are encoded, k batches per launch set
    (wdmpnn_feed_forward).  Everything is inside the timed region: generation, block plan, H2D, device
    graph build and the B=64 forwards.  Disjoint seeds per rank, no collective on the data path; value =
    edges of all ranks / max-over-ranks time."""
    from chemprop_amd.stream import NativeFeed
    enc = make_encoder(args, device)
    n = -(-graphs_per_rank // batch)
    with torch.no_grad():
        # warm-up: the first ~1000 streamed batches of a process run at half speed (HIP runtime / driver
        # warm-up of the feed's copy, event and launch paths: tools/stream_encode.py, profiles/round3_*)
        for _ in NativeFeed('polymer', batch, min(n, 1024), seed=99, device=device, rank=rank, producers=producers,
                            lean=True, slots=4 * k).encode(enc, k):
            pass
        barrier()
        t0 = time.perf_counter()
        edges = h2d = 0
        feed = NativeFeed('polymer', batch, n, seed=2024, device=device, rank=rank, producers=producers, lean=True,
                          slots=4 * k)
        for out, got, e, up in feed.encode(enc, k):
            edges += e
            h2d += up
        barrier()
        dt = time.perf_counter() - t0
    return dt, edges, n * batch, h2d, {'producers': feed.producers, 'seed_range': feed.seed_range}


def streamed_training(device, rank, world, graphs_per_rank, batch=128, producers=4, barrier=None):
    """configs[4] as data-parallel training: each rank trains MoleculeModel (depth 3, hidden 300, one
    regression task, Adam) on its own streamed batches of ``batch`` graphs (native feed: generation,
    upload and device graph build off the training thread); one flat fp32 gradient all-reduce per step
    (chemprop_amd.dp.GradBucket: RCCL over xGMI when world > 1)."""
    from chemprop_amd.dp import GradBucket, broadcast_parameters
    from chemprop_amd.model import MoleculeModel
    from chemprop_amd.stream import NativeFeed
    from chemprop_amd.train import build_optimizer, get_loss_func, train_step
    args = TrainArgs(hidden_size=300, depth=3, device=device)
    torch.manual_seed(0)
    model = MoleculeModel(args)
    initialize_weights(model)
    model = model.to(device)
    broadcast_parameters(model)
    bucket = GradBucket(model)
    opt = build_optimizer(model, 1e-4)
    loss_func = get_loss_func('regression')
    gen = torch.Generator().manual_seed(rank)
    targets = [torch.randn(batch, 1, generator=gen).tolist() for _ in range(8)]
    steps = -(-graphs_per_rank // batch)
    for i, g in enumerate(NativeFeed('polymer', batch, 10, seed=77, device=device, rank=rank, producers=producers,
                                     planes=False)):
        train_step(model, [g], targets[i % 8], loss_func, opt, bucket=bucket)
    barrier()
    t0 = time.perf_counter()
    edges = 0
    for i, g in enumerate(NativeFeed('polymer', batch, steps, seed=4048, device=device, rank=rank,
                                     producers=producers, planes=False)):
        train_step(model, [g], targets[i % 8], loss_func, opt, bucket=bucket)
        edges += g.n_bonds - 1
    barrier()
    return time.perf_counter() - t0, edges, steps


def packing_report(a, device, t_fwd):
    """Host side of one batch, outside the timed region (pack + H2D reported separately,
    and end to end): native packer time, device_graph() time (gather lists, blocks, one pinned H2D,
    device-side bond featurisation and plane split, synchronised), H2D bytes per edge, both with the
    bond rows built on the host and on the device."""
    mols = synthetic.make_batch(a.kind, a.batch, 4242)
    rep = {}
    for mode, kw in (('host_bond_features', {}), ('device_bond_features', {'device_bond_features': True})):
        BatchMolGraph(mols, **kw)
        n, t0 = 0, time.perf_counter()
        while n < 5 or time.perf_counter() - t0 < 0.5:
            g = BatchMolGraph(mols, **kw)
            n += 1
        pack = (time.perf_counter() - t0) / n
        ups = []
        for _ in range(3):
            g = BatchMolGraph(mols, **kw)
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            dg = g.device_graph(device, False, get_bond_fdim())
            torch.cuda.synchronize(device)
            ups.append(time.perf_counter() - t0)
        up = statistics.median(ups)
        E = g.n_bonds - 1
        rep[mode] = {'pack_ms': pack * 1e3, 'device_graph_ms': up * 1e3, 'h2d_bytes_per_edge': dg.h2d_bytes / E,
                     'end_to_end_edges_per_s': E / (pack + up + t_fwd)}
    rep['note'] = ('one batch of the bench workload; end_to_end = edges / (pack + device_graph + one forward), '
                   'serial on one host thread (the reference packs in 77 ms per batch, SURVEY §8(a) a2)')
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--depth', type=int, default=3)
    ap.add_argument('--hidden', type=int, default=300)
    ap.add_argument('--kind', default='polymer', choices=['polymer', 'qm9', 'zinc'])
    ap.add_argument('--n-batches', type=int, default=8, help='distinct resident batches cycled per rank')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-secondary', action='store_true', help='skip the QM9 / ZINC-shaped secondary workloads')
    ap.add_argument('--streams', type=int, default=0,
                    help='batches in flight per GPU (one HIP stream each); 0 = by batch size (default_streams)')
    ap.add_argument('--many', type=int, default=4, help='batches per MPNEncoder.forward_many call (0 = skip)')
    ap.add_argument('--variant', type=int, default=0, help='WdConfig.gemm_variant (0 = default path; 9 = f32 MFMA)')
    ap.add_argument('--stream-graphs', type=int, default=10_000_000 // 8,
                    help='configs[4]: polymer graphs streamed per rank (default 10 M / 8 GPUs); 0 = skip')
    ap.add_argument('--producers', type=int, default=0,
                    help='native generator threads per rank of the streamed workloads (0 = the cap: max(2, usable '
                         'cores // ranks per node - 2), chemprop_amd.stream.producer_cap; larger requests are capped)')
    ap.add_argument('--cpus', type=int, default=0,
                    help='run this rank on N CPUs only (sched_setaffinity before torch starts; 0 = all): the '
                         'per-rank host budget of an 8-rank node, e.g. 2 on a 16-CPU quota')
    ap.add_argument('--stream-train-graphs', type=int, default=131_072,
                    help='configs[4] as DP training: streamed graphs per rank (batches of 128); 0 = skip')
    a = ap.parse_args()

    # one process per GPU over RCCL (backend "nccl"); BENCH_BACKEND=gloo rehearses the multi-rank path
    # with several ranks on one GPU (device = local rank modulo the visible GPUs).  The process group comes
    # from chemprop_amd.dp.init_distributed, the package's one initialisation path.
    from chemprop_amd.dp import init_distributed
    env = init_distributed(os.environ.get('BENCH_BACKEND', 'nccl'), device='cuda')
    world, rank, device = env.world_size, env.rank, env.device
    from chemprop_amd.stream import producer_cap
    cap = producer_cap()
    a.producers = min(a.producers, cap) if a.producers > 0 else cap
    args = TrainArgs(hidden_size=a.hidden, depth=a.depth, device=device)

    # inputs: packed + resident in HBM before timing (featurization.py:757-813 equivalent on host)
    # (bond features rebuilt on the device from f_atoms + bond tail + b2a: SURVEY §8(f) row 2)
    graphs = [BatchMolGraph(synthetic.make_batch(a.kind, a.batch, 1000 + 7919 * rank + i), device_bond_features=True)
              for i in range(a.n_batches)]
    for g in graphs:
        g.device_graph(device, False, get_bond_fdim())
    torch.cuda.synchronize(device)
    enc = make_encoder(args, device)
    enc._gemm_variant = a.variant
    edges = [g.n_bonds - 1 for g in graphs]
    if a.streams <= 0:
        a.streams = default_streams(sum(edges) / len(edges))

    # independent batches in flight on a.streams HIP streams (round-robin): the kernels of one batch's
    # forward overlap another's ramp / drain / epilogue on the same GPU (graphs are independent units)
    # (every stream a workload uses is created here, before the native feed's stream: a stream created after it
    # can share its hardware queue)
    streams = bench_streams(device, max(a.streams, 4))[:a.streams]
    # the resident batches registered on every stream that will run them (DeviceGraph.use_on: the stream waits
    # for the upload and the caching allocator keeps the buffers for it) and their call plans cached
    # (MPNEncoder.prepare: host-side structs, no kernel) -- part of making the inputs resident, as the upload;
    # a graph's first forward otherwise pays them inside the timed region
    enc.prepare(graphs, streams)

    def step(i, prof=None):
        # (torch.cuda.set_stream, not the `with torch.cuda.stream(...)` context manager: that costs ~6 us of
        # host time per switch against 0.4 us, profiles/round5_host_breakdown.txt; the loops below restore
        # the default stream when they end)
        enc._prof = prof
        if prof is not None or len(streams) == 1:
            return enc(graphs[i % len(graphs)])
        torch.cuda.set_stream(streams[i % len(streams)])
        return enc(graphs[i % len(graphs)])

    prev_stream = torch.cuda.current_stream(device)  # (torch's default stream: every loop returns to it)

    def restore():
        torch.cuda.set_stream(prev_stream)

    def barrier():
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    if rank == 0:  # progress on stderr (stdout carries only the JSON line): long quiet phases look hung
        log(f'[bench] resident batches ready; timing {a.steps} steps on {a.streams} streams')
    with torch.no_grad():
        step(0)  # packs the weights on the default stream; the other streams wait on its event
        barrier()
        for i in range(1, a.warmup):
            step(i)
        restore()
        barrier()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        restore()
        barrier()
        elapsed = time.perf_counter() - t0
        my_edges = sum(edges[i % len(edges)] for i in range(a.steps))

        # the same K steps with one batch in flight (latency-bound: each forward waits for the last)
        single = None
        if len(streams) > 1:
            barrier()
            t2 = time.perf_counter()
            for i in range(a.steps):
                enc._prof = None
                enc(graphs[i % len(graphs)])
            barrier()
            single = time.perf_counter() - t2

        # the same K steps as MPNEncoder.forward_many calls of a.many batches on one stream (one set of
        # launches per call; the batches' tiles share one grid)
        many_dt = None
        if a.many > 1 and a.steps >= a.many:
            sets = [[graphs[(i * a.many + j) % len(graphs)] for j in range(a.many)] for i in range(len(graphs))]
            for i in range(2):
                enc.forward_many(sets[i % len(sets)])
            barrier()
            t3 = time.perf_counter()
            for i in range(a.steps // a.many):
                enc.forward_many(sets[i % len(sets)])
            barrier()
            many_dt = time.perf_counter() - t3
            many_edges = sum(g.n_bonds - 1 for i in range(a.steps // a.many) for g in sets[i % len(sets)])

        # second pass: HIP events around the dominant launches (the message-passing layers) on the
        # stream they run on
        L = _native.lib()
        pairs = a.steps  # one pair per forward around its depth - 1 layer launches (WdConfig.prof_pool)
        pool = ctypes.c_void_p()
        _native.check(L.wdmpnn_event_pool_create(pairs, ctypes.byref(pool)), 'event pool')
        barrier()
        t1 = time.perf_counter()
        for i in range(a.steps):
            step(i, (pool.value, i))
        restore()
        barrier()
        elapsed_prof = time.perf_counter() - t1
        enc._prof = None
        kernel_ms = ctypes.c_float()
        n_launch = a.steps * (a.depth - 1)
        if n_launch:  # (the span of each pair also holds the ~0.1 us gaps between the layer launches)
            _native.check(L.wdmpnn_event_pool_elapsed_ms(pool, 0, a.steps, ctypes.byref(kernel_ms)), 'events')
        L.wdmpnn_event_pool_destroy(pool)

    # configs[4]: streamed graphs (generation + upload + device build + forward, all timed), then the
    # same stream as data-parallel training with one gradient all-reduce per step
    st_dt = st_edges = st_graphs = st_h2d = tr_dt = tr_edges = tr_steps = 0
    st_info = None
    if a.stream_graphs > 0:
        if rank == 0:
            log(f'[bench] streamed workload: {a.stream_graphs} graphs per rank')
        st_dt, st_edges, st_graphs, st_h2d, st_info = streamed_workload(device, args, rank, world, a.stream_graphs,
                                                                         producers=a.producers, barrier=barrier)
        if world > 1:  # every rank's shard (batch seed range) and producer count, for the report
            infos = [None] * world
            dist.all_gather_object(infos, st_info)
            st_info = infos
        else:
            st_info = [st_info]
    if a.stream_train_graphs > 0:
        if rank == 0:
            log(f'[bench] streamed training: {a.stream_train_graphs} graphs per rank')
        tr_dt, tr_edges, tr_steps = streamed_training(device, rank, world, a.stream_train_graphs,
                                                      producers=a.producers, barrier=barrier)

    ident = device_identity(device)
    if world > 1:
        idents = [None] * world
        dist.all_gather_object(idents, ident)
    else:
        idents = [ident]
    t = torch.tensor([elapsed, elapsed_prof, single or 0.0, st_dt, tr_dt, many_dt or 0.0], dtype=torch.float64,
                     device=device)
    e = torch.tensor([my_edges, st_edges, st_graphs, st_h2d, tr_edges, many_edges if many_dt else 0.0],
                     dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
    elapsed, elapsed_prof = float(t[0]), float(t[1])
    single = float(t[2]) if single is not None else None
    total_edges = float(e[0])
    st_dt, tr_dt = float(t[3]), float(t[4])
    st_edges, st_graphs, st_h2d, tr_edges = float(e[1]), float(e[2]), float(e[3]), float(e[4])
    many_dt, many_edges = (float(t[5]), float(e[5])) if many_dt else (None, 0.0)

    if rank == 0:
        H = a.hidden
        E_avg = sum(edges[i % len(edges)] for i in range(a.steps)) / a.steps
        # dominant kernel: one message-passing layer (mpn.py:110-124), E directed bonds, hidden H.
        # Algorithmic FLOPs 2 E H^2 (W_h) + 2 E d H (weighted in-edge sums, d = CSR entries / row);
        # algorithmic bytes (fp32, each tensor once): read M_{t-1}, inp, W_h, CSR; write M_t.
        g0 = graphs[0]
        nnz = float(g0.device_graph(device, False, get_bond_fdim()).nnz_msg)
        d_avg = nnz / max(g0.n_bonds - 1, 1)
        flops_launch = 2.0 * E_avg * H * H + 2.0 * E_avg * d_avg * H
        bytes_launch = 4.0 * (3 * E_avg * H + H * H + H) + 8.0 * E_avg * d_avg + 4.0 * E_avg
        avg_launch_s = (kernel_ms.value / 1e3 / n_launch) if n_launch else float('nan')
        traffic, traffic_src = pmc_traffic('mp_layer_kernel<80')
        alone_us, alone_src = rocprof_alone('mp_layer_kernel<80')
        achieved = flops_launch / avg_launch_s / 1e12 if n_launch else None
        hbm = bytes_launch / avg_launch_s / 1e9 if n_launch else None
        line = {
            'metric': 'edges/sec MPN forward, batch=64 polymer graphs, depth=3 hidden=300',
            'value': total_edges / elapsed,
            'unit': 'edges/s',
            'n_gpus': world,
            'backend': dist.get_backend() if world > 1 else 'none (one process)',
            'distinct_devices': len({(d['pci'], d['uuid']) for d in idents}),
            'rank_devices': idents,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': elapsed / a.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'fp32',
            'arith': 'fp32-accurate GEMMs: the message-passing layers and W_o on fp16 hi/lo operand pairs (power-of-two '
                     'scales per producer tile, written by the producing kernel and copied by LDS-DMA) on fp16 MFMA '
                     '(3 products per fp32 product, fp32 accumulate); gathers, residual, activations and readout in fp32',
            'data': 'synthetic',
            'config': {'workload': f'MPNEncoder.forward on synthetic {a.kind} batches of {a.batch} graphs '
                                   f'(avg E={E_avg:.0f} directed edges), depth={a.depth}, hidden={H}, '
                                   f'{a.n_batches} resident batches cycled per rank',
                       'global_batch': a.batch * world, 'depth': a.depth, 'hidden': H,
                       'parallelism': f'dp{world} (independent graphs, no collective in the forward)',
                       'streams': a.streams,
                       'in_flight': f'{a.streams} independent batches in flight per GPU (round-robin over '
                                    f'{a.streams} HIP streams); every step is a full B={a.batch} forward'},
            'single_stream': ({'value': total_edges / single, 'ms_per_step': single / a.steps * 1e3,
                               'note': 'same steps, one batch in flight (each forward waits for the previous)'}
                              if single else None),
            'forward_many': ({'value': many_edges / many_dt, 'ms_per_step': many_dt / (a.steps // a.many * a.many) * 1e3,
                              'batches_per_call': a.many,
                              'note': 'one stream, MPNEncoder.forward_many (wdmpnn_forward_many): the batches of a '
                                      'call share one grid per kernel; every batch a full B=64 forward'}
                             if many_dt else None),
            'roofline': {'bound': 'mfma',
                         'kernel': 'mp_layer_kernel: one message-passing layer, W_h fp16-pair GEMM + in-block CSR '
                                   'gather + residual/activation (mpn.py:110-124)',
                         'achieved': achieved, 'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': achieved / FP32_MFMA_PEAK_TFLOPS if achieved else None, 'traffic': traffic,
                         'traffic_source': traffic_src,
                         'peak_note': 'fp32 dense MFMA peak; the kernel issues fp16 MFMAs (3 per fp32 product), whose '
                                      f'fp32-product equivalent peak is {BF16_MFMA_PEAK_TFLOPS / 3:.0f} TFLOP/s',
                         'avg_launch_us': avg_launch_s * 1e6, 'flops_per_launch': flops_launch,
                         'bytes_per_launch': bytes_launch, 'hbm_gbs': hbm,
                         'hbm_frac': hbm / HBM_PEAK_GBS if hbm else None,
                         'launches_timed': n_launch,
                         'in_flight': {'avg_launch_us': avg_launch_s * 1e6,
                                       'frac': achieved / FP32_MFMA_PEAK_TFLOPS if achieved else None,
                                       'source': f'HIP events around the layer launches, {a.streams} batches in '
                                                 'flight (a second pass of the timed loop)'},
                         'alone': ({'avg_launch_us': alone_us,
                                    'frac': flops_launch / (alone_us * 1e-6) / 1e12 / FP32_MFMA_PEAK_TFLOPS,
                                    'source': alone_src + ', one batch in flight'}
                                   if alone_us else None)},
            'host_cpus': {'pinned': PINNED_CPUS, 'usable': _usable_cores(1)[0]},
        }
        line['forward'] = forward_roofline(graphs, a, elapsed / a.steps)
        if st_dt > 0:
            line['streamed'] = {
                'workload': 'configs[4]: synthetic polymer graphs streamed per rank in batches of 64 (native '
                            'generation on producer threads, compact upload, device graph build, forward; all '
                            'inside the timed region), disjoint seeds per rank, no data-path collective',
                'graphs': st_graphs, 'graphs_per_rank': a.stream_graphs, 'n_gpus': world,
                'value': st_edges / st_dt, 'unit': 'edges/s', 'graphs_per_s': st_graphs / st_dt, 'seconds': st_dt,
                'h2d_bytes_per_edge': st_h2d / st_edges, 'scaling': 'weak',
                'producers_per_rank': [i['producers'] for i in st_info], 'producer_cap': cap,
                'shard_seed_ranges': [list(i['seed_range']) for i in st_info]}
        if tr_dt > 0:
            line['streamed_training'] = {
                'workload': 'configs[4] as DP training: MoleculeModel (depth 3, hidden 300, regression, Adam) on '
                            'streamed polymer batches of 128 per rank, one flat fp32 gradient all-reduce per step '
                            f'({"RCCL" if world > 1 else "none at N=1"})',
                'steps_per_rank': tr_steps, 'n_gpus': world, 'value': tr_edges / tr_dt, 'unit': 'edges/s',
                'ms_per_step': tr_dt / tr_steps * 1e3, 'graphs_per_s': tr_steps * 128 * world / tr_dt,
                'scaling': 'weak'}
        log('[bench] packing report')
        line['packing'] = packing_report(a, device, elapsed / a.steps)
        if world == 1 and a.kind == 'polymer' and not a.no_secondary:
            # (after the streamed legs the host-bound QM9 loop below takes 15-19 instead of 10.3-10.9 us per
            # forward -- four in flight, same box, round 6; run before them it recovers and the streamed leg
            # loses 60 %: whichever workload comes second pays -- not the hardware queues (8 change nothing),
            # cause not isolated; the order stays, the north-star streamed leg first)
            log('[bench] secondary workloads (qm9, zinc, training step)')
            line['secondary'] = [secondary_workload(device, 'qm9', 64, 3, 300, 200),
                                 secondary_workload(device, 'zinc', 512, 5, 512, 30),
                                 training_workload(device), atom_messages_workload(device)]
        if not a.no_cpu and world == 1:  # the CPU leg is timed at N=1 only
            log(f'[bench] CPU baseline (~{a.cpu_seconds:.0f} s + a one-thread sample)')
            cpu = cpu_baseline(TrainArgs(hidden_size=H, depth=a.depth, device=torch.device('cpu')), graphs[0],
                               a.cpu_seconds)
            line['cpu_baseline'] = cpu
        log(f'timed {a.steps} steps: {elapsed * 1e3:.2f} ms ({elapsed / a.steps * 1e6:.1f} us/step); with events '
            f'{elapsed_prof / a.steps * 1e6:.1f} us/step')
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
