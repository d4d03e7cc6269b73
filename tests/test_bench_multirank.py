"""bench.py's multi-rank path (process group, per-rank disjoint shards, MAX / SUM reductions of the
timings and counters, per-rank producer cap, streamed DP training with one gradient all-reduce per step),
run here as four ranks on cuda:0 over gloo: the 8-GPU node runs the same code with backend 'nccl' (chemprop_amd.dp
.init_distributed is the only initialisation path).  The launcher starts in a fresh child process,
before any GPU call in that child."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_four_ranks_gloo_on_one_gpu():
    per_rank = 1280
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '4',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), 'bench.py', '--gpus', '4',
           '--steps', '5', '--warmup', '1', '--n-batches', '2', '--no-cpu', '--no-secondary',
           '--stream-graphs', str(per_rank), '--stream-train-graphs', '512']
    env = dict(os.environ, BENCH_BACKEND='gloo', MASTER_ADDR='127.0.0.1', OMP_NUM_THREADS='4')
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one JSON line
    d = json.loads(lines[0])
    assert d['n_gpus'] == 4 and d['config']['global_batch'] == 256
    # the rehearsal is four ranks on ONE device over gloo, and the line says so (the 8-GPU node's line
    # must show backend nccl and 8 distinct devices)
    assert d['backend'] == 'gloo' and d['distinct_devices'] == 1
    assert len(d['rank_devices']) == 4 and {r['ordinal'] for r in d['rank_devices']} == {0}
    assert d['value'] > 0 and d['ms_per_step'] > 0
    st = d['streamed']
    assert st['graphs'] == 4 * per_rank and st['n_gpus'] == 4
    # producers per rank capped by the node's usable cores shared over its 4 ranks
    from chemprop_amd.stream import producer_cap
    assert st['producer_cap'] == producer_cap(4)
    assert st['producers_per_rank'] == [st['producer_cap']] * 4
    # disjoint shards: rank r streams batch seeds [lo_r, hi_r), pairwise disjoint
    rng = sorted(tuple(r) for r in st['shard_seed_ranges'])
    assert len(rng) == 4 and all(hi - lo == per_rank // 64 for lo, hi in rng)
    assert all(rng[i][1] <= rng[i + 1][0] for i in range(3))
    assert d['streamed_training']['n_gpus'] == 4 and d['streamed_training']['steps_per_rank'] == 4
    assert d['roofline']['launches_timed'] == 5 * 2
