"""bench.py's measurement formulas and output contract.

* CPU: the whole-forward algorithmic bytes / FLOPs of SURVEY.md §8(d) for its representative polymer
  batch (B=64, V=2,184 atoms, E=6,144 directed bonds, H=300, T=3): 86.55 MB and 3.321 GFLOP.
* GPU: one short bench.py run prints exactly one JSON line on stdout with the driver's keys, plus
  the roofline and cpu_baseline objects."""
import json
import os
import subprocess
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_forward_roofline_matches_survey_numbers():
    import bench
    g = types.SimpleNamespace(n_bonds=6144 + 1, n_atoms=2184 + 1, a_scope=[(0, 0)] * 64)
    a = types.SimpleNamespace(hidden=300, depth=3)
    r = bench.forward_roofline([g], a, 1e-4)
    assert abs(r['algorithmic_bytes'] / 1e6 - 86.55) < 0.01
    assert abs(r['algorithmic_flops'] / 1e9 - 3.321) < 0.001
    assert r['combined_frac'] == max(r['hbm_frac'], r['mfma_fp32_frac'])


@pytest.mark.gpu
def test_bench_prints_one_contract_line():
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', '5', '--warmup', '1', '--no-cpu',
                        '--no-secondary', '--stream-graphs', '6400', '--stream-train-graphs', '1280'], cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline'):
        assert k in d, k
    assert d['n_gpus'] == 1 and d['steps'] == 5 and d['warmup'] == 1 and d['value'] > 0
    assert d['distinct_devices'] == 1 and len(d['rank_devices']) == 1 and d['rank_devices'][0]['ordinal'] == 0
    assert d['metric'] == json.load(open(os.path.join(ROOT, 'BASELINE.json')))['metric']
    rf = d['roofline']
    for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic'):
        assert k in rf, k
    assert abs(rf['frac'] - rf['achieved'] / rf['peak']) < 1e-9
    st, tr = d['streamed'], d['streamed_training']  # configs[4]: streamed forward and DP training
    assert st['graphs'] == 6400 and st['value'] > 0 and st['h2d_bytes_per_edge'] <= 16
    assert tr['steps_per_rank'] == 10 and tr['value'] > 0


def test_batches_in_flight_by_batch_size():
    """Three batches in flight for polymer-sized batches, four for QM9-sized ones (one-launch forwards
    of ~64 workgroups), one for ZINC-sized B = 512 (~30 k edges)."""
    import bench
    assert bench.default_streams(6164) == 3 and bench.default_streams(900) == 4
    assert bench.default_streams(30500) == 1


def test_usable_cores_respects_affinity_and_quota(monkeypatch, tmp_path):
    import bench
    monkeypatch.setattr(os, 'sched_getaffinity', lambda pid: set(range(256)))
    real_open = open

    def fake_open(path, *a, **k):
        if path == '/sys/fs/cgroup/cpu.max':
            f = tmp_path / 'cpu.max'
            f.write_text('1600000 100000\n')
            return real_open(f, *a, **k)
        return real_open(path, *a, **k)
    monkeypatch.setattr('builtins.open', fake_open)
    assert bench._usable_cores(16) == (16, 256, 16)
