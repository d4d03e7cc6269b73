"""The training entry point (chemprop_amd.cli, BASELINE.json configs[0]) and its host-side pieces.

CPU: polymer-string parsing, the random split, the target scaler and the NoamLR schedule against golden
vectors produced by the REAL reference functions (tools/make_host_goldens.py -> tests/golden/
host_plumbing.json); graph records round-trip through the .npz format.
GPU: ``chemprop_train --polymer`` on the committed 10-row polymer CSV runs end to end (split, scaler,
NoamLR epochs, per-epoch evaluation, best checkpoint, test scores) deterministically, and learns on a
larger synthetic polymer set."""
import json
import math
import os

import numpy as np
import pytest
import torch

from chemprop_amd import cli, polymer, synthetic
from chemprop_amd.featurization import BatchMolGraph
from chemprop_amd.graph_io import load_graphs, save_graphs
from chemprop_amd.train import NoamLR

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, 'golden', 'host_plumbing.json')))
CSV = os.path.join(HERE, 'data', 'polymer10.csv')
NPZ = os.path.join(HERE, 'data', 'polymer10_graphs.npz')


@pytest.mark.parametrize('case', range(len(GOLD['polymer_rules'])))
def test_parse_polymer_rules_matches_reference(case):
    g = GOLD['polymer_rules'][case]
    rules = list(g['rules'])
    info, deg = polymer.parse_polymer_rules(rules)
    assert [list(x) for x in info] == g['info']
    assert deg == g['degree']
    assert '~' not in rules[-1]  # the reference strips ~Xn from the last rule in place


def test_split_polymer_string_and_counts():
    s = GOLD['polymer_rules'][0]['string']
    smiles, weights, rules = polymer.split_polymer_string(s)
    assert weights == ['0.5', '0.5'] and len(rules) == 10
    assert polymer.fragment_attachments(smiles) == [['1', '2'], ['3', '4']]
    assert [polymer.count_heavy_atoms(f) for f in smiles.split('.')] == [8, 9]
    assert polymer.count_heavy_atoms('Clc1ccc([*:1])cc1Br') == 8
    with pytest.raises(ValueError):
        polymer.split_polymer_string('CC.CC|0.5|<1-2:1:1')  # two fragments, one weight (rdkit.py:31-35)
    with pytest.raises(ValueError):
        polymer.parse_polymer_rules(['1-2:0.5'])  # rdkit-free format check (featurization.py:350-351)


def test_synthetic_polymer_graph_follows_the_string():
    s = GOLD['polymer_rules'][4]['string']  # [*:1]C[*:2].[*:3]N[*:4]|0.4|0.6|<1-3:0.3:0.7<2-4:0.7:0.3~1000
    g = polymer.synthetic_polymer_graph(s, seed=1)
    assert g.n_atoms == 2 and g.w_atoms == [0.4, 0.6]
    assert abs(g.degree_of_polym - 4.0) < 1e-12
    assert sorted(set(g.w_bonds)) == [0.3, 0.7] and len(g.w_bonds) == 4
    b = BatchMolGraph([g, polymer.synthetic_polymer_graph(GOLD['polymer_rules'][0]['string'], seed=2)])
    assert b.a_scope[1][1] == 17 and b._compact is not None


@pytest.mark.parametrize('case', range(len(GOLD['split'])))
def test_random_split_matches_reference(case):
    g = GOLD['split'][case]
    if g.get('raises'):
        with pytest.raises(ValueError):
            cli.random_split(g['n'], g['sizes'], g['seed'])
        return
    assert [list(x) for x in cli.random_split(g['n'], g['sizes'], g['seed'])] == [g['train'], g['val'], g['test']]


@pytest.mark.parametrize('case', range(len(GOLD['scaler'])))
def test_standard_scaler_matches_reference(case):
    g = GOLD['scaler'][case]
    sc = cli.StandardScaler().fit(g['X'])
    assert np.allclose(sc.means, g['means'], rtol=0, atol=0) and np.allclose(sc.stds, g['stds'], rtol=0, atol=0)
    t = sc.transform(g['X']).tolist()
    assert [[None if v is None else float(v) for v in r] for r in t] == g['transform']
    tasks = len(g['X'][0])
    assert sc.inverse_transform([[0.5] * tasks, [-1.0] * tasks]).tolist() == g['inverse']


@pytest.mark.parametrize('case', range(len(GOLD['noam'])))
def test_noam_schedule_matches_reference(case):
    g = GOLD['noam'][case]
    opt = torch.optim.Adam([torch.nn.Parameter(torch.zeros(1))], lr=1e-4)
    with np.errstate(all='ignore'):
        sch = NoamLR(opt, warmup_epochs=[g['warmup_epochs']], total_epochs=[g['total_epochs']],
                     steps_per_epoch=g['steps_per_epoch'], init_lr=[1e-4], max_lr=[1e-3], final_lr=[1e-4])
        lrs = []
        for _ in range(len(g['lrs'])):
            sch.step()
            lrs.append(float(opt.param_groups[0]['lr']))
    assert all((a == b) or (math.isnan(a) and math.isnan(b)) for a, b in zip(lrs, g['lrs']))


def test_graph_records_roundtrip(tmp_path):
    mols = synthetic.make_batch('polymer', 5, 3) + synthetic.edge_case_batch(2, star_leaves=5)
    p = str(tmp_path / 'g.npz')
    save_graphs(p, mols)
    back = load_graphs(p)
    a, b = BatchMolGraph(mols), BatchMolGraph(back)
    for attr in ('f_atoms', 'f_bonds', 'w_atoms', 'w_bonds', 'b2a', 'b2revb', 'a2b'):
        assert torch.equal(getattr(a, attr), getattr(b, attr)), attr
    assert a.degree_of_polym == b.degree_of_polym


def test_fixture_rows_match_their_graphs():
    _, smiles, targets = cli.read_csv(CSV)
    graphs = load_graphs(NPZ)
    assert len(smiles) == len(graphs) == 10 and all(len(t) == 1 for t in targets)
    for s, g in zip(smiles, graphs):
        sm, w, rules = polymer.split_polymer_string(s)
        _, deg = polymer.parse_polymer_rules(rules)
        assert abs(deg - g.degree_of_polym) < 1e-9
        assert sorted(set(np.asarray(g.w_atoms).tolist())) == sorted({float(x) for x in w})


@pytest.mark.gpu
def test_chemprop_train_polymer_csv_end_to_end(tmp_path):
    argv = ['--data_path', CSV, '--graphs_path', NPZ, '--dataset_type', 'regression', '--polymer',
            '--epochs', '6', '--save_dir']
    s1 = cli.chemprop_train(argv + [str(tmp_path / 'a')])
    s2 = cli.chemprop_train(argv + [str(tmp_path / 'b')])
    assert s1 == s2 and len(s1['rmse']) == 1 and math.isfinite(s1['rmse'][0])  # deterministic
    d = tmp_path / 'a'
    for f in ('test_scores.json', 'test_scores.csv', 'test_preds.csv', 'train_val_loss_log.csv', 'model.pt',
              'best_model.pt', 'split_indices.json'):
        assert (d / f).exists(), f
    split = json.load(open(d / 'split_indices.json'))
    assert [split['train'], split['val'], split['test']] == [list(x) for x in cli.random_split(10, (0.8, 0.1, 0.1), 0)]
    sd = torch.load(d / 'best_model.pt', weights_only=True)['state_dict']
    assert 'encoder.encoder.0.W_i.weight' in sd and 'ffn.1.weight' in sd  # the reference's key names
    log = open(d / 'train_val_loss_log.csv').read().splitlines()
    assert len(log) == 7


@pytest.mark.gpu
def test_chemprop_train_learns_on_synthetic_polymers(tmp_path):
    """200 polymer rows whose target is a smooth function of the string (fractions, Xn): the training rmse
    falls well below its first-epoch value within 30 epochs (batches of 50, NoamLR with real warm-up)."""
    import csv as _csv
    rng = np.random.default_rng(5)
    rows, graphs = [], []
    for k in range(200):
        fa = float(rng.choice([0.25, 0.5, 0.75]))
        xn = float(rng.choice([1, 10, 100, 1000]))
        s = f'[*:1]c1ccc([*:2])cc1.[*:3]CC[*:4]|{fa}|{1 - fa}|<1-3:0.5:0.5<2-4:0.5:0.5<1-2:0.5:0.5~{xn:g}'
        rows.append([s, 2.0 * fa - 0.5 * np.log10(xn)])
        graphs.append(polymer.synthetic_polymer_graph(s, seed=k))
    csv_path, npz_path = str(tmp_path / 'p.csv'), str(tmp_path / 'p.npz')
    with open(csv_path, 'w', newline='') as f:
        w = _csv.writer(f)
        w.writerow(['smiles', 'y'])
        w.writerows(rows)
    save_graphs(npz_path, graphs)
    cli.chemprop_train(['--data_path', csv_path, '--graphs_path', npz_path, '--polymer', '--epochs', '30',
                        '--save_dir', str(tmp_path / 'o')])
    log = [ln.split(',') for ln in open(tmp_path / 'o' / 'train_val_loss_log.csv').read().splitlines()[1:]]
    first, last = float(log[0][2]), float(log[-1][2])  # train_avg_rmse
    spread = float(np.std([r[1] for r in rows]))
    assert last < 0.6 * first and last < 0.6 * spread, (first, last, spread)


def test_checkpoint_layout_and_scaler_roundtrip(tmp_path):
    """save_checkpoint writes the reference's layout (utils.py:47-73) with plain values only: it loads with
    weights_only=True, rebuilds the model with the same weights, and the target scaler comes back
    (load_scalers, utils.py:263-293), so saved predictions can be inverse-scaled outside the run."""
    from chemprop_amd import TrainArgs
    from chemprop_amd.model import MoleculeModel
    args = TrainArgs(hidden_size=32, depth=2, num_tasks=2, device=torch.device('cpu'))
    torch.manual_seed(0)
    m = MoleculeModel(args)
    sc = cli.StandardScaler().fit([[1.0, 2.0], [3.0, None], [5.0, 7.0]])
    p = str(tmp_path / 'ck.pt')
    cli.save_checkpoint(p, m, sc, None, args)
    raw = torch.load(p, weights_only=True)
    assert set(raw) == {'args', 'state_dict', 'data_scaler', 'features_scaler', 'atom_descriptor_scaler',
                        'bond_feature_scaler'}
    assert raw['args']['hidden_size'] == 32 and raw['features_scaler'] is None
    m2 = cli.load_checkpoint(p)
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    data_scaler, feat, _, _ = cli.load_scalers(p)
    assert feat is None
    np.testing.assert_array_equal(data_scaler.means, sc.means)
    np.testing.assert_array_equal(data_scaler.inverse_transform([[0.5, -1.0]]), sc.inverse_transform([[0.5, -1.0]]))
    # an older checkpoint's un-indexed encoder names are remapped (utils.py:114-115)
    old = {k.replace('encoder.encoder.0.', 'encoder.encoder.'): v for k, v in m.state_dict().items()}
    torch.save({'state_dict': old}, str(tmp_path / 'old.pt'))
    sd = cli.load_checkpoint(str(tmp_path / 'old.pt'))
    assert 'encoder.encoder.0.W_i.weight' in sd
