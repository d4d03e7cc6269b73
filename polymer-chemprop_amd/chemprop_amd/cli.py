"""``chemprop_train`` counterpart for the wD-MPNN on MI355X (BASELINE.json configs[0]: ``chemprop_train
--polymer`` regression on a small polymer CSV, depth 3, hidden 300).

    python -m chemprop_amd.cli --data_path polymers.csv --graphs_path polymers.npz --dataset_type regression \
        --polymer --save_dir out [--epochs 30 --batch_size 50 --depth 3 --hidden_size 300 ...]

The run follows the reference's ``cross_validate`` -> ``run_training`` -> ``train`` chain for one fold
(cross_validate.py:22-115, run_training.py:28-499, train.py:17-113), with the pieces outside the hot path
restated here:

* data: CSV with a header; the first column holds the (polymer) SMILES, the others the targets, empty
  cells = missing (utils.py get_data); graphs come pre-featurised from ``--graphs_path`` (one MolGraph
  record per row, ``chemprop_amd.graph_io``) since RDKit featurisation is out of scope here;
  ``--polymer`` checks every SMILES cell as a polymer string (``chemprop_amd.polymer``);
* split: ``split_type random`` with ``split_sizes`` and ``seed`` (data/utils.py:536-547), the default
  branch the fork lost in run_training.py:58-89 and that run_training_V0.py:74-81 still has;
* targets scaled by a StandardScaler fit on the training set (scaler.py:6-63) for regression;
* MoleculeModel + initialize_weights after ``torch.manual_seed(pytorch_seed)`` (run_training.py:36,
  model.py:39), Adam (utils.py:295-310), NoamLR stepped per batch (utils.py:490-541, nn_utils.py:115-194),
  training batches reshuffled every epoch by one ``Random(seed)`` (data.py:537-587);
* each epoch: train, evaluate validation and training sets (evaluate.py), ``train_val_loss_log.csv``,
  ``model.pt``; the best validation score (``--metric``, rmse by default) keeps ``best_model.pt``;
* test: best weights, predictions inverse-scaled, ``test_scores.json`` / ``test_scores.csv``
  (run_training.py:440-491, cross_validate.py:149-172) and ``test_preds.csv``.

The encoder runs on the HIP path (a GPU is required, like every ``chemprop_amd`` forward).  Checkpoints
(``model.pt``, ``best_model.pt``) have the layout of the reference's ``save_checkpoint`` (utils.py:47-73):
``args`` (a plain dict), ``state_dict`` (the reference's parameter names), ``data_scaler`` /
``features_scaler`` / ``atom_descriptor_scaler`` / ``bond_feature_scaler`` as ``{'means', 'stds'}`` lists
or None -- only plain types, so ``torch.load(..., weights_only=True)`` reads them; ``load_checkpoint`` and
``load_scalers`` read them back (utils.py:80-131, 263-293).
"""
from __future__ import annotations

import argparse
import csv
import json
import math
import os
import re
import sys
from random import Random
from typing import Dict, List, Optional

import numpy as np
import torch

from .args import TrainArgs
from .featurization import BatchMolGraph
from .graph_io import load_graphs
from .model import MoleculeModel
from .nn_utils import initialize_weights
from .polymer import split_polymer_string, parse_polymer_rules
from .train import NoamLR, build_optimizer, get_loss_func, train_step


class StandardScaler:
    """scaler.py:6-63 (means / stds over axis 0 ignoring missing values; nan -> 0 / 1, zero std -> 1)."""

    def __init__(self, means=None, stds=None, replace_nan_token=None):
        self.means, self.stds, self.replace_nan_token = means, stds, replace_nan_token

    def fit(self, X):
        X = np.array(X).astype(float)
        self.means = np.nanmean(X, axis=0)
        self.stds = np.nanstd(X, axis=0)
        self.means = np.where(np.isnan(self.means), np.zeros(self.means.shape), self.means)
        self.stds = np.where(np.isnan(self.stds), np.ones(self.stds.shape), self.stds)
        self.stds = np.where(self.stds == 0, np.ones(self.stds.shape), self.stds)
        return self

    def transform(self, X):
        X = np.array(X).astype(float)
        t = (X - self.means) / self.stds
        return np.where(np.isnan(t), self.replace_nan_token, t)

    def inverse_transform(self, X):
        X = np.array(X).astype(float)
        t = X * self.stds + self.means
        return np.where(np.isnan(t), self.replace_nan_token, t)


def _scaler_to_dict(sc: Optional[StandardScaler]):
    """utils.py:58-62: means / stds as plain lists (None without a scaler)."""
    if sc is None:
        return None
    conv = (lambda v: np.asarray(v, dtype=float).tolist() if v is not None else None)
    return {'means': conv(sc.means), 'stds': conv(sc.stds)}


def _plain(v):
    if isinstance(v, (bool, int, float, str)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    return str(v)  # e.g. torch.device


def save_checkpoint(path: str, model, scaler: Optional[StandardScaler] = None,
                    features_scaler: Optional[StandardScaler] = None, args=None) -> None:
    """utils.py:47-73: {'args', 'state_dict', 'data_scaler', 'features_scaler', 'atom_descriptor_scaler',
    'bond_feature_scaler'}; every value a plain type (weights_only-loadable)."""
    a = {} if args is None else {k: _plain(v) for k, v in (vars(args) if not isinstance(args, dict) else args).items()}
    torch.save({'args': a, 'state_dict': model.state_dict(), 'data_scaler': _scaler_to_dict(scaler),
                'features_scaler': _scaler_to_dict(features_scaler), 'atom_descriptor_scaler': None,
                'bond_feature_scaler': None}, path)


def load_checkpoint(path: str, device=None):
    """utils.py:80-131 for this module's checkpoints: a MoleculeModel rebuilt from the stored args with the
    stored weights (``encoder.encoder.W*`` names of older checkpoints remapped to ``encoder.encoder.0.W*``,
    utils.py:114-115).  Loaded with weights_only=True: nothing in the file is executed."""
    state = torch.load(path, map_location='cpu', weights_only=True)
    if not isinstance(state, dict) or 'state_dict' not in state:
        raise ValueError(f'{path} is not a checkpoint (no state_dict)')
    sd = {re.sub(r'^encoder\.encoder\.([Wc])', r'encoder.encoder.0.\1', k): v for k, v in state['state_dict'].items()}
    if 'args' not in state:
        return sd
    fields = set(TrainArgs.__dataclass_fields__)
    kw = {k: v for k, v in state['args'].items() if k in fields and k != 'device'}
    args = TrainArgs(**kw, device=torch.device(device) if device is not None else torch.device('cpu'))
    model = MoleculeModel(args)
    model.load_state_dict(sd)
    return model.to(args.device)


def load_scalers(path: str):
    """utils.py:263-293: (data scaler, features scaler, atom descriptor scaler, bond feature scaler)."""
    state = torch.load(path, map_location='cpu', weights_only=True)

    def mk(d, nan_token=None):
        if d is None:
            return None
        return StandardScaler(np.asarray(d['means'], dtype=float), np.asarray(d['stds'], dtype=float),
                              replace_nan_token=nan_token)
    return (mk(state.get('data_scaler')), mk(state.get('features_scaler'), 0),
            mk(state.get('atom_descriptor_scaler'), 0), mk(state.get('bond_feature_scaler'), 0))


def random_split(n: int, sizes, seed: int):
    """data/utils.py:536-547 (split_type 'random') on row indices."""
    if not (len(sizes) == 3 and sum(sizes) == 1):
        raise ValueError('Valid split sizes must sum to 1 and must have three sizes: train, validation, and test.')
    indices = list(range(n))
    Random(seed).shuffle(indices)
    train_size = int(sizes[0] * n)
    train_val_size = int((sizes[0] + sizes[1]) * n)
    return indices[:train_size], indices[train_size:train_val_size], indices[train_val_size:]


def metric_value(metric: str, targets: List[float], preds: List[float]) -> float:
    """utils.py get_metric_func for the scalar metrics."""
    from sklearn.metrics import mean_absolute_error, mean_squared_error, r2_score, roc_auc_score
    if metric == 'rmse':
        return math.sqrt(mean_squared_error(targets, preds))
    if metric == 'mse':
        return mean_squared_error(targets, preds)
    if metric == 'mae':
        return mean_absolute_error(targets, preds)
    if metric == 'r2':
        return r2_score(targets, preds)
    if metric == 'auc':
        return roc_auc_score(targets, preds)
    raise ValueError(f'Metric "{metric}" not supported.')


def evaluate_predictions(preds, targets, num_tasks: int, metrics: List[str], dataset_type: str) -> Dict[str, list]:
    """evaluate.py:11-77: per task over the rows with a target."""
    if len(preds) == 0:
        return {m: [float('nan')] * num_tasks for m in metrics}
    out = {m: [] for m in metrics}
    for i in range(num_tasks):
        vp = [preds[j][i] for j in range(len(preds)) if targets[j][i] is not None]
        vt = [targets[j][i] for j in range(len(preds)) if targets[j][i] is not None]
        if dataset_type == 'classification' and (all(t == 0 for t in vt) or all(t == 1 for t in vt) or
                                                 all(p == 0 for p in vp) or all(p == 1 for p in vp)):
            for m in metrics:
                out[m].append(float('nan'))
            continue
        if not vt:
            continue
        for m in metrics:
            out[m].append(metric_value(m, vt, vp))
    return out


def predict(model, graphs, idx, batch_size: int, scaler: Optional[StandardScaler]) -> List[List[float]]:
    """predict.py:10-68: eval, no_grad, batches in order, inverse scaling."""
    model.eval()
    preds = []
    with torch.no_grad():
        for s in range(0, len(idx), batch_size):
            g = BatchMolGraph([graphs[i] for i in idx[s:s + batch_size]])
            preds.extend(model([g]).cpu().numpy().tolist())
    if scaler is not None and preds:
        preds = scaler.inverse_transform(preds).tolist()
    return preds


def read_csv(path: str):
    with open(path) as f:
        rows = list(csv.reader(f))
    header, body = rows[0], [r for r in rows[1:] if r]
    smiles = [r[0] for r in body]
    targets = [[float(x) if x.strip() != '' else None for x in r[1:]] for r in body]
    return header, smiles, targets


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog='chemprop_train', description=__doc__.split('\n')[0])
    ap.add_argument('--data_path', required=True)
    ap.add_argument('--graphs_path', required=True, help='pre-featurised MolGraph records, one per CSV row')
    ap.add_argument('--dataset_type', default='regression', choices=['regression', 'classification'])
    ap.add_argument('--save_dir', required=True)
    ap.add_argument('--polymer', action='store_true')
    ap.add_argument('--split_type', default='random', choices=['random'])
    ap.add_argument('--split_sizes', type=float, nargs=3, default=(0.8, 0.1, 0.1))
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--pytorch_seed', type=int, default=0)
    ap.add_argument('--metric', default=None)
    ap.add_argument('--extra_metrics', nargs='*', default=[])
    ap.add_argument('--epochs', type=int, default=30)
    ap.add_argument('--batch_size', type=int, default=50)
    ap.add_argument('--warmup_epochs', type=float, default=2.0)
    ap.add_argument('--init_lr', type=float, default=1e-4)
    ap.add_argument('--max_lr', type=float, default=1e-3)
    ap.add_argument('--final_lr', type=float, default=1e-4)
    ap.add_argument('--grad_clip', type=float, default=None)
    for name, default in (('hidden_size', 300), ('depth', 3), ('ffn_num_layers', 2)):
        ap.add_argument(f'--{name}', type=int, default=default)
    ap.add_argument('--ffn_hidden_size', type=int, default=None)
    ap.add_argument('--dropout', type=float, default=0.0)
    ap.add_argument('--activation', default='ReLU')
    ap.add_argument('--aggregation', default='mean', choices=['mean', 'sum', 'norm'])
    ap.add_argument('--aggregation_norm', type=int, default=100)
    ap.add_argument('--bias', action='store_true')
    ap.add_argument('--undirected', action='store_true')
    ap.add_argument('--gpu', type=int, default=0)
    return ap.parse_args(argv)


def run_training(a: argparse.Namespace) -> Dict[str, list]:
    os.makedirs(a.save_dir, exist_ok=True)
    header, smiles, targets = read_csv(a.data_path)
    graphs = load_graphs(a.graphs_path)
    if len(graphs) != len(smiles):
        raise ValueError(f'{a.graphs_path} holds {len(graphs)} graphs for {len(smiles)} CSV rows')
    if a.polymer:  # every row must be a well-formed polymer string (data.py:695-703, featurization.py:335-364)
        for s, g in zip(smiles, graphs):
            _, _, rules = split_polymer_string(s)
            if rules:
                _, deg = parse_polymer_rules(rules)
                if not np.isclose(deg, g.degree_of_polym, rtol=1e-6):
                    raise ValueError(f'graph degree_of_polym {g.degree_of_polym} != 1 + log10(Xn) = {deg} for {s}')
    num_tasks = len(header) - 1
    metric = a.metric or ('rmse' if a.dataset_type == 'regression' else 'auc')
    metrics = [metric] + [m for m in a.extra_metrics if m != metric]
    minimize = metric in ('rmse', 'mse', 'mae')
    device = torch.device('cuda', a.gpu)
    args = TrainArgs(hidden_size=a.hidden_size, depth=a.depth, dropout=a.dropout, activation=a.activation,
                     aggregation=a.aggregation, aggregation_norm=a.aggregation_norm, bias=a.bias,
                     undirected=a.undirected, ffn_num_layers=a.ffn_num_layers,
                     ffn_hidden_size=a.ffn_hidden_size or a.hidden_size, dataset_type=a.dataset_type,
                     num_tasks=num_tasks, device=device)
    torch.manual_seed(a.pytorch_seed)
    train_idx, val_idx, test_idx = random_split(len(smiles), a.split_sizes, a.seed)
    scaler = None
    train_targets = [targets[i] for i in train_idx]
    if a.dataset_type == 'regression':
        scaler = StandardScaler().fit(train_targets)
        train_targets = scaler.transform(train_targets).tolist()
        train_targets = [[None if (x is None or (isinstance(x, float) and math.isnan(x))) else x for x in r]
                         for r in train_targets]
    model = MoleculeModel(args)
    initialize_weights(model)
    model = model.to(device)
    optimizer = build_optimizer(model, a.init_lr)
    scheduler = NoamLR(optimizer, warmup_epochs=[a.warmup_epochs], total_epochs=[a.epochs],
                       steps_per_epoch=len(train_idx) // a.batch_size, init_lr=[a.init_lr], max_lr=[a.max_lr],
                       final_lr=[a.final_lr])
    loss_func = get_loss_func(a.dataset_type)
    sampler = Random(a.seed)
    log_path = os.path.join(a.save_dir, 'train_val_loss_log.csv')
    best = math.inf if minimize else -math.inf
    best_epoch = 0
    with open(log_path, 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['epoch', 'train_loss'] + [f'train_avg_{m}' for m in metrics] + [f'val_avg_{m}' for m in metrics])
        for epoch in range(a.epochs):
            order = list(range(len(train_idx)))
            sampler.shuffle(order)
            losses = []
            for s in range(0, len(order), a.batch_size):
                pos = order[s:s + a.batch_size]
                g = BatchMolGraph([graphs[train_idx[p]] for p in pos])
                loss = train_step(model, [g], [train_targets[p] for p in pos], loss_func, optimizer, scheduler,
                                  a.dataset_type, grad_clip=a.grad_clip)
                losses.append(float(loss))
            val_scores = evaluate_predictions(predict(model, graphs, val_idx, a.batch_size, scaler),
                                              [targets[i] for i in val_idx], num_tasks, metrics, a.dataset_type)
            tr_scores = evaluate_predictions(predict(model, graphs, train_idx, a.batch_size, scaler),
                                             [targets[i] for i in train_idx], num_tasks, metrics, a.dataset_type)
            w.writerow([epoch, float(np.mean(losses)) if losses else float('nan')] +
                       [float(np.nanmean(tr_scores[m])) if tr_scores[m] else float('nan') for m in metrics] +
                       [float(np.nanmean(val_scores[m])) if val_scores[m] else float('nan') for m in metrics])
            save_checkpoint(os.path.join(a.save_dir, 'model.pt'), model, scaler, None, args)
            v = float(np.nanmean(val_scores[metric])) if val_scores[metric] else float('nan')
            if (minimize and v < best) or (not minimize and v > best) or (epoch == 0 and math.isnan(v)):
                best, best_epoch = v, epoch
                save_checkpoint(os.path.join(a.save_dir, 'best_model.pt'), model, scaler, None, args)
    ckpt = torch.load(os.path.join(a.save_dir, 'best_model.pt'), map_location=device, weights_only=True)
    model.load_state_dict(ckpt['state_dict'])
    test_targets = [targets[i] for i in test_idx]
    test_preds = predict(model, graphs, test_idx, a.batch_size, scaler)
    scores = evaluate_predictions(test_preds, test_targets, num_tasks, metrics, a.dataset_type)
    with open(os.path.join(a.save_dir, 'test_scores.json'), 'w') as f:
        json.dump(scores, f, indent=4, sort_keys=True)
    with open(os.path.join(a.save_dir, 'test_scores.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Task'] + [f'Mean {m}' for m in metrics])
        for t, name in enumerate(header[1:]):
            w.writerow([name] + [scores[m][t] if t < len(scores[m]) else '' for m in metrics])
    with open(os.path.join(a.save_dir, 'test_preds.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(header)
        for i, p in zip(test_idx, test_preds):
            w.writerow([smiles[i]] + list(p))
    with open(os.path.join(a.save_dir, 'split_indices.json'), 'w') as f:
        json.dump({'train': train_idx, 'val': val_idx, 'test': test_idx, 'best_epoch': best_epoch}, f)
    return scores


def chemprop_train(argv=None) -> Dict[str, list]:
    """Entry point (setup.py:39 ``chemprop_train`` in the reference)."""
    return run_training(parse_args(argv))


if __name__ == '__main__':
    print(json.dumps(chemprop_train(sys.argv[1:])))
