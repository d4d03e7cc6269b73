"""ORACLE — test infrastructure, not product.

CPU restatement of the reference wD-MPNN encoder forward (chemprop/models/mpn.py:66-173 of
ayildiri/polymer-chemprop @ 2025-05-09), op for op in PyTorch on CPU tensors, with the reference's
padded gathers (index_select_ND, nn_utils.py:50-67).  It is:

  * the parity checker for the HIP path (tests/, __graft_entry__.smoke()),
  * the "port" CPU baseline timed by bench.py (cpu_baseline leg),
  * pinned against the REAL reference by tests/test_oracle_golden.py, which replays the committed
    fixtures in tests/golden/ (made by tools/make_goldens.py from /root/reference in the build
    container: outputs and parameter gradients of MPNEncoder / MoleculeModel on synthetic
    featurised graphs).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this module.
Inputs: any object with the reference BatchMolGraph attributes (chemprop_amd's BatchMolGraph has
them), a dict of parameters named like the reference state_dict, and an args-like object.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F


def index_select_ND(source: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """nn_utils.py:50-67."""
    target = source.index_select(dim=0, index=index.view(-1))
    return target.view(index.size() + source.size()[1:])


KINKED = ('ReLU', 'LeakyReLU', 'PReLU', 'SELU')  # derivative jumps at 0


def activation(name: str, x: torch.Tensor, prelu_weight: Optional[torch.Tensor] = None,
               mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """nn_utils.py:70-99 (functional form).  ``mask`` (parity tests only): for the kinked activations,
    take the branch of each element from ``mask`` (True = the z > 0 branch) instead of from the sign of
    ``x``; same function away from 0, so an fp64 evaluation shares the kink decisions of an fp32 run
    whose pre-activations gave the mask (sub-ulp sign flips at 0 are then not compared)."""
    if mask is not None and name in KINKED:
        m = mask.to(x.device)
        if name == 'ReLU':
            return torch.where(m, x, torch.zeros_like(x))
        if name == 'LeakyReLU':
            return torch.where(m, x, 0.1 * x)
        if name == 'PReLU':
            return torch.where(m, x, prelu_weight * x)
        return torch.where(m, 1.0507009873554804934193349852946 * x,
                           1.0507009873554804934193349852946 * 1.6732632423543772848170429916717 * torch.expm1(x))
    if name == 'ReLU':
        return F.relu(x)
    if name == 'LeakyReLU':
        return F.leaky_relu(x, 0.1)
    if name == 'PReLU':
        return F.prelu(x, prelu_weight)
    if name == 'tanh':
        return torch.tanh(x)
    if name == 'SELU':
        return F.selu(x)
    if name == 'ELU':
        return F.elu(x)
    raise ValueError(f'Activation "{name}" not supported.')


def _linear(p: Dict[str, torch.Tensor], name: str, x: torch.Tensor) -> torch.Tensor:
    b = p.get(f'{name}.bias')
    return F.linear(x, p[f'{name}.weight'], b)


def encoder_forward(p: Dict[str, torch.Tensor], graph, args,
                    atom_descriptors_batch: Optional[List[np.ndarray]] = None, dtype=None,
                    masks: Optional[dict] = None) -> torch.Tensor:
    """mpn.py:66-173 with dropout = 0.  ``p`` keys: W_i.weight, [W_i.bias], W_h.weight, [W_h.bias],
    W_o.weight, W_o.bias, cached_zero_vector, [act_func.weight], [atom_descriptors_layer.*].
    ``dtype=torch.float64`` evaluates the same op sequence in double precision (conditioning
    reference for the parity tests); the default keeps the reference's float32.  ``masks`` = {'Z':
    [one bool tensor per message activation, mpn.py:97 then each mpn.py:123], 'Zo': bool tensor for
    mpn.py:133}: kink branches taken from another evaluation (``activation``'s ``mask``)."""
    calls = iter((masks['Z'] + [masks['Zo']]) if masks is not None else [])
    act = lambda x: activation(args.activation, x, p.get('act_func.weight'), next(calls, None))  # noqa: E731
    if atom_descriptors_batch is not None:  # mpn.py:77-79
        atom_descriptors_batch = [np.zeros([1, atom_descriptors_batch[0].shape[1]])] + list(atom_descriptors_batch)
        atom_descriptors_batch = torch.from_numpy(np.concatenate(atom_descriptors_batch, axis=0)).float()
        if dtype is not None:
            atom_descriptors_batch = atom_descriptors_batch.to(dtype)
    f_atoms, f_bonds, w_atoms, w_bonds, a2b, b2a, b2revb, a_scope, b_scope, degree_of_polym = \
        graph.get_components(atom_messages=args.atom_messages)  # mpn.py:81-82
    if dtype is not None:
        f_atoms, f_bonds, w_atoms, w_bonds = (t.to(dtype) for t in (f_atoms, f_bonds, w_atoms, w_bonds))
    if args.atom_messages:
        a2a = graph.get_a2a()  # mpn.py:89-90
        inp = _linear(p, 'W_i', f_atoms)  # mpn.py:93-94
    else:
        inp = _linear(p, 'W_i', f_bonds)  # mpn.py:95-96
    message = act(inp)  # mpn.py:97
    for _ in range(args.depth - 1):  # mpn.py:100
        if args.undirected:
            message = (message + message[b2revb]) / 2  # mpn.py:101-102
        if args.atom_messages:  # mpn.py:104-108
            nei_a_message = index_select_ND(message, a2a)
            nei_f_bonds = index_select_ND(f_bonds, a2b)
            message = torch.cat((nei_a_message, nei_f_bonds), dim=2).sum(dim=1)
        else:  # mpn.py:110-120
            nei_a_message = index_select_ND(message, a2b)
            nei_a_weight = index_select_ND(w_bonds, a2b)
            nei_a_message = nei_a_message * nei_a_weight[..., None]
            a_message = nei_a_message.sum(dim=1)
            rev_message = message[b2revb]
            message = a_message[b2a] - rev_message
        message = _linear(p, 'W_h', message)  # mpn.py:122
        message = act(inp + message)  # mpn.py:123
    a2x = a2a if args.atom_messages else a2b  # mpn.py:126-131
    nei_a_message = index_select_ND(message, a2x)
    nei_a_weight = index_select_ND(w_bonds, a2x)
    a_message = (nei_a_message * nei_a_weight[..., None]).sum(dim=1)
    a_input = torch.cat([f_atoms, a_message], dim=1)  # mpn.py:132
    atom_hiddens = act(_linear(p, 'W_o', a_input))  # mpn.py:133
    if atom_descriptors_batch is not None:  # mpn.py:137-143
        if len(atom_hiddens) != len(atom_descriptors_batch):
            raise ValueError('The number of atoms is different from the length of the extra atom features')
        atom_hiddens = torch.cat([atom_hiddens, atom_descriptors_batch], dim=1)
        atom_hiddens = _linear(p, 'atom_descriptors_layer', atom_hiddens)
    mol_vecs = []  # mpn.py:146-171
    for i, (a_start, a_size) in enumerate(a_scope):
        if a_size == 0:
            mol_vecs.append(p['cached_zero_vector'])
            continue
        cur = atom_hiddens.narrow(0, a_start, a_size)
        w = w_atoms.narrow(0, a_start, a_size)
        mol_vec = w[..., None] * cur
        if args.aggregation == 'mean':
            mol_vec = mol_vec.sum(dim=0) / w.sum(dim=0)
        elif args.aggregation == 'sum':
            mol_vec = mol_vec.sum(dim=0)
        elif args.aggregation == 'norm':
            mol_vec = mol_vec.sum(dim=0) / args.aggregation_norm
        mol_vecs.append(degree_of_polym[i] * mol_vec)
    return torch.stack(mol_vecs, dim=0)


def model_forward(p: Dict[str, torch.Tensor], graphs: list, args, features_batch=None, training=False):
    """model.py:152-194 + mpn.py:210-289 for encoders named encoder.encoder.<k>.* and ffn.<i>.*."""
    encs = []
    for k, g in enumerate(graphs):
        k_enc = 0 if args.mpn_shared else k
        pre = f'encoder.encoder.{k_enc}.'
        sub = {n[len(pre):]: t for n, t in p.items() if n.startswith(pre)}
        encs.append(encoder_forward(sub, g, args))
    out = torch.cat(encs, dim=1)
    if args.use_input_features:
        out = torch.cat([out, torch.from_numpy(np.stack(features_batch)).float()], dim=1)
    idx = sorted({int(n.split('.')[1]) for n in p if n.startswith('ffn.')})
    for j, i in enumerate(idx):
        out = F.linear(out, p[f'ffn.{i}.weight'], p[f'ffn.{i}.bias'])
        if j < len(idx) - 1:
            out = activation(args.activation, out, p.get('ffn.2.weight'))
    if args.dataset_type == 'classification' and not training:
        out = torch.sigmoid(out)
    return out
