"""MoleculeModel (``chemprop/models/model.py:14-194``): the encoder runs on the HIP library, the
small FFN head stays PyTorch (~1 % of the forward).  Module layout and
state_dict keys (``encoder.encoder.0.*``, ``ffn.1.*``, ``ffn.4.*`` ...) match the reference."""
from __future__ import annotations

from typing import List

import numpy as np
import torch
import torch.nn as nn

from .mpn import MPN
from .nn_utils import get_activation_function, initialize_weights


class _Exp(nn.Module):
    def forward(self, x):
        return torch.exp(x)


class MoleculeModel(nn.Module):
    def __init__(self, args):
        super(MoleculeModel, self).__init__()
        self.classification = args.dataset_type == 'classification'
        self.multiclass = args.dataset_type == 'multiclass'
        self.output_size = args.num_tasks * (args.multiclass_num_classes if self.multiclass else 1)
        if self.classification:
            self.sigmoid = nn.Sigmoid()
        if self.multiclass:
            self.multiclass_softmax = nn.Softmax(dim=2)
        self.create_encoder(args)
        self.create_ffn(args)
        initialize_weights(self)

    def create_encoder(self, args) -> None:
        """model.py:41-55."""
        self.encoder = MPN(args)
        if getattr(args, 'checkpoint_frzn', None) is not None:
            frozen = (list(self.encoder.encoder.children())[0].parameters() if args.freeze_first_only
                      else self.encoder.parameters())
            for param in frozen:
                param.requires_grad = False

    def create_ffn(self, args) -> None:
        """model.py:57-121: Dropout/Linear/act stack (same module indices as the reference)."""
        self.multiclass = args.dataset_type == 'multiclass'
        if self.multiclass:
            self.num_classes = args.multiclass_num_classes
        if args.features_only:
            first = args.features_size
        else:
            first = args.hidden_size * args.number_of_molecules + (args.features_size if args.use_input_features else 0)
        if getattr(args, 'atom_descriptors', None) == 'descriptor':
            first += args.atom_descriptors_size
        dropout = nn.Dropout(args.dropout)
        activation = get_activation_function(args.activation)
        if args.ffn_num_layers == 1:
            layers = [dropout, nn.Linear(first, self.output_size)]
        else:
            layers = [dropout, nn.Linear(first, args.ffn_hidden_size)]
            for _ in range(args.ffn_num_layers - 2):
                layers += [activation, dropout, nn.Linear(args.ffn_hidden_size, args.ffn_hidden_size)]
            layers += [activation, dropout, nn.Linear(args.ffn_hidden_size, self.output_size)]
        if args.dataset_type == 'spectra':
            layers.append(nn.Softplus() if args.spectra_activation == 'softplus' else _Exp())
        self.ffn = nn.Sequential(*layers)
        if getattr(args, 'checkpoint_frzn', None) is not None and args.frzn_ffn_layers > 0:
            for param in list(self.ffn.parameters())[0:2 * args.frzn_ffn_layers]:
                param.requires_grad = False

    def fingerprint(self, batch, features_batch: List[np.ndarray] = None, atom_descriptors_batch: List[np.ndarray] = None,
                    atom_features_batch: List[np.ndarray] = None, bond_features_batch: List[np.ndarray] = None,
                    fingerprint_type='MPN') -> torch.FloatTensor:
        """model.py:123-150."""
        enc = self.encoder(batch, features_batch, atom_descriptors_batch, atom_features_batch, bond_features_batch)
        if fingerprint_type == 'MPN':
            return enc
        if fingerprint_type == 'last_FFN':
            return self.ffn[:-1](enc)
        raise ValueError(f'Unsupported fingerprint type {fingerprint_type}.')

    def forward(self, batch, features_batch: List[np.ndarray] = None, atom_descriptors_batch: List[np.ndarray] = None,
                atom_features_batch: List[np.ndarray] = None, bond_features_batch: List[np.ndarray] = None,
                return_embeddings: bool = False):
        """model.py:152-194."""
        emb = self.encoder(batch, features_batch, atom_descriptors_batch, atom_features_batch, bond_features_batch)
        out = self.ffn(emb)
        if self.classification and not self.training:
            out = self.sigmoid(out)
        if self.multiclass:
            out = out.reshape((out.size(0), -1, self.num_classes))
            if not self.training:
                out = self.multiclass_softmax(out)
        return (out, emb) if return_embeddings else out
