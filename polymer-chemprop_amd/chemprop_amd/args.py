"""The subset of ``chemprop.args.TrainArgs`` (args.py:219-650) that the hot path and the model head
read, with the reference's defaults.  Any object with these attributes (e.g. a
real reference ``TrainArgs``) can be passed instead."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import torch


@dataclass
class TrainArgs:
    # MPNEncoder (mpn.py:24-64)
    atom_messages: bool = False          # args.py:323
    hidden_size: int = 300               # args.py:312
    bias: bool = False                   # args.py:310
    depth: int = 3                       # args.py:314
    dropout: float = 0.0                 # args.py:319
    undirected: bool = False             # args.py:325
    activation: str = 'ReLU'             # args.py:321
    aggregation: str = 'mean'            # args.py:356
    aggregation_norm: int = 100          # args.py:358
    atom_descriptors: Optional[str] = None
    atom_descriptors_size: int = 0
    device: torch.device = field(default_factory=lambda: torch.device('cuda' if torch.cuda.is_available() else 'cpu'))
    # MPN (mpn.py:189-208)
    features_only: bool = False
    use_input_features: bool = False
    overwrite_default_atom_features: bool = False
    overwrite_default_bond_features: bool = False
    mpn_shared: bool = False
    number_of_molecules: int = 1
    # MoleculeModel (model.py:23-121)
    dataset_type: str = 'regression'
    num_tasks: int = 1
    multiclass_num_classes: int = 3
    features_size: int = 0
    ffn_num_layers: int = 2
    ffn_hidden_size: Optional[int] = None
    spectra_activation: str = 'exp'
    checkpoint_frzn: Optional[str] = None
    freeze_first_only: bool = False
    frzn_ffn_layers: int = 0
    polymer: bool = False
    # optimizer (args.py:397-407, utils.py:295-310)
    init_lr: float = 1e-4
    optimizer: str = 'adam'
    weight_decay: float = 0.0

    def __post_init__(self):
        if self.ffn_hidden_size is None:  # args.py:584-585
            self.ffn_hidden_size = self.hidden_size
