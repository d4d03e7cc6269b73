"""chemprop_amd — MI355X-native wD-MPNN encoder (the hot path of ayildiri/polymer-chemprop).

Drop-in replacements for ``chemprop.models.mpn.MPNEncoder`` / ``MPN``,
``chemprop.models.model.MoleculeModel``, ``chemprop.features.featurization.BatchMolGraph`` and
``chemprop.nn_utils.index_select_ND``, computed by hand-written gfx950 HIP kernels in
``libwdmpnn.so`` (C-ABI: include/wdmpnn.h).
"""
from .args import TrainArgs
from .featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim, mol2graph
from .model import MoleculeModel
from .mpn import MPN, MPNEncoder
from .nn_utils import get_activation_function, index_select_ND, initialize_weights

__all__ = ['TrainArgs', 'BatchMolGraph', 'get_atom_fdim', 'get_bond_fdim', 'mol2graph', 'MoleculeModel', 'MPN',
           'MPNEncoder', 'get_activation_function', 'index_select_ND', 'initialize_weights']
