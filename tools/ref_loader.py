"""Load the reference hot path (mpn.py, nn_utils.py, featurization.py, model.py) from /root/reference.

Used ONLY by tools/make_goldens.py in the build container to produce the committed fixtures under
tests/golden/.  Nothing on the GPU box imports this (the reference does not exist there).

Recipe: the package root ``chemprop/__init__.py`` pulls tap/tensorboardX/hyperopt/
RDKit, none of which is installed, so each needed file is loaded by path under stub parent packages.
RDKit is replaced by a stub exposing only the enum values ``featurization.py:27-33`` reads when it
builds ``Featurization_parameters`` (they fix list lengths, hence ATOM_FDIM=133).  The stub is never
used to featurise atoms: inputs are synthetic featurised graphs.  No bytecode is written into the
reference tree (``sys.dont_write_bytecode``).
"""
from __future__ import annotations

import enum
import importlib.util
import os
import sys
import types

REF = os.environ.get('WDMPNN_REFERENCE', '/root/reference')


def _stub_rdkit():
    rdkit = types.ModuleType('rdkit')
    chem = types.ModuleType('rdkit.Chem')
    rdchem = types.ModuleType('rdkit.Chem.rdchem')

    class HybridizationType(enum.IntEnum):
        UNSPECIFIED = 0
        S = 1
        SP = 2
        SP2 = 3
        SP3 = 4
        SP3D = 5
        SP3D2 = 6
        OTHER = 7

    class BondType(enum.IntEnum):
        UNSPECIFIED = 0
        SINGLE = 1
        DOUBLE = 2
        TRIPLE = 3
        AROMATIC = 12

    class _Placeholder:
        pass

    rdchem.HybridizationType = HybridizationType
    rdchem.BondType = BondType
    rdchem.Atom = _Placeholder
    rdchem.Bond = _Placeholder
    rdchem.Mol = _Placeholder
    rdchem.RWMol = _Placeholder
    chem.rdchem = rdchem
    chem.Mol = _Placeholder
    chem.Atom = _Placeholder
    chem.Bond = _Placeholder
    rdkit.Chem = chem
    sys.modules['rdkit'] = rdkit
    sys.modules['rdkit.Chem'] = chem
    sys.modules['rdkit.Chem.rdchem'] = rdchem


def _load(name: str, relpath: str):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    """Return a namespace with the reference's featurization, nn_utils, mpn and model modules."""
    sys.dont_write_bytecode = True
    if 'chemprop.models.mpn' in sys.modules:
        m = sys.modules
        return types.SimpleNamespace(featurization=m['chemprop.features.featurization'],
                                     nn_utils=m['chemprop.nn_utils'], mpn=m['chemprop.models.mpn'],
                                     model=m['chemprop.models.model'])
    _stub_rdkit()
    pkg = types.ModuleType('chemprop')
    pkg.__path__ = []
    sys.modules['chemprop'] = pkg
    args = types.ModuleType('chemprop.args')
    args.TrainArgs = object
    sys.modules['chemprop.args'] = args
    _load('chemprop.rdkit', 'chemprop/rdkit.py')
    feats_pkg = types.ModuleType('chemprop.features')
    feats_pkg.__path__ = []
    sys.modules['chemprop.features'] = feats_pkg
    featurization = _load('chemprop.features.featurization', 'chemprop/features/featurization.py')
    for name in ('BatchMolGraph', 'get_atom_fdim', 'get_bond_fdim', 'mol2graph'):
        setattr(feats_pkg, name, getattr(featurization, name))
    nn_utils = _load('chemprop.nn_utils', 'chemprop/nn_utils.py')
    models_pkg = types.ModuleType('chemprop.models')
    models_pkg.__path__ = [os.path.join(REF, 'chemprop/models')]
    sys.modules['chemprop.models'] = models_pkg
    mpn = _load('chemprop.models.mpn', 'chemprop/models/mpn.py')
    model = _load('chemprop.models.model', 'chemprop/models/model.py')
    return types.SimpleNamespace(featurization=featurization, nn_utils=nn_utils, mpn=mpn, model=model)
