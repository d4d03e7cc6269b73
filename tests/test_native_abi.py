"""CPU: libwdmpnn.so loads, exports every entry point include/wdmpnn.h declares, and its host-side
argument checking / workspace sizing behaves (no kernel is launched: no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

from chemprop_amd import _native, synthetic
from chemprop_amd.featurization import BatchMolGraph

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'wdmpnn.h')


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'\b(wdmpnn_\w+)\s*\(', text)))


def test_header_declares_what_binding_uses():
    assert declared_functions() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    assert os.path.exists(_native.LIB_PATH), 'build libwdmpnn.so first (__graft_entry__.build())'
    out = subprocess.run(['nm', '-D', '--defined-only', _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r'\bT (wdmpnn_\w+)', out))
    missing = set(declared_functions()) - exported
    assert not missing, missing


def test_library_loads_with_abi_version():
    L = _native.lib()
    assert L.wdmpnn_abi_version() == _native.ABI_VERSION


def test_library_is_built_for_gfx950():
    blob = open(_native.LIB_PATH, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in blob


def _structs(depth=3, hidden=300, atom_messages=False, undirected=False, act='ReLU'):
    g = BatchMolGraph(synthetic.make_batch('polymer', 4, 0))
    dg = g.device_graph('cpu', atom_messages)  # host-only: pointers are offsets, never dereferenced
    p = _native.WdParams()
    p.hidden = hidden
    for f in ('W_i', 'W_h', 'W_o', 'b_o', 'zero_vec', 'prelu'):
        setattr(p, f, 4096)
    c = _native.WdConfig()
    c.depth, c.undirected, c.activation, c.aggregation = depth, int(undirected), _native.ACTIVATIONS[act], 0
    c.aggregation_norm, c.dropout, c.save_for_backward = 100.0, 0.0, 1
    return g, dg, p, c


def test_workspace_bytes_scales_with_depth_and_hidden():
    L = _native.lib()
    sizes = []
    for depth, hidden in ((3, 300), (5, 300), (3, 512)):
        g, dg, p, c = _structs(depth, hidden)
        n = ctypes.c_size_t()
        _native.check(L.wdmpnn_workspace_bytes(ctypes.byref(dg.struct), ctypes.byref(p), ctypes.byref(c),
                                               ctypes.byref(n)), 'ws')
        sizes.append(n.value)
        # save_for_backward: depth x (Z, M) message layers + (Zo, h) atom layers, fp32
        assert n.value >= 4 * hidden * (2 * depth * g.n_bonds + 2 * g.n_atoms)
    assert sizes[1] > sizes[0] and sizes[2] > sizes[0]


@pytest.mark.parametrize('bad', ['depth', 'dropout', 'activation', 'atom_undirected', 'prelu'])
def test_argument_errors_are_reported(bad):
    L = _native.lib()
    g, dg, p, c = _structs()
    s = _native.WdGraph.from_buffer_copy(dg.struct)
    if bad == 'depth':
        c.depth = 0
    elif bad == 'dropout':
        c.dropout = 1.0
    elif bad == 'activation':
        c.activation = 42
    elif bad == 'prelu':
        c.activation = _native.ACTIVATIONS['PReLU']
        p.prelu = 0
    else:
        s.atom_messages = 1
        c.undirected = 1
    n = ctypes.c_size_t()
    rc = L.wdmpnn_workspace_bytes(ctypes.byref(s), ctypes.byref(p), ctypes.byref(c), ctypes.byref(n))
    assert rc < 0
    assert L.wdmpnn_last_error().decode()
    with pytest.raises((ValueError, NotImplementedError)):
        _native.check(rc, 'x')


def test_forward_rejects_small_workspace_without_launching():
    L = _native.lib()
    g, dg, p, c = _structs()
    rc = L.wdmpnn_forward(ctypes.byref(dg.struct), ctypes.byref(p), ctypes.byref(c), 4096, 16, 4096, None)
    assert rc == -1002
    assert 'workspace' in L.wdmpnn_last_error().decode()


def test_encoder_refuses_cpu_execution():
    from chemprop_amd import TrainArgs, MPNEncoder
    enc = MPNEncoder(TrainArgs(device=torch.device('cpu')), 133, 147)
    with pytest.raises(RuntimeError, match='HIP path only'):
        enc(BatchMolGraph(synthetic.make_batch('qm9', 2, 0)))
