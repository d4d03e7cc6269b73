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


# ---------------------------------------------------------------------------------------------------
# Load-time kernel check (wdmpnn_self_check, ABI 11).  Round 5 lost a process to an experiment library
# whose gfx950 code object lacked slab_reduce_multi_kernel while its host code launched it (the HIP
# runtime aborts at such a launch).  These tests read the library's two kernel lists independently of
# the C++ check (pure-Python ELF / offload-bundle parsing), and check that a library with a kernel
# missing from its code object is refused with NativeError instead of crashing later.
# ---------------------------------------------------------------------------------------------------
import struct  # noqa: E402


def _sections(blob, base=0):
    shoff, = struct.unpack_from('<Q', blob, base + 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from('<HHH', blob, base + 0x3a)
    secs = [struct.unpack_from('<IIQQQQIIQQ', blob, base + shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]

    def name(n):
        return blob[base + stro + n:blob.index(b'\0', base + stro + n)].decode()
    return {name(s[0]): s for s in secs}, secs


def _symbols(blob, base=0):
    _, secs = _sections(blob, base)
    st = next(s for s in secs if s[1] == 2)  # SHT_SYMTAB
    strtab = secs[st[6]]
    out = []
    for o in range(0, st[5], 24):
        n, = struct.unpack_from('<I', blob, base + st[4] + o)
        if n:
            a = base + strtab[4] + n
            out.append(blob[a:blob.index(b'\0', a)].decode())
    return out


def _gfx950_object(blob):
    named, _ = _sections(blob)
    off = named['.hip_fatbin'][4]
    assert blob[off:off + 24] == b'__CLANG_OFFLOAD_BUNDLE__'
    n, = struct.unpack_from('<Q', blob, off + 24)
    p = off + 32
    for _ in range(n):
        o, size, tl = struct.unpack_from('<QQQ', blob, p)
        triple = blob[p + 24:p + 24 + tl].decode()
        p += 24 + tl
        if 'gfx950' in triple:
            return off + o, size
    raise AssertionError('no gfx950 code object')


def _kernel_lists(path):
    blob = open(path, 'rb').read()
    host = set()
    for s in _symbols(blob):
        m = re.match(r'^(_Z.*?)(\d+)__device_stub__(.*)$', s)
        if m:
            host.add(f'{m.group(1)}{int(m.group(2)) - 15}{m.group(3)}')
    base, _size = _gfx950_object(blob)
    dev = {s[:-3] for s in _symbols(blob, base) if s.endswith('.kd')}
    return host, dev


def test_code_object_holds_every_launched_kernel():
    """Every kernel the host code registers (its __device_stub__ symbols) has a kernel descriptor in the
    gfx950 code object, and the C++ check counts the same lists."""
    host, dev = _kernel_lists(_native.LIB_PATH)
    assert host and host <= dev, sorted(host - dev)[:5]
    assert any('slab_reduce_multi_kernel' in k for k in host)
    L = _native.lib()
    nh, nd = ctypes.c_int32(), ctypes.c_int32()
    assert L.wdmpnn_self_check(ctypes.byref(nh), ctypes.byref(nd)) == 0
    assert (nh.value, nd.value) == (len(host), len(dev))


def test_library_missing_a_kernel_is_refused(tmp_path):
    """A copy of the library with one kernel renamed inside its gfx950 code object only (the host still
    launches the old name: what a device pass built from an older source gives) must make
    _native.lib() raise NativeError naming the kernel; nothing is launched."""
    blob = bytearray(open(_native.LIB_PATH, 'rb').read())
    base, size = _gfx950_object(bytes(blob))
    old, new = b'slab_reduce_multi_kernel', b'slab_reduce_multi_kernex'
    region = bytes(blob[base:base + size])
    assert region.count(old) >= 2  # symbol names and the metadata note
    blob[base:base + size] = region.replace(old, new)
    broken = tmp_path / 'libwdmpnn.so'
    broken.write_bytes(bytes(blob))
    host, dev = _kernel_lists(str(broken))
    assert sorted(k for k in host - dev) and all('slab_reduce_multi_kernel' in k for k in host - dev)
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from chemprop_amd import _native\n'
            'try:\n    _native.lib()\nexcept _native.NativeError as e:\n    print("REFUSED", e)\n'
            'else:\n    print("LOADED")\n') % os.path.join(ROOT, 'polymer-chemprop_amd')
    env = dict(os.environ, WDMPNN_LIB=str(broken))
    out = subprocess.run(['python3', '-c', code], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.startswith('REFUSED'), out.stdout
    assert 'slab_reduce_multi_kernel' in out.stdout and 'absent from the gfx950 code object' in out.stdout
