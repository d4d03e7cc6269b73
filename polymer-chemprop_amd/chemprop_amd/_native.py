"""ctypes binding of libwdmpnn.so (include/wdmpnn.h).

The library is the product: there is no CPU or PyTorch fallback.  If ``libwdmpnn.so`` is missing
or fails to load, :func:`lib` raises, and every GPU entry point of the package raises with it.

``torch`` is imported before the library is loaded so that the library's ``libamdhip64.so.7``
dependency resolves (by SONAME) to the HIP runtime torch already loaded: one runtime, one set of
device pointers and streams.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t, c_uint64, c_void_p

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('WDMPNN_LIB', os.path.join(HERE, 'libwdmpnn.so'))

ACTIVATIONS = {'ReLU': 0, 'LeakyReLU': 1, 'PReLU': 2, 'tanh': 3, 'SELU': 4, 'ELU': 5}
ACT_IDENTITY = 6
AGGREGATIONS = {'mean': 0, 'sum': 1, 'norm': 2}
ABI_VERSION = 11
GRAPH_LEAN = 1  # WDMPNN_GRAPH_LEAN
GRAPH_NO_PLANES = 2  # WDMPNN_GRAPH_NO_PLANES
ERR_UNSUPPORTED = -1003  # WD_ERR_UNSUPPORTED

EXPORTED_SYMBOLS = ('wdmpnn_abi_version', 'wdmpnn_last_error', 'wdmpnn_workspace_bytes',
                    'wdmpnn_backward_workspace_bytes', 'wdmpnn_forward', 'wdmpnn_backward',
                    'wdmpnn_index_select_rows', 'wdmpnn_event_pool_create', 'wdmpnn_event_pool_destroy',
                    'wdmpnn_event_pool_elapsed_ms', 'wdmpnn_packed_params_bytes', 'wdmpnn_pack_params',
                    'wdmpnn_plane_bytes', 'wdmpnn_split_planes', 'wdmpnn_split_planes_rows',
                    'wdmpnn_build_bond_features', 'wdmpnn_index_select_rows_backward',
                    'wdmpnn_saved_layout', 'wdmpnn_graph_bytes', 'wdmpnn_build_graph', 'wdmpnn_adam_step', 'wdmpnn_head_mse', 'wdmpnn_scale', 'wdmpnn_build_graph_ex',
                    'wdmpnn_forward_many', 'wdmpnn_feed_slot_bytes', 'wdmpnn_feed_create', 'wdmpnn_feed_next',
                    'wdmpnn_feed_release', 'wdmpnn_feed_forward_workspace_bytes', 'wdmpnn_feed_forward',
                    'wdmpnn_feed_destroy', 'wdmpnn_adam_step_repack', 'wdmpnn_self_check')


class WdCsr(Structure):
    _fields_ = [('ptr', c_void_p), ('idx', c_void_p), ('coef', c_void_p)]


class WdGraph(Structure):
    _fields_ = [('n_atoms', c_int32), ('n_bonds', c_int32), ('n_mols', c_int32), ('atom_fdim', c_int32),
                ('bond_fdim', c_int32), ('ld_atoms', c_int32), ('ld_bonds', c_int32), ('bond_col0', c_int32),
                ('f_atoms', c_void_p), ('f_bonds', c_void_p), ('w_atoms', c_void_p), ('mol_start', c_void_p),
                ('mol_size', c_void_p), ('degree_of_polym', c_void_p),
                ('msg_gather', WdCsr), ('bond_feat_gather', WdCsr), ('atom_gather', WdCsr), ('b2revb', c_void_p),
                ('msg_gather_t', WdCsr), ('bond_feat_gather_t', WdCsr), ('atom_gather_t', WdCsr),
                ('atom_desc', c_void_p), ('desc_dim', c_int32), ('atom_messages', c_int32),
                ('f_atoms_x6', c_void_p), ('f_bonds_x6', c_void_p),
                ('n_blocks', c_int32), ('blocks', c_void_p), ('bond_blk_row', c_void_p), ('f_atoms_blk_x6', c_void_p),
                ('msg_ell_idx', c_void_p), ('msg_ell_coef', c_void_p), ('atom_ell_idx', c_void_p),
                ('atom_ell_coef', c_void_p), ('atom_codes', c_void_p), ('bond_src_blk', c_void_p),
                ('bond_tail', c_void_p), ('atom_feat_sum_x6', c_void_p),
                ('blk_max_bonds', c_int32), ('blk_max_atoms', c_int32)]


class WdParams(Structure):
    _fields_ = [('hidden', c_int32), ('W_i', c_void_p), ('b_i', c_void_p), ('W_h', c_void_p), ('b_h', c_void_p),
                ('W_o', c_void_p), ('b_o', c_void_p), ('W_d', c_void_p), ('b_d', c_void_p), ('prelu', c_void_p),
                ('zero_vec', c_void_p), ('packed', c_void_p), ('packed_bytes', c_size_t)]


class WdConfig(Structure):
    _fields_ = [('depth', c_int32), ('undirected', c_int32), ('activation', c_int32), ('aggregation', c_int32),
                ('aggregation_norm', c_float), ('dropout', c_float), ('seed', c_uint64),
                ('save_for_backward', c_int32), ('prof_slot', c_int32), ('prof_pool', c_void_p),
                ('gemm_variant', c_int32)]


class WdCompact(Structure):
    _fields_ = [('n_mols', c_int32), ('n_atoms', c_int32), ('n_bonds', c_int32), ('n_blocks', c_int32),
                ('atom_fdim', c_int32), ('bond_fdim', c_int32), ('nnz_msg', c_int32), ('nnz_agg', c_int32),
                ('mols', c_void_p), ('xn', c_void_p), ('atoms', c_void_p), ('pairs', c_void_p), ('blocks', c_void_p),
                ('block_nnz', c_void_p)]


class WdFeedSpec(Structure):
    _fields_ = [('kind', c_int32), ('batch', c_int32), ('n_batches', c_int64), ('seed', c_uint64),
                ('producers', c_int32), ('slots', c_int32), ('target_blocks', c_int32), ('flags', c_int32),
                ('atom_fdim', c_int32), ('bond_fdim', c_int32), ('pinned', c_void_p), ('device', c_void_p)]


class WdFeedBatch(Structure):
    _fields_ = [('index', c_int64), ('n_mols', c_int32), ('n_atoms', c_int32), ('n_bonds', c_int32),
                ('n_blocks', c_int32), ('nnz_msg', c_int32), ('reserved', c_int32), ('h2d_bytes', c_size_t)]


class WdSaved(Structure):
    _fields_ = [('depth', c_int32), ('rows', c_int32), ('atom_rows', c_int32), ('ld', c_int32),
                ('z', c_size_t * 32), ('zo', c_size_t)]


class WdGrads(Structure):
    _fields_ = [(n, c_void_p) for n in ('W_i', 'b_i', 'W_h', 'b_h', 'W_o', 'b_o', 'W_d', 'b_d', 'prelu')]


class WdAdamTensor(Structure):
    _fields_ = [('param', c_void_p), ('grad', c_void_p), ('exp_avg', c_void_p), ('exp_avg_sq', c_void_p),
                ('numel', c_int64)]


class WdAdamHyper(Structure):
    _fields_ = [('lr', c_float), ('beta1', c_float), ('beta2', c_float), ('eps', c_float), ('weight_decay', c_float),
                ('step', c_int32), ('decoupled', c_int32)]


class WdHead(Structure):
    _fields_ = [('x', c_void_p), ('ld_x', c_int32), ('B', c_int32), ('F', c_int32), ('Hf', c_int32), ('T', c_int32),
                ('W1', c_void_p), ('b1', c_void_p), ('W2', c_void_p), ('b2', c_void_p),
                ('table', c_void_p), ('ld_table', c_int32), ('inv_n', c_float), ('act', c_int32),
                ('a', c_void_p), ('dh', c_void_p), ('dout', c_void_p), ('lossrow', c_void_p), ('dx', c_void_p),
                ('dW1', c_void_p), ('db1', c_void_p), ('dW2', c_void_p), ('db2', c_void_p), ('loss', c_void_p),
                ('loss_kind', c_int32)]


class NativeError(RuntimeError):
    pass


_LIB = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the HIP library; raise if it is missing or has the wrong ABI."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise NativeError(f'libwdmpnn.so not found at {LIB_PATH}: build it with '
                          f'`python -c "import __graft_entry__ as g; g.build()"` (no CPU fallback exists)')
    L = ctypes.CDLL(LIB_PATH)
    L.wdmpnn_abi_version.restype = c_int
    L.wdmpnn_last_error.restype = c_char_p
    L.wdmpnn_workspace_bytes.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig), POINTER(c_size_t)]
    L.wdmpnn_backward_workspace_bytes.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig),
                                                  POINTER(c_size_t)]
    L.wdmpnn_forward.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig), c_void_p, c_size_t,
                                 c_void_p, c_void_p]
    L.wdmpnn_backward.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig), c_void_p, c_size_t,
                                  c_void_p, c_void_p, c_size_t, POINTER(WdGrads), c_void_p]
    L.wdmpnn_index_select_rows.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_void_p, c_void_p]
    L.wdmpnn_index_select_rows_backward.argtypes = [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int64, c_void_p,
                                                    c_void_p]
    L.wdmpnn_packed_params_bytes.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig),
                                             POINTER(c_size_t)]
    L.wdmpnn_pack_params.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig), c_void_p, c_size_t,
                                     c_void_p]
    L.wdmpnn_saved_layout.argtypes = [POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig), POINTER(WdSaved)]
    L.wdmpnn_graph_bytes.argtypes = [POINTER(WdCompact), POINTER(c_size_t)]
    L.wdmpnn_build_graph.argtypes = [POINTER(WdCompact), c_void_p, c_size_t, POINTER(WdGraph), c_void_p]
    L.wdmpnn_plane_bytes.argtypes = [c_int32, c_int32, POINTER(c_size_t)]
    L.wdmpnn_split_planes.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_size_t, c_void_p]
    L.wdmpnn_split_planes_rows.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_void_p, c_size_t,
                                           c_void_p]
    L.wdmpnn_build_bond_features.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                             c_int32, c_void_p, c_int32, c_void_p]
    L.wdmpnn_build_graph_ex.argtypes = [POINTER(WdCompact), c_void_p, c_size_t, POINTER(WdGraph), c_int32, c_void_p]
    L.wdmpnn_head_mse.argtypes = [POINTER(WdHead), c_void_p]
    L.wdmpnn_forward_many.argtypes = [c_int32, POINTER(WdGraph), POINTER(WdParams), POINTER(WdConfig),
                                      POINTER(c_void_p), POINTER(c_size_t), POINTER(c_void_p), c_void_p]
    L.wdmpnn_feed_slot_bytes.argtypes = [c_int32, c_int32, c_int32, c_int32, POINTER(c_size_t), POINTER(c_size_t)]
    L.wdmpnn_feed_create.argtypes = [POINTER(WdFeedSpec), POINTER(c_void_p)]
    L.wdmpnn_feed_next.argtypes = [c_void_p, c_void_p, POINTER(WdGraph), POINTER(WdFeedBatch)]
    L.wdmpnn_feed_release.argtypes = [c_void_p, c_void_p]
    L.wdmpnn_feed_forward_workspace_bytes.argtypes = [c_void_p, POINTER(WdParams), POINTER(WdConfig), c_int32,
                                                      POINTER(c_size_t)]
    L.wdmpnn_feed_forward.argtypes = [c_void_p, c_int32, POINTER(WdParams), POINTER(WdConfig), c_void_p, c_size_t,
                                      c_void_p, c_int64, c_void_p, POINTER(c_int32), POINTER(c_int64),
                                      POINTER(c_int64), POINTER(c_int64)]
    L.wdmpnn_feed_destroy.argtypes = [c_void_p]
    L.wdmpnn_scale.argtypes = [POINTER(c_void_p), POINTER(c_int64), c_int32, c_void_p, c_void_p]
    L.wdmpnn_adam_step.argtypes = [POINTER(WdAdamTensor), c_int32, POINTER(WdAdamHyper), c_void_p]
    L.wdmpnn_adam_step_repack.argtypes = [POINTER(WdAdamTensor), c_int32, POINTER(WdAdamHyper), POINTER(WdGraph),
                                          POINTER(WdParams), POINTER(WdConfig), c_void_p, c_size_t, c_void_p]
    L.wdmpnn_event_pool_create.argtypes = [c_int32, POINTER(c_void_p)]
    L.wdmpnn_event_pool_destroy.argtypes = [c_void_p]
    L.wdmpnn_event_pool_elapsed_ms.argtypes = [c_void_p, c_int32, c_int32, POINTER(c_float)]
    for fn in ('wdmpnn_packed_params_bytes', 'wdmpnn_pack_params', 'wdmpnn_event_pool_create', 'wdmpnn_event_pool_destroy', 'wdmpnn_event_pool_elapsed_ms',
               'wdmpnn_workspace_bytes', 'wdmpnn_backward_workspace_bytes', 'wdmpnn_forward', 'wdmpnn_backward',
               'wdmpnn_index_select_rows', 'wdmpnn_plane_bytes', 'wdmpnn_split_planes', 'wdmpnn_split_planes_rows',
               'wdmpnn_build_bond_features', 'wdmpnn_adam_step', 'wdmpnn_head_mse', 'wdmpnn_scale', 'wdmpnn_build_graph_ex') + \
            ('wdmpnn_forward_many', 'wdmpnn_feed_slot_bytes', 'wdmpnn_feed_create', 'wdmpnn_feed_next',
             'wdmpnn_feed_release', 'wdmpnn_feed_forward_workspace_bytes', 'wdmpnn_feed_forward',
             'wdmpnn_feed_destroy', 'wdmpnn_adam_step_repack'):
        getattr(L, fn).restype = c_int
    v = L.wdmpnn_abi_version()
    if v != ABI_VERSION:
        raise NativeError(f'libwdmpnn ABI {v} != expected {ABI_VERSION}; rebuild the library')
    # the load-time kernel check (wdmpnn.h, ABI 11): a library whose gfx950 code object lacks a kernel its
    # host code launches would abort the process at that launch; refuse it here instead
    L.wdmpnn_self_check.argtypes = [POINTER(c_int32), POINTER(c_int32)]
    L.wdmpnn_self_check.restype = c_int
    n_host, n_dev = c_int32(0), c_int32(0)
    if L.wdmpnn_self_check(ctypes.byref(n_host), ctypes.byref(n_dev)) != 0:
        raise NativeError(f'{LIB_PATH}: ' + L.wdmpnn_last_error().decode(errors='replace'))
    _LIB = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().wdmpnn_last_error().decode(errors='replace')
        if rc in (-1000, -1001):
            raise ValueError(f'{what}: {msg}')
        if rc == -1003:
            raise NotImplementedError(f'{what}: {msg}')
        raise NativeError(f'{what} failed ({rc}): {msg}')


def ptr(t) -> int:
    """Device pointer of a tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


_HIP = None
HIP_HOST_MALLOC_MAPPED = 0x2
HIP_HOST_MALLOC_COHERENT = 0x40000000


def _hip():
    global _HIP
    if _HIP is None:
        h = ctypes.CDLL('libamdhip64.so.7')
        h.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
        h.hipHostGetDevicePointer.restype = ctypes.c_int
        h.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        h.hipHostMalloc.restype = ctypes.c_int
        h.hipHostFree.argtypes = [ctypes.c_void_p]
        h.hipHostFree.restype = ctypes.c_int
        _HIP = h
    return _HIP


class CoherentHostBuffer:
    """Pinned host memory that GPU kernels read directly (hipHostMalloc mapped + coherent: the device
    reads it uncached over PCIe, so a host rewrite between two launches is always seen, without the
    L2-invalidation assumption a non-coherent pinned buffer would need).  ``array`` is a float32 numpy
    view, ``device_ptr`` its device address."""

    def __init__(self, shape):
        import numpy as np
        n = int(np.prod(shape)) * 4
        h = _hip()
        p = ctypes.c_void_p()
        if h.hipHostMalloc(ctypes.byref(p), max(n, 4), HIP_HOST_MALLOC_MAPPED | HIP_HOST_MALLOC_COHERENT) != 0:
            raise NativeError('hipHostMalloc (mapped, coherent) failed')
        self._p = p.value
        self.array = np.ctypeslib.as_array((ctypes.c_float * max(n // 4, 1)).from_address(self._p))[:n // 4]
        self.array = self.array.reshape(shape)
        self.device_ptr = host_device_ptr(self._p)

    def __del__(self):
        if getattr(self, '_p', None) and _HIP is not None:
            _HIP.hipHostFree(ctypes.c_void_p(self._p))
            self._p = None


def host_device_ptr(p: int) -> int:
    """Device address of pinned host memory at ``p`` (hipHostGetDevicePointer on the HIP runtime torch
    loaded), 0 if that memory is not mapped for the device: a kernel may then read it over PCIe directly."""
    _hip()
    d = ctypes.c_void_p()
    if _HIP.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(p), 0) != 0:
        return 0
    return d.value or 0


_RAW_STREAM = getattr(torch._C, '_cuda_getCurrentRawStream', None)


def current_stream(device) -> int:
    """The raw hipStream_t of ``device``'s current stream (torch's raw accessor: no Stream object is built,
    a few us less host time per call on the training step's path)."""
    if _RAW_STREAM is not None and isinstance(device, torch.device) and device.index is not None:
        return _RAW_STREAM(device.index)
    return torch.cuda.current_stream(device).cuda_stream
