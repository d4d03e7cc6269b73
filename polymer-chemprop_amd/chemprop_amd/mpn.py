"""MPNEncoder / MPN with the reference's constructor, state_dict keys and forward signatures
(``chemprop/models/mpn.py:14-289``), computed by the HIP library (libwdmpnn.so).

The encoder's whole forward (mpn.py:66-173) is one ``wdmpnn_forward`` call; its gradient is one
``wdmpnn_backward`` call (autograd.Function below).  Parameters stay ordinary ``nn.Linear`` /
``nn.Parameter`` objects so optimisers, checkpoints (``encoder.encoder.0.W_i.weight`` ...) and
``load_checkpoint``'s key remapping (utils.py:114-115) work unchanged.
"""
from __future__ import annotations

import ctypes
import weakref
from functools import reduce
from typing import List, Union

import numpy as np
import torch
import torch.nn as nn
from torch.optim.optimizer import register_optimizer_step_post_hook

from . import _native
from .featurization import BatchMolGraph, get_atom_fdim, get_bond_fdim, mol2graph
from .nn_utils import get_activation_function

# optimizer steps taken in this process (any torch.optim optimizer): part of the packed-weight cache
# key, since fused / capturable optimizers write the parameters without bumping their version counters
_OPT_STEPS = [0]


def _count_optimizer_step(optimizer, args, kwargs):
    _OPT_STEPS[0] += 1


register_optimizer_step_post_hook(_count_optimizer_step)


def _dropout_seed() -> int:
    """64-bit counter-hash seed for one training forward's dropout masks, drawn from torch's default
    CPU generator (so ``torch.manual_seed`` reproduces the masks) and mixed with the data-parallel
    rank (ranks with the same seed still draw different masks).  No device sync."""
    s = int(torch.randint(0, 2 ** 62, (1,)).item())
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        s ^= (torch.distributed.get_rank() + 1) * 0x9E3779B97F4A7C15
    return s & 0xFFFFFFFFFFFFFFFF


def _f32(t):
    if t is None:
        return None
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise TypeError('chemprop_amd expects contiguous float32 parameters')
    return t


def _forward_call(gstruct, cfg, pstruct, hidden_out, device, pre_launch=None):
    """One wdmpnn_forward on the current stream into caller-owned (caching-allocator) buffers.
    ``pre_launch`` (the weight pack of a training forward) is enqueued after the host-side preparation,
    right before the forward, so that the GPU does not idle between the two."""
    L = _native.lib()
    nbytes = ctypes.c_size_t()
    _native.check(L.wdmpnn_workspace_bytes(ctypes.byref(gstruct), ctypes.byref(pstruct), ctypes.byref(cfg),
                                           ctypes.byref(nbytes)), 'MPNEncoder workspace')
    ws = torch.empty(max(nbytes.value, 256), dtype=torch.uint8, device=device)
    out = torch.empty((gstruct.n_mols, hidden_out), dtype=torch.float32, device=device)
    if pre_launch is not None:
        pre_launch()
    _native.check(L.wdmpnn_forward(ctypes.byref(gstruct), ctypes.byref(pstruct), ctypes.byref(cfg), ws.data_ptr(),
                                   nbytes.value, out.data_ptr(), _native.current_stream(device)),
                  'MPNEncoder forward')
    return out, ws, nbytes.value


class _EncoderFunction(torch.autograd.Function):
    """Forward = wdmpnn_forward, backward = wdmpnn_backward (parameter gradients only: the graph
    features are inputs without gradient, as in the reference training loop)."""

    @staticmethod
    def forward(ctx, enc, gstruct, cfg, pstruct, keep, hidden_out, device, W_i, b_i, W_h, b_h, W_o, b_o, W_d, b_d,
                prelu):
        out, ws, ws_bytes = _forward_call(gstruct, cfg, pstruct, hidden_out, device, pre_launch=keep[3])
        if cfg.save_for_backward:
            ctx.save_for_backward(W_i, b_i, W_h, b_h, W_o, b_o, W_d, b_d, prelu)
            ctx.ws, ctx.ws_bytes, ctx.gstruct, ctx.cfg, ctx.p, ctx.keep = ws, ws_bytes, gstruct, cfg, pstruct, keep
        return out

    @staticmethod
    def backward(ctx, dout):
        W_i, b_i, W_h, b_h, W_o, b_o, W_d, b_d, prelu = ctx.saved_tensors
        want = ctx.needs_input_grad
        first = 7  # position of W_i in forward's arguments
        out = {}
        for k, (name, t) in enumerate((('W_i', W_i), ('b_i', b_i), ('W_h', W_h), ('b_h', b_h), ('W_o', W_o),
                                       ('b_o', b_o), ('W_d', W_d), ('b_d', b_d), ('prelu', prelu))):
            if name in ('W_h', 'b_h') and ctx.cfg.depth == 1:
                continue  # unused when depth == 1 (mpn.py:100 loop body never runs): no gradient, like autograd
            if t is not None and want[first + k]:
                out[name] = torch.empty_like(t)
        _backward_call(ctx.gstruct, ctx.p, ctx.cfg, ctx.ws, ctx.ws_bytes, dout, out)
        # ctx.ws stays alive until autograd frees ctx: a second backward through the same graph
        # (retain_graph=True) reads the same saved forward state
        return (None,) * 7 + tuple(out.get(n) for n in ('W_i', 'b_i', 'W_h', 'b_h', 'W_o', 'b_o', 'W_d', 'b_d',
                                                         'prelu'))


def _backward_call(gstruct, pstruct, cfg, ws, ws_bytes, dout, grads):
    """One wdmpnn_backward into the tensors of ``grads`` (name -> tensor, names of WdGrads; absent names
    are not computed)."""
    L = _native.lib()
    dev = dout.device
    dout = dout.contiguous()
    nbytes = ctypes.c_size_t()
    _native.check(L.wdmpnn_backward_workspace_bytes(ctypes.byref(gstruct), ctypes.byref(pstruct), ctypes.byref(cfg),
                                                    ctypes.byref(nbytes)), 'MPNEncoder backward workspace')
    scratch = torch.empty(max(nbytes.value, 256), dtype=torch.uint8, device=dev)
    g = _native.WdGrads()
    for name, t in grads.items():
        setattr(g, name, t.data_ptr())
    _native.check(L.wdmpnn_backward(ctypes.byref(gstruct), ctypes.byref(pstruct), ctypes.byref(cfg), ws.data_ptr(),
                                    ws_bytes, dout.data_ptr(), scratch.data_ptr(), nbytes.value, ctypes.byref(g),
                                    _native.current_stream(dev)), 'MPNEncoder backward')


def saved_preactivations(out: torch.Tensor):
    """The fp32 pre-activations a training forward saved for its backward (introspection for tests and
    debugging; ``wdmpnn_saved_layout``): ``{'Z': [Z_0 .. Z_{depth-1}] ([rows, H] each, natural row order
    with the pad row 0: Z_0 = W_i output mpn.py:96, Z_t = input + W_h(message) mpn.py:123), 'Zo': the
    W_o pre-activation [n_atoms, H] (mpn.py:133)}``.  ``out`` must come from ``MPNEncoder.forward``
    with gradients enabled."""
    ctx = out.grad_fn
    if ctx is None or not hasattr(ctx, 'ws'):
        raise ValueError('not the output of a training-mode MPNEncoder forward')
    lay = _native.WdSaved()
    _native.check(_native.lib().wdmpnn_saved_layout(ctypes.byref(ctx.gstruct), ctypes.byref(ctx.p),
                                                    ctypes.byref(ctx.cfg), ctypes.byref(lay)), 'saved layout')
    H = ctx.p.hidden
    ws = ctx.ws

    def view(off, rows):
        return ws[off:off + rows * lay.ld * 4].view(torch.float32).view(rows, lay.ld)[:, :H]

    return {'Z': [view(lay.z[t], lay.rows) for t in range(lay.depth)], 'Zo': view(lay.zo, lay.atom_rows)}


class MPNEncoder(nn.Module):
    """mpn.py:14-173.  Same constructor arguments, attributes, parameters and forward signature."""

    def __init__(self, args, atom_fdim: int, bond_fdim: int):
        super(MPNEncoder, self).__init__()
        self.atom_fdim = atom_fdim
        self.bond_fdim = bond_fdim
        self.atom_messages = args.atom_messages
        self.hidden_size = args.hidden_size
        self.bias = args.bias
        self.depth = args.depth
        self.dropout = args.dropout
        self.layers_per_message = 1
        self.undirected = args.undirected
        self.device = args.device
        self.aggregation = args.aggregation
        self.aggregation_norm = args.aggregation_norm
        self.activation = args.activation

        self.dropout_layer = nn.Dropout(p=self.dropout)
        self.act_func = get_activation_function(args.activation)
        self.cached_zero_vector = nn.Parameter(torch.zeros(self.hidden_size), requires_grad=False)
        input_dim = self.atom_fdim if self.atom_messages else self.bond_fdim
        self.W_i = nn.Linear(input_dim, self.hidden_size, bias=self.bias)
        w_h_input_size = self.hidden_size + self.bond_fdim if self.atom_messages else self.hidden_size
        self.W_h = nn.Linear(w_h_input_size, self.hidden_size, bias=self.bias)
        self.W_o = nn.Linear(self.atom_fdim + self.hidden_size, self.hidden_size)
        if getattr(args, 'atom_descriptors', None) == 'descriptor':
            self.atom_descriptors_size = args.atom_descriptors_size
            self.atom_descriptors_layer = nn.Linear(self.hidden_size + self.atom_descriptors_size,
                                                    self.hidden_size + self.atom_descriptors_size)
        if self.aggregation not in _native.AGGREGATIONS:
            raise ValueError(f'Aggregation "{self.aggregation}" not supported.')
        if self.atom_messages and self.undirected:
            raise NotImplementedError('undirected=True with atom_messages=True indexes atom messages with bond '
                                      'indices in the reference (mpn.py:101-102) and is not supported')
        self._prof = None  # (event pool, first pair): bench.py measurement hook, see WdConfig.prof_pool
        self._pack_cache = None  # (parameter-version key, packed weight buffer)
        self._gemm_variant = 0  # WdConfig.gemm_variant (0 = split-plane default; 9 = f32-MFMA A/B)
        self._plan_token = object()  # this encoder's key in DeviceGraph.encoder_plans
        self._infer_configs = {}  # plan key -> WdConfig of the inference call (_infer)

    def __getstate__(self):
        """Copies (copy.deepcopy, pickle) drop the device-side caches: packed weights, workspaces, plans."""
        state = self.__dict__.copy()
        for k in ('_ws_by_stream', '_many_plan'):
            state.pop(k, None)
        state.update(_pack_cache=None, _train_pack=None, _infer_configs={}, _plan_token=object())
        return state

    def _config(self, save: bool) -> _native.WdConfig:
        c = _native.WdConfig()
        c.depth = self.depth
        c.undirected = int(bool(self.undirected))
        c.activation = _native.ACTIVATIONS[self.activation]
        c.aggregation = _native.AGGREGATIONS[self.aggregation]
        c.aggregation_norm = float(self.aggregation_norm)
        p = float(self.dropout) if self.training else 0.0
        c.dropout = p
        if p > 0.0:
            c.seed = _dropout_seed()
        c.save_for_backward = int(bool(save))
        if self._prof is not None:
            c.prof_pool, c.prof_slot = self._prof
        c.gemm_variant = self._gemm_variant
        return c

    def _param_tuple(self):
        """(W_i, b_i, W_h, b_h, W_o, b_o, W_d, b_d, prelu) read straight from the submodules' parameter
        dicts: the same tensors as ``self.W_i.weight`` ..., without nn.Module.__getattr__ (≈ 8 µs of host
        time per forward for the nine lookups)."""
        m = self._modules
        wi, wh, wo = m['W_i']._parameters, m['W_h']._parameters, m['W_o']._parameters
        act = m['act_func']
        return (wi['weight'], wi.get('bias'), wh['weight'], wh.get('bias'), wo['weight'], wo.get('bias'), None,
                None, act._parameters['weight'] if isinstance(act, nn.PReLU) else None)

    def _infer(self, mol_graph: BatchMolGraph):
        """Inference call path (no autograd, no dropout, no descriptors, no profiling hook).  Everything a
        call derives from the (graph, encoder configuration) pair -- the graph struct, the config, the
        workspace size -- is a plan cached on the DeviceGraph, the config itself once per encoder, and the
        workspace is this encoder's per-stream buffer: a repeated forward costs one output allocation and
        one C-ABI call, and a graph's first forward, or its first on another stream, little more (bench.py
        times 20 forwards that are mostly such first uses, predict.py:30-40 only first uses).  Returns None
        when the call needs the general path."""
        d = self.__dict__
        if d.get('_prof') is not None or '_plan_token' not in d or (self.training and self.dropout > 0):
            return None
        params = self._param_tuple()
        device = params[0].device
        if device.type != 'cuda':
            return None  # the general path raises
        if params[8] is not None and params[8].numel() != 1:
            return None
        # (the graph's DeviceGraph for this encoder's mode, memoised in the graph's device cache under a short
        # key: device_graph's own lookup builds a device string and its key per call, ~0.5 us of host time)
        cache = mol_graph._device_cache
        dkey = ('infer', device.index, d['atom_messages'], d['bond_fdim'], d['bias'])
        dg = cache.get(dkey)
        if dg is None:
            dg = cache[dkey] = mol_graph.device_graph(device, d['atom_messages'], d['bond_fdim'], not d['bias'])
        sid = _native.current_stream(device)
        if sid not in dg._streams:
            dg.use_on(torch.cuda.current_stream(device))
        ckey = (self._plan_token, d['atom_fdim'], d['bond_fdim'], d['hidden_size'], d['depth'], d['undirected'],
                d['activation'], d['aggregation'], d['aggregation_norm'], d['_gemm_variant'])
        plan = dg.encoder_plans.get(ckey)
        if plan is None:
            plan = self._new_infer_plan(dg, ckey, params, device, sid)
        pstruct, _ = self._packed_params(plan[4], plan[5], params, device, sid=sid)
        ws = self._stream_workspace(sid, plan[2], device)
        out = torch.empty((plan[3], d['hidden_size']), dtype=torch.float32, device=device)
        _native.check(_native.lib().wdmpnn_forward(plan[0], ctypes.byref(pstruct), plan[1], ws.data_ptr(), plan[2],
                                                   out.data_ptr(), sid), 'MPNEncoder forward')
        return out

    def prepare(self, graphs, streams=()) -> None:
        """Host-side setup for inference on resident graphs (no counterpart in the reference): each graph's
        DeviceGraph built and registered on ``streams`` (and the current stream), and its call plan -- graph and
        config structs, workspace size -- cached, so that its first forward costs the host what a repeat does.
        Runs no kernel besides the weight pack a first forward would enqueue.  Optional; forward never needs it."""
        d = self.__dict__
        params = self._param_tuple()
        device = params[0].device
        if device.type != 'cuda' or '_plan_token' not in d:
            return
        cur = torch.cuda.current_stream(device)
        sid = cur.cuda_stream
        ckey = (self._plan_token, d['atom_fdim'], d['bond_fdim'], d['hidden_size'], d['depth'], d['undirected'],
                d['activation'], d['aggregation'], d['aggregation_norm'], d['_gemm_variant'])
        with torch.no_grad():
            for g in graphs:
                dg = g.device_graph(device, d['atom_messages'], d['bond_fdim'], not d['bias'])
                for s_ in list(streams) + [cur]:
                    dg.use_on(s_)
                if dg.encoder_plans.get(ckey) is None:
                    self._new_infer_plan(dg, ckey, params, device, sid)

    def _new_infer_plan(self, dg, ckey, params, device, sid):
        """(graph struct ref, config ref, workspace bytes, molecules, graph struct, config) of an inference
        call on ``dg``, stored on it under ``ckey`` (shared by ``_infer`` and ``forward_many``)."""
        gs = self._graph_struct(dg)
        cfg = self._infer_configs.get(ckey)
        if cfg is None:
            cfg = self._infer_configs[ckey] = self._config(False)
        pstruct, _ = self._packed_params(gs, cfg, params, device, sid=sid)
        nbytes = ctypes.c_size_t()
        _native.check(_native.lib().wdmpnn_workspace_bytes(ctypes.byref(gs), ctypes.byref(pstruct),
                                                           ctypes.byref(cfg), ctypes.byref(nbytes)),
                      'MPNEncoder workspace')
        plan = (ctypes.byref(gs), ctypes.byref(cfg), max(nbytes.value, 256), gs.n_mols, gs, cfg)
        dg.encoder_plans[ckey] = plan
        return plan

    def _stream_workspace(self, sid: int, nbytes: int, device) -> torch.Tensor:
        """This encoder's inference workspace for the stream ``sid`` (current at the call), grown to the
        largest request.  Calls on one stream run in order, so they share one buffer safely; each stream has
        its own (allocated while it is current: the caching allocator ties the block to it)."""
        wss = self.__dict__.setdefault('_ws_by_stream', {})
        ws = wss.get(sid)
        if ws is None or ws.numel() < nbytes:
            wss[sid] = ws = None  # (the old buffer is released before the larger one is allocated)
            wss[sid] = ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return ws

    # ---------------------------------------------------------------- direct training step (train.py)
    def _direct_names(self):
        """(name, parameter) pairs the native backward fills, in WdGrads order (no descriptors)."""
        base = self._param_tuple()
        names = ('W_i', 'b_i', 'W_h', 'b_h', 'W_o', 'b_o', 'W_d', 'b_d', 'prelu')
        return [(n, t) for n, t in zip(names, base) if t is not None]

    def _train_forward(self, mol_graph):
        """The training forward of ``forward`` (save_for_backward) without autograd: (out, state) for
        :meth:`_train_backward`.  Used by ``train.train_step``'s direct path, whose fused head computes the
        encoder's output gradient itself."""
        base = self._param_tuple()
        device = base[0].device
        dg = mol_graph.device_graph(device, self.atom_messages, self.bond_fdim)
        dg.use_on(torch.cuda.current_stream(device))
        gs = self._graph_struct(dg)
        params = [_f32(t) for t in base[:6]] + [None, None, _f32(base[8])]
        cfg = self._config(True)
        pstruct, packed, pack = self._train_pack_for(gs, cfg, params, device)
        out, ws, ws_bytes = _forward_call(gs, cfg, pstruct, self.hidden_size, device, pre_launch=pack)
        return out, (gs, cfg, pstruct, ws, ws_bytes, packed, dg)

    def _train_pack_for(self, gs, cfg, params, device):
        """The direct training step's packed weights: one persistent buffer, rewritten by the optimizer's
        own pass when it is a :class:`train.HipAdam` step through ``wdmpnn_adam_step_repack`` (which then
        re-keys it to the parameters' post-step state); packed afresh (the returned launch, enqueued before
        the forward) whenever the key differs -- the first step, a parameter written any other way (version
        counters, another optimizer's step), other feature sizes or another stream."""
        sid = _native.current_stream(device)
        key = (tuple((t.data_ptr(), t._version, id(t)) if t is not None else None for t in params), _OPT_STEPS[0],
               self._parameters['cached_zero_vector'].data_ptr(), gs.atom_fdim, gs.bond_fdim, gs.desc_dim,
               gs.atom_messages, device, sid)
        tp = self.__dict__.get('_train_pack')
        # (the weak references: a Parameter that replaced a freed one at the same address, object id and
        # version still forces a repack)
        if tp is not None and tp['key'] == key and all(r is None if t is None else r() is t
                                                        for r, t in zip(tp['refs'], params)):
            tp['gs'], tp['cfg'] = gs, cfg
            return tp['p'], tp['buf'], None
        pstruct, buf, launch = self._packed_params(gs, cfg, params, device, cache=False, defer=True)
        buf.zero_()  # (the layout's alignment gaps too: a repacked buffer is bytewise a fresh pack)
        self._train_pack = {'key': key, 'p': pstruct, 'buf': buf, 'gs': gs, 'cfg': cfg,
                            'refs': tuple(None if t is None else weakref.ref(t) for t in params),
                            'ptrs': frozenset(t.data_ptr() for t in params[:6] if t is not None)}
        return pstruct, buf, launch

    def _repacked_by_optimizer(self, tp) -> None:
        """Called by HipAdam after ``wdmpnn_adam_step_repack`` rewrote ``tp['buf']`` from the updated
        weights: valid at the optimizer-step count the step's post hook is about to set."""
        k = tp['key']
        tp['key'] = k[:1] + (_OPT_STEPS[0] + 1,) + k[2:]

    def _train_backward(self, state, dout, grads) -> None:
        """wdmpnn_backward of a :meth:`_train_forward` into ``grads`` (name -> tensor, WdGrads names)."""
        gs, cfg, pstruct, ws, ws_bytes, packed, dg = state
        _backward_call(gs, pstruct, cfg, ws, ws_bytes, dout, grads)

    def forward_many(self, mol_graphs: List[BatchMolGraph]) -> List[torch.Tensor]:
        """Inference forward of several independent batches in one set of launches
        (``wdmpnn_forward_many``: embed, the depth - 1 layers and W_o + readout each launched once per
        8 batches, their tiles in one grid).  ``[self(g) for g in mol_graphs]`` with the same outputs
        (bitwise) and a fraction of the launches and host time: for callers that hold several batches
        at once (prediction over a dataset, chemprop/train/predict.py:30-40 loops one forward per batch).
        Gradient-enabled calls, atom messages, descriptors and graphs outside the fused layout take the
        one-batch path per graph."""
        graphs = list(mol_graphs)
        if not graphs:
            return []
        d = self.__dict__
        params = self._param_tuple()
        device = params[0].device
        fused = (not torch.is_grad_enabled() or not any(t is not None and t.requires_grad for t in params)) and \
            device.type == 'cuda' and d.get('_prof') is None and not (self.training and self.dropout > 0) and \
            not d['atom_messages'] and (params[8] is None or params[8].numel() == 1)
        if not fused:
            return [self(g) for g in graphs]
        stream = torch.cuda.current_stream(device)
        ckey = (self._plan_token, d['atom_fdim'], d['bond_fdim'], d['hidden_size'], d['depth'], d['undirected'],
                d['activation'], d['aggregation'], d['aggregation_norm'], d['_gemm_variant'])
        dgs = [g.device_graph(device, False, d['bond_fdim']) for g in graphs]
        for dg in dgs:
            dg.use_on(stream)
        # one cached plan, for a repeated call on the same graphs (it holds their DeviceGraphs: a cache of
        # many would keep the device memory of graphs the caller has dropped)
        key = (ckey, tuple(id(dg) for dg in dgs))
        last = d.get('_many_plan')
        plan = last[1] if last is not None and last[0] == key else None
        if plan is None or any(a is not b for a, b in zip(plan[0], dgs)):
            # a new set of graphs: each graph's struct and workspace size come from its inference plan
            # (built once per graph and encoder configuration, shared with _infer), so a set costs a copy
            # of its structs, not a workspace query per graph
            sid = stream.cuda_stream
            fparams = tuple(_f32(t) for t in params)
            structs = (_native.WdGraph * len(dgs))()
            sz = ctypes.sizeof(_native.WdGraph)
            sizes, offs, rows, total = [], [], [], 0
            for k, dg in enumerate(dgs):
                gp = dg.encoder_plans.get(ckey)
                if gp is None:
                    gp = self._new_infer_plan(dg, ckey, fparams, device, sid)
                ctypes.memmove(ctypes.byref(structs, k * sz), gp[0], sz)
                offs.append(total)
                sizes.append(gp[2])
                total += (gp[2] + 255) & ~255
                rows.append(gp[3])
            cfg = gp[5]
            plan = (dgs, structs, cfg, (ctypes.c_size_t * len(dgs))(*sizes), offs, max(total, 256), rows,
                    np.cumsum([0] + rows).tolist())
            d['_many_plan'] = (key, plan)
        dgs_, structs, cfg, sizes, offs, total, rows, row0 = plan
        pstruct, _ = self._packed_params(structs[0], cfg, params, device, stream=stream)
        ws = self._stream_workspace(stream.cuda_stream, total, device)  # (the encoder's buffer for this stream)
        out = torch.empty((row0[-1], d['hidden_size']), dtype=torch.float32, device=device)
        base, obase, H = ws.data_ptr(), out.data_ptr(), d['hidden_size']
        n = len(dgs_)
        wptr = (ctypes.c_void_p * n)(*[base + o for o in offs])
        optr = (ctypes.c_void_p * n)(*[obase + 4 * H * r for r in row0[:-1]])
        rc = _native.lib().wdmpnn_forward_many(n, structs, ctypes.byref(pstruct), ctypes.byref(cfg), wptr, sizes, optr,
                                               stream.cuda_stream)
        if rc == _native.ERR_UNSUPPORTED:
            return [self(g) for g in graphs]
        _native.check(rc, 'MPNEncoder forward_many')
        return [out[row0[k]:row0[k + 1]] for k in range(n)]

    def _graph_struct(self, dg):
        """The WdGraph copy this encoder passes (feature sizes checked against the encoder's), cached on
        the DeviceGraph per (atom_fdim, bond_fdim)."""
        gs = dg.encoder_structs.get((self.atom_fdim, self.bond_fdim))
        if gs is None:
            gs = self._new_graph_struct(dg)
            dg.encoder_structs[(self.atom_fdim, self.bond_fdim)] = gs
        return gs

    def _new_graph_struct(self, dg):
        gs = _native.WdGraph.from_buffer_copy(dg.struct)
        if gs.n_atoms > 1 and gs.atom_fdim != self.atom_fdim:
            raise ValueError(f'atom feature size {gs.atom_fdim} != encoder atom_fdim {self.atom_fdim}')
        if gs.n_bonds > 1 and gs.bond_fdim != self.bond_fdim:
            raise ValueError(f'bond feature size {gs.bond_fdim} != encoder bond_fdim {self.bond_fdim}')
        gs.atom_fdim, gs.bond_fdim = self.atom_fdim, self.bond_fdim
        return gs

    def forward(self, mol_graph: BatchMolGraph, atom_descriptors_batch: List[np.ndarray] = None) -> torch.FloatTensor:
        """mpn.py:66-173 -> [num_molecules, hidden_size (+ atom_descriptors_size)]."""
        if atom_descriptors_batch is None and not torch.is_grad_enabled():
            out = self._infer(mol_graph)
            if out is not None:
                return out
        base = self._param_tuple()
        device = base[0].device
        if device.type != 'cuda':
            raise RuntimeError('chemprop_amd.MPNEncoder runs on the MI355X HIP path only: move the model to a '
                               'GPU (model.to("cuda"))')
        # (atom messages: the fused atom-row path's arrays only for a bias-free inference forward)
        grad = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in base)
        dg = mol_graph.device_graph(device, self.atom_messages, self.bond_fdim, not self.bias and not grad)
        dg.use_on(torch.cuda.current_stream(device))
        # descriptors are per call: their struct is never cached
        gs = self._graph_struct(dg) if atom_descriptors_batch is None else self._new_graph_struct(dg)
        desc = None
        hidden_out = self.hidden_size
        if atom_descriptors_batch is not None:  # mpn.py:77-79, 136-143
            if not hasattr(self, 'atom_descriptors_layer'):
                raise ValueError('atom descriptors given but the encoder has no atom_descriptors_layer')
            d = atom_descriptors_batch[0].shape[1]
            rows = np.concatenate([np.zeros([1, d])] + list(atom_descriptors_batch), axis=0)
            if rows.shape[0] != gs.n_atoms:
                raise ValueError('The number of atoms is different from the length of the extra atom features')
            if any(n == 0 for _, n in mol_graph.a_scope):
                raise RuntimeError('stack expects each tensor to be equal size (empty molecule with atom '
                                   'descriptors, mpn.py:149 vs 171)')
            padded = np.zeros((-(-rows.shape[0] // 128) * 128, -(-d // 32) * 32), np.float32)
            padded[:rows.shape[0], :d] = rows
            desc = torch.from_numpy(padded).to(device)
            gs.atom_desc, gs.desc_dim = desc.data_ptr(), d
            hidden_out += d
        act_w = base[8]
        if act_w is not None and act_w.numel() != 1:
            raise NotImplementedError('PReLU with num_parameters > 1')
        params = list(base[:6])
        if desc is not None:
            params += [self.atom_descriptors_layer.weight, self.atom_descriptors_layer.bias]
        else:
            params += [None, None]
        params += [act_w]
        params = [_f32(t) for t in params]
        save = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in params)
        cfg = self._config(save)
        if not save:  # inference: the same C-ABI call without the autograd.Function wrapper
            pstruct, packed = self._packed_params(gs, cfg, params, device, cache=True)
            return _forward_call(gs, cfg, pstruct, hidden_out, device)[0]
        # training: the weights are repacked every call; the pack is enqueued right before the forward
        pstruct, packed, pack = self._packed_params(gs, cfg, params, device, cache=False, defer=True)
        # the autograd context keeps the device graph alive with the packed weights and descriptors: the
        # backward reads its buffers through raw pointers (gs), and the caller may drop the BatchMolGraph
        # before calling backward (``model([BatchMolGraph(mols)]).sum().backward()``)
        return _EncoderFunction.apply(self, gs, cfg, pstruct, (packed, desc, dg, pack), hidden_out, device, *params)

    def invalidate_packed_params(self) -> None:
        """Drop the cached padded weights (the inference cache and the direct training step's persistent
        pack).  Needed only after writing the parameters in a way that bypasses both their version counters
        and ``torch.optim`` / :class:`train.HipAdam` -- ``p.data.copy_(...)``, ``p.data[...] = ...``: writes
        through ``.data`` do not bump ``p._version``.  Reassigned parameters and ``load_state_dict`` are
        handled without it (object identity in the key; the caches are dropped on load)."""
        self._pack_cache = None
        self._train_pack = None

    def _load_from_state_dict(self, *args, **kwargs):
        """nn.Module hook of ``load_state_dict``: the loaded values invalidate every packed copy."""
        self.invalidate_packed_params()
        return super()._load_from_state_dict(*args, **kwargs)

    def _packed_params(self, gs, cfg, params, device, cache=True, stream=None, defer=False, sid=None):
        """WdParams + the padded weight copies (wdmpnn_pack_params).  Inference caches them per
        (parameter pointer, version counter, optimizer-step generation): fused optimizers update the
        weights without bumping version counters, so every ``Optimizer.step`` also bumps
        ``_OPT_STEPS``.  A training forward through autograd repacks and leaves no cache behind (the direct
        step keeps its own persistent pack, :meth:`_train_pack_for`).  ``sid``: the raw
        id of the current stream (the inference path's cheaper alternative to ``stream``)."""
        key = (tuple((t.data_ptr(), t._version, id(t)) if t is not None else None for t in params), _OPT_STEPS[0],
               self._parameters['cached_zero_vector'].data_ptr(), gs.atom_fdim, gs.bond_fdim, gs.desc_dim,
               gs.atom_messages, device, cfg.gemm_variant not in (9, 12)) if cache else None  # (+ W_o's pair tiles)
        cached = self._pack_cache if cache else None
        if cached is not None and cached[0] == key:
            if sid is None:
                if stream is None:
                    stream = torch.cuda.current_stream(device)
                sid = stream.cuda_stream
            if sid not in cached[4]:  # packed on another stream: order after the pack and keep the buffer
                if stream is None:    # alive for this stream's kernels
                    stream = torch.cuda.current_stream(device)
                if not cached[3].query():
                    stream.wait_event(cached[3])
                cached[1].record_stream(stream)
                cached[4].add(sid)
            return cached[2], cached[1]
        if sid is not None and stream is None:
            stream = torch.cuda.current_stream(device)
        params = [_f32(t) for t in params]  # also after model.half() / .double(): never pack other dtypes
        p = _native.WdParams()
        p.hidden = self.hidden_size
        p.W_i, p.b_i, p.W_h, p.b_h, p.W_o, p.b_o, p.W_d, p.b_d, p.prelu = map(_native.ptr, params)
        p.zero_vec = _native.ptr(_f32(self.cached_zero_vector))
        L = _native.lib()
        nbytes = ctypes.c_size_t()
        _native.check(L.wdmpnn_packed_params_bytes(ctypes.byref(gs), ctypes.byref(p), ctypes.byref(cfg),
                                                   ctypes.byref(nbytes)), 'pack size')
        buf = torch.empty(nbytes.value, dtype=torch.uint8, device=device)

        def launch():
            _native.check(L.wdmpnn_pack_params(ctypes.byref(gs), ctypes.byref(p), ctypes.byref(cfg), buf.data_ptr(),
                                               nbytes.value, stream.cuda_stream if stream is not None
                                               else _native.current_stream(device)), 'pack params')
        if defer:  # (training: the caller enqueues it on the current stream, before the forward)
            p.packed, p.packed_bytes = buf.data_ptr(), buf.numel()
            self._pack_cache = None
            return p, buf, launch
        launch()
        p.packed, p.packed_bytes = buf.data_ptr(), buf.numel()
        if cache:  # (a training forward uses its packed weights on this stream only: no event)
            if stream is None:
                stream = torch.cuda.current_stream(device)
            ev = torch.cuda.Event()
            ev.record(stream)
            self._pack_cache = (key, buf, p, ev, {stream.cuda_stream})
        else:
            self._pack_cache = None
        return p, buf


class MPN(nn.Module):
    """mpn.py:176-289."""

    def __init__(self, args, atom_fdim: int = None, bond_fdim: int = None):
        super(MPN, self).__init__()
        self.atom_fdim = atom_fdim or get_atom_fdim(overwrite_default_atom=args.overwrite_default_atom_features)
        self.bond_fdim = bond_fdim or get_bond_fdim(overwrite_default_atom=args.overwrite_default_atom_features,
                                                    overwrite_default_bond=args.overwrite_default_bond_features,
                                                    atom_messages=args.atom_messages)
        self.features_only = args.features_only
        self.use_input_features = args.use_input_features
        self.device = args.device
        self.atom_descriptors = args.atom_descriptors
        self.overwrite_default_atom_features = args.overwrite_default_atom_features
        self.overwrite_default_bond_features = args.overwrite_default_bond_features
        if self.features_only:
            return
        if args.mpn_shared:
            self.encoder = nn.ModuleList([MPNEncoder(args, self.atom_fdim, self.bond_fdim)] * args.number_of_molecules)
        else:
            self.encoder = nn.ModuleList([MPNEncoder(args, self.atom_fdim, self.bond_fdim)
                                          for _ in range(args.number_of_molecules)])

    def forward(self, batch, features_batch: List[np.ndarray] = None, atom_descriptors_batch: List[np.ndarray] = None,
                atom_features_batch: List[np.ndarray] = None,
                bond_features_batch: List[np.ndarray] = None) -> torch.FloatTensor:
        if type(batch[0]) != BatchMolGraph:
            batch = [[mols[i] for mols in batch] for i in range(len(batch[0]))]
            if self.atom_descriptors == 'feature' and len(batch) > 1:
                raise NotImplementedError('Atom/bond descriptors are currently only supported with one molecule '
                                          'per input (i.e., number_of_molecules = 1).')
            batch = [mol2graph(b) for b in batch]
        dev = self.encoder[0].W_i.weight.device if not self.features_only else torch.device(self.device)
        if self.use_input_features:
            features_batch = torch.from_numpy(np.stack(features_batch)).float().to(dev)
            if self.features_only:
                return features_batch
        if self.atom_descriptors == 'descriptor':
            if len(batch) > 1:
                raise NotImplementedError('Atom descriptors are currently only supported with one molecule '
                                          'per input (i.e., number_of_molecules = 1).')
            encodings = [enc(ba, atom_descriptors_batch) for enc, ba in zip(self.encoder, batch)]
        else:
            encodings = [enc(ba) for enc, ba in zip(self.encoder, batch)]
        output = reduce(lambda x, y: torch.cat((x, y), dim=1), encodings)
        if self.use_input_features:
            if len(features_batch.shape) == 1:
                features_batch = features_batch.view(1, -1)
            output = torch.cat([output, features_batch], dim=1)
        return output
