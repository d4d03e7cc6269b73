"""Training-step counterpart of the reference loop.

* ``train_step`` / ``train`` follow ``chemprop/train/train.py:17-113``: mask / targets from
  ``None`` entries, target and data weights, ``loss_func(preds, targets) * w_t * w_d * mask``,
  ``loss.sum() / mask.sum()``, backward, optional ``clip_grad_norm_``, ``optimizer.step()``,
  per-batch scheduler step; plus the DP all-reduce of :mod:`chemprop_amd.dp` between backward and
  the optimizer step.
* ``NoamLR`` restates ``chemprop/nn_utils.py:115-194``; ``get_loss_func`` ``utils.py:338-364``
  (regression / classification / multiclass); ``build_optimizer`` ``utils.py:295-310``.
"""
from __future__ import annotations

import ctypes
from typing import Callable, List, Optional, Sequence, Union

import numpy as np
import torch
import torch.nn as nn
from torch.optim import Adam, Optimizer
from torch.optim.lr_scheduler import _LRScheduler

from .dp import GradBucket


class NoamLR(_LRScheduler):
    """nn_utils.py:115-194: linear warm-up from init_lr to max_lr over warmup_epochs, then
    exponential decay to final_lr at total_epochs."""

    def __init__(self, optimizer: Optimizer, warmup_epochs: List[Union[float, int]], total_epochs: List[int],
                 steps_per_epoch: int, init_lr: List[float], max_lr: List[float], final_lr: List[float]):
        assert len(optimizer.param_groups) == len(warmup_epochs) == len(total_epochs) == len(init_lr) == \
            len(max_lr) == len(final_lr)
        self.num_lrs = len(optimizer.param_groups)
        self.optimizer = optimizer
        self.warmup_epochs = np.array(warmup_epochs)
        self.total_epochs = np.array(total_epochs)
        self.steps_per_epoch = steps_per_epoch
        self.init_lr = np.array(init_lr)
        self.max_lr = np.array(max_lr)
        self.final_lr = np.array(final_lr)
        self.current_step = 0
        self.lr = init_lr
        self.warmup_steps = (self.warmup_epochs * self.steps_per_epoch).astype(int)
        self.total_steps = self.total_epochs * self.steps_per_epoch
        self.linear_increment = (self.max_lr - self.init_lr) / self.warmup_steps
        self.exponential_gamma = (self.final_lr / self.max_lr) ** (1 / (self.total_steps - self.warmup_steps))
        super(NoamLR, self).__init__(optimizer)

    def get_lr(self) -> List[float]:
        return list(self.lr)

    def step(self, current_step: int = None):
        self.current_step = self.current_step + 1 if current_step is None else current_step
        for i in range(self.num_lrs):
            if self.current_step <= self.warmup_steps[i]:
                self.lr[i] = self.init_lr[i] + self.current_step * self.linear_increment[i]
            elif self.current_step <= self.total_steps[i]:
                self.lr[i] = self.max_lr[i] * (self.exponential_gamma[i] ** (self.current_step - self.warmup_steps[i]))
            else:
                self.lr[i] = self.final_lr[i]
            self.optimizer.param_groups[i]['lr'] = self.lr[i]


def get_loss_func(dataset_type: str) -> nn.Module:
    """utils.py:338-364 (no alternative losses, no spectra)."""
    if dataset_type == 'classification':
        return nn.BCEWithLogitsLoss(reduction='none')
    if dataset_type == 'regression':
        return nn.MSELoss(reduction='none')
    if dataset_type == 'multiclass':
        return nn.CrossEntropyLoss(reduction='none')
    raise ValueError(f'Dataset type "{dataset_type}" not supported.')


# the direct training step's packed weights rewritten by HipAdam's own pass (wdmpnn_adam_step_repack);
# False: a pack launch before every training forward (the A/B and test switch)
ADAM_REPACK = True


class HipAdam(Optimizer):
    """torch.optim.Adam / AdamW (no amsgrad, no maximize) whose update is ONE HIP launch per 16
    parameters (``wdmpnn_adam_step``): torch's fused Adam kernel took 40 us per training step for the
    355 k parameters of the default model (profiles/round2_train_kernel_trace_v2.txt), this one a few.
    Same per-element arithmetic as torch's fused Adam; lr / weight_decay / betas / eps are read from the
    param groups at every step, so schedulers (NoamLR) work unchanged.  State per parameter:
    ``step`` (int), ``exp_avg``, ``exp_avg_sq`` (as torch's Adam).  Writes its parameters through raw
    pointers (no version-counter bump): the encoders' packed-weight caches are keyed on the optimizer-step
    count instead.  A write of an encoder parameter through ``.data`` between steps needs
    ``MPNEncoder.invalidate_packed_params()``."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 decoupled: bool = False):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0) or weight_decay < 0.0:
            raise ValueError('invalid Adam hyperparameter')
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self.decoupled = bool(decoupled)
        self._tables = {}  # parameter pointers of one launch -> its ctypes tensor table
        self._repack = None  # (encoder, its training pack) for the next step (train_step's direct path)

    def repack_next(self, encoder) -> None:
        """Have the next :meth:`step` also rewrite ``encoder``'s training pack (the packed weight copies its
        direct training forward reads) from the updated weights, instead of a pack launch before the next
        forward (``wdmpnn_adam_step_repack``).  No effect unless the encoder's six weights are updated in
        one call of that step."""
        tp = encoder.__dict__.get('_train_pack')
        self._repack = (encoder, tp) if tp is not None and ADAM_REPACK else None

    @torch.no_grad()
    def step(self, closure=None):
        from . import _native
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        L = _native.lib()
        state = self.state
        rp, self._repack = self._repack, None
        for group in self.param_groups:
            ps = [(p, state[p]) for p in group['params'] if p.grad is not None]
            if not ps:
                continue
            # torch's Adam keeps one step count per parameter: a parameter that had no gradient on some
            # steps lags behind the others, so the launches are grouped by step count (usually one group)
            by_step = {}
            for p, st in ps:
                if 'exp_avg' not in st:
                    if p.device.type != 'cuda' or p.dtype != torch.float32 or not p.is_contiguous():
                        raise TypeError('HipAdam expects contiguous float32 CUDA parameters')
                    st['step'] = 0
                    st['exp_avg'] = torch.zeros_like(p)
                    st['exp_avg_sq'] = torch.zeros_like(p)
                by_step.setdefault(int(st['step']) + 1, []).append((p, st))
            for step, sub in by_step.items():
                key = tuple(p.data_ptr() for p, _ in sub)
                tab = self._tables.get(key)
                if tab is None:
                    tab = (_native.WdAdamTensor * len(sub))()
                    for k, (p, st) in enumerate(sub):
                        tab[k].param, tab[k].exp_avg, tab[k].exp_avg_sq = p.data_ptr(), st['exp_avg'].data_ptr(), \
                            st['exp_avg_sq'].data_ptr()
                        tab[k].numel = p.numel()
                    self._tables[key] = tab
                for k, (p, st) in enumerate(sub):
                    g = p.grad
                    if g.is_sparse or g.dtype != torch.float32 or not g.is_contiguous():
                        raise TypeError('HipAdam expects dense contiguous float32 gradients')
                    tab[k].grad = g.data_ptr()
                    st['step'] = step
                h = _native.WdAdamHyper(float(group['lr']), float(group['betas'][0]), float(group['betas'][1]),
                                        float(group['eps']), float(group['weight_decay']), step, int(self.decoupled))
                sid = _native.current_stream(sub[0][0].device)
                if rp is not None and rp[1]['ptrs'] <= frozenset(key) and rp[1]['key'][-1] == sid:
                    enc, tp = rp
                    rp = None
                    rc = L.wdmpnn_adam_step_repack(tab, len(sub), ctypes.byref(h), ctypes.byref(tp['gs']),
                                                   ctypes.byref(tp['p']), ctypes.byref(tp['cfg']), tp['buf'].data_ptr(),
                                                   tp['buf'].numel(), sid)
                    if rc != _native.ERR_UNSUPPORTED:
                        _native.check(rc, 'adam step + repack')
                        enc._repacked_by_optimizer(tp)
                        continue
                _native.check(L.wdmpnn_adam_step(tab, len(sub), ctypes.byref(h), sid), 'adam step')
        return loss

    def load_state_dict(self, state_dict) -> None:
        super().load_state_dict(state_dict)
        self._tables.clear()  # the moment buffers were replaced: rebuild the pointer tables


def build_optimizer(model: nn.Module, args=1e-4, weight_decay: float = 0.0) -> Optimizer:
    """utils.py:295-310: Adam (or AdamW when ``args.optimizer == 'adamw'``) over all parameters.
    ``args`` is a TrainArgs-like object (``init_lr``, optional ``weight_decay`` / ``optimizer``) as in
    the reference, or a plain learning rate.  On a GPU the update runs as :class:`HipAdam` (same update
    rule, one HIP launch per step)."""
    if isinstance(args, (int, float)):
        lr, wd, kind = float(args), weight_decay, 'adam'
    else:
        lr, wd, kind = args.init_lr, getattr(args, 'weight_decay', 0.0), getattr(args, 'optimizer', 'adam')
    params = list(model.parameters())
    groups = [{'params': params, 'lr': lr, 'weight_decay': wd}]
    if bool(params) and all(p.device.type == 'cuda' and p.dtype == torch.float32 for p in params):
        return HipAdam(groups, lr=lr, weight_decay=wd, decoupled=kind == 'adamw')
    if kind == 'adamw':
        return torch.optim.AdamW(groups)
    return Adam(groups)


# pinned host tables of batch_loss, a ring of _PINNED_RING per (device, shape): allocating pinned memory
# every step costs more than the rest of the loss.  A buffer is refilled after the event of its last copy,
# which with a ring is several steps old (one buffer made every step wait for the previous step's forward:
# the host could not run ahead of the GPU)
_PINNED_TABLES = {}
_PINNED_RING = 4


def _host_table(rows: np.ndarray, dev: torch.device, zero_copy: bool = False):
    """rows (float32 [B][2T]) -> device tensor through a reused pinned buffer (asynchronous copy).
    ``zero_copy``: no copy; returns (device address of the pinned buffer, its event) or None when the
    buffer is not mapped for the device -- the caller's kernel reads the rows over PCIe, and the caller
    records the event after that kernel's launch (the buffer is refilled only after it)."""
    if dev.type != 'cuda':
        return None if zero_copy else torch.from_numpy(rows).to(dev)
    key = (dev, rows.shape, zero_copy)
    ring = _PINNED_TABLES.get(key)
    if ring is None:
        ring = _PINNED_TABLES[key] = [0, [None] * _PINNED_RING]
    i = ring[0]
    ring[0] = (i + 1) % _PINNED_RING
    ent = ring[1][i]
    if ent is None:
        from . import _native
        if zero_copy:
            # the kernel reads the rows in place: coherent mapped memory (torch's pinned buffers are
            # non-coherent, and a rewritten slot read again at the same device address would then rely
            # on the dispatch invalidating stale L2 lines)
            cb = _native.CoherentHostBuffer(rows.shape)
            ent = ring[1][i] = (cb, torch.cuda.Event(), cb.device_ptr)
        else:
            buf = torch.empty(rows.shape, dtype=torch.float32, pin_memory=True)
            ent = ring[1][i] = (buf, torch.cuda.Event(), 0)
    else:
        ent[1].synchronize()  # (this buffer's last reader, _PINNED_RING steps ago)
    buf, ev, dptr = ent
    if zero_copy:
        buf.array[...] = rows
        return (dptr, ev) if dptr else None
    buf.numpy()[...] = rows
    table = buf.to(dev, non_blocking=True)
    ev.record(torch.cuda.current_stream(dev))
    return table


def _loss_table(target_batch, target_weights, data_weights, dev, zero_copy: bool = False):
    """train.py:46-74's targets and weights as one device table [B][2T] (targets | w = target weight *
    data weight * mask, rounded once to fp32) and the host count mask.sum()."""
    n_b = len(target_batch)
    n_t = len(target_batch[0]) if n_b else 0
    # missing targets are None (train.py:47-48); numpy's float conversion would turn them into NaN, so the
    # mask comes from an object array (a NaN target stays a NaN, as in the reference).  Fast path: a batch
    # that converts to floats without any NaN had neither (mask of ones, the same table)
    tgt = None
    try:
        tgt = np.asarray(target_batch, dtype=np.float64)
        if tgt.shape != (n_b, n_t) or np.isnan(tgt).any():
            tgt = None
    except (TypeError, ValueError):
        tgt = None
    if tgt is not None:
        mask = np.ones((n_b, n_t))
    else:
        obj = np.array(target_batch, dtype=object).reshape(n_b, n_t)
        present = obj != None  # noqa: E711 (elementwise)
        tgt = np.where(present, obj, 0.0).astype(np.float64)
        mask = present.astype(np.float64)
    tw = np.ones(n_t) if target_weights is None else np.asarray(target_weights, dtype=np.float64)
    dw = np.ones(n_b) if data_weights is None else np.asarray(data_weights, dtype=np.float64)
    # targets and W travel as one host table (one pinned, asynchronous copy: pageable copies would each
    # stall the host until the forward has drained)
    rows = np.concatenate([tgt, tw[None, :] * dw[:, None] * mask], axis=1).astype(np.float32)
    if zero_copy:
        return _host_table(rows, dev, True), n_t, int(mask.sum()), rows.shape
    return _host_table(rows, dev), n_t, int(mask.sum())


def batch_loss(preds: torch.Tensor, target_batch: Sequence[Sequence[Optional[float]]], loss_func: Callable,
               dataset_type: str = 'regression', target_weights: Sequence[float] = None,
               data_weights: Sequence[float] = None) -> torch.Tensor:
    """train.py:46-74: ``(loss_func(preds, targets) * target_weights * data_weights * mask).sum() /
    mask.sum()``.  The three weight factors are multiplied on the host into one weight table W, and
    ``mask.sum()`` is a host count: two fewer device ops forward and backward, the same loss (W is
    rounded once to fp32 instead of twice)."""
    table, n_t, n_mask = _loss_table(target_batch, target_weights, data_weights, preds.device)
    targets, w = table[:, :n_t], table[:, n_t:]
    if dataset_type == 'multiclass':
        targets = targets.long()
        loss = torch.cat([loss_func(preds[:, j, :], targets[:, j]).unsqueeze(1) for j in range(preds.size(1))],
                         dim=1) * w
    else:
        loss = loss_func(preds, targets) * w
    return loss.sum() / float(n_mask)


# ------------------------------------------------------------------------------------------------
# Fused FFN head + masked MSE loss (wdmpnn_head_mse).  The reference's step evaluates ffn(emb) (model.py:
# 57-121), loss_func(preds, targets) * weights and .sum() / mask.sum() (train.py:55-74) and autograd runs
# their backward: ~25 small torch ops whose host time left the GPU idle for most of the step
# (profiles/round2_train_kernel_trace_v3.txt).  For the default head (two Linear layers, an activation, no
# active dropout; MSELoss for regression, BCEWithLogitsLoss for classification) the loss and every gradient of the head come from two HIP
# launches in the forward; the backward scales them by the loss's incoming gradient (one launch).
# ------------------------------------------------------------------------------------------------
def _head_act(m: nn.Module) -> Optional[int]:
    """WdActivation of an FFN activation module the fused head supports (not PReLU), else None."""
    if type(m) is nn.ReLU:
        return 0
    if type(m) is nn.LeakyReLU and m.negative_slope == 0.1:
        return 1
    if type(m) is nn.Tanh:
        return 3
    if type(m) is nn.SELU:
        return 4
    if type(m) is nn.ELU and m.alpha == 1.0:
        return 5
    return None


def _fusable_head(model: nn.Module, loss_func: Callable, dataset_type: str):
    """(Linear 1, Linear 2, activation code) when the step's head + loss can run fused, else None."""
    from .model import MoleculeModel
    if dataset_type == 'regression' and type(loss_func) is nn.MSELoss and loss_func.reduction == 'none':
        kind = 0
    elif dataset_type == 'classification' and type(loss_func) is nn.BCEWithLogitsLoss and \
            loss_func.reduction == 'none' and loss_func.weight is None and loss_func.pos_weight is None:
        kind = 1  # (the FFN's logits: MoleculeModel applies the sigmoid only outside training, model.py:186-188)
    else:
        return None
    if not isinstance(model, MoleculeModel) or type(model).forward is not MoleculeModel.forward:
        return None
    ffn = model.ffn
    if len(ffn) != 5:
        return None
    d0, l1, act, d1, l2 = ffn
    if type(d0) is not nn.Dropout or type(d1) is not nn.Dropout or type(l1) is not nn.Linear \
            or type(l2) is not nn.Linear:
        return None
    if model.training and (d0.p > 0 or d1.p > 0):
        return None
    code = _head_act(act)
    if code is None:
        return None
    for t in (l1.weight, l1.bias, l2.weight, l2.bias):
        if t is not None and (t.device.type != 'cuda' or t.dtype != torch.float32 or not t.is_contiguous()):
            return None
    if l1.in_features > 4096 or l1.out_features > 4096 or l2.out_features > 64:
        return None
    return l1, l2, code, kind


class _HeadMSE(torch.autograd.Function):
    """loss = sum(w (W2 act(W1 x + b1) + b2 - y)^2) / n, with every gradient computed in the forward."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, table, inv_n, act, kind):
        from . import _native
        x = x.contiguous()
        dev = x.device
        B, F = x.shape
        Hf, T = W1.shape[0], W2.shape[0]
        scratch = torch.empty(B * (2 * Hf + T + 1), dtype=torch.float32, device=dev)
        dx = torch.empty_like(x)
        dW1, dW2 = torch.empty_like(W1), torch.empty_like(W2)
        db1 = torch.empty_like(b1) if b1 is not None else None
        db2 = torch.empty_like(b2) if b2 is not None else None
        loss = torch.empty((), dtype=torch.float32, device=dev)
        ptr = _native.ptr
        sp = scratch.data_ptr()
        h = _native.WdHead(ptr(x), F, B, F, Hf, T, ptr(W1), ptr(b1), ptr(W2), ptr(b2), ptr(table), table.shape[1],
                           float(inv_n), act, sp, sp + 4 * B * Hf, sp + 8 * B * Hf, sp + 4 * B * (2 * Hf + T),
                           ptr(dx), ptr(dW1), ptr(db1), ptr(dW2), ptr(db2), ptr(loss), kind)
        _native.check(_native.lib().wdmpnn_head_mse(ctypes.byref(h), _native.current_stream(dev)), 'FFN head + loss')
        ctx.grads = (dx, dW1, db1, dW2, db2)
        return loss

    @staticmethod
    def backward(ctx, gl):
        from . import _native
        grads, ctx.grads = ctx.grads, None  # (sole owner: autograd adopts the tensors instead of copying)
        live = [g for g in grads if g is not None]
        gl = gl.to(torch.float32).contiguous()
        ptrs = (ctypes.c_void_p * len(live))(*[g.data_ptr() for g in live])
        ns = (ctypes.c_int64 * len(live))(*[g.numel() for g in live])
        _native.check(_native.lib().wdmpnn_scale(ptrs, ns, len(live), gl.data_ptr(),
                                                 _native.current_stream(gl.device)), 'scale')
        return grads + (None, None, None, None)


def head_loss(emb: torch.Tensor, head, target_batch, target_weights=None, data_weights=None) -> torch.Tensor:
    """``batch_loss(model.ffn(emb), ...)`` for a head accepted by ``_fusable_head`` (regression with MSE,
    classification with BCE on logits)."""
    l1, l2, act, kind = head
    table, n_t, n_mask = _loss_table(target_batch, target_weights, data_weights, emb.device)
    if n_t != l2.out_features:
        raise ValueError(f'{n_t} targets per row for {l2.out_features} outputs')
    if table.shape[0] != emb.shape[0] or emb.dim() != 2 or emb.shape[1] != l1.in_features:
        raise ValueError(f'{table.shape[0]} target rows for encodings of shape {tuple(emb.shape)} '
                         f'(FFN input {l1.in_features})')
    inv_n = 1.0 / n_mask if n_mask else float('inf')
    return _HeadMSE.apply(emb, l1.weight, l1.bias, l2.weight, l2.bias, table, inv_n, act, kind)


def _grad_buffer(p: torch.Tensor) -> torch.Tensor:
    """The tensor a direct step writes p's gradient into: p.grad when it can be overwritten in place (a
    GradBucket view, or the last step's gradient), else a fresh one (installed as p.grad)."""
    g = p.grad
    if g is None or g.shape != p.shape or g.dtype != torch.float32 or not g.is_contiguous() or g.device != p.device:
        g = torch.empty_like(p)
        p.grad = g
    return g


def _direct_encoder(model: nn.Module, mol_batch, features_batch, head):
    """The MPNEncoder when the step can skip autograd: one molecule per input, no extra features or
    descriptors, depth >= 2, every parameter trainable and written by the direct step (the encoder's
    native gradients and the fused head's); else None."""
    from .model import MoleculeModel
    from .mpn import MPNEncoder
    if not isinstance(model, MoleculeModel) or type(model).forward is not MoleculeModel.forward:
        return None
    mpn = model.encoder
    if features_batch is not None or mpn.features_only or mpn.use_input_features or mpn.atom_descriptors or \
            len(mpn.encoder) != 1 or not isinstance(mol_batch, (list, tuple)) or len(mol_batch) != 1:
        return None
    enc = mpn.encoder[0]
    if type(enc) is not MPNEncoder or enc.depth < 2 or enc.atom_messages or hasattr(enc, 'atom_descriptors_layer'):
        return None
    if type(mol_batch[0]).__name__ != 'BatchMolGraph':
        return None
    ids = []
    if not _all_trainable(model, enc.cached_zero_vector, ids):
        return None
    # the direct step skips zero_grad and overwrites only the gradients it computes: any other trainable
    # parameter (a future addition to the model) would keep a stale gradient, so it must not exist
    l1, l2 = head[:2]
    written = {id(t) for _, t in enc._direct_names()} | {id(t) for t in (l1.weight, l1.bias, l2.weight, l2.bias)
                                                          if t is not None}
    if len(ids) != len(written) or not written.issuperset(ids):
        return None
    return enc


def _all_trainable(mod: nn.Module, skip, ids: list) -> bool:
    """Every parameter of ``mod`` and its submodules (but ``skip``) requires grad (their ids appended to
    ``ids``): ``named_parameters``'s test on the raw module dicts (its generators and memo sets cost tens of
    us per step)."""
    for p in mod._parameters.values():
        if p is not None and p is not skip:
            if not p.requires_grad:
                return False
            ids.append(id(p))
    for m in mod._modules.values():
        if m is not None and not _all_trainable(m, skip, ids):
            return False
    return True


def _direct_step(model, enc, graph, head, target_batch, target_weights, data_weights, bucket=None) -> torch.Tensor:
    """Forward, loss and every gradient of a fused-head step without the autograd engine: the encoder's
    training forward, wdmpnn_head_mse (loss, d loss / d encoding, the head's gradients) and the encoder's
    backward on that gradient (the incoming gradient of the loss is 1), each written straight into the
    parameters' .grad buffers.  The same launches as the autograd path minus its host gaps (the engine
    hand-off, the gradient-seed fill and the scale by 1; profiles/round3_*)."""
    from . import _native
    l1, l2, act, kind = head
    out, state = enc._train_forward(graph)
    # the loss table read by the head kernel straight from its pinned host buffer (no copy launch in the
    # step: the copy kernel and its gap were ~10 us, profiles/round4_train_kernel_trace_v1.txt)
    zc, n_t, n_mask, tshape = _loss_table(target_batch, target_weights, data_weights, out.device, zero_copy=True)
    if zc is None:
        table, n_t, n_mask = _loss_table(target_batch, target_weights, data_weights, out.device)
        tab_ptr, tshape = table.data_ptr(), tuple(table.shape)
    else:
        tab_ptr = zc[0]
    if n_t != l2.out_features:
        raise ValueError(f'{n_t} targets per row for {l2.out_features} outputs')
    if tshape[0] != out.shape[0] or out.shape[1] != l1.in_features:
        raise ValueError(f'{tshape[0]} target rows for encodings of shape {tuple(out.shape)} '
                         f'(FFN input {l1.in_features})')
    inv_n = 1.0 / n_mask if n_mask else float('inf')
    dev = out.device
    B, F = out.shape
    Hf, T = l1.weight.shape[0], l2.weight.shape[0]
    scratch = torch.empty(B * (2 * Hf + T + 1), dtype=torch.float32, device=dev)
    dx = torch.empty_like(out)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    dW1, dW2 = _grad_buffer(l1.weight), _grad_buffer(l2.weight)
    db1 = _grad_buffer(l1.bias) if l1.bias is not None else None
    db2 = _grad_buffer(l2.bias) if l2.bias is not None else None
    ptr = _native.ptr
    sp = scratch.data_ptr()
    h = _native.WdHead(ptr(out), F, B, F, Hf, T, ptr(l1.weight), ptr(l1.bias), ptr(l2.weight), ptr(l2.bias), tab_ptr,
                       tshape[1], float(inv_n), act, sp, sp + 4 * B * Hf, sp + 8 * B * Hf, sp + 4 * B * (2 * Hf + T),
                       ptr(dx), ptr(dW1), ptr(db1), ptr(dW2), ptr(db2), ptr(loss), kind)
    _native.check(_native.lib().wdmpnn_head_mse(ctypes.byref(h), _native.current_stream(dev)), 'FFN head + loss')
    if zc is not None:
        zc[1].record(torch.cuda.current_stream(dev))  # (the pinned buffer's last reader)
    if bucket is not None:  # the head's gradients are enqueued: their all-reduce overlaps the encoder backward
        bucket.start_early()
    enc._train_backward(state, dx, {n: _grad_buffer(p) for n, p in enc._direct_names()})
    return loss


def train_step(model: nn.Module, mol_batch, target_batch, loss_func: Callable, optimizer: Optimizer,
               scheduler: _LRScheduler = None, dataset_type: str = 'regression', features_batch=None,
               target_weights=None, data_weights=None, grad_clip: float = None,
               bucket: GradBucket = None, fused_head: bool = True, direct: bool = True) -> torch.Tensor:
    """One optimisation step (train.py:55-86).  With ``bucket`` the gradients are averaged over the
    data-parallel ranks (one all-reduce) before clipping and the optimizer step.  ``fused_head``: the
    default regression / classification head + loss run as ``wdmpnn_head_mse`` (same loss and gradients within fp32
    summation order; ``False`` = the torch ops of the reference).  ``direct``: with the fused head and a
    plain one-molecule encoder, skip the autograd engine (``_direct_step``: the same launches and results,
    bitwise, without the engine's host gaps).  The direct step keeps one packed copy of the encoder weights
    across steps (rewritten by :class:`HipAdam`); after writing an encoder parameter through ``.data`` call
    ``MPNEncoder.invalidate_packed_params()`` (reassigned parameters and ``load_state_dict`` are detected)."""
    if not model.training:  # (module.train() walks every submodule: the reference sets it once per epoch)
        model.train()
    head = _fusable_head(model, loss_func, dataset_type) if fused_head else None
    enc = _direct_encoder(model, mol_batch, features_batch, head) if head is not None and direct else None
    if enc is not None:
        # every trainable parameter's gradient is overwritten: no zeroing, no autograd
        if bucket is not None:
            bucket.attach()
        loss = _direct_step(model, enc, mol_batch[0], head, target_batch, target_weights, data_weights, bucket)
    else:
        if bucket is not None:
            bucket.zero()
        else:
            optimizer.zero_grad(set_to_none=True)  # (the optimizer holds every model parameter: build_optimizer)
        if head is not None:  # the default regression head: ffn + loss + their gradients as two HIP launches
            loss = head_loss(model.encoder(mol_batch, features_batch), head, target_batch, target_weights,
                             data_weights)
        else:
            preds = model(mol_batch, features_batch)
            loss = batch_loss(preds, target_batch, loss_func, dataset_type, target_weights, data_weights)
        loss.backward()
    if bucket is not None:
        # the rest of the bucket behind the last gradient kernel (the direct step launched the head's
        # segment before the encoder backward, so that one overlaps the backward on the GPU); with RCCL
        # finish_allreduce makes the compute stream, not the host, wait for both before the update
        bucket.start_allreduce()
        bucket.finish_allreduce()
    if grad_clip:
        nn.utils.clip_grad_norm_(model.parameters(), grad_clip)
    if enc is not None and isinstance(optimizer, HipAdam):
        optimizer.repack_next(enc)
    optimizer.step()
    if scheduler is not None and isinstance(scheduler, (NoamLR, torch.optim.lr_scheduler.CosineAnnealingLR,
                                                        torch.optim.lr_scheduler.CyclicLR)):
        scheduler.step()
    return loss.detach()


def train(model: nn.Module, batches, loss_func: Callable, optimizer: Optimizer, scheduler: _LRScheduler = None,
          dataset_type: str = 'regression', grad_clip: float = None, bucket: GradBucket = None) -> List[float]:
    """One epoch over ``batches`` = iterable of (mol_batch, target_batch[, features_batch]) (train.py:17-113
    without logging); returns the per-batch losses (one host sync per batch, like loss.item())."""
    losses = []
    for item in batches:
        mol_batch, target_batch = item[0], item[1]
        features_batch = item[2] if len(item) > 2 else None
        loss = train_step(model, mol_batch, target_batch, loss_func, optimizer, scheduler, dataset_type,
                          features_batch, grad_clip=grad_clip, bucket=bucket)
        losses.append(float(loss))
    return losses
