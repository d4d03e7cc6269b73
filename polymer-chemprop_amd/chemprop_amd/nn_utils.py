"""Hot-path helpers of ``chemprop/nn_utils.py`` with the same names and semantics.

``index_select_ND`` (nn_utils.py:50-67) runs the HIP row-gather kernel (``wdmpnn_index_select_rows``)
on device tensors; the encoder itself does not call it (its gathers are fused into the GEMM tile
loads), it is kept for callers of the reference helper.  ``get_activation_function``
(nn_utils.py:70-99) and ``initialize_weights`` (nn_utils.py:102-112) are module factories / init rules
and stay PyTorch.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _native


class _IndexSelectND(torch.autograd.Function):
    @staticmethod
    def forward(ctx, source, index):
        ctx.save_for_backward(index)
        ctx.n_src = source.shape[0]
        src = source.contiguous()
        idx = index.reshape(-1).to(torch.int64).contiguous()
        row_len = 1
        for s in src.shape[1:]:
            row_len *= s
        out = torch.empty((idx.numel(),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        if idx.numel():
            lo, hi = int(idx.min()), int(idx.max())
            if lo < 0 or hi >= src.shape[0]:
                raise IndexError(f'index out of range in self (index {lo if lo < 0 else hi}, size {src.shape[0]})')
        _native.check(_native.lib().wdmpnn_index_select_rows(src.data_ptr(), src.shape[0], row_len, idx.data_ptr(),
                                                             idx.numel(), out.data_ptr(),
                                                             _native.current_stream(src.device)),
                      'index_select_ND')
        return out.view(tuple(index.shape) + tuple(src.shape[1:]))

    @staticmethod
    def backward(ctx, grad):
        """Transposed gather on the HIP path (wdmpnn_index_select_rows_backward): every source row sums
        its selected positions' gradients in position order, deterministic and atomics-free (autograd
        of the reference's index_select scatter-adds them)."""
        (index,) = ctx.saved_tensors
        tail = tuple(grad.shape[index.dim():])
        g = torch.empty((ctx.n_src,) + tail, dtype=grad.dtype, device=grad.device)
        idx = index.reshape(-1).to(torch.int64)
        _, perm = torch.sort(idx, stable=True)
        ptr = torch.searchsorted(idx[perm], torch.arange(ctx.n_src + 1, device=idx.device, dtype=torch.int64))
        gr = grad.contiguous()
        row_len = 1
        for s in tail:
            row_len *= s
        _native.check(_native.lib().wdmpnn_index_select_rows_backward(
            gr.data_ptr(), idx.numel(), row_len, perm.data_ptr(), ptr.data_ptr(), ctx.n_src, g.data_ptr(),
            _native.current_stream(grad.device)), 'index_select_ND backward')
        return g, None


def index_select_ND(source: torch.Tensor, index: torch.Tensor) -> torch.Tensor:
    """nn_utils.py:50-67: ``source[index]`` reshaped to ``index.shape + source.shape[1:]``.

    Device tensors only (float32 source): the HIP kernel is the implementation, there is no CPU path.
    """
    if source.device.type != 'cuda':
        raise RuntimeError('chemprop_amd.index_select_ND runs on the MI355X HIP path only (device tensors)')
    if source.dtype != torch.float32:
        raise TypeError('index_select_ND: float32 source expected')
    return _IndexSelectND.apply(source, index.to(source.device))


def get_activation_function(activation: str) -> nn.Module:
    """nn_utils.py:70-99."""
    if activation == 'ReLU':
        return nn.ReLU()
    elif activation == 'LeakyReLU':
        return nn.LeakyReLU(0.1)
    elif activation == 'PReLU':
        return nn.PReLU()
    elif activation == 'tanh':
        return nn.Tanh()
    elif activation == 'SELU':
        return nn.SELU()
    elif activation == 'ELU':
        return nn.ELU()
    else:
        raise ValueError(f'Activation "{activation}" not supported.')


def initialize_weights(model: nn.Module) -> None:
    """nn_utils.py:102-112: 1-D parameters -> 0, others -> xavier_normal_."""
    for param in model.parameters():
        if param.dim() == 1:
            nn.init.constant_(param, 0)
        else:
            nn.init.xavier_normal_(param)
