"""Data parallelism over the GPUs of one node.

The reference has no distributed code; this module is the build's DP layer:
one process per GPU, ``torch.distributed`` with backend ``nccl`` (= RCCL on ROCm, over xGMI) on
GPUs and ``gloo`` on CPU (tests).  Molecules are independent, so:

* forward throughput shards batches across ranks with no collective (rank r takes r, r+N, ...);
* training is plain DP: identical initial parameters (broadcast from rank 0), local forward +
  backward on the rank's own batch, then ONE all-reduce of a flat fp32 gradient bucket
  (354,901 params = 1.42 MB at the default config), divided by the world size.

The gradients of every parameter are views into the bucket, so autograd accumulates straight into
it and the all-reduce needs no pack/unpack copies.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Iterable, List, Sequence, TypeVar

import torch
import torch.distributed as dist
import torch.nn as nn

T = TypeVar('T')


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device('cpu')

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def init_distributed(backend: str = None, device: str = None) -> DistEnv:
    """Read RANK / WORLD_SIZE / LOCAL_RANK (torch.distributed.run) and initialise the process group.
    Single process (no env): no process group, rank 0 of 1.

    ``backend``: 'nccl' (RCCL over xGMI, the multi-GPU default) or 'gloo'.  ``device``: 'cuda' puts the
    rank on GPU ``LOCAL_RANK % visible GPUs`` (several ranks may share one GPU: the gloo rehearsal of the
    multi-GPU path), 'cpu' keeps it on the host; default: cuda with nccl, cpu with gloo.  This is the one
    initialisation path of the package: bench.py and the DP training tests call it, so the 8-GPU run
    differs from the rehearsal only in the backend string."""
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if backend is None:
        backend = 'nccl' if torch.cuda.is_available() else 'gloo'
    if device is None:
        device = 'cuda' if backend == 'nccl' else 'cpu'
    if device == 'cuda':
        ordinal = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(ordinal)
        dev = torch.device('cuda', ordinal)
    else:
        dev = torch.device('cpu')
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        kwargs = {'device_id': dev} if backend == 'nccl' else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kwargs)
    return DistEnv(rank, world, local, dev)


def shard(items: Sequence[T], rank: int, world_size: int) -> List[T]:
    """Round-robin shard: rank r gets items r, r + N, r + 2N, ...  (disjoint, covering)."""
    return list(items[rank::world_size])


def broadcast_parameters(module: nn.Module, src: int = 0) -> None:
    """Make every rank start from rank ``src``'s parameters and buffers."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src)


class GradBucket:
    """One flat fp32 gradient buffer for all trainable parameters (grads are views into it).

    The buffer has two segments: the *early* parameters first (default: a MoleculeModel's FFN head,
    whose gradients the direct training step has finished before it enqueues the encoder backward),
    then the rest.  :meth:`start_early` all-reduces the early segment while the encoder backward still
    runs on the compute stream (RCCL runs the collective on its own stream, ordered after the work
    enqueued so far); :meth:`start_allreduce` then launches the rest and :meth:`finish_allreduce` waits
    for both.  Every rank issues the same two collectives in the same order (the early one from
    :meth:`start_allreduce` when :meth:`start_early` was not called), so ranks on different step paths
    stay matched."""

    def __init__(self, module: nn.Module, early: Sequence[nn.Parameter] = None):
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError('module has no trainable parameters')
        if early is None:
            ffn = getattr(module, 'ffn', None)
            early = list(ffn.parameters()) if isinstance(ffn, nn.Module) else []
        ids = {id(p) for p in early}
        self.params = [p for p in params if id(p) in ids] + [p for p in params if id(p) not in ids]
        self.n_early = sum(p.numel() for p in self.params if id(p) in ids)
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.buffer = torch.zeros(n, dtype=torch.float32, device=dev)
        self._works = []
        self._early_started = False
        off = 0
        for p in self.params:
            if p.dtype != torch.float32:
                raise TypeError('GradBucket expects float32 parameters')
            p.grad = self.buffer[off:off + p.numel()].view_as(p)
            off += p.numel()

    def zero(self) -> None:
        """Zero in place (keeps the views; use instead of ``zero_grad(set_to_none=True)``)."""
        self.buffer.zero_()
        for p, v in zip(self.params, self._views()):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v  # a grad replaced by an optimizer / user: re-attach the view

    def attach(self) -> None:
        """Re-attach the views as the parameters' gradients without zeroing (a step that overwrites every
        gradient: train.py's direct path)."""
        for p, v in zip(self.params, self._views()):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def _views(self) -> Iterable[torch.Tensor]:
        off = 0
        for p in self.params:
            yield self.buffer[off:off + p.numel()].view_as(p)
            off += p.numel()

    @staticmethod
    def _multi_rank() -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def _launch(self, seg: torch.Tensor) -> None:
        if self.buffer.is_cuda and dist.get_backend() == 'gloo':
            # gloo stages CUDA tensors through host memory; measured on ROCm: without draining the
            # producing stream first it can read the bucket before the backward kernels have written
            # it (RCCL orders the collective after the stream's work by itself)
            torch.cuda.current_stream(self.buffer.device).synchronize()
        self._works.append(dist.all_reduce(seg, op=dist.ReduceOp.SUM, async_op=True))

    def start_early(self) -> None:
        """Launch the early segment's all-reduce (async_op) once its gradients are enqueued: on RCCL it
        overlaps the rest of the backward.  No-op on one rank or without an early segment."""
        if self.n_early and not self._early_started and self._multi_rank():
            self._launch(self.buffer[:self.n_early])
            self._early_started = True

    def start_allreduce(self) -> None:
        """Launch the sum over ranks of what :meth:`start_early` has not launched (async_op) once the
        backward's last gradient kernel is enqueued; :meth:`finish_allreduce` waits for every launched
        collective (on the stream, not the host, with RCCL) and divides by the world size."""
        for p, v in zip(self.params, self._views()):
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                if self._early_started:
                    raise RuntimeError('a gradient was replaced after its segment was all-reduced')
                v.copy_(p.grad)  # autograd created a fresh tensor: fold it into the bucket
                p.grad = v
        if self._multi_rank():
            # the same collectives on every rank whichever step path it took (the direct step calls
            # start_early, the autograd path does not): with an early segment always two, early then rest,
            # so ranks never disagree on the count or sizes of their all-reduces
            if self.n_early and not self._early_started:
                self._launch(self.buffer[:self.n_early])
            if self.n_early < self.buffer.numel():
                self._launch(self.buffer[self.n_early:])

    def finish_allreduce(self) -> None:
        works, self._works, self._early_started = self._works, [], False
        for w in works:
            w.wait()  # (RCCL: the current stream waits for the collective's stream)
        if works:
            self.buffer.div_(dist.get_world_size())

    def allreduce_mean(self) -> None:
        """Sum the bucket over ranks (one collective) and divide by the world size."""
        self.start_allreduce()
        self.finish_allreduce()

    @property
    def nbytes(self) -> int:
        return self.buffer.numel() * 4
