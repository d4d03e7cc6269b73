"""Streamed synthetic batches (BASELINE.json configs[4]: 10 M random polymer graphs sharded data-parallel
over the GPUs of a node; SURVEY §8(d) "10 M-graph DP", §7 "materialised f_bonds would be ~564 GB").

Nothing is materialised: every batch is generated on the fly, per rank, from its own seed, in compact
form (include/wdmpnn.h "Compact graphs": ~14 bytes per directed edge) and expanded on the GPU.

    producer threads (native, GIL released)     feed stream                compute stream
    generate + block plan + stage  --pinned-->  H2D + wdmpnn_build_graph  --event-->  forward / train step

* ``producers`` threads run ``_wdpack.generate_stage`` (csrc/compact.hpp) for batches t, t + P, ...
  into a ring of R pinned host slots.  Batch i goes to slot i % R, and only on that slot's turn: the slot
  carries the index of the next batch allowed to write it (i, then i + R once the consumer has issued
  the H2D of batch i), so batches arrive in order whatever the thread timing.  A slot is rewritten only
  after the H2D that read it has completed (its CUDA event), so nothing is copied twice and nothing is
  overwritten early.
* The consumer (the caller's thread) takes the batches in order.  It enqueues the batch's H2D and graph
  build on a feed stream; the caller's forward waits on the graph's ready event on its own stream
  (``DeviceGraph.use_on``), so batch i + 1 is uploaded and built while batch i is encoded.
* Seeds: batch i of rank r uses ``seed + (r << 32) + i``: ranks never share a batch (disjoint shards, no
  collective on the data path).
"""
from __future__ import annotations

import threading
from typing import Iterator, Optional

import torch

from .featurization import BLK_TARGET, BatchMolGraph, _packer, upload_compact

KINDS = {'polymer': 0, 'qm9': 1, 'zinc': 2}
_MAX_ATOMS = {'polymer': 48, 'qm9': 9, 'zinc': 37}


def stage_capacity(kind: str, batch_size: int) -> int:
    """Bytes of one staged image for a batch of ``batch_size`` graphs of ``kind`` (upper bound)."""
    a = _MAX_ATOMS[kind]
    pairs = a + a // 5 + (10 if kind == 'polymer' else 0)
    return batch_size * (16 * a + 16 * pairs + 16 + 4 + 40) + 16 + 8 * 256


class StreamedBatches:
    """Iterator over ``n_batches`` generated batches of ``batch_size`` graphs as device-resident
    ``BatchMolGraph`` objects (their graph built on the GPU).  ``keep_host`` also keeps each batch's
    compact arrays (``batch._compact``) so that a test can check it against the oracle."""

    def __init__(self, kind: str, batch_size: int, n_batches: int, seed: int, device, rank: int = 0,
                 producers: int = 4, slots: Optional[int] = None, keep_host: bool = False,
                 target_blocks: int = BLK_TARGET, lean: bool = False):
        if kind not in KINDS:
            raise ValueError(f'unknown kind {kind!r}')
        self.kind, self.B, self.n, self.device = kind, int(batch_size), int(n_batches), torch.device(device)
        self.seed0 = (int(seed) + (int(rank) << 32)) & 0xFFFFFFFFFFFFFFFF
        self.P = max(1, int(producers))
        self.R = max(self.P + 2, int(slots or 0))
        self.keep = keep_host
        self.lean = bool(lean)  # inference-only device graphs (upload_compact lean)
        self.target = target_blocks
        self.cap = stage_capacity(kind, self.B)
        self.host = [torch.empty(self.cap, dtype=torch.uint8, pin_memory=True) for _ in range(self.R)]
        self.info = [None] * self.R
        self.full = [threading.Event() for _ in range(self.R)]
        self.turn = list(range(self.R))  # per slot: the batch index allowed to write it next
        self.cv = threading.Condition()
        self.copy_done = [None] * self.R  # CUDA event after the H2D that read the slot
        self.feed = torch.cuda.Stream(self.device)
        self.error = None
        self.stop = False
        self.threads = [threading.Thread(target=self._produce, args=(t,), daemon=True) for t in range(self.P)]
        for th in self.threads:
            th.start()

    def _produce(self, t: int) -> None:
        P = _packer()
        try:
            for i in range(t, self.n, self.P):
                s = i % self.R
                with self.cv:
                    while self.turn[s] != i:
                        if self.stop:
                            return
                        self.cv.wait(0.1)
                if self.copy_done[s] is not None:
                    self.copy_done[s].synchronize()  # the previous H2D out of this slot has run
                res = P.generate_stage(KINDS[self.kind], self.B, (self.seed0 + i) & 0xFFFFFFFFFFFFFFFF, self.target,
                                       self.host[s].data_ptr(), self.cap, self.keep)
                if res is None:
                    raise RuntimeError('generated molecule exceeds a block')
                info, arrays = res if self.keep else (res, None)
                if not info[0]:
                    raise RuntimeError(f'staged batch larger than the slot ({info[3]} > {self.cap} bytes)')
                self.info[s] = (i, info, arrays)
                self.full[s].set()
        except BaseException as e:  # surfaced by the consumer
            self.error = e
            for ev in self.full:
                ev.set()

    def __iter__(self) -> Iterator[BatchMolGraph]:
        try:
            for i in range(self.n):
                s = i % self.R
                self.full[s].wait()
                if self.error is not None:
                    raise RuntimeError('stream producer failed') from self.error
                self.full[s].clear()
                idx, info, arrays = self.info[s]
                if idx != i:
                    raise RuntimeError(f'stream slot {s} holds batch {idx}, expected {i}')
                with torch.cuda.stream(self.feed):
                    dg = upload_compact(self.device, self.host[s], info, 133, 147, lean=self.lean)
                    ev = torch.cuda.Event()
                    ev.record(self.feed)
                self.copy_done[s] = ev
                with self.cv:
                    self.turn[s] = i + self.R
                    self.cv.notify_all()
                yield _device_batch(dg, info, arrays)
        finally:
            self.close()

    def close(self) -> None:
        with self.cv:
            self.stop = True
            self.cv.notify_all()
        for th in self.threads:
            th.join()


def _device_batch(dg, info, arrays) -> BatchMolGraph:
    """A BatchMolGraph whose device graph is already built (scope sizes only on the host; with
    ``arrays`` the compact arrays too, decoded on access like ``BatchMolGraph.from_compact``)."""
    if arrays is not None:
        g = BatchMolGraph.from_compact(*arrays)
    else:
        g = BatchMolGraph.__new__(BatchMolGraph)
        g.overwrite_default_atom_features = g.overwrite_default_bond_features = False
        g.atom_fdim, g.bond_fdim = 133, 147
        g._compact = None
        g._a2b = g._gathers = g.b2b = g.a2a = None
        g._device_cache = {}
    n_mols, n_atoms, n_bonds = info[1][:3]
    g.n_atoms, g.n_bonds, g.n_mols = n_atoms, n_bonds, n_mols
    dev = str(dg.device)
    g._device_cache[(dev, False, None)] = dg
    g._device_cache[(dev, False, 147)] = dg
    return g
