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

import ctypes
import os
import threading
from typing import Iterator, Optional, Tuple

import torch

from .featurization import BLK_TARGET, BatchMolGraph, _packer, upload_compact

KINDS = {'polymer': 0, 'qm9': 1, 'zinc': 2}
_MAX_ATOMS = {'polymer': 48, 'qm9': 9, 'zinc': 37}


def usable_cores(fallback: int = 1) -> Tuple[int, int, Optional[int]]:
    """(usable, affinity, quota): the CPUs this process may run on -- its affinity set, capped by the
    cgroup v2 CPU quota (a GPU box shares its host: the affinity set can list every CPU of the machine
    while the quota is its share)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or fallback
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, period = f.read().split()[:2]
        if q != 'max':
            quota = max(1, int(-(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return (min(affinity, quota) if quota else affinity), affinity, quota


def producer_cap(local_world: Optional[int] = None) -> int:
    """Generator threads one rank may run: max(2, usable cores // ranks on this node - 2) (the ranks of a
    node share its cores; two stay for the rank's feeder and Python threads).  A rank's stream saturates
    at ~4 producers (profiles/round3_stream_sweep.txt), so the cap only bites on small CPU shares."""
    if local_world is None:
        local_world = int(os.environ.get('LOCAL_WORLD_SIZE', '1'))
    return max(2, usable_cores()[0] // max(1, local_world) - 2)


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


class _FeedGraph:
    """DeviceGraph of a batch handed out by a NativeFeed: device memory owned by the feed's slot (valid
    until the feed reuses the slot, after the consumer's release), already waited for on ``home``.  The
    feed marks it expired when it releases the slot: any later use raises instead of reading a slot that
    may hold another batch."""

    def __init__(self, struct, info, device, home):
        self.struct = struct
        self.device = device
        self.buffer = None
        self.views = {}
        self.encoder_structs = {}
        self.encoder_plans = {}
        self.home_stream = home
        self._streams = {home}
        self._ready = None
        self.n_edges = info.n_bonds - 1
        self.h2d_bytes = int(info.h2d_bytes)
        self.nnz_msg = info.nnz_msg
        self.built_on_device = True
        self.lean = False
        self.index = info.index
        self.expired = False

    def use_on(self, stream) -> None:
        if self.expired:
            raise RuntimeError(f'streamed batch {self.index} was released: a NativeFeed batch is valid only until '
                               'the next one is requested (encode it inside the loop, or copy what you keep)')
        sid = stream.cuda_stream
        if sid in self._streams:
            return
        if self._ready is None:  # order the other stream after the home stream's wait on the build
            self._ready = torch.cuda.Event()
            self._ready.record(torch.cuda.ExternalStream(self.home_stream, device=self.device))
        stream.wait_event(self._ready)
        self._streams.add(sid)


class NativeFeed:
    """Streamed synthetic batches produced natively (``wdmpnn_feed_*``, csrc/feed.hpp): ``producers``
    generator threads stage compact batches into pinned slots, a feed thread uploads each one and builds
    its device graph on its own HIP stream; this object only hands out finished graphs (no Python in the
    data path, no GIL held by the pipeline).  Batch i of rank r is generated from
    ``seed + (r << 32) + i``, like :class:`StreamedBatches`, whose order and content it reproduces.

    * iteration yields device-resident ``BatchMolGraph`` objects in order; the batch handed out last is
      released (its slot may be reused) when the next one is requested, after the work enqueued for it on
      the current stream -- a batch kept past that point (``list(feed)``, a look-ahead) raises on use;
    * the feed's threads write its pinned and device buffers from creation on: iterate it to the end, or
      ``close()`` it (a ``with`` block, or garbage collection, does so) before dropping it;
    * :meth:`encode` runs the whole stream through an encoder's fused inference forward, ``k`` batches
      per launch set (``wdmpnn_feed_forward``)."""

    def __init__(self, kind: str, batch_size: int, n_batches: int, seed: int, device, rank: int = 0,
                 producers: int = 4, slots: Optional[int] = None, lean: bool = False,
                 target_blocks: int = BLK_TARGET, atom_fdim: int = 133, bond_fdim: int = 147,
                 planes: bool = True):
        from . import _native
        if kind not in KINDS:
            raise ValueError(f'unknown kind {kind!r}')
        self.L = L = _native.lib()
        self.device = torch.device(device)
        self.kind, self.B, self.n = kind, int(batch_size), int(n_batches)
        self.producers = min(max(1, int(producers)), producer_cap())  # (threads per rank: producer_cap)
        self.R = max(int(slots or 0), self.producers + 2, 4)
        hb, db = ctypes.c_size_t(), ctypes.c_size_t()
        _native.check(L.wdmpnn_feed_slot_bytes(KINDS[kind], self.B, atom_fdim, bond_fdim, ctypes.byref(hb),
                                               ctypes.byref(db)), 'feed slot bytes')
        self.pinned = torch.empty(self.R * hb.value, dtype=torch.uint8, pin_memory=True)
        self.arena = torch.empty(self.R * db.value + 256, dtype=torch.uint8, device=self.device)
        base = (self.arena.data_ptr() + 255) & ~255
        spec = _native.WdFeedSpec()
        spec.kind, spec.batch, spec.n_batches = KINDS[kind], self.B, self.n
        spec.seed = (int(seed) + (int(rank) << 32)) & 0xFFFFFFFFFFFFFFFF
        spec.producers, spec.slots, spec.target_blocks = self.producers, self.R, int(target_blocks)
        # planes=False: no bf16 plane tiles of the feature rows (WDMPNN_GRAPH_NO_PLANES) -- the fused forward
        # and backward of these categorical-code graphs never read them (training streams)
        spec.flags = (_native.GRAPH_LEAN if lean else 0) | (0 if planes else _native.GRAPH_NO_PLANES)
        spec.atom_fdim, spec.bond_fdim = atom_fdim, bond_fdim
        spec.pinned, spec.device = self.pinned.data_ptr(), base
        self.lean = bool(lean)
        self.fdims = (atom_fdim, bond_fdim)
        self.seed_range = (spec.seed, spec.seed + self.n)  # batch i: seed_range[0] + i
        self.handle = ctypes.c_void_p()
        _native.check(L.wdmpnn_feed_create(ctypes.byref(spec), ctypes.byref(self.handle)), 'feed create')
        self._native = _native

    def __enter__(self):
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # (interpreter shutdown)
            pass

    def __iter__(self) -> Iterator[BatchMolGraph]:
        L, check = self.L, self._native.check
        prev = None
        try:
            while True:
                stream = torch.cuda.current_stream(self.device)
                if prev is not None:
                    prev.expired = True
                    prev._streams = set()  # (so the inference path's stream check reaches use_on, which raises)
                check(L.wdmpnn_feed_release(self.handle, stream.cuda_stream), 'feed release')
                g = self._native.WdGraph()
                info = self._native.WdFeedBatch()
                rc = L.wdmpnn_feed_next(self.handle, stream.cuda_stream, ctypes.byref(g), ctypes.byref(info))
                if rc == 1:
                    return
                check(rc, 'feed next')
                dg = prev = _FeedGraph(g, info, self.device, stream.cuda_stream)
                dg.lean = self.lean
                yield _device_batch(dg, ((True,), (info.n_mols, info.n_atoms, info.n_bonds)), None)
        finally:
            self.close()

    def encode(self, enc, k: int = 8):
        """Run every remaining batch through ``enc``'s fused inference forward, k batches per launch set.
        Yields (out [rows, H] tensor, batches, directed edges, H2D bytes) per call."""
        nat = self._native
        L = self.L
        try:  # (the setup too: a failure there still stops the feed's threads)
            params = enc._param_tuple()
            stream = torch.cuda.current_stream(self.device)
            cfg = enc._config(False)
            dummy = nat.WdGraph()  # sizes only: the packed-parameter layout depends on the feature widths
            dummy.n_atoms = dummy.n_bonds = 1
            dummy.atom_fdim, dummy.bond_fdim = self.fdims
            dummy.ld_atoms = dummy.ld_bonds = -(-max(self.fdims) // 32) * 32
            dummy.f_atoms = dummy.f_bonds = self.arena.data_ptr() & ~255
            pstruct, _ = enc._packed_params(dummy, cfg, tuple(t for t in params), self.device, stream=stream)
            wsb = ctypes.c_size_t()
            nat.check(L.wdmpnn_feed_forward_workspace_bytes(self.handle, ctypes.byref(pstruct), ctypes.byref(cfg), k,
                                                            ctypes.byref(wsb)), 'feed workspace')
            H = enc.hidden_size
            got, rows, edges, h2d = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            while True:
                ws = torch.empty(wsb.value, dtype=torch.uint8, device=self.device)
                out = torch.empty((k * self.B, H), dtype=torch.float32, device=self.device)
                nat.check(L.wdmpnn_feed_forward(self.handle, k, ctypes.byref(pstruct), ctypes.byref(cfg), ws.data_ptr(),
                                                wsb.value, out.data_ptr(), k * self.B, stream.cuda_stream,
                                                ctypes.byref(got), ctypes.byref(rows), ctypes.byref(edges),
                                                ctypes.byref(h2d)), 'feed forward')
                if got.value == 0:
                    return
                yield out[:rows.value], got.value, edges.value, h2d.value
        finally:
            self.close()

    def close(self) -> None:
        """Stop the feed's threads and free its native state (idempotent).  The pinned and device buffers
        stay referenced by this object until then, so nothing native writes freed memory."""
        if getattr(self, 'handle', None):
            torch.cuda.current_stream(self.device).synchronize()  # the slots' last readers
            self.L.wdmpnn_feed_destroy(self.handle)
            self.handle = ctypes.c_void_p()
