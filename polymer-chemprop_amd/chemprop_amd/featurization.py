"""BatchMolGraph with the reference's API plus a CSR-packed, device-resident layout.

Reference: ``chemprop/features/featurization.py`` (``BatchMolGraph`` 742-875, ``get_atom_fdim`` 68-75,
``get_bond_fdim`` 150-167, ``mol2graph`` 878-898).

``BatchMolGraph(mol_graphs)`` accepts objects with the attributes of the reference ``MolGraph``
(``f_atoms, f_bonds, w_atoms, w_bonds, a2b, b2a, b2revb, n_atoms, n_bonds, degree_of_polym,
overwrite_default_*``) and exposes the same public attributes and methods (``n_atoms, n_bonds,
a_scope, b_scope, max_num_bonds, degree_of_polym, atom_fdim, bond_fdim, f_atoms, f_bonds, w_atoms,
w_bonds, a2b, b2a, b2revb, get_components, get_a2a, get_b2b``) with identical values: index 0 is the
zero pad atom / bond (featurization.py:767-781), ``a2b`` is padded with 0 to ``max_num_bonds``
(featurization.py:802-809).  Packing is vectorised numpy instead of per-element Python loops
(featurization.py:782-811 take ~77 ms per 64 polymers).

``device_graph(device, ...)`` adds what the HIP kernels consume: row-gather lists (CSR, int32 + fp32
coefficients) that express the reference's padded gathers and their transposes, and the float
arrays with 16-byte aligned row strides, all in ONE device buffer filled by one pinned H2D copy.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import _native

# featurization.py:19-45 defaults: ATOM_FDIM = 133, BOND_FDIM = 14
_PARAMS = {'ATOM_FDIM': 133, 'EXTRA_ATOM_FDIM': 0, 'BOND_FDIM': 14, 'EXTRA_BOND_FDIM': 0}


def get_atom_fdim(overwrite_default_atom: bool = False) -> int:
    """featurization.py:68-75."""
    return (not overwrite_default_atom) * _PARAMS['ATOM_FDIM'] + _PARAMS['EXTRA_ATOM_FDIM']


def get_bond_fdim(atom_messages: bool = False, overwrite_default_bond: bool = False,
                  overwrite_default_atom: bool = False) -> int:
    """featurization.py:150-167."""
    return (not overwrite_default_bond) * _PARAMS['BOND_FDIM'] + _PARAMS['EXTRA_BOND_FDIM'] + \
        (not atom_messages) * get_atom_fdim(overwrite_default_atom=overwrite_default_atom)


def set_extra_atom_fdim(extra: int) -> None:
    _PARAMS['EXTRA_ATOM_FDIM'] = extra


def set_extra_bond_fdim(extra: int) -> None:
    _PARAMS['EXTRA_BOND_FDIM'] = extra


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


CSR_PAD = 8  # WdCsr: idx / coef readable 8 entries past the end (branch-free first-8 fetch)
BLK_BONDS, BLK_ATOMS, BLK_MOLS = 128, 64, 64  # molecule-block capacity of the fused forward (WdGraph.blocks)
BLK_TARGET = 64  # blocks a batch is spread over at least (x 4-5 column tiles = one workgroup per CU)


class Csr:
    """Row-gather list: row r = sum_{e in [ptr[r], ptr[r+1])} coef[e] * source[idx[e]]."""

    def __init__(self, ptr: np.ndarray, idx: np.ndarray, coef: np.ndarray):
        self.ptr = np.ascontiguousarray(ptr, dtype=np.int32)
        self.idx = np.ascontiguousarray(idx, dtype=np.int32)
        self.coef = np.ascontiguousarray(coef, dtype=np.float32)

    @property
    def rows(self) -> int:
        return len(self.ptr) - 1

    @staticmethod
    def from_rows(row_of_entry: np.ndarray, idx: np.ndarray, coef: np.ndarray, n_rows: int) -> 'Csr':
        """Build from unsorted (row, idx, coef) triples; entries keep their order within a row."""
        order = np.argsort(row_of_entry, kind='stable')
        counts = np.bincount(row_of_entry, minlength=n_rows)
        ptr = np.zeros(n_rows + 1, np.int64)
        np.cumsum(counts, out=ptr[1:])
        return Csr(ptr, idx[order], coef[order])

    def transpose(self, n_src_rows: int) -> 'Csr':
        """Gradient of the gather: dSrc[j] = sum over entries (r, j, c) of c * dRow[r]."""
        rows = np.repeat(np.arange(self.rows, dtype=np.int64), np.diff(self.ptr))
        return Csr.from_rows(self.idx.astype(np.int64), rows, self.coef, n_src_rows)

    def apply(self, source: np.ndarray) -> np.ndarray:
        """Host evaluation (used by the CPU tests of the packing logic)."""
        rows = np.repeat(np.arange(self.rows), np.diff(self.ptr))
        out = np.zeros((self.rows,) + source.shape[1:], np.float64)
        np.add.at(out, rows, self.coef[:, None].astype(np.float64) * source[self.idx].astype(np.float64))
        return out


ELLW = 8  # gather entries per row held in the block-local ELL form (WdGraph.*_ell_*)


def ell_rows(c: 'Csr', rows_p: int, base: np.ndarray, width: int = ELLW):
    """First ``width`` entries of every CSR row in block-local form (WdGraph.*_ell_idx / *_ell_coef):
    index idx - base[row] as uint8 (< 128), coefficient; unused slots (index 0, coef 0); bit 7 of the
    last slot set on rows with more entries (the kernels take the rest from the CSR list).  Built by
    the native packer (csrc/packer.cpp ``ell``)."""
    idx, coef = _packer().ell(c.ptr, c.idx, c.coef, int(rows_p), np.ascontiguousarray(base[:c.rows], np.int64),
                              int(width))
    return np.frombuffer(idx, np.uint8), np.frombuffer(coef, np.float32)


def _packer():
    """The native packer extension (built in-tree by __graft_entry__.build()); no Python fallback."""
    try:
        from . import _wdpack
    except ImportError as e:  # pragma: no cover - exercised only on an unbuilt tree
        raise ImportError('chemprop_amd._wdpack is not built: run `python -c "import __graft_entry__ as g; '
                          'g.build()"` (g++ csrc/packer.cpp)') from e
    return _wdpack


class DeviceGraph:
    """Device-resident packed graph + the ctypes ``WdGraph`` pointing into it.

    Its uploads and device-side builds run on the stream current at ``device_graph()`` time (the home
    stream) and end with an event.  ``use_on(stream)`` makes another stream wait for that event and
    records the graph's allocations as used by that stream (``record_stream``), so a graph may be
    encoded on any stream and freed while another stream still reads it."""

    def __init__(self, buffer: torch.Tensor, views: Dict[str, torch.Tensor], struct: '_native.WdGraph'):
        self.buffer = buffer
        self.views = views
        self.struct = struct
        self.device = buffer.device
        self.encoder_structs = {}  # (atom_fdim, bond_fdim) -> the WdGraph copy an encoder passes (mpn.py)
        self.encoder_plans = {}  # (encoder token, encoder config) -> cached inference call (MPNEncoder._infer)
        self.ready = None  # event after the uploads / builds on the home stream
        self.home_stream = None
        self._streams = set()

    def finish(self) -> None:
        """Record the ready event on the current (home) stream; called once the graph is built."""
        if self.device.type == 'cuda':
            st = torch.cuda.current_stream(self.device)
            self.ready = torch.cuda.Event()
            self.ready.record(st)
            self.home_stream = st.cuda_stream
            self._streams.add(st.cuda_stream)

    def use_on(self, stream) -> None:
        """Order ``stream`` after the graph's build and keep its memory alive for that stream's work.
        (Callers on a hot path test ``sid in dg._streams`` with the raw stream id first: a repeat costs
        nothing.)"""
        sid = stream.cuda_stream
        if sid in self._streams:
            return
        if self.ready is not None and not self.ready.query():  # (a finished build needs no wait)
            stream.wait_event(self.ready)
        cached = self.__dict__.get('_owners')
        if cached is None or cached[0] != len(self.views):
            # one tensor per distinct allocation (the views share a few), found once: the per-view storage
            # walk cost a first use on a stream tens of us of host time
            seen, owners = set(), []
            for t in [self.buffer] + list(self.views.values()):
                if t is None:
                    continue
                base = t.untyped_storage().data_ptr()
                if base not in seen:
                    seen.add(base)
                    owners.append(t)
            cached = self._owners = (len(self.views), owners)
        for t in cached[1]:
            t.record_stream(stream)
        self._streams.add(sid)


class BatchMolGraph:
    """featurization.py:742-875; the tables are concatenated by the native packer (csrc/packer.cpp)."""

    def __init__(self, mol_graphs: Sequence, device_bond_features: bool = False, check_bond_features: bool = False,
                 compact: bool = True, block_target: int = BLK_TARGET):
        """``device_bond_features``: keep only the bond-feature tail of every f_bonds
        row on the host (the reference builds each row as ``f_atoms[b2a] ‖ bond features``,
        featurization.py:467-468, 545-546, 616-617); ``check_bond_features`` verifies that layout while
        packing (ValueError otherwise).  Without it the full rows are packed and the layout is checked
        here before the compact form is used.

        ``compact`` (default): when every row is in the reference's categorical layout (one-hot atom
        columns + mass, binary bond columns, bonds in reverse pairs, featurization.py:190-250, 469-480)
        the batch also gets its compact codes (include/wdmpnn.h "Compact graphs", ~14 bytes per edge) and
        ``device_graph`` builds every device array from them on the GPU (``wdmpnn_build_graph``).
        Other batches (extra / overwritten features, atom messages, molecules larger than a block) take
        the host-built path: gather lists packed here, fp32 rows uploaded.

        ``block_target``: the molecule blocks a small batch is spread over at least (``molecule_blocks``).
        The default (BLK_TARGET) cuts a small batch into many part-filled blocks, so that ONE forward spreads
        over the CUs; batches that are encoded several per launch (``MPNEncoder.forward_many``) are better
        packed into full blocks (``block_target=1``): the launch then has enough workgroups anyway and each
        one streams W_h once for a full block instead of a sliver.  Results do not depend on the plan."""
        self.block_target = int(block_target)
        self.overwrite_default_atom_features = mol_graphs[0].overwrite_default_atom_features
        self.overwrite_default_bond_features = mol_graphs[0].overwrite_default_bond_features
        self.atom_fdim = get_atom_fdim(overwrite_default_atom=self.overwrite_default_atom_features)
        self.bond_fdim = get_bond_fdim(overwrite_default_bond=self.overwrite_default_bond_features,
                                       overwrite_default_atom=self.overwrite_default_atom_features)
        fa_w = next((len(g.f_atoms[0]) for g in mol_graphs if g.n_atoms), self.atom_fdim)
        fb_w = next((len(g.f_bonds[0]) for g in mol_graphs if g.n_bonds), self.bond_fdim)
        # native packer (csrc/packer.cpp): concatenation at the reference's offsets, pad row 0
        # (featurization.py:767-793), a2b as CSR (deg + in_idx in slot order)
        tail_from = int(fa_w) if device_bond_features else 0
        (f_atoms, f_bonds, w_atoms, w_bonds, b2a, b2revb, deg, in_idx, na, nb) = \
            _packer().pack(mol_graphs, int(fa_w), int(fb_w), tail_from, bool(check_bond_features))
        na = np.frombuffer(na, np.int64)
        nb = np.frombuffer(nb, np.int64)
        V, E = int(na.sum()), int(nb.sum())
        f_atoms = np.frombuffer(f_atoms, np.float32).reshape(V + 1, fa_w)
        f_bonds = np.frombuffer(f_bonds, np.float32).reshape(E + 1, fb_w - tail_from)
        w_atoms = np.frombuffer(w_atoms, np.float32)
        w_bonds = np.frombuffer(w_bonds, np.float32)
        b2a = np.frombuffer(b2a, np.int64)
        b2revb = np.frombuffer(b2revb, np.int64)
        deg = np.frombuffer(deg, np.int64)
        a_off = 1 + np.concatenate([[0], np.cumsum(na)[:-1]]).astype(np.int64)
        b_off = 1 + np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64)
        self.n_atoms = V + 1
        self.n_bonds = E + 1
        self.a_scope: List[Tuple[int, int]] = [(int(s), int(n)) for s, n in zip(a_off, na)]
        self.b_scope: List[Tuple[int, int]] = [(int(s), int(n)) for s, n in zip(b_off, nb)]
        self.degree_of_polym = [g.degree_of_polym for g in mol_graphs]
        in_ptr = np.zeros(V + 2, np.int64)
        np.cumsum(deg, out=in_ptr[1:])
        self._in_ptr = in_ptr
        self._in_idx = np.frombuffer(in_idx, np.int64)
        self._deg = deg
        self.max_num_bonds = max(1, int(deg.max()) if len(deg) else 0)  # featurization.py:802-803

        self._np = dict(f_atoms=f_atoms, w_atoms=w_atoms, w_bonds=w_bonds, b2a=b2a, b2revb=b2revb)
        if device_bond_features:
            self._np['bond_tail'] = f_bonds  # [E+1][fb_w - fa_w]; the full rows are rebuilt on demand
            self._f_bonds = None
        else:
            self._np['f_bonds'] = f_bonds
            self._f_bonds = torch.from_numpy(f_bonds)
        self.f_atoms = torch.from_numpy(f_atoms)
        self.w_atoms = torch.from_numpy(w_atoms)
        self.w_bonds = torch.from_numpy(w_bonds)
        self.b2a = torch.from_numpy(b2a)
        self.b2revb = torch.from_numpy(b2revb)
        self._a2b = None
        self._gathers = None
        self.b2b = None
        self.a2a = None
        self._device_cache: Dict[tuple, DeviceGraph] = {}
        self._compact = None  # (mols, xn, atoms, pairs) bytearrays, or None
        self._compact_why = 'disabled'
        if compact:
            self._compact_why = self._encode_compact(na, nb, device_bond_features)

    def _encode_compact(self, na: np.ndarray, nb: np.ndarray, tail_mode: bool) -> str:
        """Compact codes of the packed batch (csrc/compact.hpp ``encode``); returns why not, or ''."""
        fa = self._np['f_atoms']
        rows = self._np['bond_tail'] if tail_mode else self._np['f_bonds']  # full rows: layout checked natively
        tail_w = rows.shape[1] if tail_mode else rows.shape[1] - fa.shape[1]
        if tail_w < 0:
            return 'bond rows narrower than atom rows'
        res = _packer().compact_encode(fa, rows, self._np['w_atoms'], self._np['w_bonds'], self._np['b2a'],
                                       self._np['b2revb'], self._deg, self._in_idx, na, nb,
                                       np.asarray(self.degree_of_polym, np.float64), int(fa.shape[1]), int(tail_w))
        if res[0] is None:
            return res[1]
        self._compact = tuple(res)
        self._compact_dims = (int(fa.shape[1]), int(fa.shape[1] + tail_w))
        return ''

    @classmethod
    def from_compact(cls, mols, xn, atoms, pairs, atom_fdim: int = 133, bond_fdim: int = 147) -> 'BatchMolGraph':
        """A batch given in compact form (e.g. ``chemprop_amd.stream``'s native generator): scope arrays
        now, the reference's tables (f_atoms, f_bonds, a2b, ...) decoded natively on first access."""
        self = cls.__new__(cls)
        self.overwrite_default_atom_features = False
        self.overwrite_default_bond_features = False
        self.atom_fdim, self.bond_fdim = int(atom_fdim), int(bond_fdim)
        m = np.frombuffer(mols, np.int32).reshape(-1, 4)
        self.n_atoms = len(atoms) // 16
        self.n_bonds = 1 + 2 * (len(pairs) // 16)
        self.a_scope = [(int(a), int(n)) for a, n in zip(m[:, 0], m[:, 1])]
        self.b_scope = [(int(b), int(n)) for b, n in zip(m[:, 2], m[:, 3])]
        self.degree_of_polym = np.frombuffer(xn, np.float32).astype(np.float64).tolist()
        self._compact = (mols, xn, atoms, pairs)
        self._compact_dims = (self.atom_fdim, self.bond_fdim)
        self._compact_why = ''
        self._a2b = None
        self._gathers = None
        self.b2b = None
        self.a2a = None
        self._device_cache = {}
        return self

    _LAZY = ('f_atoms', 'w_atoms', 'w_bonds', 'b2a', 'b2revb', '_np', '_deg', '_in_idx', '_in_ptr', '_f_bonds',
             'max_num_bonds')

    def __getattr__(self, name):
        # only reached for attributes not set yet: a from_compact batch decodes its tables once
        if name in BatchMolGraph._LAZY and self.__dict__.get('_compact') is not None and '_np' not in self.__dict__:
            self._decode_compact()
            return self.__dict__[name]
        raise AttributeError(name)

    def _decode_compact(self) -> None:
        fa_w, fb_w = self._compact_dims
        (f_atoms, tail, w_atoms, w_bonds, b2a, b2revb, deg, in_idx, _, _) = \
            _packer().compact_decode(*self._compact, fa_w, fb_w)
        V1, E1 = self.n_atoms, self.n_bonds
        self._np = dict(f_atoms=np.frombuffer(f_atoms, np.float32).reshape(V1, fa_w),
                        w_atoms=np.frombuffer(w_atoms, np.float32), w_bonds=np.frombuffer(w_bonds, np.float32),
                        b2a=np.frombuffer(b2a, np.int64), b2revb=np.frombuffer(b2revb, np.int64),
                        bond_tail=np.frombuffer(tail, np.float32).reshape(E1, fb_w - fa_w))
        self._f_bonds = None
        self._deg = np.frombuffer(deg, np.int64)
        self._in_idx = np.frombuffer(in_idx, np.int64)
        in_ptr = np.zeros(V1 + 1, np.int64)
        np.cumsum(self._deg, out=in_ptr[1:])
        self._in_ptr = in_ptr
        self.max_num_bonds = max(1, int(self._deg.max()) if len(self._deg) else 0)
        self.f_atoms = torch.from_numpy(self._np['f_atoms'])
        self.w_atoms = torch.from_numpy(self._np['w_atoms'])
        self.w_bonds = torch.from_numpy(self._np['w_bonds'])
        self.b2a = torch.from_numpy(self._np['b2a'])
        self.b2revb = torch.from_numpy(self._np['b2revb'])

    # ------------------------------------------------------------------ reference API
    @property
    def f_bonds(self) -> torch.Tensor:
        """[n_bonds, bond_fdim] float32 (featurization.py:806); with device_bond_features, assembled on
        first access from f_atoms[b2a] ‖ bond tail (the layout the reference builds)."""
        if self._f_bonds is None:
            self._np['f_bonds'] = self._host_f_bonds()
            self._f_bonds = torch.from_numpy(self._np['f_bonds'])
        return self._f_bonds

    def _host_f_bonds(self) -> np.ndarray:
        fa, tail = self._np['f_atoms'], self._np['bond_tail']
        return np.ascontiguousarray(np.concatenate([fa[self._np['b2a']], tail], axis=1))

    @property
    def a2b(self) -> torch.Tensor:
        """[n_atoms, max_num_bonds] LongTensor padded with 0 (featurization.py:809)."""
        if self._a2b is None:
            V1 = self.n_atoms
            a2b = np.zeros((V1, self.max_num_bonds), np.int64)
            rows = np.repeat(np.arange(V1), self._deg)
            slot = np.arange(len(self._in_idx)) - np.repeat(self._in_ptr[:-1], self._deg)
            a2b[rows, slot] = self._in_idx
            self._a2b = torch.from_numpy(a2b)
        return self._a2b

    def get_components(self, atom_messages: bool = False):
        """featurization.py:815-846: the 10-tuple in the reference's order."""
        if atom_messages:
            f_bonds = self.f_bonds[:, -get_bond_fdim(atom_messages=atom_messages,
                                                     overwrite_default_atom=self.overwrite_default_atom_features,
                                                     overwrite_default_bond=self.overwrite_default_bond_features):]
        else:
            f_bonds = self.f_bonds
        return self.f_atoms, f_bonds, self.w_atoms, self.w_bonds, self.a2b, self.b2a, self.b2revb, \
            self.a_scope, self.b_scope, self.degree_of_polym

    def get_b2b(self) -> torch.Tensor:
        """featurization.py:848-860."""
        if self.b2b is None:
            b2b = self.a2b[self.b2a]
            revmask = (b2b != self.b2revb.unsqueeze(1).repeat(1, b2b.size(1))).long()
            self.b2b = b2b * revmask
        return self.b2b

    def get_a2a(self) -> torch.Tensor:
        """featurization.py:862-875."""
        if self.a2a is None:
            self.a2a = self.b2a[self.a2b]
        return self.a2a

    # ------------------------------------------------------------------ gather lists
    def _entries_of_in(self, atoms: np.ndarray):
        """(row position, bond id) pairs of in(atoms[r]) for every r, in a2b slot order."""
        counts = self._deg[atoms]
        rows = np.repeat(np.arange(len(atoms), dtype=np.int64), counts)
        starts = np.repeat(self._in_ptr[atoms], counts)
        slot = np.arange(len(rows), dtype=np.int64) - np.repeat(np.cumsum(counts) - counts, counts)
        return rows, self._in_idx[starts + slot]

    def _native_gathers(self):
        """(msg, agg, msg_t, agg_t) built by the native packer (csrc/packer.cpp ``gathers``), cached."""
        if self._gathers is None:
            out = _packer().gathers(self._np['b2a'], self._np['b2revb'], self._np['w_bonds'], self._deg,
                                    self._in_idx)
            self._gathers = tuple(Csr(np.frombuffer(p, np.int32), np.frombuffer(i, np.int32),
                                      np.frombuffer(c, np.float32)) for p, i, c in out)
        return self._gathers

    def bond_message_gather(self) -> Csr:
        """mpn.py:112-120 as a row gather over bonds, built natively (csrc/packer.cpp ``gathers``; the
        numpy restatement it is tested against is oracle/pack_ref.bond_message_gather):
        X_b = sum_{j in in(b2a[b])} w_j M_j - M_{b2revb[b]}.  The reverse bond normally is in
        in(b2a[b]); its coefficient becomes w_rev - 1 and is dropped when 0 (w = 1 bonds)."""
        return self._native_gathers()[0]

    def atom_message_gather(self) -> Tuple[Csr, Csr]:
        """mpn.py:104-108 (atom messages): nei_a = sum over a2b slots of M[a2a] (pad slots gather atom 0,
        whose message is act(b_i) != 0 with bias, hence the (0, max_num_bonds - deg) entry), and the
        bond-feature part sum_{j in in(a)} f_bonds[j]."""
        V1 = self.n_atoms
        atoms = np.arange(V1, dtype=np.int64)
        rows, j = self._entries_of_in(atoms)
        b2a = self._np['b2a']
        pad = self.max_num_bonds - self._deg
        prow = atoms[pad > 0]
        msg = Csr.from_rows(np.concatenate([rows, prow]), np.concatenate([b2a[j], np.zeros(len(prow), np.int64)]),
                            np.concatenate([np.ones(len(rows)), pad[prow]]).astype(np.float32), V1)
        feat = Csr.from_rows(rows, j, np.ones(len(rows), np.float32), V1)
        return msg, feat

    def atom_aggregate_gather(self, atom_messages: bool = False) -> Csr:
        """mpn.py:126-131: A_a = sum_{slots} M[a2x] * w_bonds[a2x] (a2x = a2b, or a2a in atom-message
        mode where the weights are w_bonds indexed by ATOM ids, a reference quirk kept as is)."""
        if not atom_messages:  # native (oracle/pack_ref.atom_aggregate_gather restates it)
            return self._native_gathers()[1]
        V1 = self.n_atoms
        rows, j = self._entries_of_in(np.arange(V1, dtype=np.int64))
        w = self._np['w_bonds']
        src = self._np['b2a'][j]
        if len(src) and src.max() >= len(w):
            raise IndexError('atom_messages readout indexes w_bonds with atom ids (mpn.py:128) and an atom id '
                             'exceeds the number of bonds')
        coef = w[src]
        keep = coef != 0.0
        return Csr.from_rows(rows[keep], src[keep], coef[keep], V1)

    def molecule_blocks(self, target_blocks: int = None):
        """Consecutive molecules grouped greedily into blocks of <= BLK_BONDS bond rows, <= BLK_ATOMS atom
        rows and <= BLK_MOLS molecules (WdGraph.blocks, int32 [n_blocks, 8]); None when a molecule alone
        exceeds a limit.  A batch too small to give ``target_blocks`` full blocks is cut into smaller
        ones (fill limit: the 16-row-rounded share of the bond rows, never below the largest molecule):
        every block is one workgroup per column tile, and the kernels skip the empty 16-row groups, so
        small batches spread over more CUs instead of a few full blocks."""
        if target_blocks is None:
            target_blocks = getattr(self, 'block_target', BLK_TARGET)
        nb = np.array([n for _, n in self.b_scope], np.int64)
        big = int(nb.max()) if len(nb) else 0
        share = -(-int(nb.sum()) // max(1, target_blocks))
        cap_b = min(BLK_BONDS, max(big, -(-share // 16) * 16))
        rows = []
        cur = None
        for i, ((as_, an), (bs, bn)) in enumerate(zip(self.a_scope, self.b_scope)):
            if bn > BLK_BONDS or an > BLK_ATOMS:
                return None
            if cur is not None and cur[1] + bn <= cap_b and cur[3] + an <= BLK_ATOMS and i - cur[4] < BLK_MOLS:
                cur[1] += bn
                cur[3] += an
                cur[5] = i + 1
            else:
                if cur is not None:
                    rows.append(cur)
                cur = [bs, bn, as_, an, i, i + 1, 0, 0]
        if cur is not None:
            rows.append(cur)
        return np.array(rows, np.int32).reshape(-1, 8)

    # ------------------------------------------------------------------ device packing
    def _device_graph_compact(self, device):
        """The compact path of ``device_graph``: plan + image (native, one pinned buffer), one H2D,
        one build launch; None when a molecule exceeds a block."""
        host = torch.empty(_stage_bound(self._compact), dtype=torch.uint8, pin_memory=True)
        info = _packer().compact_stage(*self._compact, *self._compact_dims,
                                       getattr(self, 'block_target', BLK_TARGET), host.data_ptr(),
                                       host.numel())
        if info is None:
            return None
        assert info[0], 'staged image larger than its bound'
        return upload_compact(device, host, info, *self._compact_dims)

    def device_graph(self, device, atom_messages: bool = False, bond_fdim: int = None,
                     atom_blocks: bool = True) -> DeviceGraph:
        """Pack (once per device/mode) into one device buffer; returns the cached DeviceGraph.
        ``atom_blocks`` (atom messages only): also build what the molecule-blocked fused atom-message
        forward reads (blocks, block-local ELL lists, per-atom bond-feature sums).  Only a bias-free
        inference forward can take that path (wdmpnn.hip get_dims), so the encoder asks for them only
        then: a training or biased graph skips their host work and upload."""
        device = torch.device(device)
        atom_blocks = bool(atom_blocks) or not atom_messages
        key = (str(device), bool(atom_messages), bond_fdim) if atom_blocks else \
            (str(device), True, bond_fdim, 'no_blocks')
        dg = self._device_cache.get(key)
        if dg is not None:
            return dg
        if self._compact is not None and not atom_messages and device.type == 'cuda' and \
                (bond_fdim is None or bond_fdim == self._compact_dims[1]):
            dg = self._device_graph_compact(device)
            if dg is not None:
                self._device_cache[key] = dg
                return dg
        fa = self._np['f_atoms']
        tail = self._np.get('bond_tail')
        dev_bonds = tail is not None and device.type == 'cuda'  # rebuild f_bonds on the device
        if atom_messages:
            nb_used = bond_fdim if bond_fdim is not None else get_bond_fdim(atom_messages=True)
            src = tail if tail is not None and nb_used <= tail.shape[1] else self.f_bonds.numpy()
            fb = src[:, src.shape[1] - nb_used:]
            dev_bonds = False
        elif tail is not None and not dev_bonds:
            fb = self.f_bonds.numpy()
        else:
            fb = tail if dev_bonds else self._np['f_bonds']
        Fa = fa.shape[1]
        Fb = Fa + tail.shape[1] if dev_bonds else fb.shape[1]
        lda, ldb = _round_up(Fa, 32), _round_up(Fb, 32)
        fa_p = np.zeros((_round_up(fa.shape[0], 128), lda), np.float32)  # rows to the GEMM tile, K to 32
        fa_p[:fa.shape[0], :Fa] = fa
        rows_b = _round_up(fb.shape[0], 128)
        if dev_bonds:  # upload the tail + b2a only (pad rows: source atom 0 = the zero pad row, tail 0)
            fb_p = np.zeros((rows_b, tail.shape[1]), np.float32)
            fb_p[:tail.shape[0]] = tail
            b2a_p = np.zeros(rows_b, np.int32)
            b2a_p[:tail.shape[0]] = self._np['b2a']
        else:
            fb_p = np.zeros((rows_b, ldb), np.float32)
            fb_p[:fb.shape[0], :Fb] = fb
        a_start = np.array([s for s, _ in self.a_scope], np.int32)
        a_size = np.array([n for _, n in self.a_scope], np.int32)
        xn = np.array(self.degree_of_polym, np.float32)
        if atom_messages:
            msg, feat = self.atom_message_gather()
            msg_rows = self.n_atoms
        else:
            msg, feat = self.bond_message_gather(), None
            msg_rows = self.n_bonds
        agg = self.atom_aggregate_gather(atom_messages)
        blocks = self.molecule_blocks() if atom_blocks else None
        msg_blk = msg
        if atom_messages and blocks is not None and len(blocks):
            # the fused atom-message layers (wdmpnn.hip get_dims: bias-free models only) gather a2a neighbours
            # inside the block: their ELL lists drop the pad slots (atom 0, whose message is zero without
            # biases); msg keeps each row's real entries first, so a longer row continues in msg past the
            # ELL width (the kernel skips its pad entry)
            rows, j = self._entries_of_in(np.arange(self.n_atoms, dtype=np.int64))
            msg_blk = Csr.from_rows(rows, self._np['b2a'][j], np.ones(len(rows), np.float32), self.n_atoms)
        if blocks is not None and len(blocks):
            # every gather of a block's rows must stay inside the block (block-diagonal batches)
            bond_blk = np.full(fb_p.shape[0], -1, np.int32)
            atom_blk = np.full(fa_p.shape[0], -1, np.int32)
            blk_of_bond = np.full(fb_p.shape[0], -1, np.int64)
            blk_of_atom = np.full(fa_p.shape[0], -1, np.int64)
            for (start, count, cap, blk_row, blk_of) in ((blocks[:, 0], blocks[:, 1], BLK_BONDS, bond_blk, blk_of_bond),
                                                         (blocks[:, 2], blocks[:, 3], BLK_ATOMS, atom_blk, blk_of_atom)):
                k = np.repeat(np.arange(len(blocks)), count)  # rows of a block are contiguous from its start
                within = np.arange(len(k)) - np.repeat(np.cumsum(count) - count, count)
                rows = np.repeat(start, count) + within
                blk_row[rows] = cap * k + within
                blk_of[rows] = k
            # (bond mode: msg rows are bonds gathering bonds, agg rows atoms gathering bonds; atom mode: both
            # gather atoms into atom rows)
            src_of = blk_of_atom if atom_messages else blk_of_bond
            for c, rb in ((msg_blk, blk_of_atom if atom_messages else blk_of_bond), (agg, blk_of_atom)):
                row = np.repeat(np.arange(len(c.ptr) - 1), np.diff(c.ptr))
                if len(row) and not np.array_equal(rb[row], src_of[c.idx]):
                    blocks = None
                    break
        if atom_messages:
            msg_t = msg.transpose(msg_rows)
            agg_t = agg.transpose(msg_rows)
        else:
            msg_t, agg_t = self._native_gathers()[2:]
        arrays = [('f_atoms', fa_p), ('bond_tail' if dev_bonds else 'f_bonds', fb_p), ('w_atoms', self._np['w_atoms']),
                  ('mol_start', a_start), ('mol_size', a_size), ('xn', xn),
                  ('b2revb', self._np['b2revb'].astype(np.int32))]
        if dev_bonds:
            arrays.append(('b2a', b2a_p))
        if atom_messages and feat is not None and blocks is not None and len(blocks):
            # per atom the sum of its in-bonds' feature rows (mpn.py:105-106 summed over the a2b slots): a
            # function of the graph alone, made here with the feature planes (WdGraph.atom_feat_sum_x6);
            # fp32, added in slot order -- the gather kernel's order
            fs = np.zeros((fa_p.shape[0], fb_p.shape[1]), np.float32)
            deg = np.diff(feat.ptr)
            for k in range(int(deg.max(initial=0))):
                rows_k = np.nonzero(deg > k)[0]
                fs[rows_k] += fb_p[feat.idx[feat.ptr[rows_k] + k]]
            arrays.append(('atom_feat_sum', fs))
        if blocks is not None and len(blocks):
            arrays += [('blocks', blocks), ('bond_blk_row', bond_blk), ('atom_blk_row', atom_blk)]
            bstart = np.zeros(len(blocks) + 1, np.int64)  # first row of the gathered kind per block (-1: row 0)
            bstart[:-1] = blocks[:, 2] if atom_messages else blocks[:, 0]
            mrows, mblk = (fa_p.shape[0], blk_of_atom) if atom_messages else (fb_p.shape[0], blk_of_bond)
            for name, c, rows_p, rb in (('msg_ell', msg_blk, mrows, mblk), ('agg_ell', agg, fa_p.shape[0], blk_of_atom)):
                ell_idx, ell_coef = ell_rows(c, rows_p, bstart[rb[:len(c.ptr) - 1]])
                arrays += [(name + '_idx', ell_idx), (name + '_coef', ell_coef)]
            # per bond row: its source atom (b2a) as a block-local atom index (the fused layer's X[b] =
            # A[src(b)] - P[rev(b)], mpn.py:119-120); rows outside the blocks 0
            src_blk = np.zeros(fb_p.shape[0], np.uint8)
            nb = len(self._np['b2a'])
            inb = np.nonzero(blk_of_bond[:nb] >= 0)[0]
            src_blk[inb] = (self._np['b2a'][inb] - blocks[blk_of_bond[inb], 2]).astype(np.uint8)
            arrays.append(('bond_src_blk', src_blk))
        csrs = [('msg', msg), ('agg', agg), ('msg_t', msg_t), ('agg_t', agg_t)]
        if feat is not None:
            csrs.append(('feat', feat))
        for name, c in csrs:  # idx / coef carry CSR_PAD readable dummy entries past ptr[rows] (header)
            arrays += [(f'{name}_ptr', c.ptr), (f'{name}_idx', np.concatenate([c.idx, np.zeros(CSR_PAD, np.int32)])),
                       (f'{name}_coef', np.concatenate([c.coef, np.zeros(CSR_PAD, np.float32)]))]
        offsets, total = {}, 0
        for name, a in arrays:
            offsets[name] = total
            total += (a.nbytes + 255) & ~255
        total = max(total, 256)
        host = torch.empty(total, dtype=torch.uint8, pin_memory=device.type == 'cuda' and torch.cuda.is_available())
        hv = host.numpy()
        for name, a in arrays:
            hv[offsets[name]:offsets[name] + a.nbytes] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        buf = host.to(device, non_blocking=True)
        base = buf.data_ptr() if device.type == 'cuda' else 0
        views = {name: buf[offsets[name]:offsets[name] + a.nbytes] for name, a in arrays}
        # the pinned staging block goes back to torch's caching host allocator, which records the copy's
        # stream event and recycles the block only after the copy has run: later batches reuse pinned
        # memory instead of pinning fresh pages
        del host, hv

        def P(name):
            return base + offsets[name]

        def csr(name):
            return _native.WdCsr(P(f'{name}_ptr'), P(f'{name}_idx'), P(f'{name}_coef'))

        if dev_bonds:  # f_bonds = f_atoms[b2a] ‖ tail, built on the device from the uploaded pieces
            fbd = torch.empty(rows_b * ldb, dtype=torch.float32, device=device)
            _native.check(_native.lib().wdmpnn_build_bond_features(
                P('f_atoms'), lda, Fa, fa_p.shape[0], P('b2a'), P('bond_tail'), fb_p.shape[1], fb_p.shape[1], rows_b,
                fbd.data_ptr(), ldb, _native.current_stream(device)), 'device bond features')
            views['f_bonds'] = fbd
            offsets['f_bonds'] = fbd.data_ptr() - base
        s = _native.WdGraph()
        s.n_atoms, s.n_bonds, s.n_mols = self.n_atoms, self.n_bonds, len(self.a_scope)
        s.atom_fdim, s.bond_fdim, s.ld_atoms, s.ld_bonds, s.bond_col0 = Fa, Fb, lda, ldb, 0
        s.f_atoms, s.f_bonds, s.w_atoms = P('f_atoms'), P('f_bonds'), P('w_atoms')
        s.mol_start, s.mol_size, s.degree_of_polym = P('mol_start'), P('mol_size'), P('xn')
        s.msg_gather, s.atom_gather = csr('msg'), csr('agg')
        s.msg_gather_t, s.atom_gather_t = csr('msg_t'), csr('agg_t')
        if feat is not None:
            s.bond_feat_gather = csr('feat')
        s.b2revb = P('b2revb')
        s.atom_desc, s.desc_dim = 0, 0
        s.atom_messages = int(bool(atom_messages))
        if device.type == 'cuda':  # bf16x3 plane tiles of the features for the split GEMMs (exact copies)
            L = _native.lib()
            plane_srcs = [('f_atoms', fa_p.shape[0], lda), ('f_bonds', rows_b, ldb)]
            if 'atom_feat_sum' in offsets:
                plane_srcs.append(('atom_feat_sum', fa_p.shape[0], ldb))
            for name, rows, ld in plane_srcs:
                nbytes = ctypes.c_size_t()
                _native.check(L.wdmpnn_plane_bytes(rows, ld, ctypes.byref(nbytes)), 'plane bytes')
                planes = torch.empty(max(nbytes.value, 256), dtype=torch.uint8, device=device)
                _native.check(L.wdmpnn_split_planes(P(name), ld, rows, ld, planes.data_ptr(), nbytes.value,
                                                    _native.current_stream(device)), f'{name} planes')
                views[name + '_x6'] = planes
                setattr(s, name + '_x6', planes.data_ptr())
            if blocks is not None and len(blocks):  # f_atoms planes in the molecule-blocked atom layout
                out_rows = BLK_ATOMS * len(blocks)
                nbytes = ctypes.c_size_t()
                _native.check(L.wdmpnn_plane_bytes(out_rows, lda, ctypes.byref(nbytes)), 'plane bytes')
                planes = torch.empty(max(nbytes.value, 256), dtype=torch.uint8, device=device)
                _native.check(L.wdmpnn_split_planes_rows(P('f_atoms'), lda, fa_p.shape[0], lda, P('atom_blk_row'),
                                                         out_rows, planes.data_ptr(), nbytes.value,
                                                         _native.current_stream(device)), 'blocked f_atoms planes')
                views['f_atoms_blk_x6'] = planes
                s.n_blocks, s.blocks, s.bond_blk_row = len(blocks), P('blocks'), P('bond_blk_row')
                s.blk_max_bonds, s.blk_max_atoms = int(blocks[:, 1].max()), int(blocks[:, 3].max())
                s.msg_ell_idx, s.msg_ell_coef = P('msg_ell_idx'), P('msg_ell_coef')
                s.atom_ell_idx, s.atom_ell_coef = P('agg_ell_idx'), P('agg_ell_coef')
                if not atom_messages:
                    s.bond_src_blk = P('bond_src_blk')
                s.f_atoms_blk_x6 = planes.data_ptr()
        dg = DeviceGraph(buf, views, s)
        dg.finish()
        dg.host_csr = dict(csrs)
        dg.n_edges = self.n_bonds - 1
        dg.h2d_bytes = total
        dg.nnz_msg = int(msg.ptr[-1])
        dg.built_on_device = False
        self._device_cache[key] = dg
        return dg


def upload_compact(device, staged: torch.Tensor, info, atom_fdim: int, bond_fdim: int,
                   lean: bool = False) -> DeviceGraph:
    """H2D of a staged compact image (pinned host tensor from ``compact_stage`` / ``generate_stage``)
    on the current stream, then ``wdmpnn_build_graph`` into one device buffer: the DeviceGraph of the
    batch.  ``info`` = (copied, counts, offsets, total) as the native stage functions return it.
    ``lean``: an inference-only graph (WDMPNN_GRAPH_LEAN: no dense feature rows, planes or transposed
    gathers); a training forward or an unblocked path on it raises NotImplementedError."""
    _, (n_mols, n_atoms, n_bonds, n_blocks, nnz_msg, nnz_agg), off, total = info
    buf = staged[:total].to(device, non_blocking=True)
    base = buf.data_ptr()
    c = _native.WdCompact()
    c.n_mols, c.n_atoms, c.n_bonds, c.n_blocks = n_mols, n_atoms, n_bonds, n_blocks
    c.atom_fdim, c.bond_fdim, c.nnz_msg, c.nnz_agg = atom_fdim, bond_fdim, nnz_msg, nnz_agg
    c.mols, c.xn, c.atoms, c.pairs, c.blocks, c.block_nnz = (base + o for o in off)
    L = _native.lib()
    nbytes = ctypes.c_size_t()
    _native.check(L.wdmpnn_graph_bytes(ctypes.byref(c), ctypes.byref(nbytes)), 'graph bytes')
    gbuf = torch.empty(nbytes.value, dtype=torch.uint8, device=device)
    s = _native.WdGraph()
    _native.check(L.wdmpnn_build_graph_ex(ctypes.byref(c), gbuf.data_ptr(), nbytes.value, ctypes.byref(s),
                                          _native.GRAPH_LEAN if lean else 0, _native.current_stream(device)),
                  'device graph build')
    if n_blocks:  # the block plan's largest blocks, read from the staged image (WdGraph.blk_max_*)
        blk = np.frombuffer(staged.numpy(), np.int32, count=8 * n_blocks, offset=off[4]).reshape(n_blocks, 8)
        s.blk_max_bonds, s.blk_max_atoms = int(blk[:, 1].max()), int(blk[:, 3].max())
    dg = DeviceGraph(gbuf, {'compact': buf}, s)
    dg.finish()
    dg.n_edges = n_bonds - 1
    dg.h2d_bytes = total
    dg.nnz_msg = nnz_msg
    dg.built_on_device = True
    dg.lean = bool(lean)
    return dg


def _stage_bound(arrays) -> int:
    """Upper bound of a staged image's bytes (blocks <= molecules)."""
    n_mols = len(arrays[1]) // 4
    return sum(len(a) for a in arrays) + 40 * (n_mols + 1) + 6 * 256


def mol2graph(mols, atom_features_batch=(None,), bond_features_batch=(None,),
              overwrite_default_atom_features: bool = False, overwrite_default_bond_features: bool = False):
    """featurization.py:878-898.  SMILES -> MolGraph needs RDKit; this package consumes featurised
    graphs (MolGraph-like objects), so pass a BatchMolGraph / MolGraph list instead."""
    raise NotImplementedError('mol2graph needs RDKit-based MolGraph featurisation, which is outside the '
                              'accelerated hot path; build MolGraph objects with the reference featuriser '
                              'and wrap them in chemprop_amd.featurization.BatchMolGraph')
