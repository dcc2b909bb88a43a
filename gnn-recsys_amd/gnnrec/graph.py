"""Device-resident CSR heterographs and blocks — the graph objects the drop-in
modules consume (replacing DGL 0.5.2's DGLHeteroGraph / block objects).

HeteroGraph  a full user–item(–sport) heterograph (reference
             src/builder.py:377-383 `create_graph` -> dgl.heterograph).  COO per
             canonical etype in eid order; reverse relations share the forward
             eid order (src/utils_data.py:205-238).  The dst-major CSR that the
             aggregation kernel reads is built once per relation and cached.
Block        a sampled computation block (DGL `to_block`): per node type the dst
             nodes are the prefix of the src nodes; per relation a dst-major CSR
             over LOCAL ids plus the global eid of every edge
             (reference src/sampling.py:153-161, consumed at
             src/train/run.py:112,340 and src/model.py:415-421).
RelGraph     one relation of either, as ConvLayer.forward sees it
             (DGL's `g[stype, etype, dtype]`): CSR + per-edge data in CSR order.
PairGraph    pos_g / neg_g of the edge loader: COO over the seed nodes.

Data layout in HBM: CSR indptr int64 [n_dst+1], indices int32 [E] (local src
row), eids int64 [E]; features fp32 row-major.  See DESIGN.md §layout.
"""
from __future__ import annotations

import contextlib
from typing import Dict, Iterable, Optional, Tuple

import torch

from . import ops

NID = "_ID"
EID = "_ID"
CEType = Tuple[str, str, str]


class LazyRows:
    """Rows of a table at ids, gathered when first read (ops.gather_rows; a negative id gives
    a zero row).  A static-shape batch's block data (sampling, static_shapes=True) is held
    this way: a captured training step that reads it gathers it INSIDE its graph from the
    batch's captured ids — so the loader neither gathers it nor hands it over, and data the
    model never reads (a `mean` model's block edge data) is never moved."""

    __slots__ = ("table", "ids")

    def __init__(self, table: torch.Tensor, ids: torch.Tensor):
        self.table, self.ids = table, ids

    def get(self) -> torch.Tensor:
        return ops.gather_rows(self.table, self.ids)


class _FrameDict(dict):
    """ntype/etype-keyed feature store with DGL-like access.  A LazyRows value is gathered
    on first read and replaced by its tensor."""

    def __getitem__(self, key):
        v = dict.__getitem__(self, key)
        if isinstance(v, LazyRows):
            v = v.get()
            dict.__setitem__(self, key, v)
        return v

    def get(self, key, default=None):
        return self[key] if key in self else default

    def items(self):
        return [(k, self[k]) for k in list(self.keys())]

    def values(self):
        return [self[k] for k in list(self.keys())]

    def pop(self, key, *default):
        if key in self:
            v = self[key]
            dict.__delitem__(self, key)
            return v
        return dict.pop(self, key, *default)

    def lazy_items(self):
        """(key, value) with LazyRows values left unread."""
        return list(dict.items(self))


class _TypeAccessor:
    def __init__(self, frames: dict, resolve):
        self._frames = frames
        self._resolve = resolve

    def __getitem__(self, key):
        class _View:
            pass

        v = _View()
        v.data = self._frames[self._resolve(key)]
        return v


class _MultiTypeData:
    """g.ndata / g.edata / block.srcdata: data['field'] -> {type: tensor}."""

    def __init__(self, frames: dict, single_key=None):
        self._frames = frames
        self._single = single_key

    def __getitem__(self, field):
        res = {t: f[field] for t, f in self._frames.items() if field in f}
        if self._single is not None:
            return res[self._single]
        return res

    def __setitem__(self, field, value):
        if isinstance(value, dict):
            for t, v in value.items():
                self._frames[t][field] = v
        elif self._single is not None:
            self._frames[self._single][field] = value
        else:
            raise ValueError("multi-type data needs a {type: tensor} dict")

    def __contains__(self, field):
        return any(field in f for f in self._frames.values())

    def keys(self):
        ks = []
        for f in self._frames.values():
            ks.extend(k for k in f if k not in ks)
        return ks


def build_csr(src: torch.Tensor, dst: torch.Tensor, n_dst: int):
    """dst-major CSR with in-row order = eid order.  -> indptr, indices(int32), eids.

    Row f3 (reference src/builder.py:377-383 -> dgl.heterograph, whose in-CSR keeps the
    edges of a row in edge-id order): on a HIP device the library's stable radix sort of
    the dst ids (gnnrec_csr_build).  A graph still held in host memory (assembled on the
    CPU before .to(device), as the reference builds its graphs) gets the same CSR from a
    host stable sort; nothing on the device path falls back to it."""
    src = torch.as_tensor(src, dtype=torch.int64)
    dst = torch.as_tensor(dst, dtype=torch.int64, device=src.device)
    if dst.device.type == 'cuda':
        return ops.csr_build(src, dst, n_dst)
    order = torch.argsort(dst, stable=True)
    indptr = torch.zeros(n_dst + 1, dtype=torch.int64)
    torch.cumsum(torch.bincount(dst, minlength=n_dst), 0, out=indptr[1:])
    return indptr, src[order].to(torch.int32), order


class RelGraph:
    """One relation as ConvLayer sees it: CSR over local ids + edge data in CSR order."""

    is_block = True

    def __init__(self, cetype: CEType, indptr, indices, n_src: int, n_dst: int,
                 edata: Optional[dict] = None, eids: Optional[torch.Tensor] = None,
                 transposed: Optional[tuple] = None):
        self.cetype = cetype
        # (indptr_t, dst rows int32, 1/deg(dst) per edge): the source-major CSR the
        # aggregation backward gathers over, when the sampler built it with the block
        self.transposed = transposed
        self.canonical_etypes = [cetype]
        self.indptr = indptr
        self.indices = indices
        self.eids = eids
        self.n_src = n_src
        self.n_dst = n_dst
        self.edata = edata if edata is not None else {}

    def number_of_edges(self):
        return int(self.indices.numel())

    num_edges = number_of_edges

    def number_of_dst_nodes(self):
        return self.n_dst

    def number_of_src_nodes(self):
        return self.n_src

    def in_degrees_i32(self) -> torch.Tensor:
        return (self.indptr[1:] - self.indptr[:-1]).to(torch.int32)


class HeteroGraph:
    """Full heterograph on one device (COO + cached dst-major CSR per relation)."""

    is_block = False

    def __init__(self, data_dict: Dict[CEType, Tuple[torch.Tensor, torch.Tensor]],
                 num_nodes_dict: Optional[Dict[str, int]] = None, device=None):
        """data_dict: {(src type, relation, dst type): (src ids, dst ids)} — the reference's
        `graph_schema` (src/utils_data.py:204-238).  num_nodes_dict: nodes per type; types it
        omits (all of them when None) get max id + 1 over every relation they appear in,
        as dgl.heterograph infers them (0 for a type with no edges)."""
        self._coo = {}
        for ce, (s, d) in data_dict.items():
            if len(ce) != 3:
                raise ValueError(f"edge type {ce!r} must be a (src type, relation, dst type) "
                                 f"triple")
            s = torch.as_tensor(s, dtype=torch.int64, device=device)
            d = torch.as_tensor(d, dtype=torch.int64, device=device)
            if s.shape != d.shape or s.dim() != 1:
                raise ValueError(f"src/dst of {ce} must be 1-D id arrays of one length")
            self._coo[tuple(ce)] = (s, d)
        self.canonical_etypes = list(self._coo.keys())
        self._num_nodes = dict(num_nodes_dict or {})
        inferred: Dict[str, int] = {}
        for ce, (s, d) in self._coo.items():
            for nt, ids in ((ce[0], s), (ce[2], d)):
                if nt in self._num_nodes:
                    continue
                n = int(ids.max()) + 1 if ids.numel() else 0
                inferred[nt] = max(inferred.get(nt, 0), n)
        for ce, (s, d) in self._coo.items():  # ids must lie in [0, N)
            for nt, ids in ((ce[0], s), (ce[2], d)):
                if nt in self._num_nodes and ids.numel() and not ids.is_meta and (
                        int(ids.min()) < 0 or int(ids.max()) >= self._num_nodes[nt]):
                    raise ValueError(f"{ce}: {nt} ids outside [0, {self._num_nodes[nt]})")
        self._num_nodes.update(inferred)
        for ce in self.canonical_etypes:
            for nt in (ce[0], ce[2]):
                self._num_nodes.setdefault(nt, 0)
        self.ntypes = sorted(self._num_nodes)
        self.etypes = [ce[1] for ce in self.canonical_etypes]
        self._ndata = {nt: _FrameDict() for nt in self.ntypes}
        self._edata = {ce: _FrameDict() for ce in self.canonical_etypes}
        self._csr = {}
        self._csr_edata = {}
        self._edge_rec = {}
        self.nodes = _TypeAccessor(self._ndata, lambda k: k)
        self.edges = _TypeAccessor(self._edata, self.to_canonical_etype)
        self.device = torch.device(device) if device is not None else (
            next(iter(self._coo.values()))[0].device if self._coo else torch.device("cpu"))

    # ---- metadata -----------------------------------------------------
    def to_canonical_etype(self, etype) -> CEType:
        if isinstance(etype, tuple):
            return etype
        hits = [ce for ce in self.canonical_etypes if ce[1] == etype]
        if len(hits) != 1:
            raise KeyError(f"edge type {etype!r} not found or ambiguous")
        return hits[0]

    def num_nodes(self, ntype: Optional[str] = None) -> int:
        if ntype is None:
            return sum(self._num_nodes.values())
        return self._num_nodes[ntype]

    number_of_nodes = num_nodes

    def num_edges(self, etype=None) -> int:
        if etype is None:
            return sum(int(s.numel()) for s, _ in self._coo.values())
        return int(self._coo[self.to_canonical_etype(etype)][0].numel())

    number_of_edges = num_edges

    @property
    def ndata(self):
        return _MultiTypeData(self._ndata)

    @property
    def edata(self):
        single = self.canonical_etypes[0] if len(self.canonical_etypes) == 1 else None
        return _MultiTypeData(self._edata, single)

    @contextlib.contextmanager
    def local_scope(self):
        saved_n = {nt: _FrameDict(f) for nt, f in self._ndata.items()}
        saved_e = {ce: _FrameDict(f) for ce, f in self._edata.items()}
        try:
            yield self
        finally:
            for nt in self._ndata:
                self._ndata[nt].clear()
                self._ndata[nt].update(saved_n[nt])
            for ce in self._edata:
                self._edata[ce].clear()
                self._edata[ce].update(saved_e[ce])

    # ---- structure ------------------------------------------------------
    def all_edges(self, form="uv", order="eid", etype=None):
        ce = self.to_canonical_etype(etype if etype is not None else self.canonical_etypes[0])
        s, d = self._coo[ce]
        if form == "uv":
            return s, d
        if form == "eid":
            return torch.arange(s.numel(), device=s.device)
        return s, d, torch.arange(s.numel(), device=s.device)

    def find_edges(self, eids, etype=None):
        ce = self.to_canonical_etype(etype if etype is not None else self.canonical_etypes[0])
        s, d = self._coo[ce]
        eids = torch.as_tensor(eids, dtype=torch.int64, device=s.device)
        return s[eids], d[eids]

    def in_csr(self, etype):
        """(indptr int64, indices int32, eids int64) of the dst-major CSR, cached."""
        ce = self.to_canonical_etype(etype)
        if ce not in self._csr:
            s, d = self._coo[ce]
            self._csr[ce] = build_csr(s, d, self._num_nodes[ce[2]])
        return self._csr[ce]

    def in_csr_global(self, etype):
        """CSR for sampling: (indptr, src global ids int32, eids) -- the cached in_csr
        arrays themselves (the sampler widens ids to int64 as it copies them)."""
        return self.in_csr(etype)

    def edge_records(self, etype) -> Optional[torch.Tensor]:
        """The in-CSR's edges as packed 8-byte records for the fused sampler, cached:
        rec[e] = eids[e] << 32 | indices[e] (include/gnnrec.h gnnrec_sample_rel.edge_rec) —
        a fanout pick reads one record (one cache line) instead of a line of each array.
        None when an eid does not fit 31 bits (the sampler then reads the two arrays)."""
        ce = self.to_canonical_etype(etype)
        if ce not in self._edge_rec:
            _ip, ix, eid = self.in_csr(ce)
            rec = None
            if eid.numel() < (1 << 31) and eid.is_cuda:
                rec = (eid << 32) | ix.to(torch.int64)  # ids >= 0: no sign bits to mask
            self._edge_rec[ce] = rec
        return self._edge_rec[ce]

    def in_degrees(self, etype) -> torch.Tensor:
        indptr = self.in_csr(etype)[0]
        return indptr[1:] - indptr[:-1]

    def rel_graph(self, etype) -> RelGraph:
        ce = self.to_canonical_etype(etype)
        indptr, indices, eids = self.in_csr(ce)
        cache = self._csr_edata.setdefault(ce, {})
        edata = {}
        for k, v in self._edata[ce].items():
            hit = cache.get(k)
            if hit is None or hit[0] is not v:  # (re)permute into CSR order once per tensor
                hit = (v, v[eids] if v.numel() else v)
                cache[k] = hit
            edata[k] = hit[1]
        return RelGraph(ce, indptr, indices, self._num_nodes[ce[0]], self._num_nodes[ce[2]], edata,
                        eids)

    def __getitem__(self, key) -> RelGraph:
        return self.rel_graph(key if isinstance(key, tuple) and len(key) == 3 else key)

    def has_edges_between(self, u, v, etype=None) -> torch.Tensor:
        """Membership of (u[i], v[i]) in relation etype: a bool tensor (reference
        src/train/run.py:95-101,160-166, the false-negative mask; DGL's has_edges_between).
        On a HIP device, one binary search per query over the relation's source-sorted
        in-CSR (gnnrec_csr_has_edges; the CSR is built once by the library's radix sort and
        cached).  A graph still in host memory answers with a host sort + search."""
        ce = self.to_canonical_etype(etype if etype is not None else self.canonical_etypes[0])
        s, d = self._coo[ce]
        if s.is_cuda:
            cache = self._csr_edata.setdefault(("_member",) + ce, {})
            if "csr" not in cache:
                cache["csr"] = ops.membership_csr(s, d, self._num_nodes[ce[0]],
                                                  self._num_nodes[ce[2]])
            indptr, indices = cache["csr"]
            return ops.has_edges(indptr, indices, self._num_nodes[ce[0]], u, v)
        u = torch.as_tensor(u, dtype=torch.int64).reshape(-1)
        v = torch.as_tensor(v, dtype=torch.int64).reshape(-1)
        n_src = self._num_nodes[ce[0]]
        key = torch.sort(d * n_src + s).values
        ok = (u >= 0) & (u < n_src) & (v >= 0) & (v < self._num_nodes[ce[2]])
        q = v * n_src + u
        if key.numel() == 0:
            return torch.zeros_like(q, dtype=torch.bool)
        pos = torch.searchsorted(key, q).clamp(max=key.numel() - 1)
        return (key[pos] == q) & ok

    def to(self, device):
        g = HeteroGraph({ce: (s.to(device), d.to(device)) for ce, (s, d) in self._coo.items()},
                        self._num_nodes, device=device)
        for nt, f in self._ndata.items():
            for k, v in f.items():
                g._ndata[nt][k] = v.to(device)
        for ce, f in self._edata.items():
            for k, v in f.items():
                g._edata[ce][k] = v.to(device)
        return g


def create_graph(graph_schema: Dict[CEType, Tuple[object, object]], device=None,
                 num_nodes_dict: Optional[Dict[str, int]] = None) -> HeteroGraph:
    """Drop-in for the reference's `create_graph(graph_schema)` (src/builder.py:377-383,
    `dgl.heterograph(graph_schema)`): the relation -> (src ids, dst ids) dict built by
    DataLoader.graph_schema (src/utils_data.py:204-238, numpy arrays or tensors), node
    counts inferred per type as max id + 1 unless given."""
    return HeteroGraph(graph_schema, num_nodes_dict, device=device)


class Block:
    """A sampled computation block (DGL to_block output, restated)."""

    is_block = True
    static = False  # fixed-capacity block (BlockSampler static shapes): -1-padded rows

    def __init__(self, src_nid: Dict[str, torch.Tensor], num_dst: Dict[str, int],
                 rels: Dict[CEType, Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]):
        self.ntypes = sorted(src_nid)
        self.srctypes = self.ntypes
        self.dsttypes = self.ntypes
        self.canonical_etypes = list(rels.keys())
        self._num_dst = dict(num_dst)
        self._rels = rels
        self._src = {nt: _FrameDict({NID: src_nid[nt]}) for nt in self.ntypes}
        self._dst = {nt: _FrameDict({NID: src_nid[nt][: num_dst[nt]]}) for nt in self.ntypes}
        self._edata = {ce: _FrameDict({EID: rels[ce][2]}) for ce in self.canonical_etypes}
        self._t = {}  # ce -> source-major CSR of the relation (sampler, training loaders)
        # static blocks: ('dst' | 'src', ntype) -> the real row count on the device (int64 [1])
        self._live = {}

    @property
    def srcdata(self):
        return _MultiTypeData(self._src)

    @property
    def dstdata(self):
        return _MultiTypeData(self._dst)

    @property
    def edata(self):
        return _MultiTypeData(self._edata)

    def number_of_src_nodes(self, ntype):
        return int(self._src[ntype][NID].numel())

    def number_of_dst_nodes(self, ntype):
        return self._num_dst[ntype]

    def num_edges(self, etype):
        return int(self._rels[etype][1].numel())

    number_of_edges = num_edges

    def rel_graph(self, ce) -> RelGraph:
        indptr, indices, eids = self._rels[ce]
        edata = _FrameDict({k: v for k, v in self._edata[ce].lazy_items() if k != EID})
        return RelGraph(ce, indptr, indices, self.number_of_src_nodes(ce[0]), self._num_dst[ce[2]],
                        edata, eids, self._t.get(ce))

    def __getitem__(self, ce) -> RelGraph:
        return self.rel_graph(ce)

    def to(self, device):
        b = Block({nt: self._src[nt][NID].to(device) for nt in self.ntypes}, self._num_dst,
                  {ce: tuple(t.to(device) for t in r) for ce, r in self._rels.items()})
        for nt in self.ntypes:
            for k, v in self._src[nt].items():
                b._src[nt][k] = v.to(device)
        for ce in self.canonical_etypes:
            for k, v in self._edata[ce].items():
                b._edata[ce][k] = v.to(device)
        b._t = {ce: tuple(t.to(device) for t in v) for ce, v in self._t.items()}
        return b


def _stamp(t: torch.Tensor):
    """Identity of a tensor's contents: storage, in-place version, size."""
    return (t.data_ptr(), t._version, t.numel(), t.device)


class PairGraph:
    """pos_g / neg_g: edges over compacted seed nodes (DGL compact_graphs output)."""

    is_block = False
    static = False      # node lists at a fixed capacity, -1 past the real nodes
    node_counts = None  # static: the real node count per type (device scalars)

    def __init__(self, edges: Dict[CEType, Tuple[torch.Tensor, torch.Tensor]],
                 node_ids: Dict[str, torch.Tensor]):
        self._coo = {tuple(ce): (s, d) for ce, (s, d) in edges.items()}
        self.canonical_etypes = list(self._coo.keys())
        self.ntypes = sorted(node_ids)
        self._ndata = {nt: _FrameDict({NID: node_ids[nt]}) for nt in self.ntypes}
        self._edata = {ce: _FrameDict() for ce in self.canonical_etypes}
        self.nodes = _TypeAccessor(self._ndata, lambda k: k)
        # K when this is the negative graph of negative_sampler.Uniform(K): every etype's
        # sources are the positive graph's repeated K times (EdgeDataLoader sets it)
        self._repeats = None

    @property
    def src_repeats_pos(self):
        """K when marked as negative_sampler.Uniform(K)'s negative graph, else None."""
        return None if self._repeats is None else self._repeats[0]

    @src_repeats_pos.setter
    def src_repeats_pos(self, K):
        """Mark (or unmark: None) the graph's CURRENT source tensors as the positives'
        sources repeated K times.  The mark holds per etype only while that tensor is the
        one marked, unmodified (src_repeats): a replaced or edited edge list falls back to
        the per-edge cosine instead of trusting a stale mark."""
        self._repeats = None if K is None else (
            int(K), {ce: _stamp(s) for ce, (s, _d) in self._coo.items()})

    def src_repeats(self, etype, src) -> Optional[int]:
        """K if `src` is still the marked source tensor of `etype`, else None."""
        r = self._repeats
        if r is None or r[1].get(tuple(etype)) != _stamp(src):
            return None
        return r[0]

    @property
    def ndata(self):
        return _MultiTypeData(self._ndata)

    @property
    def edata(self):
        return _MultiTypeData(self._edata)

    def all_edges(self, form="uv", order="eid", etype=None):
        return self._coo[etype if etype is not None else self.canonical_etypes[0]]

    def edges(self, etype=None):
        return self.all_edges(etype=etype)

    def num_edges(self, etype):
        return int(self._coo[etype][0].numel())

    number_of_edges = num_edges

    def num_nodes(self, ntype):
        return int(self._ndata[ntype][NID].numel())

    @contextlib.contextmanager
    def local_scope(self):
        yield self

    def to(self, device):
        p = PairGraph({ce: (s.to(device), d.to(device)) for ce, (s, d) in self._coo.items()},
                      {nt: self._ndata[nt][NID].to(device) for nt in self.ntypes})
        for ce, f in self._edata.items():
            for k, v in f.items():
                p._edata[ce][k] = v.to(device)
        if self._repeats is not None and all(
                self.src_repeats(ce, s) is not None for ce, (s, _d) in self._coo.items()):
            p.src_repeats_pos = self._repeats[0]  # the copies hold the same values
        return p


def rel_graphs(g) -> Iterable[Tuple[CEType, RelGraph]]:
    for ce in g.canonical_etypes:
        yield ce, g.rel_graph(ce)
