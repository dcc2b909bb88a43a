"""Full-graph inference embedding pass (rows a5/a6/e of SURVEY.md §8).

Replaces reference src/train/run.py:311-349 `get_embeddings` as driven by
main_inference.py:123-152 (NodeDataLoader over every user and item,
MultiLayerFullNeighborSampler, 128-seed batches).  With full neighbourhoods
and eval-mode dropout that loop computes, for every node, the L-layer
ConvModel output over its complete L-hop neighbourhood; here the same
function is computed LAYER-WISE over the whole graph (every edge aggregated
once per layer instead of once per batch that touches it), which is the
reference run with one batch containing every node.

Sharding (P ranks, one per GPU, RCCL over xGMI):
  * the large node type (users) is partitioned into contiguous ranges; every
    relation INTO users is aggregated by the owner of the destination row
    (sources read from the replicated item table);
  * relations into the replicated types (items, sports) are aggregated from
    the edges each rank holds (its users' edges, or an eid range) into a
    partial table of every destination row, then reduce-scattered (sum, or max
    for pool aggregators) to the row owner, which divides by the GLOBAL
    in-degree inside the projection GEMM's operand load and projects;
  * the projected replicated rows are all-gathered for the next layer.
Per layer each rank moves 2·(P−1)/P·N_item·d·4 bytes instead of the
(P−1)/P·(N_user+N_item)·d·4 of an all-gather-everything scheme, and the
collectives overlap the user-side aggregation (async RCCL work handles).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from . import _lib, ops
from .dist import Exchange, degree_ranges, even_ranges, multi_rank, padded_shard
from .graph import HeteroGraph, build_csr


# --------------------------------------------------------- single process ---
@torch.no_grad()
def full_graph_embeddings(g: HeteroGraph, model, feats: Optional[Dict[str, torch.Tensor]] = None,
                          embedding_layer: Optional[bool] = None) -> Dict[str, torch.Tensor]:
    """Layer-wise full-graph pass on one device: {ntype: [N, out_dim]}."""
    if feats is None:
        feats = g.ndata['features']
    if embedding_layer is None:
        embedding_layer = model.embedding_layer
    h = model.embed(feats) if embedding_layer else dict(feats)
    for layer in model.layers:
        h = layer(g, h)
    return h


@torch.no_grad()
def get_embeddings(g, out_dim: int, trained_model, nodeloader_test, num_batches_valid: int = 0,
                   cuda: bool = True, device=None, embedding_layer: bool = True):
    """Drop-in for reference src/train/run.py:311-349 (minibatch loop over a node loader)."""
    dev = device if device is not None else torch.device('cuda')
    y = {nt: torch.zeros(g.num_nodes(nt), out_dim, device=dev) for nt in g.ntypes}
    for input_nodes, output_nodes, blocks in nodeloader_test:
        blocks = [b.to(dev) for b in blocks]
        input_features = blocks[0].srcdata['features']
        if embedding_layer:
            input_features = trained_model.embed(input_features)
        h = trained_model.get_repr(blocks, input_features)
        for ntype in h.keys():
            y[ntype][output_nodes[ntype]] = h[ntype]
    return y


# ------------------------------------------------------------- sharded ------
class RelShard:
    """One relation's edges held by this rank, as a dst-major CSR."""

    def __init__(self, ce, kind: str, indptr, indices, weights, n_rows: int, global_edges: int,
                 deg_own: Optional[torch.Tensor] = None, segs: Optional[list] = None):
        self.ce = ce
        self.kind = kind              # 'local_dst' (dst rows owned here) | 'partial'
        self.indptr = indptr
        self.indices = indices
        self.weights = weights        # float32 per edge in CSR order, or None
        self.n_rows = n_rows
        self.global_edges = global_edges
        self.deg_own = deg_own        # int32 global in-degree of the owned dst rows ('partial')
        self.segs = segs              # 'partial' + segments: [(indptr, indices, weights)] per
                                      # owned segment, in segment order

    @property
    def local_edges(self) -> int:
        return int(self.indices.numel())


def _planned(indptr: torch.Tensor, split: int = ops.DEFAULT_SPLIT) -> torch.Tensor:
    """A shard CSR with its heavy-row plan computed once, at setup (one host readback):
    the pass then launches the plain aggregation kernel when no row is heavy, instead of
    the device-planned form's plan / chunk / combine launches on every pass (C5: 32 extra
    launches per layer, ≈1.5 ms)."""
    if indptr.is_cuda:
        ops.split_plan(indptr, split)
    return indptr


# Source-range tiles are reduced by the plain aggregation kernel, never by the fused one, so
# their heavy rows can be chunked finer than the fused kernel's eligibility threshold
# (DEFAULT_SPLIT): one wave per 512 edges instead of per 2048 spreads a Zipf head over 4x
# the waves — C4 --zipf 1.0 pass 164.2 -> 142.6 ms (split 256: 146.3, 1024: 149.1); the
# uniform configs have no tile row that long.  Every rank uses the same split, so the
# deterministic tree stays bitwise P-invariant.
TILE_SPLIT = 512


class GraphShard:
    """This rank's share of a heterograph for the sharded full-graph pass."""

    def __init__(self, rank: int, world: int, ptype: str, num_nodes: Dict[str, int],
                 canonical_etypes: List[tuple], device, segments: Optional[int] = None,
                 ptype_weight: Optional[torch.Tensor] = None):
        """segments: split every 'partial' relation's edges into this many fixed key ranges
        (source id of the partitioned type, else edge id), `segments // world` per rank, so
        ShardedFullGraphPass(deterministic=True) sums the same partials in the same tree at
        any world size dividing `segments` (bitwise-equal outputs at P=1/2/4/8).

        ptype_weight: per-node weight of the partitioned type (its in-degree summed over
        relations, + 1): the contiguous id ranges are then balanced by cumulative weight
         instead of by node count.  With `segments`, the segment key ranges are
        the weight-balanced ones and every rank's range is the union of its segments, so the
        boundaries still nest at every world size."""
        if segments is not None and (segments < world or segments % world or
                                     segments & (segments - 1)):
            raise ValueError(f"segments={segments} must be a power of two and a multiple of "
                             f"the world size {world}")
        self.segments = segments
        self.rank, self.world, self.ptype = rank, world, ptype
        self.num_nodes = dict(num_nodes)
        self.canonical_etypes = list(canonical_etypes)
        self.device = torch.device(device)
        n_p = num_nodes[ptype]
        if ptype_weight is not None and ptype_weight.numel() != n_p:
            raise ValueError(f"ptype_weight has {ptype_weight.numel()} entries for {n_p} nodes")
        split = (lambda parts: degree_ranges(ptype_weight, parts)) if ptype_weight is not None \
            else (lambda parts: even_ranges(n_p, parts))
        self.balance = "degree" if ptype_weight is not None else "count"
        if segments is not None:
            self.seg_bounds = split(segments)
            k = segments // world
            self.bounds = [self.seg_bounds[r * k] for r in range(world + 1)]
        else:
            self.seg_bounds = None
            self.bounds = split(world)
        self.p_lo, self.p_hi = self.bounds[rank], self.bounds[rank + 1]
        self.shard_rows = {nt: padded_shard(n, world) for nt, n in num_nodes.items()
                           if nt != ptype}
        self.rels: Dict[tuple, RelShard] = {}
        self._in_edges = {}  # ce -> (src, dst - block start): this rank's rows' in-edges
        self._full_rows = {}

    @property
    def ptype_pad(self) -> int:
        """Rows per rank of the partitioned table gathered in rank order (the largest range)."""
        b = self.bounds
        return max(b[r + 1] - b[r] for r in range(self.world))

    def full_in_rows(self, ce):
        """(indptr [S+1], indices int32) of a relation into a replicated type over this
        rank's block of destination rows (own_slice): EVERY in-edge of those rows in edge-id
        order (the reference's mailbox order).  Sources of the partitioned type are numbered
        as rows of its table all-gathered with `ptype_pad` rows per rank; sources of a
        replicated type are its rows.  What a reducer that does not split into per-rank
        partials (the LSTM) runs over at P > 1.  Built once from the graph the shard came
        from (GraphShard.from_graph)."""
        hit = self._full_rows.get(ce)
        if hit is not None:
            return hit
        s_t, _, d_t = ce
        if d_t == self.ptype:
            raise ValueError(f"full_in_rows: {ce} ends in the partitioned type")
        if ce not in self._in_edges:
            raise NotImplementedError(
                "a relation whose reducer does not split into per-rank partials (lstm) needs "
                "the whole in-neighbourhood of the rows a rank owns: build the shard with "
                "GraphShard.from_graph")
        src, dst = self._in_edges[ce]
        S = self.shard_rows[d_t]
        if s_t == self.ptype:
            bounds = torch.tensor(self.bounds, dtype=torch.int64, device=src.device)
            owner = torch.searchsorted(bounds, src, right=True) - 1
            src = owner * self.ptype_pad + (src - bounds[owner])
        indptr, indices, _ = build_csr(src, dst, S)
        hit = (indptr.to(self.device), indices.to(self.device))
        self._full_rows[ce] = hit
        return hit

    @property
    def n_own(self) -> int:
        return self.p_hi - self.p_lo

    def padded_rows(self, nt) -> int:
        return self.shard_rows[nt] * self.world

    def own_slice(self, nt):
        S = self.shard_rows[nt]
        return slice(self.rank * S, (self.rank + 1) * S)

    def local_edge_count(self) -> int:
        return sum(r.local_edges for r in self.rels.values())

    def global_edge_count(self) -> int:
        return sum(r.global_edges for r in self.rels.values())

    def add_relation(self, ce, src: torch.Tensor, dst: torch.Tensor, eid: torch.Tensor,
                     global_edges: int, weights: Optional[torch.Tensor] = None,
                     dst_global_deg: Optional[torch.Tensor] = None):
        """Register this rank's edges of relation ce.

        src/dst are GLOBAL ids of the edges this rank holds; for relations into
        ptype they must be exactly the edges whose dst is owned here."""
        s_t, _, d_t = ce
        dev = self.device
        if d_t == self.ptype:
            if s_t == self.ptype:
                raise NotImplementedError("relations between two rows of the partitioned type "
                                          "need the full partitioned table (not in the schema)")
            rows = dst - self.p_lo
            indptr, indices, order = build_csr(src, rows, self.n_own)
            w = None if weights is None else weights[order].float().contiguous()
            self.rels[ce] = RelShard(ce, 'local_dst', _planned(indptr.to(dev)), indices.to(dev),
                                     None if w is None else w.to(dev), self.n_own, global_edges)
            return
        src_loc = src - self.p_lo if s_t == self.ptype else src
        n_rows = self.padded_rows(d_t)
        indptr, indices, order = build_csr(src_loc, dst, n_rows)
        w = None if weights is None else weights[order].float().contiguous()
        deg = torch.zeros(n_rows, dtype=torch.int32, device=dst_global_deg.device)
        deg[: dst_global_deg.numel()] = dst_global_deg.to(torch.int32)
        segs = None
        if self.segments is not None:
            # key ranges fixed by the global sizes alone: the source id when the source is
            # the partitioned type (rank ranges are unions of them), else the edge id (the
            # edge split of from_graph); each segment's rows keep the edges' input order
            k = self.segments // self.world
            if s_t == self.ptype:
                key, bounds = src, self.seg_bounds
            else:
                key, bounds = eid, even_ranges(global_edges, self.segments)
            segs = []
            for sg in range(self.rank * k, (self.rank + 1) * k):
                sel = (key >= bounds[sg]) & (key < bounds[sg + 1])
                ip, ix, od = build_csr(src_loc[sel], dst[sel], n_rows)
                ws = None if weights is None else weights[sel][od].float().contiguous().to(dev)
                segs.append((_planned(ip.to(dev), TILE_SPLIT), ix.to(dev), ws))
        self.rels[ce] = RelShard(ce, 'partial', _planned(indptr.to(dev)), indices.to(dev),
                                 None if w is None else w.to(dev), n_rows, global_edges,
                                 deg[self.own_slice(d_t)].contiguous().to(dev), segs)

    @classmethod
    def from_graph(cls, g: HeteroGraph, rank: int, world: int, ptype: str = 'user', device=None,
                   weight_field: Optional[str] = 'occurrence', segments: Optional[int] = None,
                   balance: str = 'degree'):
        """Shard a full HeteroGraph held by every rank (tests / moderate graphs).
        balance: 'degree' (ranges balanced by the partitioned type's in-degree over all
        relations + 1) or 'count' (equal node counts)."""
        dev = device if device is not None else g.device
        weight = None
        if balance == 'degree':
            weight = ptype_in_degree(g, ptype)
        elif balance != 'count':
            raise ValueError(f"balance must be 'degree' or 'count', not {balance!r}")
        sh = cls(rank, world, ptype, {nt: g.num_nodes(nt) for nt in g.ntypes},
                 g.canonical_etypes, dev, segments, weight)
        for ce in g.canonical_etypes:
            s, d = g.all_edges(etype=ce)
            if ce[2] != ptype:
                # full_in_rows' input: every in-edge (edge-id order) of this rank's block of
                # the replicated destination rows — kept instead of the whole graph
                S = sh.shard_rows[ce[2]]
                sel = (d >= rank * S) & (d < (rank + 1) * S)
                sh._in_edges[ce] = (s[sel], d[sel] - rank * S)
            E = s.numel()
            eid = torch.arange(E, device=s.device)
            w = g._edata[ce].get(weight_field) if weight_field else None
            if ce[2] == ptype:
                keep = (d >= sh.p_lo) & (d < sh.p_hi)
            elif ce[0] == ptype:
                keep = (s >= sh.p_lo) & (s < sh.p_hi)
            else:
                lo, hi = even_ranges(E, world)[rank], even_ranges(E, world)[rank + 1]
                keep = (eid >= lo) & (eid < hi)
            gdeg = torch.bincount(d, minlength=g.num_nodes(ce[2])) if ce[2] != ptype else None
            sh.add_relation(ce, s[keep], d[keep], eid[keep], E,
                            None if w is None else w[keep], gdeg)
        return sh

    def local_features(self, feats: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Full per-type feature tables -> this rank's inputs (own ptype rows, padded tables)."""
        out = {}
        for nt, x in feats.items():
            if nt == self.ptype:
                out[nt] = x[self.p_lo:self.p_hi].contiguous().to(self.device)
            else:
                t = torch.zeros((self.padded_rows(nt), x.shape[1]), dtype=x.dtype,
                                device=self.device)
                t[: x.shape[0]] = x.to(self.device)
                out[nt] = t
        return out


def ptype_in_degree(g: HeteroGraph, ptype: str) -> torch.Tensor:
    """In-degree of every `ptype` node summed over the relations into it, + 1 (the
    partition weight of GraphShard: a row costs its edges plus its own read/write)."""
    w = torch.ones(g.num_nodes(ptype), dtype=torch.int64, device=g.device)
    for ce in g.canonical_etypes:
        if ce[2] == ptype:
            _, d = g.all_edges(etype=ce)
            w += torch.bincount(d, minlength=w.numel())
    return w


RESERVE_CUS = 16  # of 256: room for RCCL's channel blocks beside the aggregation


class ShardedFullGraphPass:
    """Layer-wise full-graph ConvModel pass over a GraphShard (one rank's view).

    Streams (when `overlap` and the tensors live on a HIP device):
      main  aggregation kernels and the replicated-type GEMMs;
      side  the projection GEMMs of the partitioned type (users), which are
            MFMA-bound and run concurrently with the HBM-bound aggregation of
            the other relation (events order every hand-off);
      RCCL  reduce-scatter / all-gather, issued async_op=True.
    Order per layer: partial aggregation (the item-dst tiles) first.  At world size 1
    the items' tree + projection GEMMs then go to the side stream under the user-dst
    launch (C5 157.8 -> 157.0 ms, C4 -0.1 ms: the persistent user-side launch holds every
    CU, so the GEMM blocks mostly find room only between launches; reserving CUs for them
    costs the HBM-bound launch more — 32 CUs: C5 160.7 ms); GNNREC_OWNED_SIDE=0 restores
    user-side-first on one stream.  With several ranks the reduce-scatter overlaps the
    user-dst aggregation and the all-gather the next layer's partial aggregation.

    `ops_backend` defaults to the HIP ops (gnnrec.ops); tests on CPU ranks
    inject a checker backend with the same signatures."""

    def __init__(self, model, shard: GraphShard, exchange: Optional[Exchange] = None,
                 ops_backend=None, overlap: bool = True, fold_embedding: bool = True,
                 deterministic: bool = False, concurrency=None):
        self.model = model
        # deterministic: outputs bitwise independent of the world size (needs a shard built
        # with `segments`): replicated-type sums are per-segment partials folded in a fixed
        # pairwise tree (locally, then across ranks after an all-to-all) and every kernel
        # choice is made from global sizes (the embedding fold depends on neither, so it
        # stays on).  Costs the fused launch on the replicated side at one rank and the
        # partials' extra HBM passes.
        if deterministic and shard.segments is None:
            raise ValueError("deterministic=True needs a GraphShard built with segments")
        self.deterministic = deterministic
        # fold the partitioned type's NodeEmbedding into the first layer's fused launches
        # (one rank, mean/sum reducers): its 10M-row GEMM and table disappear
        self.fold_embedding = fold_embedding
        self._fold = {}  # nt -> (W_emb, b_emb) while h[nt] holds that type's raw features
        self._folded_types = set()  # types whose embedding was folded in the last run
        # folded weights per relation, kept across passes and rebuilt only when a parameter
        # changes (its version counter): no weight products inside a timed pass, and the
        # side-stream GEMMs read tensors that live as long as the runner
        self._fold_cache = {}
        self.shard = shard
        self.ex = exchange if exchange is not None else Exchange()
        self.ops = ops_backend if ops_backend is not None else ops
        self.overlap = overlap
        # keyed by the id of the tensor being produced (a layer's input and output tables
        # of one node type are alive together; keying by ntype would make a consumer of
        # the input wait for the producer of the output)
        self._pending = {}   # id(table) -> RCCL work producing it
        self._ready = {}     # id(table) -> event on the side stream producing it
        self.side = (torch.cuda.Stream(device=shard.device)
                     if overlap and shard.device.type == 'cuda' else None)
        # (reserve_cus, dynamic) of the row kernels (ops.set_concurrency) during the pass:
        # rows come from the device work queue (each XCD on its own contiguous range; C4
        # one GPU 149 -> 144 ms), and with several ranks RESERVE_CUS CUs stay free so
        # RCCL's kernels find room, while aggregation blocks that start behind one take
        # fewer rows instead of ending the launch a collective late
        # (tools/probe_comm_overlap.py).  Default on HIP devices: (0, True) at one rank,
        # (RESERVE_CUS, True) at several with overlap on.
        if concurrency is None and shard.device.type == 'cuda':
            concurrency = (RESERVE_CUS if multi_rank(self.ex) and self.side is not None else 0,
                           True)
        self.concurrency = concurrency
        self.timers = None  # optional callable(tag) -> context manager (bench)
        self.side_delay_us = 0  # tests: a delay kernel ahead of every side-stream task
        self.capture = None  # optional list: every layer's output tables are appended (tests)
        self.progress = None  # optional callable(layer index) at every layer's start (bench)
        self.fused = set()  # relations whose aggregation ran with the projection fused
        self.pair_fused = set()  # (ce_a, ce_b) run as one two-relation launch
        self.pair_raw = set()  # ... of them, the one-table form (gnnrec_spmm_pair_f32)
        self.tile_pairs = set()  # (relation a, relation b) whose tiles ran as one launch
        self._pool = {}  # scratch tables reused across passes (_scratch)
        self._scratch_ev = {}  # scratch key -> event of the side-stream work reading it
        self._last, self._replicate_last = False, True

    def _scratch(self, key, shape, device):
        """A per-runner scratch table reused by every pass (tile partials, unfused
        aggregates): the pass allocates the same shapes every time, and tables that the
        side-stream GEMMs read (record_stream) would otherwise park freed blocks in the
        caching allocator until that stream catches up, growing the pool by tens of GB per
        pass and stalling on fresh hipMallocs (C5: reserved 17 -> 175 GiB over 10 passes, 2 s
        host stalls).  Reuse is ordered by the pass itself: a partial is read by the tree and
        the exchange, which the owner's GEMM waits for, before the next layer's tiles write
        it; an aggregate is read by the side-stream GEMM whose output the next layer waits
        for before it reaches the same relation."""
        t = self._pool.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != torch.device(device):
            t = torch.empty(shape, dtype=torch.float32, device=device)
            self._pool[key] = t
        return t

    def _par(self) -> int:
        """Scratch set of this layer's replicated-type partials: alternating by layer when
        the previous layer's tree + GEMMs may still read theirs on the side stream."""
        return self._layer_idx % 2 if getattr(self, '_owned_side', False) else 0

    def _get(self, h, nt):
        """h[nt], ready for reading on the CURRENT stream.  A table is produced either by a
        collective (its work handle in _pending) or on the side stream (its event in
        _ready), and may be read on both streams — at one rank the replicated table is read
        by the side stream's tree + GEMMs and by main's item->user launch — so readiness is
        never consumed by the first reader: a waited work becomes an event recorded on the
        stream that waited, kept in _ready for every later reader (until the layer that
        reads the table is done, _prune_ready)."""
        t = h[nt]
        key = id(t)
        cur = torch.cuda.current_stream(self.shard.device) if t.is_cuda else None
        ev = self._ready.get(key)
        if ev is not None and cur is not None:
            cur.wait_event(ev)
        w = self._pending.pop(key, None)
        if w is not None:
            w.wait()
            if cur is not None:
                ev = torch.cuda.Event()
                ev.record(cur)
                self._ready[key] = ev
        return t

    def _prune_ready(self, h):
        """Drop readiness of tables no longer in h (a freed table's id can be reused)."""
        live = {id(t) for t in h.values()}
        self._ready = {k: v for k, v in self._ready.items() if k in live}

    def _side_delay(self):
        """Test hook (side_delay_us): hold the side stream before its work, so a reader
        that skips a wait on it reads the table before it is written."""
        if self.side_delay_us and self.side is not None:
            self.ops.hold_cus(8, self.side_delay_us, stream=self.side)

    def _time(self, tag):
        import contextlib
        return self.timers(tag) if self.timers is not None else contextlib.nullcontext()

    def _on_side(self, fn, *tensors):
        """Run fn() on the side stream after everything queued on main; returns its event."""
        if self.side is None:
            fn()
            return None
        main = torch.cuda.current_stream(self.shard.device)
        self.side.wait_stream(main)
        for t in tensors:  # keep the allocator from recycling them under the side stream
            t.record_stream(self.side)
        with torch.cuda.stream(self.side):
            self._side_delay()
            fn()
            ev = torch.cuda.Event()
            ev.record(self.side)
        return ev

    @torch.no_grad()
    def run(self, feats: Dict[str, torch.Tensor], embedding_layer: Optional[bool] = None,
            replicate_output: bool = True):
        """feats: this rank's inputs (see GraphShard.local_features) -> this rank's outputs:
        {ptype: [n_own, out]} and the replicated types as full padded tables, or — with
        replicate_output=False — as this rank's own row block of them (own_slice), so the
        last layer's all-gather is skipped and every type's output stays partitioned."""
        mode = getattr(self.ops, 'concurrency', None)
        if self.concurrency is None or mode is None:
            return self._run(feats, embedding_layer, replicate_output)
        with mode(*self.concurrency):
            return self._run(feats, embedding_layer, replicate_output)

    def _run(self, feats, embedding_layer, replicate_output):
        m, O, sh = self.model, self.ops, self.shard
        self._replicate_last = replicate_output
        self._pending.clear()
        self._ready.clear()
        self._fold.clear()
        self._folded_types.clear()
        if embedding_layer is None:
            embedding_layer = m.embedding_layer
        h = dict(feats)
        if embedding_layer:
            embeds = [(nt, getattr(m, nt + '_embed', None)) for nt in ('item', 'sport', 'user')]
            for nt, mod in embeds:
                if mod is None or nt not in h:
                    continue
                W, b, x = mod.proj_feats.weight, mod.proj_feats.bias, h[nt]
                if self.fold_embedding and m.layers and self._foldable(m.layers[0], h, nt, W):
                    self._fold[nt] = (W, b)
                    self._folded_types.add(nt)
                    continue  # h[nt] stays the raw features
                if nt == sh.ptype and self.side is not None:
                    y = torch.empty((x.shape[0], W.shape[0]), dtype=torch.float32, device=x.device)
                    self._ready[id(y)] = self._on_side(
                        lambda: O.gemm(x, W, bias=b, out=y), x, y)
                    h[nt] = y
                else:
                    h[nt] = O.gemm(x, W, bias=b)
        # one rank with a side stream: the replicated type's tree + projection GEMMs run on
        # the side stream under the partitioned type's (HBM-bound) aggregation of the same
        # layer; the tile partials then alternate between two scratch sets by layer parity
        self._owned_side = not multi_rank(self.ex) and self.side is not None and \
            os.environ.get("GNNREC_OWNED_SIDE", "1") != "0"
        for i, layer in enumerate(m.layers):
            self._layer_idx = i
            self._last = i == len(m.layers) - 1
            if self.progress is not None:
                self.progress(i)
            h = self._layer(layer, h)
            self._prune_ready(h)
            if self.capture is not None:
                for nt in list(h):
                    self._get(h, nt)
                self.capture.append(dict(h))
        for nt in list(h):
            self._get(h, nt)
        return h

    def _foldable(self, hconv, h, nt, W_emb) -> bool:
        """A node type's NodeEmbedding (the partitioned users, and the replicated items,
        whose 1M-row embedding GEMM every rank would otherwise repeat) folds into every
        first-layer relation that touches nt: as the destination (W_self·W_e, bias W_self·b_e — fused kernel or GEMM
        alike) and as the source when the reducer is linear in the source rows and adds one
        b_e per non-empty row: mean, no fc_preagg (non-linear), no edge weights (they would
        scale b_e).  Needs the HIP backend (bias_nonempty) and W_e square at the fused width.
        Nothing here depends on the world size, so the deterministic mode folds too."""
        if getattr(self.ops, 'can_spmm_project', None) is None or \
                tuple(W_emb.shape) != (ops.FUSED_D, ops.FUSED_D):
            return False
        for ces in self._active(hconv, h).values():
            for ce in ces:
                if nt not in (ce[0], ce[2]):
                    continue
                preagg, weighted, reduce = hconv.mods[ce[1]]._plan_rel(ce)
                if reduce == 'lstm' or ce[0] == ce[2]:
                    return False
                if ce[0] == nt and (preagg or weighted or reduce != 'mean'):
                    return False
        return True

    def _folded(self, mod, ce):
        """(W_self, W_neigh, bias, bias_nonempty) of a fused launch, with a NodeEmbedding
        (W_e, b_e) folded in where its node type's raw features stand in for h:
        (x W_eᵀ + b_e) W_sᵀ = x (W_s W_e)ᵀ + W_s b_e; mean/sum over x[src] then W_n W_e,
        plus W_n b_e on rows that have neighbours."""
        Ws, Wn = mod.fc_self.weight, mod.fc_neigh.weight
        fd, fs = self._fold.get(ce[2]), self._fold.get(ce[0])
        if fd is None and fs is None:  # the parameters themselves: the ops detach them, and
            return Ws, Wn, None, None   # their transposes stay cached on them (ops._transposed)

        def ver(*ts):
            return tuple((id(t), t._version) for t in ts)

        key = ver(Ws, Wn, *(fd or ()), *(fs or ()))
        hit = self._fold_cache.get(ce)
        if hit is not None and hit[0] == key:
            return hit[1]
        Ws, Wn = Ws.detach(), Wn.detach()
        O, bias, bias_ne = self.ops, None, None
        # W @ W_e = linear(W, W_eᵀ); W @ b_e = linear(b_eᵀ, W) — the HIP GEMM, not vendor BLAS
        if fd is not None:
            We, be = fd[0].detach(), fd[1].detach()
            Ws, bias = (O.gemm(Ws, We.t().contiguous()),
                        O.gemm(be.view(1, -1).contiguous(), Ws).view(-1))
        if fs is not None:
            We, be = fs[0].detach(), fs[1].detach()
            Wn, bias_ne = (O.gemm(Wn, We.t().contiguous()),
                           O.gemm(be.view(1, -1).contiguous(), Wn).view(-1))
        self._fold_cache[ce] = (key, (Ws, Wn, bias, bias_ne))
        return Ws, Wn, bias, bias_ne

    @staticmethod
    def _attn(hconv, T, n_rows, device):
        """kwargs of the attention accumulate modes for dst type T (empty otherwise): the
        type's attention vector and a fresh per-row (running max, running sum) state."""
        if hconv.aggregate != 'attention':
            return {}
        return {'attn_vec': hconv.attn[T],
                'attn_state': torch.empty((n_rows, 2), dtype=torch.float32, device=device)}

    def _active(self, hconv, h):
        active: Dict[str, list] = {}
        for ce in self.shard.canonical_etypes:
            rs = self.shard.rels[ce]
            if rs.global_edges == 0 or ce[0] not in h or ce[2] not in h:
                continue
            active.setdefault(ce[2], []).append(ce)
        return active

    def _message(self, mod, ce, h, preagg):
        src = self._get(h, ce[0])
        return self.ops.gemm(src, mod.fc_preagg.weight, relu=True) if preagg else src

    def _partials(self, hconv, h, active):
        """user->item style relations: partial aggregates of the local edges -> reduce-scatter."""
        sh, O = self.shard, self.ops
        partials = {}
        for T, ces in active.items():
            if T == sh.ptype:
                continue
            tree_rels = []
            for ce in ces:
                mod = hconv.mods[ce[1]]
                preagg, weighted, reduce = mod._plan_rel(ce)
                rs = sh.rels[ce]
                msg = self._message(mod, ce, h, preagg)
                can_fuse = getattr(O, 'can_spmm_project', None)
                if self.deterministic and reduce in ('sum', 'mean'):
                    tree_rels.append((ce, rs, msg, weighted, reduce))
                    continue
                if rs.segs is not None and reduce != 'lstm':
                    # source-range tiles: each tile gathers from a slice of the source table
                    # small enough to stay in the Infinity Cache; accumulated in place
                    op = 'max' if reduce == 'max' else 'sum'
                    part = self._scratch(('part', ce, self._par()), (rs.n_rows, msg.shape[1]),
                                         msg.device)
                    for j, (ip, ix, w) in enumerate(rs.segs):
                        with self._time('spmm_tile'):
                            O.spmm(ip, ix, msg, op, edge_weight=w if weighted else None,
                                   empty_neginf=op == 'max', out=part, accumulate=j > 0,
                                   split=TILE_SPLIT)
                    own, work = self.ex.reduce_scatter_rows(part, op, async_op=self.overlap)
                    partials[ce] = (own, work, reduce)
                    continue
                if not multi_rank(self.ex) and reduce != 'lstm' and can_fuse is not None and \
                        not self.deterministic:
                    self_rows = self._get(h, T)
                    if can_fuse(rs.indptr, msg, self_rows, mod.fc_self.weight,
                                mod.fc_neigh.weight):
                        # one rank: no partials to exchange, aggregate + project in _owned
                        partials[ce] = ('fused', msg, reduce, weighted)
                        continue
                if reduce == 'lstm':
                    # the recurrence runs over each destination's whole in-edge sequence and
                    # does not split into per-rank partials: at P > 1 the owner of a block of
                    # destination rows runs it over their every in-edge, from the partitioned
                    # table all-gathered (every row: this reducer is off the reference's
                    # hyper-parameter space and is not sized for C4)
                    if multi_rank(self.ex):
                        ip, ix = sh.full_in_rows(ce)
                        src = self._gather_ptype(msg) if ce[0] == sh.ptype else msg
                        own = self._lstm(mod, ip, ix, src)
                    else:
                        own = self._lstm(mod, rs.indptr, rs.indices, msg)
                    partials[ce] = (own, None, reduce)
                    continue
                with self._time('spmm'):
                    part = O.spmm(rs.indptr, rs.indices, msg, 'max' if reduce == 'max' else 'sum',
                                  edge_weight=rs.weights if weighted else None,
                                  empty_neginf=reduce == 'max')
                own, work = self.ex.reduce_scatter_rows(part, 'max' if reduce == 'max' else 'sum',
                                                        async_op=self.overlap)
                partials[ce] = (own, work, reduce)
            partials.update(self._tree_partials(tree_rels))
        return partials

    def _lstm(self, mod, indptr, indices, m):
        """ConvLayer._lstm_reducer (src/model.py:106-121) over a CSR on this pass's backend."""
        L = mod.lstm
        return self.ops.lstm_aggregate(indptr, indices, m, L.weight_ih_l0, L.weight_hh_l0,
                                       L.bias_ih_l0, L.bias_hh_l0)

    def _gather_ptype(self, rows):
        """This rank's rows of the partitioned type -> the table of every rank's rows,
        `ptype_pad` rows per rank in rank order (GraphShard.full_in_rows numbers them)."""
        sh = self.shard
        S = sh.ptype_pad
        pad = torch.zeros((S, rows.shape[1]), dtype=rows.dtype, device=rows.device)
        pad[: rows.shape[0]] = rows
        out = torch.empty((S * self.ex.ws, rows.shape[1]), dtype=rows.dtype, device=rows.device)
        out, work = self.ex.all_gather_rows(pad, out, async_op=True)
        if work is not None:  # RCCL / the emulation: the current stream waits for it
            work.wait()
        return out

    def _tree_partials(self, rels):
        """Σ over each relation's segments in one fixed pairwise tree: the rank folds its
        own contiguous block of segments (a subtree), the all-to-all hands every owner the
        P subtree roots of its rows in rank order, and the owner folds those.  The tree is
        the same at every world size dividing the segment count.

        Relations into one destination type (C5: clicks and buys into items) run their
        tiles interleaved, tile j of every relation before tile j+1, so a relation's tile
        finds the source slice the previous relation's tile j just gathered from still
        partly in the Infinity Cache; each relation's result is unchanged (same kernels,
        same inputs)."""
        # the tree's leaf pairs are formed in the kernel (tile 2i+1 accumulated onto tile 2i:
        # the same single add), the upper levels by _tree_sum
        parts = {ce: [] for ce, *_ in rels}
        n_seg = max((len(rs.segs) for _, rs, *_ in rels), default=0)
        pairs = self._tile_pairs(rels)
        for j in range(n_seg):
            for item in pairs:
                if len(item) == 2:  # two relations, one launch per tile (gnnrec_spmm_csr2_f32)
                    (ca, ra, msg, weighted, _), (cb, rb, *_r) = item
                    self.tile_pairs.add((ca, cb))
                    sa, sb = ra.segs[j], rb.segs[j]
                    csr_a = (sa[0], sa[1], sa[2] if weighted else None)
                    csr_b = (sb[0], sb[1], sb[2] if weighted else None)
                    with self._time('spmm_tile2'):
                        if j % 2 == 0:
                            shp = (ra.n_rows, msg.shape[1])
                            pa, pb = self.ops.spmm2(
                                csr_a, csr_b, msg, 'sum',
                                out_a=self._scratch(('tile', ca, j, self._par()), shp,
                                                    msg.device),
                                out_b=self._scratch(('tile', cb, j, self._par()), shp,
                                                    msg.device))
                            parts[ca].append(pa)
                            parts[cb].append(pb)
                        else:
                            self.ops.spmm2(csr_a, csr_b, msg, 'sum', out_a=parts[ca][-1],
                                           out_b=parts[cb][-1], accumulate=True)
                    continue
                ce, rs, msg, weighted, _ = item[0]
                if j >= len(rs.segs):
                    continue
                ip, ix, w = rs.segs[j]
                ew = w if weighted else None
                with self._time('spmm_tile'):
                    if j % 2 == 0:
                        parts[ce].append(self.ops.spmm(
                            ip, ix, msg, 'sum', edge_weight=ew, split=TILE_SPLIT,
                            out=self._scratch(('tile', ce, j, self._par()),
                                              (rs.n_rows, msg.shape[1]), msg.device)))
                    else:
                        self.ops.spmm(ip, ix, msg, 'sum', edge_weight=ew, out=parts[ce][-1],
                                      accumulate=True, split=TILE_SPLIT)
        out = {}
        for ce, rs, msg, weighted, reduce in rels:
            if not multi_rank(self.ex) and self._owned_side:
                # one rank, owner work on the side stream: the whole tree is folded there
                # (_owned), off the main stream that runs the pair launch's inputs next
                out[ce] = (parts[ce], None, reduce, 'tree_local')
                continue
            blocks, work = self.ex.all_to_all_rows(_tree_sum(parts[ce], self.ops),
                                                   async_op=self.overlap)
            out[ce] = (blocks, work, reduce, 'tree')  # the owner's fold waits for the exchange
        return out

    def _tile_pairs(self, rels):
        """Relations of one destination type grouped for the tile launches: two relations
        that gather from the same table with the same segments and no heavy tile rows run as
        one launch per tile (ops.spmm2: C5's clicks and buys); the rest alone.  Each pair's
        partials are bitwise those of separate launches."""
        pair_ok = getattr(self.ops, 'spmm2', None) is not None
        out, used = [], set()
        for i, a in enumerate(rels):
            if i in used:
                continue
            used.add(i)
            for k in range(i + 1, len(rels)):
                b = rels[k]
                if not pair_ok or k in used or b[2] is not a[2] or b[3] != a[3] or \
                        b[1].n_rows != a[1].n_rows or len(b[1].segs) != len(a[1].segs) or \
                        a[2].shape[1] > 256 or a[2].shape[1] % 4:
                    continue
                segs = a[1].segs + b[1].segs
                if any(not sg[0].is_cuda or ops.split_plan(sg[0], TILE_SPLIT) is not None
                       for sg in segs):
                    continue
                if a[3] and any(sg[2] is None for sg in segs):
                    continue
                used.add(k)
                out.append((a, b))
                break
            else:
                out.append((a,))
        return out

    def _local(self, hconv, h, active, out):
        """item->user style relations: dst rows owned here; GEMMs on the side stream."""
        sh, O = self.shard, self.ops
        T = sh.ptype
        ces = active.get(T, [])
        if not ces:
            return
        if len(ces) == 2 and self._pair(hconv, h, ces, out):
            return
        R = len(ces)
        # the self rows of the partitioned type were produced on the side stream (or by main
        # when not overlapping): the side-stream GEMM is ordered after them without making
        # the main stream wait, so this relation's aggregation can start right away
        self_rows = h[T] if self.side is not None else self._get(h, T)
        o = None
        ev = None
        can_fuse = getattr(O, 'can_spmm_project', None)
        for j, ce in enumerate(ces):
            mod = hconv.mods[ce[1]]
            preagg, weighted, reduce = mod._plan_rel(ce)
            rs = sh.rels[ce]
            msg = self._message(mod, ce, h, preagg)
            acc, div = hconv.accum_mode(j, R)
            avg = (rs.global_edges / max(sh.num_nodes[T], 1)) if self.deterministic else None
            # a pre-projected low-degree relation fuses even beside a side stream: its
            # MFMA runs the self half only (C5 bought-by: 10.6 + 0.4 ms vs 7.6 ms gather +
            # a 7 ms GEMM contending with the tiles for HBM)
            pre = reduce != 'lstm' and getattr(O, 'preproject_pays', None) is not None and \
                O.preproject_pays(msg.shape[0], rs.n_rows, reduce)
            if reduce != 'lstm' and can_fuse is not None and can_fuse(
                    rs.indptr, msg, self_rows, mod.fc_self.weight, mod.fc_neigh.weight,
                    avg_deg=avg, gemm_overlaps=self.side is not None and not pre):
                # aggregation and projection in one launch on the main stream: the self rows
                # must be ready here (they may come from the side stream)
                self_rows = self._get(h, T)
                if ev is not None:  # an earlier relation's projection ran on the side stream
                    torch.cuda.current_stream(self.shard.device).wait_event(ev)
                    ev = None
                if o is None:
                    o = torch.empty((sh.n_own, mod._out_feats), dtype=torch.float32,
                                    device=msg.device)
                    akw = self._attn(hconv, T, sh.n_own, o.device)
                Ws, Wn, bias, bias_ne = self._folded(mod, ce)
                vkw = {} if avg is None else {'avg_deg': avg}  # same kernel on every rank
                if O.fused_preprojects(rs.indptr, msg, self_rows, reduce, avg):
                    with self._time('preproject'):
                        msg = O.preproject(msg, Wn, out=self._scratch(
                            ('pre', ce), (msg.shape[0], Wn.shape[0]), msg.device))
                    Wn = None
                with self._time(self._fused_tag(rs, avg)):
                    O.spmm_project(rs.indptr, rs.indices, msg, self_rows, Ws, Wn, reduce,
                                   rs.weights if weighted else None, relu=True,
                                   l2norm=bool(mod.norm), accum=acc, out_div=div, out=o,
                                   bias=bias, bias_nonempty=bias_ne, **akw, **vkw)
                self.fused.add(ce)
                continue
            with self._time('spmm'):
                ev_prev = self._scratch_ev.pop(('agg', ce), None)
                if ev_prev is not None:  # the last side-stream GEMM that read this scratch
                    torch.cuda.current_stream(self.shard.device).wait_event(ev_prev)
                a = (self._lstm(mod, rs.indptr, rs.indices, msg) if reduce == 'lstm' else
                     O.spmm(rs.indptr, rs.indices, msg, reduce,
                            edge_weight=rs.weights if weighted else None,
                            out=self._scratch(('agg', ce), (rs.n_rows, msg.shape[1]),
                                              msg.device)))
            if o is None:
                o = torch.empty((sh.n_own, mod._out_feats), dtype=torch.float32, device=a.device)
                akw = self._attn(hconv, T, sh.n_own, o.device)

            Ws, Wn, bias, bias_ne = self._folded(mod, ce)
            # a folded source-side embedding adds W_n b_e on rows that have neighbours
            fkw = {} if bias_ne is None else {'bias_nonempty': bias_ne,
                                              'a2_deg': self._local_deg(rs)}

            def proj(Ws=Ws, Wn=Wn, bias=bias, mod=mod, a=a, acc=acc, div=div, o=o, akw=akw,
                     fkw=fkw):
                O.gemm(self_rows, Ws, a, Wn, bias, relu=True, l2norm=bool(mod.norm), accum=acc,
                       out_div=div, out=o, **akw, **fkw)
            ev = self._on_side(proj, self_rows, a, o, *akw.values(), *fkw.values(),
                               *(t for t in (Ws, Wn, bias) if t is not None))
            if ev is not None:
                self._scratch_ev[('agg', ce)] = ev
        out[T] = o
        if ev is not None:
            self._ready[id(o)] = ev

    def _pair_stage(self, plan, h):
        """The pair launch's inputs: both relations' messages pre-projected (the source
        tables × W_neigh,r, into per-relation scratch), the self weights and biases."""
        O = self.ops
        msgs = [self._message(mod, ce, h, preagg) for mod, ce, _, preagg, _, _ in plan]
        rels, Wself, biases = [], [], []
        for (mod, ce, rs, _, weighted, reduce), msg in zip(plan, msgs):
            Ws, Wn, bias, bias_ne = self._folded(mod, ce)
            with self._time('preproject'):
                Y = O.preproject(msg, Wn, out=self._scratch(
                    ('pre', ce), (msg.shape[0], Wn.shape[0]), msg.device))
            rels.append((rs.indptr, rs.indices, Y, reduce, rs.weights if weighted else None,
                         bias_ne))
            Wself.append(Ws)
            biases.append(bias)
        return rels, Wself, biases

    def _pair(self, hconv, h, ces, out) -> bool:
        """Exactly two relations into the partitioned type, both linear (sum / mean) with a
        source table at most half the destination count (C5: clicked-by and bought-by
        from the 1M items into the 10M users): both source tables pre-projected, then one
        spmm_project2 launch reads each user row once and writes it once (C5 user side
        39.0 ms vs 41.0 ms for the two fused launches).
        In deterministic mode the decision uses the global user count (same on every
        rank); the HeteroGraphConv combine runs in the kernel (sum, mean as /2, max, the
        attention softmax over the two relations)."""
        sh, O = self.shard, self.ops
        T = sh.ptype
        plan = self._pair_plan(hconv, h, ces)
        if plan is None:
            return False
        mod = plan[0][0]
        from .nn import _pair_combine
        combine, div = _pair_combine(hconv.aggregate)
        if self._pair_raw(plan):
            # both relations gather the SAME raw source table: no pre-projection, the four
            # projections in the launch's MFMA epilogue (gnnrec_spmm_pair_f32) — the gathered
            # working set is one 512 MB table at C5 instead of two pre-projected ones
            X = self._get(h, plan[0][1][0])
            self_rows = self._get(h, T)
            rels, Wts = [], []
            for m, ce, rs, _, weighted, reduce in plan:
                Ws, Wn, bias, bias_ne = self._folded(m, ce)
                rels.append((rs.indptr, rs.indices, reduce, rs.weights if weighted else None,
                             bias_ne))
                Wts.append((Ws, Wn, bias))
            o = torch.empty((sh.n_own, mod._out_feats), dtype=torch.float32,
                            device=self_rows.device)
            with self._time('spmm_pair'):
                O.spmm_pair(rels[0], rels[1], X, self_rows, Wts[0][0], Wts[0][1], Wts[1][0],
                            Wts[1][1], Wts[0][2], Wts[1][2], relu=True,
                            l2norm=bool(mod.norm), combine=combine, out_div=div, out=o,
                            attn_vec=hconv.attn[T] if combine == 'attention' else None)
            self.pair_fused.add((ces[0], ces[1]))
            self.pair_raw.add((ces[0], ces[1]))
            out[T] = o
            return True
        rels, Wself, biases = self._pair_stage(plan, h)
        self_rows = self._get(h, T)
        o = torch.empty((sh.n_own, mod._out_feats), dtype=torch.float32,
                        device=self_rows.device)
        with self._time('spmm_project2'):
            O.spmm_project2(rels[0], rels[1], self_rows, Wself[0], Wself[1], biases[0],
                            biases[1], relu=True, l2norm=bool(mod.norm), combine=combine,
                            out_div=div, out=o,
                            attn_vec=hconv.attn[T] if combine == 'attention' else None)
        self.pair_fused.add((ces[0], ces[1]))
        out[T] = o
        return True

    def _pair_raw(self, plan) -> bool:
        """The pair gathers one raw table (gnnrec_spmm_pair_f32) when GNNREC_PAIR_RAW=1, both
        relations come from the same source type with no fc_preagg (their messages are that
        table itself) and the backend has the op.  Off by default: at C5 the pre-projected
        launch plus its GEMMs is 0.5 ms faster per pass (csrc/spmm_pair_mfma.hip)."""
        return getattr(self.ops, 'spmm_pair', None) is not None and \
            os.environ.get("GNNREC_PAIR_RAW", "0") != "0" and \
            plan[0][1][0] == plan[1][1][0] and not plan[0][3] and not plan[1][3]

    def _pair_plan(self, hconv, h, ces):
        """The two relations of a pair launch, or None (shapes and layouts only: nothing is
        launched or waited for)."""
        sh, O = self.shard, self.ops
        T = sh.ptype
        if getattr(O, 'spmm_project2', None) is None or \
                hconv.aggregate not in ('sum', 'mean', 'max', 'attention'):
            return None
        n_dec = sh.num_nodes[T] if self.deterministic else sh.n_own
        plan = []
        for ce in ces:
            mod = hconv.mods[ce[1]]
            preagg, weighted, reduce = mod._plan_rel(ce)
            rs = sh.rels[ce]
            src = h.get(ce[0])
            if reduce not in ('sum', 'mean') or src is None or \
                    not O.preproject_pays(src.shape[0], n_dec, reduce):
                return None
            plan.append((mod, ce, rs, preagg, weighted, reduce))
        if bool(plan[0][0].norm) != bool(plan[1][0].norm):
            return None
        # eligibility from the tables' shapes and layouts before anything is launched or
        # waited for (a message is the source table itself, or fc_preagg's fresh output of
        # the same shape): a refused pair costs no GEMM and no main-stream wait
        for mod, ce, rs, _, _, _ in plan:
            if not O.can_spmm_project(rs.indptr, h[ce[0]], h[T], mod.fc_self.weight,
                                      mod.fc_neigh.weight):
                return None
        return plan

    def _fused_tag(self, rs, avg):
        """timer tag of a fused launch: 'spmm_project' (VALU kernel) or 'spmm_project_mfma'."""
        fv = getattr(self.ops, 'fused_variant', None)
        return 'spmm_project_mfma' if fv is not None and fv(rs.indptr, avg) == 'mfma' \
            else 'spmm_project'

    @staticmethod
    def _local_deg(rs):
        """int32 in-degrees of a locally owned relation's rows (cached on the relation)."""
        if getattr(rs, '_deg_i32', None) is None:
            rs._deg_i32 = (rs.indptr[1:] - rs.indptr[:-1]).to(torch.int32)
        return rs._deg_i32

    def _owned(self, hconv, h, active, partials, out):
        """owners project their replicated rows, then all-gather the table."""
        sh, O = self.shard, self.ops
        for T, ces in active.items():
            if T == sh.ptype:
                continue
            R = len(ces)
            o = None
            self_rows = self._get(h, T)[sh.own_slice(T)]
            akw = self._attn(hconv, T, self_rows.shape[0], self_rows.device)
            for j, ce in enumerate(ces):
                mod = hconv.mods[ce[1]]
                acc, div = hconv.accum_mode(j, R)
                if isinstance(partials[ce][0], str):  # ('fused', msg, reduce, weighted)
                    _, msg, reduce, weighted = partials[ce]
                    rs = sh.rels[ce]
                    if o is None:
                        o = torch.empty((self_rows.shape[0], mod._out_feats),
                                        dtype=torch.float32, device=msg.device)
                    Ws, Wn, bias, bias_ne = self._folded(mod, ce)
                    with self._time(self._fused_tag(rs, None)):
                        O.spmm_project(rs.indptr, rs.indices, msg, self_rows, Ws, Wn, reduce,
                                       rs.weights if weighted else None, relu=True,
                                       l2norm=bool(mod.norm), accum=acc, out_div=div, out=o,
                                       bias=bias, bias_nonempty=bias_ne, **akw)
                    self.fused.add(ce)
                    continue
                own, work, reduce = partials[ce][:3]
                if work is not None:
                    work.wait()
                if len(partials[ce]) == 4 and partials[ce][3] == 'tree_local':
                    own = _tree_sum(own, self.ops)  # one rank: the segments' whole tree
                elif len(partials[ce]) == 4:  # deterministic: fold the P subtree roots
                    own = _tree_sum(list(own.unbind(0)), self.ops)
                if o is None:
                    o = torch.empty((own.shape[0], mod._out_feats), dtype=torch.float32,
                                    device=own.device)
                Ws, Wn, bias, bias_ne = self._folded(mod, ce)
                fkw = {} if bias_ne is None else {'bias_nonempty': bias_ne}
                O.gemm(self_rows, Ws, own, Wn, bias, relu=True,
                       l2norm=bool(mod.norm), accum=acc, out_div=div, out=o,
                       a2_deg=sh.rels[ce].deg_own,
                       a2_mode=(_lib.A2_NONE if reduce == 'lstm' else
                                _lib.A2_ZERO_DEG if reduce == 'max' else _lib.A2_DIV_DEG),
                       **akw, **fkw)
            if not multi_rank(self.ex) or (self._last and not self._replicate_last):
                out[T] = o  # the owned rows ARE the table (one rank), or stay partitioned
                continue
            table = torch.empty((sh.padded_rows(T), o.shape[1]), dtype=torch.float32,
                                device=o.device)
            table, work = self.ex.all_gather_rows(o, table, async_op=self.overlap)
            if work is not None:
                self._pending[id(table)] = work
            out[T] = table

    def _owned_on_side(self, hconv, h, active, partials, out):
        """_owned on the side stream (one rank): ordered after the tiles queued on main,
        its outputs handed to later main-stream readers by an event (_get)."""
        main = torch.cuda.current_stream(self.shard.device)
        self.side.wait_stream(main)
        produced = {}
        with torch.cuda.stream(self.side):
            self._side_delay()
            self._owned(hconv, h, active, partials, produced)
            ev = torch.cuda.Event()
            ev.record(self.side)
        for T, t in produced.items():
            t.record_stream(main)  # read on main later: not recycled under it
            self._ready[id(t)] = ev
            out[T] = t

    def _layer(self, hconv, h):
        active = self._active(hconv, h)
        out = {}
        if self._owned_side:
            # tiles (main) -> tree + GEMMs of the replicated type (side) under the
            # partitioned type's launch (main), whose inputs are the previous layer's
            # (the tiles' tree is folded on the side stream too: the partitioned type's
            # launch follows the tiles at once — C4 143.2 -> 142.9 ms, C5 152.3 -> 151.5)
            partials = self._partials(hconv, h, active)
            self._owned_on_side(hconv, h, active, partials, out)
            self._local(hconv, h, active, out)
            self._fold.clear()
            return out
        if multi_rank(self.ex):
            partials = self._partials(hconv, h, active)
            self._local(hconv, h, active, out)
        else:
            self._local(hconv, h, active, out)
            partials = self._partials(hconv, h, active)
        self._owned(hconv, h, active, partials, out)
        self._fold.clear()  # a folded embedding only stands in for the first layer's input
        return out


def _tree_sum(parts: List[torch.Tensor], O) -> torch.Tensor:
    """Pairwise tree ((p0+p1)+(p2+p3))+... over a power-of-two list, in order, in place into
    the left operand: subtrees of up to 8 leaves folded by one tree_sum_ kernel each (every
    table read once; the same additions as one add kernel per node, bitwise)."""
    parts = [p.contiguous() for p in parts]
    tree = getattr(O, "tree_sum_", None)
    aligned = all(p.data_ptr() % 16 == 0 and p.numel() % 4 == 0 for p in parts)
    while len(parts) > 1:
        g = min(8, len(parts))
        if tree is not None and aligned:
            parts = [tree(parts[i:i + g]) for i in range(0, len(parts), g)]
        else:
            parts = [O.add_(parts[i], parts[i + 1]) for i in range(0, len(parts), 2)]
    return parts[0]


def gather_partitioned(shard: GraphShard, rows: torch.Tensor, exchange: Exchange) -> torch.Tensor:
    """Assemble the full [N_ptype, d] table from every rank's owned rows (tests/tools)."""
    if exchange.ws == 1:
        return rows
    import torch.distributed as dist
    b = shard.bounds
    S = max(b[r + 1] - b[r] for r in range(exchange.ws))
    pad = torch.zeros((S, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    pad[: rows.shape[0]] = rows
    parts = [torch.empty_like(pad) for _ in range(exchange.ws)]
    dist.all_gather(parts, pad, group=exchange.group)
    return torch.cat([parts[r][: b[r + 1] - b[r]] for r in range(exchange.ws)], 0)


@torch.no_grad()
def inference_ondemand(graph, trained_model, user_ids='all', k: int = 10,
                       already_bought_dict=None, remove_already_bought: bool = True,
                       pred: str = 'cos', use_popularity: bool = False,
                       weight_popularity: float = 1.0, embedding_layer=None):
    """Embedding pass + recommendations on the device, the hot part of reference
    main_inference.py:20-175 (`inference_ondemand`): full-graph embeddings of every
    user and item (:123-152), then top-k per requested user with already-bought items
    removed (:153-166).  `graph` is a HeteroGraph (or a path written by gnnrec.io).

    Returns (recs {user: np.ndarray[k]}, embeddings {ntype: tensor})."""
    import numpy as np

    from .io import read_graph
    from .recs import create_already_bought, get_recs
    g = read_graph(graph, device=torch.device('cuda')) if isinstance(graph, str) else graph
    trained_model.eval()
    h = full_graph_embeddings(g, trained_model, embedding_layer=embedding_layer)
    if isinstance(user_ids, str) and user_ids == 'all':
        user_ids = np.arange(g.num_nodes('user'))
    if already_bought_dict is None:
        users = torch.as_tensor(user_ids, device=g.device)
        s, _ = g.all_edges(etype='buys')
        bought = torch.nonzero(torch.isin(s, users)).squeeze(1)
        already_bought_dict = create_already_bought(g, bought, etype='buys')
    out_dim = h['item'].shape[1]
    recs = get_recs(g, h, trained_model, out_dim, k, list(np.asarray(user_ids).tolist()),
                    already_bought_dict, remove_already_bought, True, g.device, pred,
                    use_popularity, weight_popularity)
    return recs, h
