"""GPU block sampling and loaders — drop-ins for the DGL 0.5.2 dataloading API
used by reference src/sampling.py:117-243 and main_inference.py:124-138.

  MultiLayerFullNeighborSampler(n_layers)        sampling.py:157, main_inference.py:129
  MultiLayerNeighborSampler(fanouts, replace=False)  sampling.py:159
  negative_sampler.Uniform(k)                    sampling.py:163-165
  NodeDataLoader(g, nids, sampler, batch_size, shuffle, drop_last, ...)  :209-241
  EdgeDataLoader(g, eids, sampler, exclude='reverse_types', reverse_etypes,
                 g_sampling, negative_sampler, batch_size, shuffle, ...)  :167-207

Everything runs on the device in the caller's process: per relation the
in-edges of the seeds are counted, scanned and copied by the HIP sampler
(gnnrec_sample_count/fill — fanout choices by a counter hash, eid exclusion
after sampling as DGL's BlockSampler does), then per node type the sources
are relabelled by mark/scan/compact (dst prefix first, new ids ascending).
There are no DataLoader worker processes, no pinned host copies and no
per-batch host->device transfer of blocks (reference run.py:104-107, 338-339).
`num_workers > 0` (the reference's asynchronous DataLoader workers) samples
ahead instead: one host thread builds the next batches on a second HIP stream
while the caller's stream runs the training step, and each batch is handed over
through a stream event (at most `num_workers` batches in flight).  Sampling in
that thread draws from the CUDA generator concurrently with the caller, so the
batch sequence is reproducible only when the caller draws no random numbers
(dropout 0).  `pin_memory` is accepted and ignored.
"""
from __future__ import annotations

import queue
import threading
import weakref
from typing import Dict, List, Optional

import torch

from . import ops
from .graph import Block, EID, HeteroGraph, LazyRows, NID, PairGraph

# The loaders' draws from torch's default CUDA generator (negatives, an epoch's shuffle) and a
# hipGraph capture (capture.CapturedTrainStep) exclude each other: while a capture is under
# way torch refuses a draw from any stream that is not capturing ("Offset increment outside
# graph capture"), and a sampling thread's draws are exactly that.
RNG_LOCK = threading.RLock()


def _mix(*xs) -> int:
    h = 0x9E3779B97F4A7C15
    for x in xs:
        h = ((h ^ (int(x) & 0xFFFFFFFFFFFFFFFF)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        h ^= h >> 31
    return h


class BlockSampler:
    """Multi-layer block sampler base (DGL BlockSampler.sample_blocks semantics)."""

    def __init__(self, num_layers: int, fanouts=None, replace: bool = False, seed: int = None):
        if replace:
            raise NotImplementedError("sampling with replacement is not used by the reference")
        self.num_layers = num_layers
        self.fanouts = fanouts
        self.seed = int(seed) if seed is not None else int(torch.initial_seed())
        self._calls = 0
        self._relabelers = {}
        self._exclude_masks = {}
        # bounded fanouts: every block of a call in one fused op (ops.sample_blocks); False
        # keeps the per-layer ops (the blocks are bitwise the same; tests compare the two)
        self.fused = True
        # the fused sampler reads the CSR as packed 8-byte edge records (HeteroGraph
        # .edge_records) when every eid fits 31 bits; False: the index and eid arrays
        # (bitwise the same blocks; tests compare the two)
        self.packed = True
        # static-shape blocks hold their block data as LazyRows (gathered when read); False:
        # gathered by the sampler call like the exact blocks' (the same values)
        self.lazy_static_data = True
        self._sb_scratch = {}
        self._stamp = 1
        # the first block's source-major CSRs (sample_blocks(transposes=True)) are skipped
        # for first blocks of at least this many source rows: a model that folds its
        # NodeEmbeddings into the first layer (nn.ConvModel._folded_first_layer) never reads
        # them there and sets the bound it folds from (None: always build them)
        self.first_transposes_below = None

    def _fanout(self, block_id: int, ce) -> int:
        if self.fanouts is None:
            return -1
        f = self.fanouts[block_id]
        if isinstance(f, dict):
            f = f.get(ce, f.get(ce[1], -1))
        return -1 if f is None else int(f)

    def _relabeler(self, g, nt):
        key = (id(g), nt)
        r = self._relabelers.get(key)
        if r is None:
            r = ops.Relabeler(g.num_nodes(nt), g.device)
            self._relabelers[key] = r
        return r

    def _mask(self, g, ce):
        key = (id(g), ce)
        m = self._exclude_masks.get(key)
        if m is None:
            m = torch.zeros(g.num_edges(ce), dtype=torch.uint8, device=g.device)
            self._exclude_masks[key] = m
        return m

    def _mask_rows(self, g, ce):
        """Per dst node of ce: 1 on the dst of an excluded eid (set and cleared with the
        mask): the sampler kernels check eids only for those seeds."""
        key = (id(g), ce, 'rows')
        m = self._exclude_masks.get(key)
        if m is None:
            m = torch.zeros(g.num_nodes(ce[2]), dtype=torch.uint8, device=g.device)
            self._exclude_masks[key] = m
        return m

    def _fused_ok(self, g) -> bool:
        """Every block of a call in one ops.sample_blocks: bounded fanouts (0..64) for every
        block and relation, on a HIP device, within the fused op's limits."""
        if not self.fused or g.device.type != "cuda" or self.fanouts is None:
            return False
        ces = g.canonical_etypes
        if not (1 <= self.num_layers <= ops.SB_MAX_STEPS and len(ces) <= ops.SB_MAX_RELS
                and 1 <= len(g.ntypes) <= ops.SB_MAX_TYPES):
            return False
        return all(0 <= self._fanout(b, ce) <= ops.SB_MAX_FANOUT
                   for b in range(self.num_layers) for ce in ces)

    def _edge_recs(self, g, ces):
        """The packed edge records of every relation (HeteroGraph.edge_records), or [] —
        the fused sampler then reads the index and eid arrays (the same picks and blocks)."""
        if not self.packed or not hasattr(g, "edge_records"):
            return []
        recs = [g.edge_records(ce) for ce in ces]
        return [] if any(r is None for r in recs) else recs

    def _sample_fused(self, g, seeds, exclude_eids, transposes, static=False, hints=None,
                      overflow=None):
        """sample_blocks through gnnrec_sample_blocks: 1 + 3L launches and one host read for
        all L blocks (bitwise the blocks of the per-layer path, _one_block).

        static: the blocks at their capacities, nothing read back (include/gnnrec.h, static
        shapes): seeds may hold -1 padding; block s has seed_cap + D destination rows per
        type (the last D are its dump rows, at most 2048 edges each) and node_cap + D'
        source rows (the last D' are the next block's dump rows), so every layer's output is
        the next block's source table."""
        ces, nts = list(g.canonical_etypes), list(g.ntypes)
        tix = {nt: i for i, nt in enumerate(nts)}
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        L = self.num_layers
        scratch = []
        for nt in nts:
            key = (id(g), nt)
            sc = self._sb_scratch.get(key)
            if sc is None:
                sc = self._sb_scratch[key] = ops.SampleScratch(g.num_nodes(nt), g.device)
            scratch.append(sc)
        if self._stamp + L + 3 >= (1 << 32):  # never in practice: restart the stamps
            for sc in self._sb_scratch.values():
                sc.pos.zero_()
            self._stamp = 1
        stamp = self._stamp
        self._stamp += L + 1
        excl = [None] * len(ces)
        for ce, e in (exclude_eids or {}).items():
            ce = g.to_canonical_etype(ce)
            e = torch.as_tensor(e, dtype=torch.int64, device=g.device).reshape(-1)
            if e.numel():
                excl[ces.index(ce)] = (e, g._coo[ce][1], self._mask(g, ce),
                                       self._mask_rows(g, ce))
        csrs = [g.in_csr_global(ce) for ce in ces]
        # step s samples block L-1-s (the output block first), with that block's keys
        fans = [[self._fanout(L - 1 - s, ce) for ce in ces] for s in range(L)]
        keys = [[_mix(self.seed, self._calls, L - 1 - s, r) for r in range(len(ces))]
                for s in range(L)]
        NT, R = len(nts), len(ces)
        # the block data (DGL copies it at block creation; the reference reads
        # blocks[0].srcdata['features']) is gathered inside the call, behind the sampler and
        # ahead of its one size read; static: -1 ids -> zero rows
        etab = [(ce, k, v if v.dim() < 2 or v[0].is_contiguous() else v.contiguous())
                for ce in ces for k, v in g._edata[ce].items()]
        ntab = [(nt, k, v if v.dim() < 2 or v[0].is_contiguous() else v.contiguous())
                for nt in nts for k, v in g._ndata[nt].items()]
        lazy = static and self.lazy_static_data
        # static: the real counts stay on the device (sizes_out: [L + 1][T] node counts, the
        # seed counts first, then [L][R] edge counts) and drive the kernels over the blocks
        dsz = torch.empty((L + 1) * len(nts) + L * len(ces), dtype=torch.int64,
                          device=g.device) if static else None
        steps, sizes, data = ops.sample_blocks(
            [c[0] for c in csrs], [c[1] for c in csrs], [c[2] for c in csrs],
            [tix[ce[0]] for ce in ces], [tix[ce[2]] for ce in ces], excl,
            [g.num_nodes(nt) for nt in nts], [seeds.get(nt, empty) for nt in nts], scratch,
            fans, keys, stamp, static_shapes=static, sizes_out=dsz,
            node_cap_hint=[[(hints or {}).get((s_, nt), 0) for nt in nts] for s_ in range(L)]
            if hints else None, overflow=overflow,
            # static: the block data is left to LazyRows (gathered when read: inside a
            # captured step's graph, from its captured ids), not gathered here
            edge_tables=[] if lazy else [(v, ces.index(ce)) for ce, _k, v in etab],
            node_tables=[] if lazy else [(v, tix[nt]) for nt, _k, v in ntab],
            edge_recs=self._edge_recs(g, ces))
        blocks = []
        for s_, (o_ip, src_loc, o_eid, nodes) in enumerate(steps):
            rels = {}
            for r, ce in enumerate(ces):
                ip, loc, eid = o_ip[r], src_loc[r], o_eid[r]
                if static:  # sizes = seed caps, node caps [L x T], edge caps [L x R], dump rows
                    ip._gnnrec_nnz = int(sizes[NT + L * NT + s_ * R + r])
                    if 0 <= fans[s_][r] <= ops.DEFAULT_SPLIT:  # dump rows: <= 2048 edges
                        ip._gnnrec_split_plan = (ops.DEFAULT_SPLIT, None)
                else:
                    ip._gnnrec_nnz = int(sizes[(L + 1) * NT + s_ * R + r])
                    if 0 <= fans[s_][r] <= ops.DEFAULT_SPLIT:
                        ip._gnnrec_split_plan = (ops.DEFAULT_SPLIT, None)  # no heavy rows
                rels[ce] = (ip, loc, eid)
            if static:
                dump = [int(sizes[NT + L * NT + L * R + s_ * NT + t]) for t in range(NT)]
                num_dst = {nt: int(sizes[s_ * NT + t]) + dump[t] for t, nt in enumerate(nts)}
            else:
                num_dst = {nt: int(sizes[s_ * NT + t]) for t, nt in enumerate(nts)}
            b = Block(dict(zip(nts, nodes)), num_dst, rels)
            if static:
                # the destination ids are the step's seed slots (-1: padding rows, the dump
                # rows last), not the source prefix: a padding row may sit over a real source
                b.static = True
                # the real destination / source counts (device): the aggregation gathers the
                # real rows only, and the backward's transposed gathers the real sources
                for t, nt in enumerate(nts):
                    b._live[('dst', nt)] = dsz.narrow(0, s_ * NT + t, 1)
                    b._live[('src', nt)] = dsz.narrow(0, (s_ + 1) * NT + t, 1)
                for ce in ces:
                    rels[ce][0]._gnnrec_live = b._live[('dst', ce[2])]
                for t, nt in enumerate(nts):
                    if s_ == 0:
                        dst_ids = torch.cat([seeds.get(nt, empty),
                                             empty.new_full((dump[t],), -1)])
                    else:
                        dst_ids = steps[s_ - 1][3][t]
                    b._dst[nt][NID] = dst_ids
            blocks.insert(0, b)
        if lazy:  # -1 ids (padding edges / source slots) read as zero rows
            for b in blocks:
                for ce, k, v in etab:
                    b._edata[ce][k] = LazyRows(v, b._rels[ce][2])
            for nt, k, v in ntab:
                blocks[0]._src[nt][k] = LazyRows(v, blocks[0]._src[nt][NID])
        else:
            it = iter(data)
            for s_ in range(L):
                b = blocks[L - 1 - s_]
                for ce, k, _v in etab:
                    b._edata[ce][k] = next(it)
            for nt, k, _v in ntab:
                blocks[0]._src[nt][k] = next(it)
        if transposes:
            for block_id, b in enumerate(blocks):
                if block_id > 0 or self._first_transposes(b):
                    _add_transposes(b)
        return blocks

    def _first_transposes(self, block) -> bool:
        lim = self.first_transposes_below
        return lim is None or sum(block.number_of_src_nodes(nt) for nt in block.ntypes) < lim

    def sample_blocks(self, g: HeteroGraph, seed_nodes: Dict[str, torch.Tensor],
                      exclude_eids: Optional[Dict[tuple, torch.Tensor]] = None,
                      transposes: bool = False, static_shapes: bool = False,
                      node_cap_hint=None, overflow=None) -> List[Block]:
        """transposes: also build every relation's source-major CSR (Block._t), which the
        training backward gathers over — in the sampling thread (num_workers > 0), off the
        training thread (EdgeDataLoader, transposed_blocks=True).
        static_shapes: the blocks at fixed capacities with nothing read back (seeds may hold
        -1 padding; _sample_fused) — the batches of a captured training step.
        node_cap_hint {(step, ntype): capacity} and overflow (an int64 device flag): tighter
        static node capacities than the provable ones, and the flag a batch that does not fit
        them raises (EdgeDataLoader learns them from its first exact batches)."""
        self._calls += 1
        seeds = {nt: torch.as_tensor(v, dtype=torch.int64, device=g.device)
                 for nt, v in seed_nodes.items()}
        if static_shapes and not self._fused_ok(g):
            raise ValueError("static_shapes needs the fused sampler: bounded fanouts (0..64) "
                             "on a HIP device within its limits")
        if self._fused_ok(g):
            blocks = self._sample_fused(g, seeds, exclude_eids, transposes, static_shapes,
                                        node_cap_hint, overflow)
            for b in blocks:
                b._sampler = weakref.ref(self)
            return blocks
        masks = {}
        if exclude_eids:
            for ce, eids in exclude_eids.items():
                ce = g.to_canonical_etype(ce)
                m = self._mask(g, ce)
                m.index_fill_(0, eids, 1)  # (m[eids] = 1 copies the scalar: a host sync)
                rows = self._mask_rows(g, ce)
                dst = g.find_edges(eids, ce)[1]
                rows.index_fill_(0, dst, 1)
                masks[ce] = (m, eids, rows, dst)
        blocks = []
        try:
            for block_id in reversed(range(self.num_layers)):
                block = self._one_block(g, seeds, block_id, masks)
                if transposes and (block_id > 0 or self._first_transposes(block)):
                    _add_transposes(block)
                blocks.insert(0, block)
                seeds = {nt: block.srcdata[NID][nt] for nt in block.ntypes
                         if block.number_of_src_nodes(nt) > 0}
        finally:
            for ce, (m, eids, rows, dst) in masks.items():
                m.index_fill_(0, eids, 0)
                rows.index_fill_(0, dst, 0)
        _copy_block_data(g, blocks)
        for b in blocks:  # (the model's fold sets first_transposes_below through it)
            b._sampler = weakref.ref(self)
        return blocks

    def _one_block(self, g, seeds, block_id, masks) -> Block:
        """One layer: counts of every relation, ONE size readback, fills; then the
        new-source marks of every node type, ONE size readback, compaction/relabel —
        issued from C++ by the gnnrec::sample_layer op (same kernels, same order, same
        keys as _one_block_py, which stays as the readable form)."""
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        ces = list(g.canonical_etypes)
        nts = list(g.ntypes)
        tix = {nt: i for i, nt in enumerate(nts)}
        csrs = [g.in_csr_global(ce) for ce in ces]
        fans = [self._fanout(block_id, ce) for ce in ces]
        rel = [self._relabeler(g, nt) for nt in nts]
        o_ip, src_loc, o_eid, src_nid, totals = ops.sample_layer(
            [c[0] for c in csrs], [c[1] for c in csrs], [c[2] for c in csrs],
            [masks.get(ce, (None,))[0] for ce in ces], [tix[ce[0]] for ce in ces],
            [tix[ce[2]] for ce in ces], fans,
            [_mix(self.seed, self._calls, block_id, r) for r in range(len(ces))],
            [seeds.get(nt, empty) for nt in nts], [r.prefix_pos for r in rel],
            [r.mark for r in rel],
            mask_rows=[masks.get(ce, (None, None, None))[2] for ce in ces])
        rels = {}
        for r, ce in enumerate(ces):
            ip = o_ip[r]
            ip._gnnrec_nnz = int(totals[r])  # edge count known on the host: no later readback
            if fans[r] is not None and 0 <= fans[r] <= ops.DEFAULT_SPLIT:
                ip._gnnrec_split_plan = (ops.DEFAULT_SPLIT, None)  # no heavy rows possible
            rels[ce] = (ip, src_loc[r], o_eid[r])
        num_dst = {nt: int(seeds.get(nt, empty).numel()) for nt in nts}
        return Block(dict(zip(nts, src_nid)), num_dst, rels)

    def _one_block_py(self, g, seeds, block_id, masks) -> Block:
        """_one_block issued from Python, op by op (the reference form of the C++ op)."""
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        plan = []
        for r_idx, ce in enumerate(g.canonical_etypes):
            dseeds = seeds.get(ce[2], empty)
            indptr, indices, eids = g.in_csr_global(ce)
            key = _mix(self.seed, self._calls, block_id, r_idx)
            mask, _e, mrows = masks.get(ce, (None, None, None))[:3]
            fan = self._fanout(block_id, ce)
            o_ip = ops.sample_count(indptr, eids, dseeds, fan, key, mask, mrows)
            plan.append((ce, indptr, indices, eids, dseeds, fan, key, (mask, mrows), o_ip))
        totals = torch.stack([p[-1][-1] for p in plan]).tolist() if plan else []
        rels = {}
        src_lists: Dict[str, list] = {}
        for (ce, indptr, indices, eids, dseeds, fan, key, mask, o_ip), tot in zip(plan, totals):
            o_src, o_eid = ops.sample_fill(indptr, indices, eids, dseeds, fan, key, o_ip, tot,
                                           *mask)
            o_ip._gnnrec_nnz = int(tot)  # edge count known on the host: no later readback
            if fan is not None and 0 <= fan <= ops.DEFAULT_SPLIT:
                o_ip._gnnrec_split_plan = (ops.DEFAULT_SPLIT, None)  # no heavy rows possible
            rels[ce] = [o_ip, o_src, o_eid]
            src_lists.setdefault(ce[0], []).append(ce)
        prefixes, ranks = {}, {}
        for nt in g.ntypes:
            prefixes[nt] = seeds.get(nt, empty)
            ranks[nt] = self._relabeler(g, nt).begin(
                prefixes[nt], [rels[ce][1] for ce in src_lists.get(nt, [])])
        n_new = torch.stack([ranks[nt][-1] for nt in g.ntypes]).tolist()
        src_nid, num_dst = {}, {}
        for nt, nn_ in zip(g.ntypes, n_new):
            ces = src_lists.get(nt, [])
            nodes, locs = self._relabeler(g, nt).finish(prefixes[nt], [rels[ce][1] for ce in ces],
                                                        ranks[nt], int(nn_))
            src_nid[nt] = nodes
            num_dst[nt] = int(prefixes[nt].numel())
            for ce, loc in zip(ces, locs):
                rels[ce][1] = loc.to(torch.int32)
        return Block(src_nid, num_dst, {ce: tuple(v) for ce, v in rels.items()})


def _copy_block_data(g, blocks) -> None:
    """Edge data into every block, node data into the input block (DGL copies features at
    block creation; the reference reads blocks[0].srcdata['features']): every table in ONE
    launch (ops.gather_rows_batch)."""
    jobs, dests = [], []
    for b in blocks:
        for ce in b.canonical_etypes:
            eid = b._edata[ce][EID]
            for k, v in g._edata[ce].items():
                jobs.append((v, eid))
                dests.append((b._edata[ce], k))
    b0 = blocks[0]
    for nt in b0.ntypes:
        ids = b0._src[nt][NID]
        for k, v in g._ndata[nt].items():
            jobs.append((v, ids))
            dests.append((b0._src[nt], k))
    if not jobs:
        return
    for (frame, k), t in zip(dests, ops.gather_rows_batch(jobs)):
        frame[k] = t


def _add_transposes(block: Block) -> None:
    """Every relation's source-major CSR of the block, one C++ call (ops.block_transposes)."""
    ces = [ce for ce in block.canonical_etypes if ops._nnz(block._rels[ce][0]) > 0]
    if not ces:
        return
    ips, ixs, ws = ops._T().block_transposes(
        [block._rels[ce][0] for ce in ces], [block._rels[ce][1] for ce in ces],
        [block.number_of_src_nodes(ce[0]) for ce in ces],
        [ops._nnz(block._rels[ce][0]) for ce in ces])
    for ce, ip, ix, w in zip(ces, ips, ixs, ws):
        ip._gnnrec_nnz = ops._nnz(block._rels[ce][0])
        live = block._live.get(('src', ce[0]))
        if live is not None:  # a static block: its real sources (rows past them are padding)
            ip._gnnrec_live = live
        block._t[ce] = (ip, ix, w)


class MultiLayerFullNeighborSampler(BlockSampler):
    """All in-edges of every seed at every layer (dgl.dataloading, reference sampling.py:157)."""

    def __init__(self, n_layers: int, return_eids: bool = False):
        super().__init__(n_layers, None)


class MultiLayerNeighborSampler(BlockSampler):
    """fanouts[i] in-edges per seed (without replacement) for block i (sampling.py:159)."""

    def __init__(self, fanouts, replace: bool = False, return_eids: bool = False, seed=None):
        super().__init__(len(fanouts), list(fanouts), replace, seed)


class _Uniform:
    """negative_sampler.Uniform(k): src repeated k times, dst uniform over the dst type."""

    def __init__(self, k: int):
        self.k = k

    def __call__(self, g: HeteroGraph, eids: Dict[tuple, torch.Tensor]):
        out = {}
        for ce, e in eids.items():
            ce = g.to_canonical_etype(ce)
            src, _ = g.find_edges(e, etype=ce)
            src = src.repeat_interleave(self.k)
            with RNG_LOCK:
                dst = torch.randint(0, g.num_nodes(ce[2]), (src.numel(),), device=src.device)
            out[ce] = (src, dst)
        return out


class _NegNS:
    Uniform = _Uniform


negative_sampler = _NegNS


def _batches(n: int, batch_size: int, shuffle: bool, drop_last: bool, device):
    with RNG_LOCK:
        order = torch.randperm(n, device=device) if shuffle else torch.arange(n, device=device)
    stop = (n // batch_size) * batch_size if drop_last else n
    for i in range(0, stop, batch_size):
        yield order[i:i + batch_size]


def _tensors(obj, out):
    """Every tensor reachable from a loader item (dicts, tuples, lists, blocks, graphs);
    a LazyRows value is left unread (not gathered, not listed)."""
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, dict):
        for v in dict.values(obj):
            _tensors(v, out)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _tensors(v, out)
    elif isinstance(obj, (Block, PairGraph)):
        _tensors(vars(obj), out)
    return out


class _Prefetch:
    """Runs a batch iterator in a host thread on its own HIP stream, `depth` batches ahead.
    Each batch is handed over with an event the consumer's stream waits on, and every
    tensor in it is recorded on the consumer's stream (so the caching allocator does not
    recycle it under work the consumer queued)."""

    _END = object()
    # the producer stream's priority (torch.cuda.Stream: lower is higher; 0 = normal)
    priority = 0

    def __init__(self, make_iter, depth: int, device, take_handoff=None):
        self.device = device
        # take_handoff() -> the event to hand the item just produced over with (recorded
        # right after its own work), or None: an event recorded when it comes out
        self.take_handoff = take_handoff
        self.stream = torch.cuda.Stream(device=device, priority=self.priority)
        # the producer starts after everything the consumer has queued, which includes the
        # tail of any earlier loader's producer (its __iter__ ends with the consumer stream
        # waiting on it): a sampler shared by several loaders (reference sampling.py:153-241
        # passes one to all five) never has two producers on its relabel scratch and masks
        self.stream.wait_stream(torch.cuda.current_stream(device))
        self.q = queue.Queue(maxsize=max(1, depth))
        self.stop = threading.Event()
        self.thread = threading.Thread(target=self._run, args=(make_iter,), daemon=True)
        self.thread.start()

    def _put(self, x):
        while not self.stop.is_set():
            try:
                self.q.put(x, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _run(self, make_iter):
        try:
            with torch.cuda.device(self.device), torch.cuda.stream(self.stream):
                for item in make_iter():
                    ev = self.take_handoff() if self.take_handoff else None
                    if ev is None:
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    if not self._put((item, ev)):
                        return
            self._put(self._END)
        except BaseException as exc:  # surfaced in the consumer
            self._put(exc)

    def __iter__(self):
        try:
            while True:
                x = self.q.get()
                if x is self._END:
                    return
                if isinstance(x, BaseException):
                    raise x
                item, ev = x
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(ev)
                for t in _tensors(item, []):
                    if t.is_cuda:
                        t.record_stream(cur)
                yield item
        finally:
            # an early exit (break, exception) must not leave the producer running: stop it,
            # wait for its host side, and order its queued kernels before the consumer's
            self.stop.set()
            self.thread.join()
            torch.cuda.current_stream(self.device).wait_stream(self.stream)


def _maybe_prefetch(loader, make_iter):
    n = int(getattr(loader, "num_workers", 0) or 0)
    dev = loader.g.device
    if n > 0 and dev.type == "cuda":
        return iter(_Prefetch(make_iter, n, dev, getattr(loader, "_take_handoff", None)))
    return make_iter()


def _split_by_type(idx, flat_ids, type_starts, n_types):
    """Batch positions -> per-type id slices, batch order kept within a type; one readback
    (none for a single edge type: the reference's training loaders batch one type)."""
    if n_types == 1:
        return [flat_ids[idx]]
    ty = torch.bucketize(idx, type_starts[1:], right=True)
    order = torch.argsort(ty, stable=True)
    ids = flat_ids[idx[order]]
    counts = torch.bincount(ty, minlength=n_types).tolist()
    out, c = [], 0
    for n in counts:
        out.append(ids[c:c + n])
        c += n
    return out


def _type_starts(ids, dev):
    starts = [0]
    for t in ids:
        starts.append(starts[-1] + t.numel())
    return torch.tensor(starts, dtype=torch.int64, device=dev)


class NodeDataLoader:
    """Yields (input_nodes, output_nodes, blocks) for batches of seed nodes."""

    def __init__(self, g: HeteroGraph, nids, block_sampler: BlockSampler, device=None,
                 batch_size: int = 1, shuffle: bool = False, drop_last: bool = False,
                 num_workers: int = 0, **kwargs):
        self.g = g
        self.sampler = block_sampler
        dev = g.device
        if not isinstance(nids, dict):
            nids = {g.ntypes[0]: nids}
        self.types = list(nids.keys())
        ids = [torch.as_tensor(nids[nt], dtype=torch.int64).to(dev) for nt in self.types]
        self.flat_ids = torch.cat(ids) if ids else torch.zeros(0, dtype=torch.int64, device=dev)
        self.type_starts = _type_starts(ids, dev)
        self.batch_size, self.shuffle, self.drop_last = batch_size, shuffle, drop_last
        self.num_workers = num_workers

    def __len__(self):
        n = self.flat_ids.numel()
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        return _maybe_prefetch(self, self._iter_batches)

    def _iter_batches(self):
        for idx in _batches(self.flat_ids.numel(), self.batch_size, self.shuffle,
                            self.drop_last, self.g.device):
            parts = _split_by_type(idx, self.flat_ids, self.type_starts, len(self.types))
            seeds = {nt: v for nt, v in zip(self.types, parts) if v.numel() > 0}
            blocks = self.sampler.sample_blocks(self.g, seeds)
            input_nodes = blocks[0].srcdata[NID]
            output_nodes = {nt: blocks[-1].dstdata[NID][nt] for nt in seeds}
            yield input_nodes, output_nodes, blocks


class EdgeDataLoader:
    """Yields (input_nodes, pos_graph, neg_graph, blocks) for batches of edges
    (or (input_nodes, pair_graph, blocks) without a negative sampler)."""

    def __init__(self, g: HeteroGraph, eids, block_sampler: BlockSampler, device=None,
                 g_sampling: Optional[HeteroGraph] = None, exclude: Optional[str] = None,
                 reverse_eids=None, reverse_etypes: Optional[dict] = None,
                 negative_sampler=None, batch_size: int = 1, shuffle: bool = False,
                 drop_last: bool = False, num_workers: int = 0, pin_memory: bool = False,
                 transposed_blocks: bool = True, static_shapes: bool = False,
                 static_caps: str = "provable", **kwargs):
        self.g = g
        self.g_sampling = g_sampling if g_sampling is not None else g
        # the training loader's blocks carry their source-major CSRs (built by the sampler,
        # in the sampling thread when num_workers > 0): the backward sorts nothing
        self.transposed_blocks = transposed_blocks
        self.sampler = block_sampler
        self.exclude = exclude
        if exclude not in (None, 'reverse_types', 'self'):
            raise NotImplementedError(f"exclude={exclude!r}")
        # the reference passes the same four-type map for every graph (src/sampling.py:180-181);
        # a pair naming two types this graph lacks (clicks / clicked-by on a buys-only graph)
        # cannot occur in a batch and is dropped.  A pair with ONE side known is a typo that
        # would silently switch reverse-edge exclusion off for the known relation (its
        # reverse edges would leak into the sampled blocks): that raises
        names = {ce[1] for ce in self.g.canonical_etypes} | set(self.g.canonical_etypes)
        self.reverse_etypes = {}
        for k, v in (reverse_etypes or {}).items():
            if (k in names) != (v in names):
                bad = v if k in names else k
                raise KeyError(f"reverse_etypes pair {k!r}: {v!r} names {bad!r}, which is not a "
                               f"relation of this graph ({sorted(n for n in names if isinstance(n, str))})")
            if k in names:
                self.reverse_etypes[self.g.to_canonical_etype(k)] = self.g.to_canonical_etype(v)
        self.negative_sampler = negative_sampler
        # the batch head (pairs, negatives, compaction) as one C++ call on the GPU for the
        # Uniform sampler; any other sampler is called as given
        self.fused_head = (g.device.type == "cuda" and
                           (negative_sampler is None or type(negative_sampler) is _Uniform))
        dev = g.device
        if not isinstance(eids, dict):
            eids = {g.canonical_etypes[0]: eids}
        self.types = [g.to_canonical_etype(k) for k in eids]
        ids = [torch.as_tensor(eids[k], dtype=torch.int64).to(dev) for k in eids]
        self.flat_ids = torch.cat(ids)
        self.type_starts = _type_starts(ids, dev)
        self.batch_size, self.shuffle, self.drop_last = batch_size, shuffle, drop_last
        self.num_workers = num_workers
        # static_shapes: every full batch at fixed shapes with nothing read back to the host
        # (_head_static + the sampler's static blocks), so a training step over it can be
        # captured once and replayed (gnnrec.capture.CapturedTrainStep); a final partial
        # batch comes in the ordinary exact form
        self.static_shapes = static_shapes
        # static_caps: 'provable' (default) — the capacities no batch can exceed (a graph-sized
        # source list where the fanout can reach most of a node type: C2 at K = 2500 pads its
        # first block's 7.3M edges to 11M); 'auto' — the first STATIC_LEARN full batches come
        # out exact, and their largest source lists x STATIC_MARGIN (+ a padding slot) become
        # the node capacities: a later batch that does not fit (the sampler's overflow flag,
        # read back in the loader's thread) is redone exactly and the capacities grow.  The
        # flag is read once the next batch's kernels are queued (_iter_batches): read at
        # once, it made the loader wait for its own kernels, queued behind the training
        # step's (profiles/r05l_captured_step_probe_learned_caps.json)
        if static_caps not in ("auto", "provable"):
            raise ValueError(f"static_caps={static_caps!r}: 'auto' or 'provable'")
        self.static_caps = static_caps
        self._node_hint = None if static_caps == "auto" else {}
        self._seen_nodes = {}
        self._learned = 0
        self._overflow = None
        self._handoff = None  # the next item's hand-off event (_iter_batches)
        self.static_redone = 0
        if static_shapes:
            if len(self.types) != 1 or not self.fused_head:
                raise ValueError("static_shapes: batches of one edge type, with "
                                 "negative_sampler.Uniform or none, on a HIP device")
            if not block_sampler._fused_ok(self.g_sampling):
                raise ValueError("static_shapes needs bounded fanouts (0..64) within the fused "
                                 "sampler's limits")
        self._cx_scratch = None

    def __len__(self):
        n = self.flat_ids.numel()
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    STATIC_LEARN = 3
    # a batch's source-list sizes are sums of ~10^5-10^6 draws: their spread across batches
    # is ~0.1-0.5 % (C2 K = 10 / 2500), so 3 % over the largest of the learned batches
    # leaves ~10 standard deviations; every padded row costs the captured step's
    # row-proportional kernels (GEMMs, weight gradients, norms, the feature gather)
    STATIC_MARGIN = 1.03

    def _learn_caps(self, blocks):
        """Record an exact batch's source-list sizes per (step, node type); after
        STATIC_LEARN of them, fix the static node capacities."""
        L = len(blocks)
        for s_ in range(L):
            b = blocks[L - 1 - s_]
            for nt in b.ntypes:
                n = b.number_of_src_nodes(nt)
                self._seen_nodes[(s_, nt)] = max(self._seen_nodes.get((s_, nt), 0), n)
        self._learned += 1
        if self._learned >= self.STATIC_LEARN:
            self._node_hint = {k: -(-int(v * self.STATIC_MARGIN + 2) // 1024) * 1024
                               for k, v in self._seen_nodes.items()}

    def _head_static(self, batch):
        """_head at fixed shapes, with no host read: the same pairs, negatives (the same
        generator draws) and compaction, each type's node list padded with -1 to its bound —
        the batch's distinct ids, at most min(n_nodes, the positive endpoints plus the
        negative destinations): a Uniform negative's source is a positive's source."""
        g = self.g
        nts = list(g.ntypes)
        tix = {nt: i for i, nt in enumerate(nts)}
        if self._cx_scratch is None:
            self._cx_scratch = [ops.CompactScratch(g.num_nodes(nt), g.device) for nt in nts]
        k = 0 if self.negative_sampler is None else self.negative_sampler.k
        pairs = []
        for ce, e in batch.items():
            coo = g._coo[ce]
            pairs.append((ce, coo[0].index_select(0, e), coo[1].index_select(0, e)))
        negs = []
        for ce, ps, _pd in pairs:
            if k:
                ns = ps.unsqueeze(1).expand(ps.numel(), k).reshape(-1)
                with RNG_LOCK:
                    nd = torch.randint(0, g.num_nodes(ce[2]), (ns.numel(),), device=g.device)
                negs.append((ce, ns, nd))
        # per etype: positive sources, negative sources, positive dsts, negative dsts — the
        # local ids come back as consecutive views of one buffer, so an etype's positive and
        # negative endpoint lists are one list each (the cosine backward reads them joined)
        neg_of = {ce: (ns, nd) for ce, ns, nd in negs}
        lists, caps, slots = [], [0] * len(nts), {}
        for ce, ps, pd in pairs:
            ns, nd = neg_of.get(ce, (None, None))
            for key, ids, nt in (('ps', ps, ce[0]), ('ns', ns, ce[0]), ('pd', pd, ce[2]),
                                 ('nd', nd, ce[2])):
                if ids is None:
                    continue
                slots[(ce, key)] = len(lists)
                lists.append((ids, tix[nt]))
                if key != 'ns':  # a negative's source is a positive's source
                    caps[tix[nt]] += ids.numel()
        caps = [min(c, g.num_nodes(nt)) for c, nt in zip(caps, nts)]
        nodes, local, count = ops.compact_ids(lists, self._cx_scratch, caps)
        node_ids = dict(zip(nts, nodes))
        pos_l, neg_l = {}, {}
        for ce, _ps, _pd in pairs:
            pos_l[ce] = (local[slots[(ce, 'ps')]], local[slots[(ce, 'pd')]])
            if ce in neg_of:
                neg_l[ce] = (local[slots[(ce, 'ns')]], local[slots[(ce, 'nd')]])
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        pos_l = {ce: pos_l.get(ce, (empty, empty)) for ce in g.canonical_etypes}
        if k:  # every etype, in graph order, as _head returns them
            neg_l = {ce: neg_l.get(ce, (empty, empty)) for ce in g.canonical_etypes}
        return node_ids, pos_l, neg_l, count

    def _compact(self, pos_edges, neg_edges):
        """DGL compact_graphs([pos, neg]): both pair graphs over the union of their nodes
        (ascending global id per type)."""
        g = self.g
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        per_type: Dict[str, list] = {}
        for edges in (pos_edges, neg_edges):
            for ce, (s, d) in edges.items():
                per_type.setdefault(ce[0], []).append(s)
                per_type.setdefault(ce[2], []).append(d)
        node_ids, local = {}, {}
        ranks = [self.sampler._relabeler(g, nt).begin(empty, per_type.get(nt, []))
                 for nt in g.ntypes]
        n_new = torch.stack([r[-1] for r in ranks]).tolist()  # one readback for all types
        for nt, rank, n in zip(g.ntypes, ranks, n_new):
            nodes, locs = self.sampler._relabeler(g, nt).finish(empty, per_type.get(nt, []),
                                                                rank, int(n))
            node_ids[nt] = nodes
            local[nt] = locs
        cursor = {nt: 0 for nt in g.ntypes}

        def take(nt):
            v = local[nt][cursor[nt]]
            cursor[nt] += 1
            return v

        pos_l = {ce: None for ce in pos_edges}
        neg_l = {ce: None for ce in neg_edges}
        for edges, dst_map in ((pos_edges, pos_l), (neg_edges, neg_l)):
            for ce in edges:
                s = take(ce[0])
                d = take(ce[2])
                dst_map[ce] = (s, d)
        return node_ids, pos_l, neg_l

    def _head(self, batch):
        """find_edges + negative_sampler.Uniform + _compact in one C++ call
        (gnnrec::edge_batch_pairs), bitwise the same pair graphs as the three steps above."""
        g = self.g
        ces, nts = list(g.canonical_etypes), list(g.ntypes)
        tix = {nt: i for i, nt in enumerate(nts)}
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        coo = [g._coo[ce] for ce in ces]
        rel = [self.sampler._relabeler(g, nt) for nt in nts]
        k = 0 if self.negative_sampler is None else self.negative_sampler.k
        with RNG_LOCK:  # (its negatives: randint on the default generator)
            nodes, ps, pd, ns, nd = ops.edge_batch_pairs(
                [c[0] for c in coo], [c[1] for c in coo], [tix[ce[0]] for ce in ces],
                [tix[ce[2]] for ce in ces], [batch.get(ce, empty) for ce in ces],
                [ces.index(ce) for ce in batch], k, [g.num_nodes(nt) for nt in nts],
                [r.prefix_pos for r in rel], [r.mark for r in rel])
        node_ids = dict(zip(nts, nodes))
        pos_l = {ce: (ps[i], pd[i]) for i, ce in enumerate(ces)}
        neg_l = {} if k == 0 else {ce: (ns[i], nd[i]) for i, ce in enumerate(ces)}
        return node_ids, pos_l, neg_l

    def __iter__(self):
        return _maybe_prefetch(self, self._iter_batches)

    def _iter_batches(self):
        """The batches in order.  A static batch's overflow flag (learned capacities) is
        read only once the NEXT batch's kernels are queued — copied to the host behind an
        event of its own — so the loader's host work for batch N + 1 overlaps batch N's
        kernels instead of waiting for them (which, in a sampling thread, queue behind the
        training step's).  Each batch is handed over with an event recorded right after
        its own work (_Prefetch takes it from _take_handoff)."""
        pending = None
        for idx in _batches(self.flat_ids.numel(), self.batch_size, self.shuffle,
                            self.drop_last, self.g.device):
            rec = self._make_batch(idx)
            if pending is not None:
                yield self._settle(pending)
                pending = None
            if rec["flag"] is None:
                yield self._settle(rec)
            else:
                pending = rec
        if pending is not None:
            yield self._settle(pending)

    def _take_handoff(self):
        ev, self._handoff = self._handoff, None
        return ev

    def _make_batch(self, idx):
        """One batch's pairs, negatives and blocks, queued; static: its overflow flag on its
        way to the host (rec['flag'], read by _settle)."""
        g = self.g
        empty = torch.zeros(0, dtype=torch.int64, device=g.device)
        parts = _split_by_type(idx, self.flat_ids, self.type_starts, len(self.types))
        batch = {ce: v for ce, v in zip(self.types, parts) if v.numel() > 0}
        static = self.static_shapes and idx.numel() == self.batch_size and \
            self._node_hint is not None
        learn = self.static_shapes and idx.numel() == self.batch_size and not static
        counts = None
        if static:
            node_ids, pos_l, neg_l, counts = self._head_static(batch)
        elif self.fused_head:
            node_ids, pos_l, neg_l = self._head(batch)
        else:  # the readable form: the same kernels, generator draws and order
            pos_edges = {ce: g.find_edges(batch[ce], etype=ce) if ce in batch
                         else (empty, empty) for ce in g.canonical_etypes}
            neg_edges = {}
            if self.negative_sampler is not None:
                neg = self.negative_sampler(g, batch)
                neg_edges = {ce: neg.get(ce, (empty, empty)) for ce in g.canonical_etypes}
            node_ids, pos_l, neg_l = self._compact(pos_edges, neg_edges)
        exclude = None
        if self.exclude == 'reverse_types':
            exclude = {}
            for ce, e in batch.items():
                exclude[ce] = e
                if ce in self.reverse_etypes:
                    exclude[self.reverse_etypes[ce]] = e
        elif self.exclude == 'self':
            exclude = dict(batch)
        hint = self._node_hint if static and self._node_hint else None
        flag = None
        if hint is not None:
            if self._overflow is None:  # two flags (and host copies): batch N's is read
                # after batch N + 1 has zeroed and set its own
                self._overflow = [torch.zeros(1, dtype=torch.int64, device=g.device)
                                  for _ in range(2)]
                self._overflow_host = [torch.zeros(1, dtype=torch.int64).pin_memory()
                                       for _ in range(2)]
                self._overflow_i = 0
            i = self._overflow_i
            self._overflow_i = 1 - i
            self._overflow[i].zero_()
        pos_g = self._pair_graph(batch, pos_l, node_ids, static)
        seeds = {nt: v for nt, v in node_ids.items() if v.numel() > 0}
        blocks = self.sampler.sample_blocks(self.g_sampling, seeds, exclude,
                                            transposes=self.transposed_blocks,
                                            static_shapes=static, node_cap_hint=hint,
                                            overflow=self._overflow[i] if hint else None)
        if hint is not None:
            self._overflow_host[i].copy_(self._overflow[i], non_blocking=True)
            flag = (self._overflow_host[i], torch.cuda.Event())
            flag[1].record()
        if learn:
            self._learn_caps(blocks)
        ready = None
        if flag is not None:  # the hand-off event of a batch settled after the next one's
            ready = torch.cuda.Event()  # kernels are queued: this batch's work only
            ready.record()
        return {"batch": batch, "pos_l": pos_l, "neg_l": neg_l, "node_ids": node_ids,
                "counts": counts, "static": static, "exclude": exclude, "pos_g": pos_g,
                "blocks": blocks, "flag": flag, "ready": ready}

    def _pair_graph(self, batch, pos_l, node_ids, static):
        pos_g = PairGraph(pos_l, node_ids)
        pos_g.static = static
        for ce, e in batch.items():
            for k, v in self.g._edata[ce].items():
                pos_g._edata[ce][k] = ops.gather_rows(v, e)
            pos_g._edata[ce][EID] = e
        return pos_g

    def _settle(self, rec):
        """The loader item of a made batch; a static batch that outgrew the learned
        capacities is redone exactly (same pairs and negatives, fresh picks) and the
        capacities grow."""
        static, pos_g, blocks, node_ids = rec["static"], rec["pos_g"], rec["blocks"], rec["node_ids"]
        self._handoff = rec["ready"]
        if rec["flag"] is not None:
            host, ev = rec["flag"]
            ev.synchronize()
            if int(host[0]):
                self.static_redone += 1
                self._node_hint = {k: -(-int(v * self.STATIC_MARGIN) // 1024) * 1024
                                   for k, v in self._node_hint.items()}
                cnt = rec["counts"].tolist()
                node_ids = {nt: v[:c] for (nt, v), c in zip(node_ids.items(), cnt)}
                static = False
                pos_g = self._pair_graph(rec["batch"], rec["pos_l"], node_ids, False)
                seeds = {nt: v for nt, v in node_ids.items() if v.numel() > 0}
                blocks = self.sampler.sample_blocks(self.g_sampling, seeds, rec["exclude"],
                                                    transposes=self.transposed_blocks)
                self._handoff = None  # the redo's work is the last queued
        # static: the real node count per type, on the device (the node lists hold -1
        # past it)
        pos_g.node_counts = dict(zip(self.g.ntypes, rec["counts"].unbind(0))) if static else None
        pos_g.static = static
        input_nodes = blocks[0].srcdata[NID]
        if self.negative_sampler is None:
            return input_nodes, pos_g, blocks
        neg_g = PairGraph(rec["neg_l"], node_ids)
        neg_g.static = static
        if type(self.negative_sampler) is _Uniform:
            # every etype's negative sources are its positive sources repeated K times
            # (in local ids too: one relabel maps both): CosinePrediction.pair scores
            # them with the grouped launch
            neg_g.src_repeats_pos = self.negative_sampler.k
        return input_nodes, pos_g, neg_g, blocks
