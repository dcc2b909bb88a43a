"""Drop-in nn.Modules for reference src/model.py, backed by the HIP kernels.

Same class names, constructor signatures, parameter names/shapes (so a
reference state_dict loads unchanged), forward signatures and error behaviour
as the reference:

  NodeEmbedding      src/model.py:10-24
  ConvLayer          src/model.py:27-237   (aggregators mean / mean_nn / pool_nn /
                                            lstm / *_edge; lstm_edge fails on the
                                            missing self.lstm exactly as the reference)
  HeteroGraphConv    DGL 0.5.2 dgl.nn.pytorch.HeteroGraphConv as used at
                     src/model.py:384-406 (relation-skip rule, sum/mean/max)
  PredictingLayer    src/model.py:240-272
  PredictingModule   src/model.py:275-305
  CosinePrediction   src/model.py:308-327
  ConvModel          src/model.py:330-470
  max_margin_loss    src/model.py:473-533

Inference (no autograd) runs entirely in HIP kernels: gather+aggregate
(gnnrec_spmm_csr_f32) then ONE fused fp32-MFMA GEMM per relation that also
applies ReLU, the zero-guarded L2 norm and the cross-relation
sum/mean/max straight into the destination buffer (no torch.stack).
With autograd active the forward values still come from the same kernels;
gradients are computed by the Functions in gnnrec/autograd.py.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple

import torch
import torch.nn as nn

from . import _lib, ops
from . import autograd as ag

USER_ITEM = ("user", "item")
# debug: check a negative graph's src_repeats_pos mark against its values before the grouped
# cosine trusts it (one device comparison and sync per etype and step; tests switch it on)
CHECK_GROUPED_PAIRS = False
_PREAGG = ("pool_nn", "pool_nn_edge", "mean_nn", "mean_nn_edge")
_KNOWN = ("mean", "mean_nn", "pool_nn", "lstm", "mean_edge", "mean_nn_edge", "pool_nn_edge",
          "lstm_edge")


def _grad_mode(*tensors, module: nn.Module = None) -> bool:
    if not torch.is_grad_enabled():
        return False
    if any(t is not None and t.requires_grad for t in tensors):
        return True
    return module is not None and any(p.requires_grad for p in module.parameters())


class NodeEmbedding(nn.Module):
    """Projects the node features into embedding space (src/model.py:10-24)."""

    def __init__(self, in_feats, out_feats):
        super().__init__()
        self.proj_feats = nn.Linear(in_feats, out_feats)

    def forward(self, node_feats):
        W, b = self.proj_feats.weight, self.proj_feats.bias
        if _grad_mode(node_feats, module=self):
            return ag.LinearFn.apply(node_feats, W, b, False, False)
        return ops.gemm(node_feats, W, bias=b)


class ConvLayer(nn.Module):
    """One relation of message passing + aggregation (src/model.py:27-237)."""

    def reset_parameters(self):
        gain = nn.init.calculate_gain('relu')
        nn.init.xavier_uniform_(self.fc_self.weight, gain=gain)
        nn.init.xavier_uniform_(self.fc_neigh.weight, gain=gain)
        if self._aggre_type in _PREAGG:
            nn.init.xavier_uniform_(self.fc_preagg.weight, gain=gain)
        if self._aggre_type == 'lstm':
            self.lstm.reset_parameters()

    def __init__(self, in_feats: Tuple[int, int], out_feats: int, dropout: float,
                 aggregator_type: str, norm):
        super().__init__()
        self._in_neigh_feats, self._in_self_feats = in_feats
        self._out_feats = out_feats
        self._aggre_type = aggregator_type
        self.dropout_fn = nn.Dropout(dropout)
        self.norm = norm
        self.fc_self = nn.Linear(self._in_self_feats, out_feats, bias=False)
        self.fc_neigh = nn.Linear(self._in_neigh_feats, out_feats, bias=False)
        if aggregator_type in _PREAGG:
            self.fc_preagg = nn.Linear(self._in_neigh_feats, self._in_neigh_feats, bias=False)
        if aggregator_type == 'lstm':
            self.lstm = nn.LSTM(self._in_neigh_feats, self._in_neigh_feats, batch_first=True)
        self.reset_parameters()

    # --- helpers -------------------------------------------------------------
    def _plan(self, graph):
        return self._plan_rel(graph.canonical_etypes[0])

    def _plan_rel(self, ce):
        """(fc_preagg applies, edge weight applies, 'mean'|'max'|'lstm') — src/model.py:143-224."""
        agg = self._aggre_type
        if agg not in _KNOWN:
            raise KeyError('Aggregator type {} not recognized.'.format(agg))
        if agg.startswith('lstm'):
            # reference :164-169 / :210-221; self.lstm exists only for 'lstm' (:103-104),
            # so 'lstm_edge' raises AttributeError here as it does in the reference
            self.lstm  # noqa: B018
            return False, False, 'lstm'
        weighted = agg.endswith('_edge') and ce[0] in USER_ITEM and ce[2] in USER_ITEM
        reduce = 'max' if agg.startswith('pool') else 'mean'
        return agg in _PREAGG, weighted, reduce

    @staticmethod
    def _edge_weight(graph):
        """graph.edata['occurrence'].float() in CSR order (src/model.py:174)."""
        w = graph.edata['occurrence']
        return w if w.dtype == torch.float32 else w.float()

    def aggregate(self, indptr, indices, m, reduce: str, ew=None, **kw):
        """Inference neighbourhood reduction over a CSR: gSpMM mean/max/sum or the LSTM."""
        if reduce == 'lstm':
            L = self.lstm
            return ops.lstm_aggregate(indptr, indices, m, L.weight_ih_l0, L.weight_hh_l0,
                                      L.bias_ih_l0, L.bias_hh_l0)
        return ops.spmm(indptr, indices, m, reduce, edge_weight=ew, **kw)

    def forward(self, graph, x):
        """Reference ConvLayer.forward(graph, (h_neigh, h_self)) -> z [n_dst, out_feats]."""
        return self._run(graph, x, None, 'store', 0.0)

    def _pre_plan(self, graph, x):
        """Inference: (message, reduce, edge weight) when this relation can run pre-projected
        inside a two-relation launch (ops.spmm_project2) — a linear reduce, the fused
        shapes, a source table at most half the destination count; else None."""
        h_neigh, h_self = x
        preagg, weighted, reduce = self._plan(graph)
        if reduce not in ('sum', 'mean') or self._dropout_active() or \
                not ops.preproject_pays(h_neigh.shape[0], graph.n_dst, reduce):
            return None
        m = ops.gemm(h_neigh, self.fc_preagg.weight, relu=True) if preagg else h_neigh
        if not ops.can_spmm_project(graph.indptr, m, h_self, self.fc_self.weight,
                                    self.fc_neigh.weight):
            return None
        return m, reduce, (self._edge_weight(graph) if weighted else None)

    def _dropout_active(self) -> bool:
        return self.training and self.dropout_fn.p > 0

    def _run(self, graph, x, out, accum: str, out_div: float, attn=None, n_self: int = 0):
        """attn: (attn_vec, attn_state) for the attention accumulate modes.  n_self > 0
        (autograd, no dropout): x[1] is the block's whole source table of the dst type and
        its first n_self rows are the dst rows."""
        av, ast = attn if attn is not None else (None, None)
        h_neigh, h_self = x
        preagg, weighted, reduce = self._plan(graph)
        if self._dropout_active():
            h_neigh = self.dropout_fn(h_neigh)
            h_self = self.dropout_fn(h_self)
        ew = self._edge_weight(graph) if weighted else None
        grad = _grad_mode(h_neigh, h_self, module=self)
        if n_self and not grad:
            h_self = h_self[:n_self]
        if grad:
            m = ag.LinearFn.apply(h_neigh, self.fc_preagg.weight, None, True, False) \
                if preagg else h_neigh
            if ag.sage_rel_fusable(m, h_self, self.fc_neigh.weight, reduce, bool(self.norm)):
                # one autograd node, one C++ call each way (ag.SageRelFn)
                return ag.SageRelFn.apply(m, h_self, self.fc_self.weight, self.fc_neigh.weight,
                                          graph.indptr, graph.indices, ew, reduce,
                                          bool(self.norm), n_self,
                                          getattr(graph, 'transposed', None))
            if reduce == 'lstm':
                L = self.lstm
                agg = ag.LstmAggFn.apply(m, L.weight_ih_l0, L.weight_hh_l0, L.bias_ih_l0,
                                         L.bias_hh_l0, graph.indptr, graph.indices)
            else:
                agg = ag.SpmmFn.apply(m, graph.indptr, graph.indices, ew, reduce, graph.n_dst)
            z = ag.SageProjectFn.apply(h_self, agg, self.fc_self.weight, self.fc_neigh.weight,
                                       bool(self.norm), n_self)
            return z if out is None else z  # caller combines relations in grad mode
        m = ops.gemm(h_neigh, self.fc_preagg.weight, relu=True) if preagg else h_neigh
        if reduce != 'lstm' and ops.can_spmm_project(graph.indptr, m, h_self, self.fc_self.weight,
                                                     self.fc_neigh.weight):
            Wn = self.fc_neigh.weight
            if ops.fused_preprojects(graph.indptr, m, h_self, reduce):
                # few source rows: project them first, the kernel runs the self half only
                m, Wn = ops.preproject(m, Wn), None
            return ops.spmm_project(graph.indptr, graph.indices, m, h_self, self.fc_self.weight,
                                    Wn, reduce, ew, relu=True,
                                    l2norm=bool(self.norm), accum=accum, out_div=out_div,
                                    out=out, attn_vec=av, attn_state=ast)
        agg = self.aggregate(graph.indptr, graph.indices, m, reduce, ew)
        return ops.gemm(h_self, self.fc_self.weight, agg, self.fc_neigh.weight, relu=True,
                        l2norm=bool(self.norm), accum=accum, out_div=out_div, out=out,
                        attn_vec=av, attn_state=ast)


class HeteroGraphConv(nn.Module):
    """DGL 0.5.2 HeteroGraphConv semantics (restated), fused cross-relation aggregate.

    Relations with zero edges in `g`, or whose src / dst type has no input, are
    skipped; the outputs of the active relations are reduced per dst type with
    sum / mean / max.  Modules live in an nn.ModuleDict keyed by relation name,
    so state_dict keys are `mods.{rel}.*` exactly as in the reference.

    aggregate='attention' (build-defined, for BASELINE config C5 — the reference offers
    only sum/mean/max, main.py:486): per dst node, a softmax over its active relations
    of a_Tᵀ z_r weighs the relation outputs z_r; one learnable vector a_T per dst type
    (`attn.{ntype}`, needs attn_dims {ntype: out_feats}).  In inference the softmax is
    accumulated online across the relation launches (running max and sum per row)."""

    def __init__(self, mods: Dict[str, nn.Module], aggregate: str = 'sum',
                 attn_dims: Dict[str, int] = None):
        super().__init__()
        self.mods = nn.ModuleDict(mods)
        if aggregate not in ('sum', 'mean', 'max', 'attention'):
            raise KeyError('Invalid cross type reducer: {}'.format(aggregate))
        self.aggregate = aggregate
        self.attn = None
        if aggregate == 'attention':
            if not attn_dims:
                raise ValueError("aggregate='attention' needs attn_dims {dst ntype: out_feats}")
            self.attn = nn.ParameterDict({nt: nn.Parameter(torch.randn(d) / d ** 0.5)
                                          for nt, d in attn_dims.items()})

    def accum_mode(self, j: int, R: int):
        """(accumulate mode, out_div) of the j-th of R active relations into one dst type."""
        if self.aggregate == 'attention':
            return ('attn_first' if j == 0 else 'attn_last' if j == R - 1 else 'attn'), 0.0
        acc = 'store' if j == 0 else ('max' if self.aggregate == 'max' else 'add')
        div = float(R) if (self.aggregate == 'mean' and j == R - 1 and R > 1) else 0.0
        return acc, div

    def _layer_node(self, g, src_inputs, dst_inputs, active, fold=None):
        """Training over a block: the whole layer as ONE autograd node (ag.HeteroSageFn,
        every relation's gradient written into one table per node type), or None.

        fold {ntype: (W_e, b_e)}: the inputs are RAW features and the types' NodeEmbeddings
        are folded into the layer — per relation W_self W_e,dst with the bias W_self b_e,dst
        on every row, W_neigh W_e,src with W_neigh b_e,src on rows with an in-edge (the
        mean of x W_eᵀ + b_e over a non-empty set is mean(x) W_eᵀ + b_e).  Only for mean
        relations without fc_preagg or edge weights; None otherwise (the caller embeds)."""
        plan = _layer_plan(self, g, src_inputs, dst_inputs, active)
        if plan is None:
            return None
        folded = None
        if fold is not None:
            if any(preagg or weighted or reduce != 'mean' or ce[0] not in fold or
                   dtype not in fold for dtype, ce, _m, _rg, preagg, weighted, reduce in plan):
                return None
            folded = _fold_weights(plan, fold)
        types = []
        for dtype, ce, *_ in plan:
            for nt in (ce[0], dtype):
                if nt not in types:
                    types.append(nt)
        tix = {nt: i for i, nt in enumerate(types)}
        rels, per, groups, order = [], [], {}, []
        for dtype, ce, mod, rg, preagg, weighted, reduce in plan:
            ew = mod._edge_weight(rg) if weighted else None
            if dtype not in groups:
                groups[dtype] = []
                order.append(dtype)
            groups[dtype].append(len(rels))
            rels.append((tix[ce[0]], tix[dtype], reduce, bool(mod.norm),
                         dst_inputs[dtype].shape[0], rg.indptr, rg.indices, ew,
                         getattr(rg, 'transposed', None)))
            if folded is None:
                per += [mod.fc_preagg.weight if preagg else None, mod.fc_self.weight,
                        mod.fc_neigh.weight, None, None]
            else:
                per += [None, *folded[len(rels) - 1]]
        spec = (len(types), tuple(rels),
                tuple((tix[dt], tuple(groups[dt]), self.aggregate) for dt in order))
        outs = ag.HeteroSageFn.apply(spec, *[src_inputs[nt] for nt in types], *per)
        return dict(zip(order, outs))

    def _pair(self, g, ces, src_inputs, h_dst, out) -> bool:
        """Inference, exactly two relations into one type, both pre-projectable
        (ConvLayer._pre_plan): one launch with the sum / mean / max / attention combine
        inside — ops.spmm_pair when both gather the same raw table, else ops.spmm_project2
        over the pre-projected tables (the sharded pass's _pair does the same)."""
        if self.aggregate not in ('sum', 'mean', 'max', 'attention'):
            return False
        mods = [self.mods[ce[1]] for ce in ces]
        if bool(mods[0].norm) != bool(mods[1].norm):
            return False
        plans = []
        for mod, ce in zip(mods, ces):
            p = mod._pre_plan(g.rel_graph(ce), (src_inputs[ce[0]], h_dst))
            if p is None:
                return False
            plans.append(p)
        combine, div = _pair_combine(self.aggregate)
        dtype = ces[0][2]
        if plans[0][0] is plans[1][0] and os.environ.get("GNNREC_PAIR_RAW", "0") != "0":
            # both messages are the one source table itself: ops.spmm_pair gathers it raw and
            # runs all four projections in its epilogue (the sharded pass's _pair_raw)
            rels = []
            for ce, (m, reduce, ew) in zip(ces, plans):
                rg = g.rel_graph(ce)
                rels.append((rg.indptr, rg.indices, reduce, ew, None))
            ops.spmm_pair(rels[0], rels[1], plans[0][0], h_dst, mods[0].fc_self.weight,
                          mods[0].fc_neigh.weight, mods[1].fc_self.weight,
                          mods[1].fc_neigh.weight, relu=True, l2norm=bool(mods[0].norm),
                          combine=combine, out_div=div, out=out,
                          attn_vec=self.attn[dtype] if combine == 'attention' else None)
            return True
        rels = []
        for mod, ce, (m, reduce, ew) in zip(mods, ces, plans):
            rg = g.rel_graph(ce)
            rels.append((rg.indptr, rg.indices, ops.preproject(m, mod.fc_neigh.weight), reduce,
                         ew, None))
        ops.spmm_project2(rels[0], rels[1], h_dst, mods[0].fc_self.weight,
                          mods[1].fc_self.weight, relu=True, l2norm=bool(mods[0].norm),
                          combine=combine, out_div=div, out=out,
                          attn_vec=self.attn[dtype] if combine == 'attention' else None)
        return True

    def forward(self, g, inputs):
        if isinstance(inputs, tuple):
            src_inputs, dst_inputs = inputs
        elif g.is_block:
            src_inputs = inputs
            dst_inputs = {k: v[:g.number_of_dst_nodes(k)] for k, v in inputs.items()}
        else:
            src_inputs = dst_inputs = inputs
        active: Dict[str, list] = {}
        for ce in g.canonical_etypes:
            stype, etype, dtype = ce
            if g.num_edges(ce) == 0:
                continue
            if stype not in src_inputs or dtype not in dst_inputs:
                continue
            active.setdefault(dtype, []).append(ce)
        grad = _grad_mode(*src_inputs.values(), *dst_inputs.values(), module=self)
        if grad and active and g.is_block and not isinstance(inputs, tuple):
            rsts = self._layer_node(g, src_inputs, dst_inputs, active)
            if rsts is not None:
                return rsts
        rsts = {}
        for dtype, ces in active.items():
            if grad:
                outs = []
                for ce in ces:
                    mod = self.mods[ce[1]]
                    if (g.is_block and not isinstance(inputs, tuple) and not mod._dropout_active()
                            and dst_inputs[dtype].shape[0] > 0):
                        # dst rows = prefix of the src table: hand over the whole table so
                        # the self-gradient needs no slice backward
                        outs.append(mod._run(g.rel_graph(ce), (src_inputs[ce[0]],
                                                               src_inputs[dtype]), None,
                                             'store', 0.0, n_self=dst_inputs[dtype].shape[0]))
                    else:
                        outs.append(mod(g.rel_graph(ce), (src_inputs[ce[0]], dst_inputs[dtype])))
                if len(outs) == 1 and self.aggregate != 'attention':
                    rsts[dtype] = outs[0]  # sum / mean / max of one relation is itself
                    continue
                if len(outs) == 2 and self.aggregate == 'sum':
                    rsts[dtype] = outs[0] + outs[1]
                    continue
                st = torch.stack(outs, 0)
                if self.aggregate == 'attention':
                    w = torch.softmax((st * self.attn[dtype]).sum(-1), dim=0)  # [R, n_dst]
                    rsts[dtype] = (w.unsqueeze(-1) * st).sum(0)
                    continue
                rsts[dtype] = (st.sum(0) if self.aggregate == 'sum' else
                               st.mean(0) if self.aggregate == 'mean' else st.max(0)[0])
                continue
            n_dst = dst_inputs[dtype].shape[0]
            out_feats = self.mods[ces[0][1]]._out_feats
            out = torch.empty((n_dst, out_feats), dtype=torch.float32,
                              device=dst_inputs[dtype].device)
            R = len(ces)
            if R == 2 and self._pair(g, ces, src_inputs, dst_inputs[dtype], out):
                rsts[dtype] = out
                continue
            attn = None
            if self.aggregate == 'attention':
                attn = (self.attn[dtype], torch.empty((n_dst, 2), dtype=torch.float32,
                                                      device=out.device))
            for j, ce in enumerate(ces):
                accum, div = self.accum_mode(j, R)
                self.mods[ce[1]]._run(g.rel_graph(ce), (src_inputs[ce[0]], dst_inputs[dtype]),
                                      out, accum, div, attn)
            rsts[dtype] = out
        return rsts


def _layer_plan(hconv, g, src_inputs, dst_inputs, active):
    """The relations of one training layer as ag.HeteroSageFn takes them, or None when a
    relation needs the per-relation path (max / LSTM reducers, dropout, attention or max
    across relations, rows wider than one GEMM block, GNNREC_TRAIN_LAYER=0)."""
    if os.environ.get("GNNREC_TRAIN_LAYER", "1") == "0" or \
            hconv.aggregate not in ('sum', 'mean'):
        return None
    rels = []
    for dtype, ces in active.items():
        if dst_inputs[dtype].shape[0] == 0:
            return None
        for ce in ces:
            mod = hconv.mods[ce[1]]
            if mod._dropout_active():
                return None
            rg = g.rel_graph(ce)
            preagg, weighted, reduce = mod._plan(rg)
            if not ag.sage_rel_fusable(src_inputs[ce[0]], src_inputs[dtype], mod.fc_neigh.weight,
                                       reduce, bool(mod.norm)):
                return None
            rels.append((dtype, ce, mod, rg, preagg, weighted, reduce))
    return rels


def _fold_weights(plan, fold):
    """Per relation of a training layer plan (W_self W_e,dst, W_neigh W_e,src, W_self b_e,dst,
    W_neigh b_e,src), autograd-tracked: per node type T every weight its embedding
    multiplies is stacked and multiplied once ([W; ...] W_e,T and [W; ...] b_e,T), so a
    layer costs two small products per node type (the C2 layer: 4 instead of 8)."""
    uses = {}  # node type -> [(relation index, 0 self | 1 neigh, W)]
    for r, (dtype, ce, mod, *_rest) in enumerate(plan):
        uses.setdefault(dtype, []).append((r, 0, mod.fc_self.weight))
        uses.setdefault(ce[0], []).append((r, 1, mod.fc_neigh.weight))
    out = [[None] * 4 for _ in plan]
    for nt, lst in uses.items():
        W_e, b_e = fold[nt]
        prods = ag.FoldFn.apply(W_e, b_e, *[W for _r, _k, W in lst])
        for i, (r, k, _W) in enumerate(lst):
            out[r][k] = prods[i]
            out[r][2 + k] = prods[len(lst) + i]
    return out


# First-block source rows from which ConvModel folds its NodeEmbeddings into the first
# training layer by default (GNNREC_TRAIN_FOLD=auto; C2: ≈0.36M rows at K = 10, ≈0.96M at
# the reference's K = 2500)
FOLD_MIN_SRC_ROWS = int(os.environ.get("GNNREC_TRAIN_FOLD_MIN_ROWS", 1 << 19))


def _pair_combine(aggregate: str):
    """(spmm_project2 combine, out_div) of a HeteroGraphConv aggregate over two relations."""
    if aggregate in ('max', 'attention'):
        return aggregate, 0.0
    return 'add', (2.0 if aggregate == 'mean' else 0.0)


class PredictingLayer(nn.Module):
    """MLP edge scorer (src/model.py:240-272)."""

    def reset_parameters(self):
        gain_relu = nn.init.calculate_gain('relu')
        gain_sigmoid = nn.init.calculate_gain('sigmoid')
        nn.init.xavier_uniform_(self.hidden_1.weight, gain=gain_relu)
        nn.init.xavier_uniform_(self.hidden_2.weight, gain=gain_relu)
        nn.init.xavier_uniform_(self.output.weight, gain=gain_sigmoid)

    def __init__(self, embed_dim: int):
        super(PredictingLayer, self).__init__()
        self.hidden_1 = nn.Linear(embed_dim * 2, 128)
        self.hidden_2 = nn.Linear(128, 32)
        self.output = nn.Linear(32, 1)
        self.relu = nn.ReLU()
        self.sigmoid = nn.Sigmoid()
        self.reset_parameters()

    def forward(self, x):
        if _grad_mode(x, module=self):
            x = ag.LinearFn.apply(x, self.hidden_1.weight, self.hidden_1.bias, True, False)
            x = ag.LinearFn.apply(x, self.hidden_2.weight, self.hidden_2.bias, True, False)
            return ag.LinearFn.apply(x, self.output.weight, self.output.bias, False, True)
        x = ops.gemm(x, self.hidden_1.weight, bias=self.hidden_1.bias, relu=True)
        x = ops.gemm(x, self.hidden_2.weight, bias=self.hidden_2.bias, relu=True)
        return ops.gemm(x, self.output.weight, bias=self.output.bias, sigmoid=True)

    def score_edges(self, h_src, h_dst, src, dst, K=None):
        """Edge scores without materialising [E, 2d]: W1[hu‖hv] = (W1a hu + b1) + W1b hv.
        K: `src` is runs of K repeats of one source (negative_sampler.Uniform's negatives:
        the grouped launch, one P row per run)."""
        d = h_src.shape[1]
        W1 = self.hidden_1.weight
        if K is not None and K >= 32 and src.numel() == (src.numel() // K) * K and \
                src.numel() >= h_src.shape[0] + h_dst.shape[0]:
            P = ops.gemm(h_src, W1[:, :d], bias=self.hidden_1.bias)
            Q = ops.gemm(h_dst, W1[:, d:])
            _, out = ops.edge_mlp_grouped(src[::K].contiguous(), None, K, dst, P, Q,
                                          self.hidden_2.weight, self.hidden_2.bias,
                                          self.output.weight.reshape(-1), self.output.bias)
            return out
        if src.numel() < h_src.shape[0] + h_dst.shape[0]:
            # fewer edges than table rows: score the gathered rows
            hu, hv = h_src.index_select(0, src), h_dst.index_select(0, dst)
            src = dst = torch.arange(src.numel(), device=src.device)
        else:
            hu, hv = h_src, h_dst
        P = ops.gemm(hu, W1[:, :d], bias=self.hidden_1.bias)
        Q = ops.gemm(hv, W1[:, d:])
        return ops.edge_mlp(src, dst, P, Q, self.hidden_2.weight, self.hidden_2.bias,
                            self.output.weight.reshape(-1), self.output.bias)


class PredictingModule(nn.Module):
    """src/model.py:275-305: scores user/item etypes of `graph` with the MLP."""

    def __init__(self, predicting_layer, embed_dim: int):
        super(PredictingModule, self).__init__()
        self.layer_nn = predicting_layer(embed_dim)

    def forward(self, graph, h):
        ratings_dict = {}
        for etype in graph.canonical_etypes:
            if etype[0] in USER_ITEM and etype[2] in USER_ITEM:
                utype, _, vtype = etype
                src_nid, dst_nid = graph.all_edges(etype=etype)
                if _grad_mode(h[utype], h[vtype], module=self):
                    cat_embed = torch.cat((h[utype][src_nid], h[vtype][dst_nid]), 1)
                    ratings = self.layer_nn(cat_embed)
                else:
                    # negative_sampler.Uniform's negative graph (the loader marks it): the
                    # grouped launch
                    K = graph.src_repeats(etype, src_nid) if hasattr(graph, 'src_repeats') \
                        else None
                    ratings = self.layer_nn.score_edges(h[utype], h[vtype], src_nid, dst_nid, K)
                ratings_dict[etype] = torch.flatten(ratings)
        return {k: torch.unsqueeze(v, 1) for k, v in ratings_dict.items()}


class CosinePrediction(nn.Module):
    """src/model.py:308-327: per-etype cosine of L2-normalised endpoints."""

    def __init__(self):
        super().__init__()

    def forward(self, graph, h):
        ratings = {}
        for etype in graph.canonical_etypes:
            if etype[0] not in h or etype[2] not in h:
                continue  # etypes whose node types have no 'h' (reference KeyError branch)
            src, dst = graph.all_edges(etype=etype)
            if _grad_mode(h[etype[0]], h[etype[2]]):
                cos = ag.CosineFn.apply(h[etype[0]], h[etype[2]], src, dst)
            else:
                cos = ops.sddmm_cos(src, dst, h[etype[0]], h[etype[2]])
            ratings[etype] = cos.unsqueeze(1)
        return ratings

    def pair(self, pos_g, neg_g, h):
        """forward(pos_g, h) and forward(neg_g, h) — the same scores — with each etype's
        positive and negative edges in ONE cosine launch each way (the pair graphs share
        their node ids): in training one backward call per etype instead of two, and no
        add of two gradients per endpoint table."""
        pos, neg = {}, {}
        for etype in pos_g.canonical_etypes:
            if etype[0] not in h or etype[2] not in h:
                continue
            ps, pd = pos_g.all_edges(etype=etype)
            if etype not in neg_g.canonical_etypes:
                pos[etype] = self.forward_one(h, etype, ps, pd)
                continue
            ns, nd = neg_g.all_edges(etype=etype)
            if ps.numel() == 0 and ns.numel() == 0:
                # an etype the batch has no pairs of: empty scores, no launches, and no
                # zero gradient for autograd to add into the endpoint tables
                pos[etype] = h[etype[0]].new_zeros((0, 1))
                neg[etype] = h[etype[0]].new_zeros((0, 1))
                continue
            # negative_sampler.Uniform's pairs (the loader marks them): every positive's
            # source repeated K times -> the grouped launch, one gathered row per edge
            K = neg_g.src_repeats(etype, ns) if hasattr(neg_g, 'src_repeats') else None
            if K is not None and (ns.numel() != ps.numel() * K or
                                  not ops.cos_grouped_ok(h[etype[0]], h[etype[2]])):
                K = None
            if K is not None and CHECK_GROUPED_PAIRS:  # debug: the mark against the values
                if not torch.equal(ns, ps.repeat_interleave(K)):
                    raise ValueError(f"{etype}: negative sources are not the positives' "
                                     f"sources repeated {K} times (stale src_repeats_pos)")
            if _grad_mode(h[etype[0]], h[etype[2]]):
                a, b = ag.CosinePairFn.apply(h[etype[0]], h[etype[2]], ps, pd, ns, nd, K)
            elif K is not None:
                a, b = ops.sddmm_cos_grouped(ps, pd, K, nd, h[etype[0]], h[etype[2]])
            else:
                cos = ops.sddmm_cos(torch.cat([ps, ns]), torch.cat([pd, nd]), h[etype[0]],
                                    h[etype[2]])
                a, b = cos[:ps.numel()], cos[ps.numel():]
            pos[etype], neg[etype] = a.unsqueeze(1), b.unsqueeze(1)
        for etype in neg_g.canonical_etypes:
            if etype not in pos and etype[0] in h and etype[2] in h:
                ns, nd = neg_g.all_edges(etype=etype)
                neg[etype] = self.forward_one(h, etype, ns, nd)
        return pos, neg

    @staticmethod
    def forward_one(h, etype, src, dst):
        if _grad_mode(h[etype[0]], h[etype[2]]):
            cos = ag.CosineFn.apply(h[etype[0]], h[etype[2]], src, dst)
        else:
            cos = ops.sddmm_cos(src, dst, h[etype[0]], h[etype[2]])
        return cos.unsqueeze(1)


class ConvModel(nn.Module):
    """Embedding layers + ConvLayers + prediction head (src/model.py:330-470)."""

    # None: GNNREC_TRAIN_FOLD decides ('auto' by default); '0' / '1' / 'auto' for this model
    train_fold = None

    def __init__(self, g, n_layers: int, dim_dict, norm: bool = True, dropout: float = 0.0,
                 aggregator_type: str = 'mean', pred: str = 'cos',
                 aggregator_hetero: str = 'sum', embedding_layer: bool = True):
        super().__init__()
        self.embedding_layer = embedding_layer
        if embedding_layer:
            self.user_embed = NodeEmbedding(dim_dict['user'], dim_dict['hidden'])
            self.item_embed = NodeEmbedding(dim_dict['item'], dim_dict['hidden'])
            if 'sport' in g.ntypes:
                self.sport_embed = NodeEmbedding(dim_dict['sport'], dim_dict['hidden'])
        self.layers = nn.ModuleList()

        def attn_dims(d):  # every ConvLayer of a layer has the same out_feats
            if aggregator_hetero != 'attention':
                return None
            return {etype[2]: d for etype in g.canonical_etypes}
        if not embedding_layer:
            self.layers.append(HeteroGraphConv(
                {etype[1]: ConvLayer((dim_dict[etype[0]], dim_dict[etype[2]]), dim_dict['hidden'],
                                     dropout, aggregator_type, norm)
                 for etype in g.canonical_etypes}, aggregate=aggregator_hetero,
                attn_dims=attn_dims(dim_dict['hidden'])))
        for _ in range(n_layers - 2):
            self.layers.append(HeteroGraphConv(
                {etype[1]: ConvLayer((dim_dict['hidden'], dim_dict['hidden']), dim_dict['hidden'],
                                     dropout, aggregator_type, norm)
                 for etype in g.canonical_etypes}, aggregate=aggregator_hetero,
                attn_dims=attn_dims(dim_dict['hidden'])))
        self.layers.append(HeteroGraphConv(
            {etype[1]: ConvLayer((dim_dict['hidden'], dim_dict['hidden']), dim_dict['out'],
                                 dropout, aggregator_type, norm)
             for etype in g.canonical_etypes}, aggregate=aggregator_hetero,
            attn_dims=attn_dims(dim_dict['out'])))
        if pred == 'cos':
            self.pred_fn = CosinePrediction()
        elif pred == 'nn':
            self.pred_fn = PredictingModule(PredictingLayer, dim_dict['out'])
        else:
            raise KeyError('Prediction function {} not recognized.'.format(pred))

    def get_repr(self, blocks, h):
        for i in range(len(blocks)):
            layer = self.layers[i]
            h = layer(blocks[i], h)
        return h

    def embed(self, h):
        """The embedding step of forward / get_embeddings (src/model.py:462-466)."""
        h = dict(h)
        h['user'] = self.user_embed(h['user'])
        h['item'] = self.item_embed(h['item'])
        if 'sport' in h.keys():
            h['sport'] = self.sport_embed(h['sport'])
        return h

    def _folded_first_layer(self, blocks, h):
        """Training: the first layer over the RAW features with the NodeEmbeddings folded
        into it (HeteroGraphConv._layer_node(fold=...)), or None.  The embedding tables of
        every source node are never formed, and the backward writes no gradient into them:
        the first block's transposed gathers and the embeddings' weight-gradient GEMMs over
        every source row disappear (the fold's weight products are per-layer 64×64 work).
        Numerically the reference's NodeEmbedding + mean up to fp32 rounding.
        GNNREC_TRAIN_FOLD: 'auto' (default) folds when the first block has at least
        FOLD_MIN_SRC_ROWS source rows — the fold's weight products cost ≈0.3 ms of host time
        per step, which a host-bound small step pays (C2 at K = 10: 2.62 → 2.92 ms without the
        sampling thread) and a GPU-bound large one recovers several times over (K = 2500:
        4.3 → 3.46 ms; profiles/r04h_train_fold_ab.md, r04l_k10_fold_ab.md); '1' always, '0'
        never (embed, then aggregate).  `model.train_fold` overrides the variable for one model
        (a captured step, whose host cost is gone, folds every block: '1')."""
        mode = self.train_fold or os.environ.get("GNNREC_TRAIN_FOLD", "auto")
        if mode == "0" or not blocks or \
                not getattr(blocks[0], 'is_block', False) or not isinstance(
                    self.layers[0], HeteroGraphConv) or not _grad_mode(module=self):
            return None
        g = blocks[0]
        if mode != "1" and sum(g.number_of_src_nodes(nt) for nt in g.ntypes) < \
                FOLD_MIN_SRC_ROWS:
            return None
        fold = {}
        for nt in h:
            emb = getattr(self, nt + '_embed', None)
            if emb is None:
                return None
            fold[nt] = (emb.proj_feats.weight, emb.proj_feats.bias)
        src = dict(h)
        dst = {k: v[:g.number_of_dst_nodes(k)] for k, v in src.items()}
        active: Dict[str, list] = {}
        for ce in g.canonical_etypes:
            if g.num_edges(ce) and ce[0] in src and ce[2] in dst:
                active.setdefault(ce[2], []).append(ce)
        if not active:
            return None
        out = self.layers[0]._layer_node(g, src, dst, active, fold=fold)
        ref = getattr(g, '_sampler', None)
        sampler = ref() if ref is not None else None
        if out is not None and sampler is not None:
            # the sampler that built these blocks stops building the first block's transposes
            # for the blocks this model folds (nothing reads them): every one under '1', those
            # of at least FOLD_MIN_SRC_ROWS source rows under 'auto' — smaller ones, which
            # the model does not fold, keep theirs for the backward
            sampler.first_transposes_below = 0 if mode == "1" else FOLD_MIN_SRC_ROWS
        return out

    def forward(self, blocks, h, pos_g, neg_g, embedding_layer: bool = True):
        start = 0
        if embedding_layer:
            h1 = self._folded_first_layer(blocks, h)
            if h1 is not None:
                h, start = h1, 1
            else:
                h = self.embed(h)
        for i in range(start, len(blocks)):
            h = self.layers[i](blocks[i], h)
        if isinstance(self.pred_fn, CosinePrediction):
            pos_score, neg_score = self.pred_fn.pair(pos_g, neg_g, h)
        else:
            pos_score = self.pred_fn(pos_g, h)
            neg_score = self.pred_fn(neg_g, h)
        return h, pos_score, neg_score


def max_margin_loss(pos_score, neg_score, delta: float, neg_sample_size: int,
                    use_recency: bool = False, recency_scores=None,
                    remove_false_negative: bool = False, negative_mask=None, cuda=False,
                    device=None):
    """Max-margin loss (src/model.py:473-533), same arguments and semantics: the mean over
    every etype of relu(neg + delta - pos - mask) (/ recency).  One HIP launch per etype
    computes the scores' sum and their gradient (gnnrec_margin_loss_f32)."""
    scores, meta = [], []
    for etype in pos_score.keys():
        neg, pos = neg_score[etype], pos_score[etype]
        mask = negative_mask[etype] if remove_false_negative else None
        rec = None
        if use_recency and recency_scores is not None and etype in recency_scores:
            rec = recency_scores[etype]
        scores += [pos, neg]
        meta.append((neg_sample_size, mask, rec))
    if not meta:
        return torch.tensor(float('nan'))
    return ag.MarginLossFn.apply((delta, meta), *scores)


def library_available() -> bool:
    return _lib.available()
