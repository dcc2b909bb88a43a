"""Autograd Functions for training through the drop-in modules.

Forward values always come from the HIP kernels (the same launches as the
inference path, so train/eval numerics agree).  Backward, all HIP:
  * aggregation: the transposed scatter (gnnrec_spmm_backward_f32, first-arg-max
    routing for max, as DGL's gSpMM backward);
  * projections: the pre-activation is recomputed by gnnrec_gemm_f32, the
    ReLU/zero-guarded-norm epilogue is differentiated by gnnrec_act_backward_f32,
    input gradients are gnnrec_gemm_f32 against the transposed weights and weight
    gradients the split-K gnnrec_gemm_tn_f32 (dW = dYᵀ X);
  * cosine head: the two reduction sides of gSDDMM's backward are weighted
    gSpMMs over the pair graph sorted by src and by dst (DGL's rule: the
    backward of an SDDMM is an SpMM on the same / reversed graph).
"""
from __future__ import annotations

import os

import torch

from . import ops


class LinearFn(torch.autograd.Function):
    """y = act(x Wᵀ + b), act ∈ {none, relu, sigmoid}; forward = gnnrec_gemm_f32."""

    @staticmethod
    def forward(ctx, x, W, b, relu: bool, sigmoid: bool):
        y = ops.gemm(x.contiguous(), W.detach(), bias=None if b is None else b.detach(),
                     relu=relu, sigmoid=sigmoid)
        ctx.save_for_backward(x, W, y)
        ctx.has_b = b is not None
        ctx.relu, ctx.sigmoid = relu, sigmoid
        return y

    @staticmethod
    def backward(ctx, gy):
        x, W, y = ctx.saved_tensors
        if ctx.relu:  # y = relu(u): y > 0 exactly where u > 0
            gy = ops.act_backward(y, gy, relu=True, l2norm=False)
        elif ctx.sigmoid:
            gy = gy * y * (1 - y)
        gy = gy.contiguous()
        gx = ops.gemm(gy, W.t().contiguous()) if ctx.needs_input_grad[0] else None
        gb = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = torch.empty(gy.shape[1], dtype=torch.float32, device=gy.device)
        if ctx.needs_input_grad[1]:
            gW = ops.gemm_tn(gy, x.contiguous(), colsum=gb)  # db from the same pass
        else:
            gW = None
            if gb is not None:
                gb = gy.sum(0)
        return gx, gW, gb, None, None


class SpmmFn(torch.autograd.Function):
    """agg = reduce_{e in row v} m[src_e] (* w_e); forward = gnnrec_spmm_csr_f32."""

    @staticmethod
    def forward(ctx, m, indptr, indices, ew, reduce: str, n_dst: int):
        out = ops.spmm(indptr, indices, m.contiguous(), reduce, edge_weight=ew)
        ctx.save_for_backward(m, indptr, indices, ew, out)
        ctx.reduce = reduce
        ctx.nnz = getattr(indptr, "_gnnrec_nnz", None)  # host edge count if already known
        return out

    @staticmethod
    def backward(ctx, g):
        m, indptr, indices, ew, out = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        if ctx.reduce in ('sum', 'mean') and os.environ.get("GNNREC_SPMM_BWD") != "atomic":
            # DGL's rule: the backward of a gSpMM is a gSpMM on the reversed graph.  The
            # block is transposed on the device (stable radix sort) and the gradient is
            # the forward's bandwidth-bound gather over that CSR: deterministic, and not
            # capped by the L2 float-atomic rate as the scatter is
            # (GNNREC_SPMM_BWD=atomic keeps the scatter)
            return (_spmm_reversed(indptr, indices, g, ew, ctx.reduce, m.shape[0], ctx.nnz),
                    None, None, None, None, None)
        gm = ops.spmm_backward(indptr, indices, g, ctx.reduce, edge_weight=ew,
                               X=m, out=out, n_src=m.shape[0])
        return gm, None, None, None, None, None


def _spmm_reversed(indptr, indices, g, ew, reduce: str, n_src: int, nnz=None):
    """grad_X[u] = Σ_{e: src_e = u} g[dst_e] · (ew_e) (/ deg(dst_e) for mean), as a sum
    gSpMM over the source-major CSR of the same edges (rows = sources)."""
    ip_t, ix_t, w_t = ops.csr_transpose(indptr, indices, n_src, edge_weight=ew,
                                        mean=reduce == 'mean', n_edges=nnz)
    if g.stride(-1) != 1:
        g = g.contiguous()
    return ops.spmm(ip_t, ix_t, g, 'sum', edge_weight=w_t)  # g may be a strided row view


class LstmAggFn(torch.autograd.Function):
    """agg[v] = LSTM over m[src of v's in-edges] (ConvLayer._lstm_reducer); forward =
    gnnrec_lstm_step_save_f32 per step, keeping every step's hidden / cell rows and gates;
    backward = back-propagation through time on the HIP kernels
    (ops.lstm_aggregate_backward: the gate Jacobian per step, dz·W_hh and the weight /
    input-projection gradients as GEMMs, dP summed per source row by an spmm)."""

    @staticmethod
    def forward(ctx, m, W_ih, W_hh, b_ih, b_hh, indptr, indices):
        out, state = ops.lstm_aggregate_train(indptr, indices, m, W_ih, W_hh, b_ih, b_hh)
        ctx.save_for_backward(m, W_ih, indptr, indices)
        ctx.state = state
        return out

    @staticmethod
    def backward(ctx, g):
        m, W_ih, indptr, indices = ctx.saved_tensors
        need = ctx.needs_input_grad
        if ctx.state is None:
            raise RuntimeError("LstmAggFn: the forward's per-step LSTM state was released by "
                               "the first backward through this graph; a second backward "
                               "(retain_graph=True) needs a fresh forward")
        dX, dW_ih, dW_hh, db = ops.lstm_aggregate_backward(indptr, indices, m, W_ih, ctx.state,
                                                          g, need_x=need[0])
        ctx.state = None
        return (dX, dW_ih if need[1] else None, dW_hh if need[2] else None,
                db if need[3] else None, db if need[4] else None, None, None)


class SageProjectFn(torch.autograd.Function):
    """z = norm?(relu(h_self W_selfᵀ + agg W_neighᵀ)); forward = fused gnnrec_gemm_f32.

    n_self > 0: h_self is a block's whole source table, whose first n_self rows are the
    destination rows (DGL blocks keep the dst nodes as the src prefix).  Its gradient then
    comes back for the whole table (zero past n_self) and autograd adds it to the table's
    other gradient directly, instead of a slice backward (zero fill + copy) and an add."""

    @staticmethod
    def forward(ctx, h_self, agg, Ws, Wn, norm: bool, n_self: int = 0):
        hs = h_self[:n_self] if n_self else h_self
        # the backward needs the epilogue's Jacobian, not the GEMM again: z = relu(u)/|relu(u)|
        # and the row norms (one fused launch) — or y = relu(u) kept before a separate
        # normalisation when the row is wider than one GEMM block
        nrm = None
        if norm and Ws.shape[0] <= ops.GEMM_ROW_N:
            nrm = torch.empty(hs.shape[0], dtype=torch.float32, device=hs.device)
            z = ops.gemm(hs.contiguous(), Ws.detach(), agg.contiguous(), Wn.detach(), relu=True,
                         l2norm=True, row_norm=nrm)
            y = z
        else:
            y = ops.gemm(hs.contiguous(), Ws.detach(), agg.contiguous(), Wn.detach(), relu=True)
            z = ops.l2_normalize_rows(y) if norm else y
        ctx.save_for_backward(h_self, agg, Ws, Wn, y, nrm)
        ctx.norm, ctx.n_self = norm, n_self
        return z

    @staticmethod
    def backward(ctx, gz):
        h_self, agg, Ws, Wn, y, nrm = ctx.saved_tensors
        need = ctx.needs_input_grad
        M = y.shape[0]
        hs = h_self[:M]
        gz = gz.contiguous()
        if nrm is not None:  # y is the normalised output
            gu = ops.act_backward_normed(y, nrm, gz, relu=True)
        else:  # y = relu(u): relu(y) = y, same mask
            gu = ops.act_backward(y, gz, relu=True, l2norm=ctx.norm)
        g_self = g_agg = None
        if need[0]:
            # contiguous [rows, d_s] with the tail past the dst rows zeroed: autograd adds it
            # to the table's other gradient with a vectorised kernel (a strided view of a
            # [rows, d_s + d_n] GEMM output took a slow strided add, more than the GEMM saved)
            g_self = torch.empty((h_self.shape[0], Ws.shape[1]), dtype=torch.float32,
                                 device=gu.device)
            ops.gemm(gu, Ws.detach().t().contiguous(), out=g_self[:M])
            if h_self.shape[0] > M:
                g_self[M:].zero_()
        if need[1]:
            g_agg = ops.gemm(gu, Wn.detach().t().contiguous())
        g_Ws = ops.gemm_tn(gu, hs.contiguous()) if need[2] else None
        g_Wn = ops.gemm_tn(gu, agg.contiguous()) if need[3] else None
        return g_self, g_agg, g_Ws, g_Wn, None, None


def _live(indptr):
    """A static-shape block's real row count on the device (sampling, static_shapes=True),
    or None: the gathers over its CSR treat the rows past it as empty."""
    return getattr(indptr, "_gnnrec_live", None)


class SageRelFn(torch.autograd.Function):
    """One sum / mean ConvLayer relation of a training step — SpmmFn and SageProjectFn as
    ONE autograd node whose forward and backward are each ONE dispatcher call
    (torch.ops.gnnrec.sage_rel_forward / sage_rel_backward, csrc/torch_ops.cpp), which issue
    the same launches as the two-node form from C++: the spmm + projection GEMM (row norms
    kept), and the epilogue Jacobian, self / neighbour input GEMMs, device CSR transpose +
    transposed gather, and the two split-K weight-gradient GEMMs.  Same values bit for bit;
    the per-launch Python wrappers and the second node per relation were most of the C2
    step's host time.  GNNREC_TRAIN_FUSED=0 keeps the two-node form."""

    @staticmethod
    def forward(ctx, m, h_self, Ws, Wn, indptr, indices, ew, reduce: str, norm: bool,
                n_self: int = 0, transposed=None):
        z, agg, nrm = ops._T().sage_rel_forward(m, h_self, n_self, Ws.detach(), Wn.detach(),
                                                indptr, indices, ew, ops.REDUCE[reduce],
                                                bool(norm), None, None, _live(indptr))
        ctx.save_for_backward(h_self, agg, Ws, Wn, z, nrm, indptr, indices, ew)
        ctx.reduce, ctx.norm, ctx.n_src = reduce, bool(norm), m.shape[0]
        ctx.nnz = ops._nnz(indptr)  # sampled blocks carry it: no readback
        # the block's source-major CSR when the sampler built it (unweighted relations)
        ctx.transposed = transposed if ew is None else None
        return z

    @staticmethod
    def backward(ctx, gz):
        h_self, agg, Ws, Wn, z, nrm, indptr, indices, ew = ctx.saved_tensors
        need = ctx.needs_input_grad
        mask = (1 if need[1] else 0) | (2 if need[0] else 0) | (4 if need[2] else 0) | \
            (8 if need[3] else 0)
        tr = ctx.transposed or (None, None, None)
        g_self, g_m, g_Ws, g_Wn, _gb, _gbne = ops._T().sage_rel_backward(
            gz, z, nrm, h_self, agg, Ws.detach(), Wn.detach(), indptr, indices, ew,
            ops.REDUCE[ctx.reduce], ctx.n_src, ctx.nnz, ctx.norm, mask, *tr,
            live_src=_live(tr[0]) if tr[0] is not None else None)
        return (g_m if need[0] else None, g_self if need[1] else None,
                g_Ws if need[2] else None, g_Wn if need[3] else None,
                None, None, None, None, None, None, None)


PER = 5  # HeteroSageFn parameters per relation: W_preagg, W_self, W_neigh, bias, bias_nonempty


class HeteroSageFn(torch.autograd.Function):
    """A whole HeteroGraphConv layer of a training step over a sampled block — every
    relation a SageRelFn-style sum / mean relation, the cross-relation sum / mean — as ONE
    autograd node.  Its backward writes each node type's input gradient ONCE: the first
    relation that reaches a table stores into it, the later ones accumulate (the transposed
    gather with GNNREC_SPMM_ACCUM, the self GEMM with ACC_ADD), so the per-relation
    gradients are never materialised and added by autograd (C3: ten full-table adds per
    step, 0.49 ms), and the engine runs one node per layer instead of one per relation.

    apply(spec, *tables, *[W_preagg_r or None, W_self_r, W_neigh_r, bias_r or None,
    bias_nonempty_r or None for r]) -> one output per dst group.  bias_r / bias_nonempty_r
    carry a NodeEmbedding folded into the first layer (nn.ConvModel._fold_plan): the tables
    are then the raw features, W_self_r = W_s W_e,dst, bias_r = W_s b_e,dst, W_neigh_r = W_n
    W_e,src, bias_nonempty_r = W_n b_e,src (rows with an in-edge: the mean of an empty set
    is 0).  spec = (n_tables, rels, groups): rels[r] = (src table, dst table, reduce,
    norm, n_dst, indptr, indices, edge weight, transposed); groups[k] = (dst table, relation
    indices, 'sum' | 'mean').  W_preagg_r: the relation's fc_preagg (messages relu(x W_preᵀ),
    src/model.py:102,151), whose input gradient is accumulated into the table as well."""

    @staticmethod
    def forward(ctx, spec, *args):
        n_t, rels, groups = spec
        tables = args[:n_t]
        per = args[n_t:]
        T = ops._T()
        zs, saved = [], []
        msgs = []
        for r, (si, di, reduce, norm, n_dst, ip, ix, ew, _tr) in enumerate(rels):
            Wp = per[PER * r]
            m = tables[si] if Wp is None else ops.gemm(tables[si].contiguous(), Wp.detach(),
                                                       relu=True)
            msgs.append(m if Wp is not None else torch.empty(0))
            Ws, Wn, b, bne = per[PER * r + 1:PER * r + PER]
            z, agg, nrm = T.sage_rel_forward(
                m, tables[di], n_dst, Ws.detach(), Wn.detach(), ip, ix, ew, ops.REDUCE[reduce],
                bool(norm), None if b is None else b.detach(),
                None if bne is None else bne.detach(), _live(ip))
            zs.append(z)
            saved += [agg, z, nrm]
        outs = []
        for _di, idx, mode in groups:
            o = zs[idx[0]]
            for r in idx[1:]:
                o = o + zs[r]
            if mode == 'mean' and len(idx) > 1:
                o = o / len(idx)
            outs.append(o)
        ctx.save_for_backward(*tables, *[t if t is not None else torch.empty(0) for t in per],
                              *saved, *msgs)
        ctx.spec = spec
        ctx.m_given = [per[PER * r] is not None for r in range(len(rels))]
        ctx.n_src = [tables[rels[r][0]].shape[0] for r in range(len(rels))]
        ctx.nnz = [ops._nnz(rel[5]) for rel in rels]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *g_outs):
        n_t, rels, groups = ctx.spec
        R = len(rels)
        sv = ctx.saved_tensors
        tables, per = sv[:n_t], sv[n_t:n_t + PER * R]
        saved, msgs = sv[n_t + PER * R:n_t + (PER + 3) * R], sv[n_t + (PER + 3) * R:]
        need = ctx.needs_input_grad[1:]  # (spec)
        need_t, need_per = need[:n_t], need[n_t:]
        T = ops._T()
        g_tab = [None] * n_t
        g_per = [None] * (PER * R)
        for gi, (_di, idx, mode) in enumerate(groups):
            g = g_outs[gi]
            if g is None:
                continue
            g = g.contiguous()
            if mode == 'mean' and len(idx) > 1:
                g = g / len(idx)
            for r in idx:
                si, di, reduce, norm, _n, ip, ix, ew, tr = rels[r]
                agg, z, nrm = saved[3 * r:3 * r + 3]
                Ws, Wn = per[PER * r + 1], per[PER * r + 2]
                given = ctx.m_given[r]  # messages through fc_preagg
                want_m = need_t[si] or (given and need_per[PER * r])
                mask = (1 if need_t[di] else 0) | (2 if want_m else 0) | \
                    (4 if need_per[PER * r + 1] else 0) | (8 if need_per[PER * r + 2] else 0) | \
                    (16 if need_per[PER * r + 3] else 0) | (32 if need_per[PER * r + 4] else 0)
                kw = {}
                if need_t[di]:
                    acc = g_tab[di] is not None
                    if not acc:
                        g_tab[di] = torch.empty((tables[di].shape[0], Ws.shape[1]),
                                                dtype=torch.float32, device=g.device)
                    kw.update(g_self_out=g_tab[di], g_self_acc=acc)
                if want_m and not given:
                    acc = g_tab[si] is not None
                    if not acc:
                        g_tab[si] = torch.empty((tables[si].shape[0], Wn.shape[1]),
                                                dtype=torch.float32, device=g.device)
                    kw.update(g_m_out=g_tab[si], g_m_acc=acc)
                t3 = tr if (tr is not None and ew is None) else (None, None, None)
                if t3[0] is not None:
                    kw.update(live_src=_live(t3[0]))
                _gs, g_m, g_Ws, g_Wn, g_b, g_bne = T.sage_rel_backward(
                    g, z, nrm, tables[di], agg, Ws.detach(), Wn.detach(), ip, ix, ew,
                    ops.REDUCE[reduce], ctx.n_src[r], ctx.nnz[r], bool(norm), mask, *t3, **kw)
                if given and want_m:  # relu(x W_preᵀ): mask, then W_pre's two gradients
                    gy = ops.act_backward(msgs[r], g_m, relu=True, l2norm=False)
                    Wp = per[PER * r]
                    if need_per[PER * r]:
                        g_per[PER * r] = ops.gemm_tn(gy, tables[si].contiguous())
                    if need_t[si]:
                        acc = g_tab[si] is not None
                        if not acc:
                            g_tab[si] = torch.empty((tables[si].shape[0], Wp.shape[1]),
                                                    dtype=torch.float32, device=g.device)
                        ops.gemm(gy, Wp.detach().t().contiguous(), out=g_tab[si],
                                 accum='add' if acc else 'store')
                if need_per[PER * r + 1]:
                    g_per[PER * r + 1] = g_Ws
                if need_per[PER * r + 2]:
                    g_per[PER * r + 2] = g_Wn
                if need_per[PER * r + 3]:
                    g_per[PER * r + 3] = g_b
                if need_per[PER * r + 4]:
                    g_per[PER * r + 4] = g_bne
        return (None, *g_tab, *g_per)


class FoldFn(torch.autograd.Function):
    """The first-layer fold's weight products for one node type (nn._fold_weights): every
    weight W_i that the type's NodeEmbedding (W_e, b_e) feeds, stacked as A = [W_1; W_2; ..],
    -> (W_1 W_e, W_2 W_e, .., W_1 b_e, W_2 b_e, ..), each a contiguous row block of A W_e /
    A b_e.  As one node its backward is the two stacked gradients and three library GEMMs —
    dW_e = Aᵀ dWF and db_e = (dBFᵀ A)ᵀ on the split-K weight-gradient GEMM, dA = dWF W_eᵀ +
    dBF b_eᵀ as one two-operand GEMM — where the per-slice autograd form (cat, matmul,
    slices) zero-filled and copied every slice's gradient and added them (≈15 launches per
    node type in a captured C2 step).  Every product runs on the library's fp32 MFMA GEMMs
    (ops.gemm / ops.gemm_tn), as the inference fold does (inference.py), not vendor BLAS."""

    @staticmethod
    def forward(ctx, W_e, b_e, *Ws):
        A = (torch.cat(Ws, 0) if len(Ws) > 1 else Ws[0]).detach().contiguous()
        W_e, b_e = W_e.detach().contiguous(), b_e.detach().contiguous()
        WF = ops.gemm(A, W_e.t().contiguous())             # A W_e = linear(A, W_eᵀ)
        BF = ops.gemm(b_e.view(1, -1), A).view(-1)         # (A b_e)ᵀ = linear(b_eᵀ, A)
        rows = [W.shape[0] for W in Ws]
        ctx.save_for_backward(A, W_e, b_e)
        ctx.rows = rows
        return (*WF.split(rows), *BF.split(rows))

    @staticmethod
    def backward(ctx, *grads):
        A, W_e, b_e = ctx.saved_tensors
        rows = ctx.rows
        n = len(rows)

        def stacked(gs, shape):
            gs = [g if g is not None else A.new_zeros(shape(r)) for g, r in zip(gs, rows)]
            return (torch.cat(gs, 0) if n > 1 else gs[0]).contiguous()
        dWF = stacked(grads[:n], lambda r: (r, W_e.shape[1]))
        dBF = stacked(grads[n:], lambda r: (r,))
        need = ctx.needs_input_grad
        dW_e = ops.gemm_tn(A, dWF) if need[0] else None
        db_e = ops.gemm_tn(dBF.view(-1, 1), A).view(-1) if need[1] else None
        dWs = [None] * n
        if any(need[2:]):
            dA = ops.gemm(dWF, W_e, dBF.view(-1, 1), b_e.view(-1, 1))
            dWs = list(dA.split(rows))
        return (dW_e, db_e, *dWs)


def sage_rel_fusable(m, h_self, Wn, reduce: str, norm: bool) -> bool:
    """SageRelFn applies: a linear reduce, fp32 row-major tables, the row norm within one
    GEMM block (ops.GEMM_ROW_N)."""
    if os.environ.get("GNNREC_TRAIN_FUSED", "1") == "0" or reduce not in ("sum", "mean") or \
            os.environ.get("GNNREC_SPMM_BWD") == "atomic":
        return False
    if norm and Wn.shape[0] > ops.GEMM_ROW_N:
        return False
    return all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 2 and t.stride(-1) == 1
               for t in (m, h_self))


class CosineFn(torch.autograd.Function):
    """cos_e = <ĥs[src_e], ĥd[dst_e]>; forward = gnnrec_sddmm_cos_f32, backward =
    gnnrec_sddmm_cos_backward_f32 (both reduction sides of the SDDMM backward as weighted
    gathers over the pair graph grouped by src / by dst, in one library call)."""

    @staticmethod
    def forward(ctx, hs, hd, src, dst):
        out = ops.sddmm_cos(src, dst, hs.contiguous(), hd.contiguous())
        ctx.save_for_backward(hs, hd, src, dst)
        return out

    @staticmethod
    def backward(ctx, g):
        hs, hd, src, dst = ctx.saved_tensors
        need = ctx.needs_input_grad
        if not (need[0] or need[1]):
            return None, None, None, None
        ga, gb = ops.sddmm_cos_backward(src, dst, hs.contiguous(), hd.contiguous(),
                                        g.reshape(-1), need[0], need[1])
        return ga, gb, None, None


def _joined(a, b):
    """torch.cat([a, b]) of two 1-d tensors — as a view when b starts where a ends in the
    same storage (no launch)."""
    if a.dim() == 1 and b.dim() == 1 and a.is_contiguous() and b.is_contiguous() and \
            a.dtype == b.dtype and a.device == b.device and \
            a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr() and \
            b.storage_offset() == a.storage_offset() + a.numel():
        return a.as_strided((a.numel() + b.numel(),), (1,), a.storage_offset())
    return torch.cat([a, b])


class CosinePairFn(torch.autograd.Function):
    """CosineFn over the positive and the negative pair graph of one etype at once (they
    share node ids): one forward launch over both edge lists, and one backward call whose
    gradients already sum both graphs' parts.  -> (cos_pos, cos_neg).
    K (optional): the negatives' sources are the positives' repeated K times
    (negative_sampler.Uniform) — the forward is then the grouped launch
    (ops.sddmm_cos_grouped: one gathered row per edge, the same bits)."""

    @staticmethod
    def forward(ctx, hs, hd, src_p, dst_p, src_n, dst_n, K=None):
        hs, hd = hs.contiguous(), hd.contiguous()
        if K is not None:
            a, b = ops.sddmm_cos_grouped(src_p, dst_p, K, dst_n, hs, hd)
        else:
            out = ops.sddmm_cos(torch.cat([src_p, src_n]), torch.cat([dst_p, dst_n]), hs, hd)
            a, b = out[:src_p.numel()], out[src_p.numel():]
        ctx.save_for_backward(hs, hd, src_p, dst_p, src_n, dst_n)
        ctx.n_pos = src_p.numel()
        ctx.K = K
        return a, b

    @staticmethod
    def backward(ctx, g_pos, g_neg):
        hs, hd, src_p, dst_p, src_n, dst_n = ctx.saved_tensors
        need = ctx.needs_input_grad
        if not (need[0] or need[1]):
            return None, None, None, None, None, None, None
        # the positive and negative lists are usually one buffer already (the static batch
        # head's compaction, MarginLossFn's gradient): a view then, no cat / copy launches.
        # The grouped backward reads only the positives' sources.
        src = src_p if ctx.K else _joined(src_p, src_n)
        dst = _joined(dst_p, dst_n)
        n_pos = ctx.n_pos
        g = None
        if g_pos is not None and g_neg is not None:
            g = _joined(g_pos.reshape(-1), g_neg.reshape(-1))
        else:
            g = torch.empty(dst.numel(), dtype=torch.float32, device=dst.device)
            for part, gp in ((g[:n_pos], g_pos), (g[n_pos:], g_neg)):
                if gp is None:
                    part.zero_()
                else:
                    part.copy_(gp.reshape(-1))
        # the grouped layout (each negative's source its positive's): the source side
        # sorts only the positives' keys
        K = ctx.K if ctx.K is not None else 0
        ga, gb = ops.sddmm_cos_backward(src, dst, hs.contiguous(), hd.contiguous(), g,
                                        need[0], need[1], groups=n_pos if K else 0, K=K)
        return ga, gb, None, None, None, None, None


class MarginLossFn(torch.autograd.Function):
    """max_margin_loss (src/model.py:473-533) over every etype at once: the forward kernel
    also writes d(sum of scores)/d(score), so the backward is one scale.
    apply(spec, pos_0, neg_0, pos_1, neg_1, ...) with spec = (delta, [(K, mask, recency)])."""

    @staticmethod
    def forward(ctx, spec, *scores):
        delta, meta = spec
        parts = [(scores[2 * i].reshape(-1), scores[2 * i + 1].reshape(-1), K, mask, rec)
                 for i, (K, mask, rec) in enumerate(meta)]
        loss, total, grads, flat = ops.margin_loss(parts, delta, flat=True)
        ctx.grads, ctx.total, ctx.flat = grads, total, flat
        ctx.shapes = [t.shape for t in scores]
        return loss

    @staticmethod
    def backward(ctx, g):
        # the unscaled gradients are views of one buffer (ops.margin_loss): one scale launch
        # for all of them, handed back as views of its result (the cosine backward then joins
        # an etype's positive and negative parts without a copy)
        scaled = ctx.flat * (g / ctx.total)
        out, off = [None], 0
        for i, (gp, gn) in enumerate(ctx.grads):
            for j, part in enumerate((gp, gn)):
                n = part.numel()
                view = scaled.narrow(0, off, n).view(ctx.shapes[2 * i + j])
                out.append(view if ctx.needs_input_grad[1 + 2 * i + j] else None)
                off += n
        return tuple(out)
