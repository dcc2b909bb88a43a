"""Recommendation scoring + top-k — drop-ins for reference
src/metrics.py (`create_ground_truth` :9-17, `create_already_bought` :20-28,
`get_recs` :31-78, `recs_to_metrics` :81-107, `get_metrics_at_k` :110-134),
consumed by main_inference.py:153-166.

The reference loops over users in Python: repeat the user embedding once per
item, cosine (or the MLP head) against every item, copy to the host, argsort,
filter already-bought items, keep k.  Here a batch of users is scored against
every item in one fp32 MFMA GEMM of L2-normalised embeddings (gnnrec_gemm_f32),
or by the re-associated MLP head (gnnrec_edge_mlp_f32), and
gnnrec_topk_rows_f32 selects the k best non-bought items per user on the
device.  Only the [users, k] result leaves the GPU.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
import torch

from . import _lib, ops


def create_ground_truth(users, items):
    """{user: [items actually bought]} (reference src/metrics.py:9-17)."""
    d = defaultdict(list)
    for u, i in zip(np.asarray(users).tolist(), np.asarray(items).tolist()):
        d[u].append(i)
    return d


def create_already_bought(g, bought_eids, etype='buys'):
    """{user: [items already bought]} from the bought edges (src/metrics.py:20-28)."""
    users, items = g.find_edges(bought_eids, etype=etype)
    return create_ground_truth(torch.as_tensor(users).cpu().numpy(),
                               torch.as_tensor(items).cpu().numpy())


def topk_rows(scores: torch.Tensor, k: int, exclude_indptr=None, exclude_indices=None):
    """Per row: k best columns by (score desc, column asc), excluded columns skipped."""
    n_rows, n_cols = scores.shape
    vals = torch.empty((n_rows, k), dtype=torch.float32, device=scores.device)
    idx = torch.empty((n_rows, k), dtype=torch.int64, device=scores.device)
    _lib.torch_ops().topk_rows(scores, k, exclude_indptr, exclude_indices, vals, idx)
    return vals, idx


def _normalize_rows(x: torch.Tensor) -> torch.Tensor:
    """x / ||x|| per row (zero rows stay zero) — the fused GEMM with an identity weight
    and its L2-norm epilogue (exact: x·I adds only zero products)."""
    eye = torch.eye(x.shape[1], dtype=torch.float32, device=x.device)
    return ops.gemm(x.contiguous(), eye, l2norm=True)


def get_recs(g, h, model, embed_dim, k, user_ids, already_bought_dict,
             remove_already_bought=True, cuda=True, device=None, pred: str = 'cos',
             use_popularity: bool = False, weight_popularity=1, batch_size: int = 1024):
    """Top-k recommendations for every user in user_ids: {user: np.ndarray[k]}."""
    if pred not in ('cos', 'nn'):
        raise KeyError(f'Prediction function {pred} not recognized.')
    dev = h['item'].device
    items = h['item'].contiguous()
    n_items = items.shape[0]
    user_ids = [int(u) for u in user_ids]
    if pred == 'cos':
        items_hat = _normalize_rows(items)
    else:
        layer = model.pred_fn.layer_nn
        W1 = layer.hidden_1.weight
        Q = ops.gemm(items, W1[:, embed_dim:])                     # item half of hidden_1
    pop = None
    if use_popularity:
        pop = g.ndata['popularity']['item'].reshape(-1).to(dev).float() * weight_popularity
    if pred == 'nn':
        batch_size = max(1, min(batch_size, (1 << 26) // max(1, n_items)))
    recs = {}
    for b0 in range(0, len(user_ids), batch_size):
        ub = user_ids[b0:b0 + batch_size]
        users = h['user'][torch.tensor(ub, device=dev)].contiguous()
        if pred == 'cos':
            scores = ops.gemm(_normalize_rows(users), items_hat)   # [B, n_items] cosine
        else:
            P = ops.gemm(users, W1[:, :embed_dim], bias=layer.hidden_1.bias)
            B = len(ub)
            src = torch.arange(B, device=dev).repeat_interleave(n_items)
            dst = torch.arange(n_items, device=dev).repeat(B)
            scores = ops.edge_mlp(src, dst, P, Q, layer.hidden_2.weight, layer.hidden_2.bias,
                                  layer.output.weight.reshape(-1),
                                  layer.output.bias).view(B, n_items)
        if pop is not None:  # softmax over items, plus weighted popularity (metrics.py:69-72)
            scores = torch.softmax(scores, dim=1) + pop
        ex_ptr = ex_idx = None
        if remove_already_bought:
            lists = [already_bought_dict.get(u, []) for u in ub]
            ip = np.zeros(len(lists) + 1, np.int64)
            np.cumsum([len(x) for x in lists], out=ip[1:])
            flat = np.fromiter((i for x in lists for i in x), dtype=np.int64, count=int(ip[-1]))
            ex_ptr = torch.from_numpy(ip).to(dev)
            ex_idx = torch.from_numpy(flat).to(dev) if flat.size else torch.zeros(1, dtype=torch.int64, device=dev)
        _, top = topk_rows(scores, k, ex_ptr, ex_idx)
        top = top.cpu().numpy()
        for r, u in enumerate(ub):
            row = top[r]
            recs[u] = row[row >= 0]
    return recs


def recs_to_metrics(recs, ground_truth_dict, g):
    """precision / recall / coverage (reference src/metrics.py:81-107)."""
    k_relevant = k_total = 0
    for uid, iids in recs.items():
        gt = set(ground_truth_dict[uid])
        k_total += len(iids)
        k_relevant += sum(1 for i in iids if i in gt)
    precision = k_relevant / k_total
    k_relevant = k_total = 0
    for uid, iids in recs.items():
        rec = set(np.asarray(iids).tolist())
        k_total += len(ground_truth_dict[uid])
        k_relevant += sum(1 for i in ground_truth_dict[uid] if i in rec)
    recall = k_relevant / k_total
    nb_recommended = len(set(int(i) for v in recs.values() for i in v))
    coverage = nb_recommended / g.num_nodes('item')
    return precision, recall, coverage


def get_metrics_at_k(h, g, model, embed_dim, ground_truth, bought_eids, k,
                     remove_already_bought=True, cuda=True, device=None, pred='cos',
                     use_popularity=False, weight_popularity=1):
    """reference src/metrics.py:110-134."""
    already_bought_dict = create_already_bought(g, bought_eids)
    users, items = ground_truth
    user_ids = np.unique(users).tolist()
    ground_truth_dict = create_ground_truth(users, items)
    recs = get_recs(g, h, model, embed_dim, k, user_ids, already_bought_dict,
                    remove_already_bought, cuda, device, pred, use_popularity, weight_popularity)
    return recs_to_metrics(recs, ground_truth_dict, g)


def MRR_neg_edges(model, blocks, pos_g, neg_g, etype, neg_sample_size):
    """Mean reciprocal rank of each positive edge among its negatives (reference
    src/metrics.py:137-157, marked "currently not used" there).  The reference passes
    `etype` where ConvModel.forward expects `embedding_layer` and reshapes the per-etype
    score dict directly; here the model runs with its own embedding_layer setting and the
    scores of `etype` are ranked: rank = #{neg >= pos} + 1 over the positive's
    neg_sample_size negatives (negatives grouped [E_pos, K], sampling.py:163-165)."""
    input_features = blocks[0].srcdata['features']
    with torch.no_grad():
        _, pos_score, neg_score = model(blocks, input_features, pos_g, neg_g,
                                        getattr(model, 'embedding_layer', True))
    if isinstance(pos_score, dict):
        ce = next(c for c in pos_score if etype in (c, c[1]))
        pos_score, neg_score = pos_score[ce], neg_score[ce]
    neg = neg_score.reshape(-1, neg_sample_size)
    rankings = torch.sum(neg >= pos_score.reshape(-1, 1), dim=1) + 1
    return float(np.mean(1.0 / rankings.cpu().numpy()))
