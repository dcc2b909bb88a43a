"""Checker backend with the gnnrec.ops signatures, computed by the CPU oracle.

TEST INFRASTRUCTURE: lets the multi-process (gloo, CPU) tests drive the
product's partition / exchange / orchestration code (gnnrec.inference) while
the per-rank arithmetic is done by oracle/ — the product itself never falls
back to this (it raises when libgnnrec.so is missing)."""
import numpy as np
import torch

from oracle import oracle


def spmm(indptr, indices, X, reduce="mean", edge_weight=None, out=None, empty_neginf=False,
         accumulate=False, split=None):  # split: the HIP op's heavy-row chunking (no-op here)
    ip = indptr.cpu().numpy()
    res = oracle.spmm_csr(ip, indices.cpu().numpy(), X.detach().cpu().numpy(), reduce,
                          None if edge_weight is None else edge_weight.cpu().numpy())
    if reduce == "max" and empty_neginf:
        res[(ip[1:] - ip[:-1]) == 0] = -np.inf
    t = torch.from_numpy(res)
    if accumulate:
        t = torch.maximum(out, t) if reduce == "max" else out + t
    if out is not None:
        out.copy_(t)
        return out
    return t


def lstm_aggregate(indptr, indices, X, W_ih, W_hh, b_ih, b_hh, out=None):
    res = torch.from_numpy(oracle.lstm_reduce(
        indptr.cpu().numpy(), indices.cpu().numpy(), X.detach().cpu().numpy(),
        *(w.detach().cpu().numpy() for w in (W_ih, W_hh, b_ih, b_hh))))
    if out is not None:
        out.copy_(res)
        return out
    return res


def _attn_update(out, t, accum, attn_vec, attn_state):
    """online softmax over relations (the product's ACC_ATTN_* semantics) in numpy."""
    z = t.numpy().astype(np.float64)
    e = z @ attn_vec.detach().cpu().numpy().astype(np.float64)
    if accum == "attn_first":
        m, ssum, acc = e, np.ones_like(e), z
    else:
        st = attn_state.cpu().numpy().astype(np.float64)
        m = np.maximum(st[:, 0], e)
        keep, new = np.exp(st[:, 0] - m), np.exp(e - m)
        ssum = st[:, 1] * keep + new
        acc = out.cpu().numpy().astype(np.float64) * keep[:, None] + z * new[:, None]
    if accum == "attn_last":
        acc = acc / ssum[:, None]
    attn_state.copy_(torch.from_numpy(np.stack([m, ssum], 1).astype(np.float32)))
    return torch.from_numpy(acc.astype(np.float32))


def gemm(A1, W1, A2=None, W2=None, bias=None, *, relu=False, l2norm=False, sigmoid=False,
         accum="store", out_div=0.0, out=None, a2_deg=None, a2_mode=0, attn_vec=None,
         attn_state=None, bias_nonempty=None):
    z = oracle.linear(A1.detach().cpu().numpy(), W1.detach().cpu().numpy(),
                      None if bias is None else bias.detach().cpu().numpy())
    if bias_nonempty is not None:
        ne = (a2_deg.cpu().numpy() > 0)[:, None]
        z = (z + np.where(ne, bias_nonempty.detach().cpu().numpy(), np.float32(0))).astype(np.float32)
    if A2 is not None:
        a2 = A2.detach().cpu().numpy().astype(np.float32)
        if a2_mode == 1:
            deg = np.maximum(a2_deg.cpu().numpy(), 1).astype(np.float32)
            a2 = a2 / deg[:, None]
        elif a2_mode == 2:
            a2 = np.where((a2_deg.cpu().numpy() == 0)[:, None], np.float32(0), a2)
        z = (z + oracle.linear(a2, W2.detach().cpu().numpy())).astype(np.float32)
    if relu:
        z = oracle.relu(z)
    if sigmoid:
        z = oracle.sigmoid(z)
    if l2norm:
        z = oracle.l2_normalize_rows_guarded(z)
    t = torch.from_numpy(np.ascontiguousarray(z, np.float32))
    if accum.startswith("attn"):
        t = _attn_update(out, t, accum, attn_vec, attn_state)
        if out is None:
            return t
        out.copy_(t)
        return out
    if out is None:
        return t
    if accum == "add":
        t = out + t
    elif accum == "max":
        t = torch.maximum(out, t)
    if out_div > 0:
        t = t / out_div
    out.copy_(t)
    return out


def add_(a, b):
    a += b
    return a
