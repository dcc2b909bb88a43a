"""Torch-facing wrappers over the gnnrec ops (include/gnnrec.h, registered with the torch
dispatcher as torch.ops.gnnrec.* by csrc/torch_ops.cpp).

Each function validates shapes/dtypes/devices on the host, allocates the output with
torch (device memory plumbing only) and launches the HIP kernel through its
torch.ops.gnnrec op on the current HIP stream, so the launches are visible to the
dispatcher, to torch.compile (meta kernels, functionalised outputs) and to HIP-graph
capture.  There is no fallback: a missing library or a CPU tensor is an error.
"""
from __future__ import annotations

import contextlib
import os

from typing import Optional

import torch

from . import _lib


def _T():
    """torch.ops.gnnrec (loads libgnnrec.so + libgnnrec_torch.so on first use)."""
    return _lib.torch_ops()

REDUCE = {"sum": _lib.REDUCE_SUM, "mean": _lib.REDUCE_MEAN, "max": _lib.REDUCE_MAX}
ACCUM = {"store": _lib.ACC_STORE, "add": _lib.ACC_ADD, "max": _lib.ACC_MAX,
         "attn_first": _lib.ACC_ATTN_FIRST, "attn": _lib.ACC_ATTN,
         "attn_last": _lib.ACC_ATTN_LAST}


def _attn_args(accum, attn_vec, attn_state, n_rows, n_cols):
    """Validated (attn_vec, attn_state) for the attention accumulate modes, else (None, None)."""
    if not accum.startswith("attn"):
        return None, None
    if attn_vec is None or attn_state is None:
        raise ValueError(f"accum={accum!r} needs attn_vec and attn_state")
    _dev(attn_vec, "attn_vec", torch.float32)
    _dev(attn_state, "attn_state", torch.float32)
    if attn_vec.numel() != n_cols or tuple(attn_state.shape) != (n_rows, 2) or \
            not attn_state.is_contiguous():
        raise ValueError(f"attention needs attn_vec [{n_cols}] and a contiguous attn_state "
                         f"[{n_rows}, 2]")
    return attn_vec.detach().contiguous(), attn_state


def _dev(t: torch.Tensor, name: str, dtype=None) -> None:
    if not (t.is_cuda or t.is_meta):  # meta: shape tracing, the ops launch nothing
        raise ValueError(f"{name} must be a HIP device tensor (got {t.device}); "
                         f"gnnrec has no CPU path")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype} (got {t.dtype})")


def _rowmajor(t: torch.Tensor, name: str) -> int:
    """Leading dimension of a 2-D tensor with unit column stride."""
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D (got shape {tuple(t.shape)})")
    if t.stride(1) != 1 and t.shape[1] > 1:
        raise ValueError(f"{name} must have unit column stride")
    return max(t.stride(0), t.shape[1], 1)


def set_concurrency(reserve_cus: int = 0, dynamic: bool = False) -> None:
    """Process-wide mode of the row kernels (spmm, spmm_project) for launches that share
    the chip with kernels on other streams (gnnrec_set_concurrency): leave `reserve_cus`
    CUs free, and hand rows out through a device work queue when `dynamic`."""
    _T().set_concurrency(int(reserve_cus), bool(dynamic))


def get_concurrency():
    """(reserve_cus, dynamic) currently in force."""
    r, d = _T().get_concurrency()
    return r, bool(d)


def rowq_stats():
    """(queued launches, launches refused a busy ring slot) since the library loaded."""
    q, b = _T().rowq_stats()
    return q, b


@contextlib.contextmanager
def concurrency(reserve_cus: int, dynamic: bool = True):
    """set_concurrency for the launches enqueued inside the block, restored after."""
    old = get_concurrency()
    set_concurrency(reserve_cus, dynamic)
    try:
        yield
    finally:
        set_concurrency(*old)


def hold_cus(blocks: int, usec: int, threads: int = 256, lds_bytes: int = 16384,
             stream=None) -> None:
    """Diagnostic: `blocks` workgroups holding `lds_bytes` of LDS each stay resident for
    `usec` µs on `stream` (default: current) — a collective kernel's footprint."""
    dev = torch.device("cuda", torch.cuda.current_device())
    sink = _hold_sink.get(dev.index)
    if sink is None:
        sink = _hold_sink[dev.index] = torch.empty(1024, dtype=torch.float32, device=dev)
    with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream(dev)):
        _T().hold_cus(int(blocks), int(threads), int(lds_bytes), int(usec), sink)


_hold_sink = {}

DEFAULT_SPLIT = 2048  # edges per chunk for rows split across wavefronts


def split_plan(indptr: torch.Tensor, split: int = DEFAULT_SPLIT):
    """Heavy-row plan for a CSR, computed once and cached on the indptr tensor.

    Returns None when no row has more than `split` edges, else
    (heavy_rows, chunk_ptr, chunk_row, n_chunks)."""
    cached = getattr(indptr, "_gnnrec_split_plan", None)
    if cached is not None and cached[0] == split:
        return cached[1]
    deg = indptr[1:] - indptr[:-1]
    heavy = torch.nonzero(deg > split).squeeze(1)
    plan = None
    if heavy.numel() > 0:
        nch = (deg[heavy] + split - 1) // split
        chunk_ptr = torch.zeros(heavy.numel() + 1, dtype=torch.int64, device=indptr.device)
        torch.cumsum(nch, 0, out=chunk_ptr[1:])
        chunk_row = torch.repeat_interleave(
            torch.arange(heavy.numel(), device=indptr.device), nch)
        plan = (heavy.contiguous(), chunk_ptr, chunk_row.contiguous(), int(chunk_ptr[-1].item()))
    try:
        indptr._gnnrec_split_plan = (split, plan)
    except AttributeError:  # pragma: no cover
        pass
    return plan


def _device_plan(indptr: torch.Tensor, split: int):
    """Device-built heavy-row plan sized from the host edge count (cached on indptr);
    None when no row can have more than `split` edges."""
    cached = getattr(indptr, "_gnnrec_dev_plan", None)
    if cached is not None and cached[0] == split:
        return cached[1]
    n_dst, E = indptr.numel() - 1, indptr._gnnrec_nnz
    cap_h = min(n_dst, E // (split + 1))
    res = None
    if cap_h > 0:
        cap_c = E // split + cap_h
        pl = torch.empty(2 + cap_h + cap_h + 1 + cap_c, dtype=torch.int64, device=indptr.device)
        _T().spmm_plan_build(indptr, split, cap_h, pl)
        res = (pl, cap_h, cap_c)
    try:
        indptr._gnnrec_dev_plan = (split, res)
    except AttributeError:  # pragma: no cover
        pass
    return res


def plan_overflows() -> int:
    """Device-built heavy-row plans that overflowed their capacities since the library
    loaded (gnnrec_spmm_plan_overflows; synchronises the device).  Such a plan's gather
    reduced every row unsplit — exact, not clipped — but a nonzero count means a CSR whose
    host edge count (`_gnnrec_nnz`) understated its edges: check it after a step."""
    return int(_T().spmm_plan_overflows())


def spmm(indptr: torch.Tensor, indices: torch.Tensor, X: torch.Tensor, reduce: str = "mean",
         edge_weight: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
         empty_neginf: bool = False, split: Optional[int] = DEFAULT_SPLIT,
         accumulate: bool = False) -> torch.Tensor:
    """a1: out[v] = reduce_{e in row v} X[indices[e]] (* edge_weight[e]).

    indptr int64 [n_dst+1], indices int32 [E] (local rows of X), X fp32 [n_src, d].
    Rows with more than `split` edges are reduced in parallel chunks (split=None: never).
    accumulate: out[v] = out[v] (+ | max) that (source-range tiles of one relation; max
    needs empty_neginf so rows without edges in the tile leave out unchanged).
    """
    T = _T()
    _dev(indptr, "indptr", torch.int64)
    _dev(indices, "indices", torch.int32)
    _dev(X, "X", torch.float32)
    if reduce not in REDUCE:
        raise KeyError(f"Aggregator reduce {reduce} not recognized.")
    n_dst = indptr.numel() - 1
    d = X.shape[1]
    _rowmajor(X, "X")
    if edge_weight is not None:
        _dev(edge_weight, "edge_weight", torch.float32)
        if edge_weight.numel() != indices.numel():
            raise ValueError("edge_weight must have one value per edge")
        edge_weight = edge_weight.contiguous()
    if out is None:
        if accumulate:
            raise ValueError("spmm: accumulate needs out")
        out = torch.empty((n_dst, d), dtype=torch.float32, device=X.device)
    else:
        _dev(out, "out", torch.float32)
        if tuple(out.shape) != (n_dst, d):
            raise ValueError(f"out must be [{n_dst}, {d}]")
    _rowmajor(out, "out")
    flags = _lib.SPMM_EMPTY_NEGINF if empty_neginf else 0
    if accumulate:
        if reduce == "max" and not empty_neginf:
            raise ValueError("spmm: max accumulation needs empty_neginf")
        flags |= _lib.SPMM_ACCUM
    if split and getattr(indptr, "_gnnrec_split_plan", None) is None and \
            getattr(indptr, "_gnnrec_nnz", None) is not None:
        # edge count known, degrees not: heavy-row plan built on the device (no readback)
        dplan = _device_plan(indptr, split)
        if dplan is not None:
            pl, cap_h, cap_c = dplan
            ws = torch.empty((cap_c, d), dtype=torch.float32, device=X.device)
            T.spmm_csr_planned(indptr, indices, edge_weight, X, REDUCE[reduce], flags, split, pl,
                               cap_h, cap_c, out, ws)
            return out
        split = None  # no row can exceed split
    plan = split_plan(indptr, split) if split else None
    if plan is None:
        T.spmm_csr(indptr, indices, edge_weight, X, REDUCE[reduce], flags, out)
        return out
    heavy, chunk_ptr, chunk_row, n_chunks = plan
    ws = torch.empty((n_chunks, d), dtype=torch.float32, device=X.device)
    T.spmm_csr_split(indptr, indices, edge_weight, X, REDUCE[reduce], flags, split, heavy,
                     chunk_ptr, chunk_row, n_chunks, out, ws)
    return out


def spmm2(csr_a, csr_b, X: torch.Tensor, reduce: str = "sum", out_a=None, out_b=None,
          accumulate: bool = False, empty_neginf: bool = False):
    """a1 for two relations into one destination type in one launch (gnnrec_spmm_csr2_f32):
    csr_* = (indptr, indices int32, edge_weight|None) over the same n_dst rows, both gathering
    from X -> (out_a, out_b), each bitwise what spmm() gives for that relation.  No heavy-row
    split: callers use it only for CSRs without heavy rows (split_plan(...) is None)."""
    (ip_a, ix_a, w_a), (ip_b, ix_b, w_b) = csr_a, csr_b
    for t, n in ((ip_a, "indptr_a"), (ip_b, "indptr_b")):
        _dev(t, n, torch.int64)
    _dev(X, "X", torch.float32)
    if reduce not in REDUCE:
        raise KeyError(f"Aggregator reduce {reduce} not recognized.")
    if (w_a is None) != (w_b is None):
        raise ValueError("spmm2: edge weights on both relations or on neither")
    n_dst, d = ip_a.numel() - 1, X.shape[1]
    if accumulate and (out_a is None or out_b is None):
        raise ValueError("spmm2: accumulate needs out_a and out_b")
    if out_a is None:
        out_a = torch.empty((n_dst, d), dtype=torch.float32, device=X.device)
    if out_b is None:
        out_b = torch.empty((n_dst, d), dtype=torch.float32, device=X.device)
    if accumulate and reduce == "max" and not empty_neginf:
        raise ValueError("spmm2: max accumulation needs empty_neginf")
    flags = (_lib.SPMM_EMPTY_NEGINF if empty_neginf else 0) | (_lib.SPMM_ACCUM if accumulate else 0)
    _T().spmm_csr2(ip_a, ix_a, None if w_a is None else w_a.contiguous(), ip_b, ix_b,
                   None if w_b is None else w_b.contiguous(), X, REDUCE[reduce], flags, out_a,
                   out_b)
    return out_a, out_b


def csr_transpose(indptr: torch.Tensor, indices: torch.Tensor, n_src: int,
                  edge_weight: Optional[torch.Tensor] = None, mean: bool = False,
                  n_edges: Optional[int] = None):
    """Source-major CSR of a dst-major block (stable: ascending edge id per source row).
    -> (indptr_t int64 [n_src+1], indices_t int32 = dst rows, ew_t float32 or None), where
    ew_t = edge_weight (· 1/deg(dst) when mean) in the transposed order."""
    T = _T()
    _dev(indptr, "indptr", torch.int64)
    _dev(indices, "indices", torch.int32)
    dev = indptr.device
    n_dst, E = indptr.numel() - 1, _nnz(indptr) if n_edges is None else int(n_edges)
    if indices.numel() < E:
        raise ValueError("csr_transpose: indices shorter than the edge count")
    if edge_weight is not None:
        _dev(edge_weight, "edge_weight", torch.float32)
        if edge_weight.numel() < E:
            raise ValueError("csr_transpose: edge_weight shorter than the edge count")
    ip_t = torch.empty(n_src + 1, dtype=torch.int64, device=dev)
    ix_t = torch.empty(E, dtype=torch.int32, device=dev)
    w_t = torch.empty(E, dtype=torch.float32, device=dev) if (edge_weight is not None or mean) else None
    nbytes = int(T.csr_transpose_workspace_bytes(E, n_src))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    T.csr_transpose(indptr, indices, edge_weight, n_src, E, bool(mean), ws, ip_t, ix_t, w_t)
    ip_t._gnnrec_nnz = E
    return ip_t, ix_t, w_t


def csr_build(src: torch.Tensor, dst: torch.Tensor, n_dst: int):
    """dst-major CSR of the COO relation (src, dst) with in-row order = edge id
    (gnnrec_csr_build: stable radix sort of the dst ids on the device).
    -> (indptr int64 [n_dst+1], indices int32 = src ids, eids int64)."""
    T = _T()
    _dev(dst, "dst", torch.int64)
    _dev(src, "src", torch.int64)
    if src.shape != dst.shape or src.dim() != 1:
        raise ValueError("csr_build: src and dst must be 1-D tensors of one length")
    dev, E = dst.device, dst.numel()
    if E and n_dst <= 0:
        raise ValueError(f"csr_build: {E} edges into {n_dst} rows")
    src, dst = src.contiguous(), dst.contiguous()
    indptr = torch.empty(n_dst + 1, dtype=torch.int64, device=dev)
    indices = torch.empty(E, dtype=torch.int32, device=dev)
    eids = torch.empty(E, dtype=torch.int64, device=dev)
    nbytes = int(T.csr_build_workspace_bytes(E, n_dst))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    T.csr_build(src, dst, n_dst, ws, indptr, indices, eids)
    indptr._gnnrec_nnz = E
    return indptr, indices, eids


def membership_csr(src: torch.Tensor, dst: torch.Tensor, n_src: int, n_dst: int):
    """The dst-major CSR of (src, dst) with every row's source ids ascending — what
    has_edges searches.  Two stable radix sorts of the library (gnnrec_csr_build): by source
    (edge ids grouped by source), then by destination over the edges in that order, so the
    second sort's stability leaves each row sorted by source.  -> (indptr, sorted_indices)."""
    _dev(src, "src", torch.int64)
    _dev(dst, "dst", torch.int64)
    if src.numel() == 0:
        return torch.zeros(n_dst + 1, dtype=torch.int64, device=src.device), \
            torch.zeros(0, dtype=torch.int32, device=src.device)
    _, _, by_src = csr_build(dst, src, n_src)
    indptr, indices, _ = csr_build(gather_rows(src, by_src), gather_rows(dst, by_src), n_dst)
    return indptr, indices


def has_edges(indptr: torch.Tensor, sorted_indices: torch.Tensor, n_src: int,
              u: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """K10: bool [n], (u[i] -> v[i]) is an edge of the relation whose membership_csr is
    (indptr, sorted_indices) (gnnrec_csr_has_edges: one binary search per query)."""
    _dev(indptr, "indptr", torch.int64)
    u = torch.as_tensor(u, dtype=torch.int64, device=indptr.device).reshape(-1).contiguous()
    v = torch.as_tensor(v, dtype=torch.int64, device=indptr.device).reshape(-1).contiguous()
    if u.numel() != v.numel():
        raise ValueError(f"has_edges: {u.numel()} sources for {v.numel()} destinations")
    out = torch.empty(u.numel(), dtype=torch.bool, device=indptr.device)
    if u.numel():
        _T().csr_has_edges(indptr, sorted_indices, int(n_src), u, v, out)
    return out


def csr_from_keys(keys: torch.Tensor, n_rows: int):
    """Rows of a COO list: -> (indptr int64 [n_rows+1], perm int32 [E]) with perm the edge
    ids grouped by keys[e] (ascending edge id inside a row).  keys: int32/int64 in [0, n_rows)."""
    T = _T()
    if keys.dtype != torch.int32:
        keys = keys.to(torch.int32)
    _dev(keys, "keys", torch.int32)
    keys = keys.contiguous()
    dev, E = keys.device, keys.numel()
    ip = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
    perm = torch.empty(E, dtype=torch.int32, device=dev)
    nbytes = int(T.csr_from_keys_workspace_bytes(E, n_rows))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    T.csr_from_keys(keys, n_rows, ws, ip, perm)
    ip._gnnrec_nnz = E
    return ip, perm


def add_(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a += b (same shape, contiguous fp32) with the library's add kernel; returns a."""
    _dev(a, "a", torch.float32)
    _dev(b, "b", torch.float32)
    if a.shape != b.shape or not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("add_: operands must be contiguous and of one shape")
    _T().add_(a, b)
    return a


def tree_sum_(parts) -> torch.Tensor:
    """parts[0] = ((p0+p1)+(p2+p3))+... over 2, 4 or 8 same-shape contiguous fp32 tables in
    one kernel pass (gnnrec_tree_sum_f32): the same additions, in the same order, as
    pairwise add_ launches level by level; returns parts[0]."""
    n = len(parts)
    if n not in (2, 4, 8):
        raise ValueError("tree_sum_: 2, 4 or 8 tables")
    a = parts[0]
    for p in parts:
        _dev(p, "part", torch.float32)
        if p.shape != a.shape or not p.is_contiguous():
            raise ValueError("tree_sum_: operands must be contiguous and of one shape")
    _T().tree_sum_(a, list(parts[1:]))
    return a


def l2_normalize_rows(y: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = y / ‖y‖ per row, rows with ‖y‖ == 0 unchanged (src/model.py:230-235), one
    wave per row (gnnrec_row_epilogue_f32)."""
    _dev(y, "y", torch.float32)
    M, N = y.shape
    _rowmajor(y, "y")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=y.device)
    _T().row_epilogue(y, 1, ACCUM["store"], 0.0, None, None, out)
    return out


def spmm_backward(indptr, indices, grad_out, reduce, edge_weight=None, X=None, out=None,
                  grad_X=None, n_src=None):
    """Gradient of spmm w.r.t. its source rows (accumulated into grad_X, created if None)."""
    _dev(grad_out, "grad_out", torch.float32)
    n_dst, d = grad_out.shape
    if grad_X is None:
        grad_X = torch.zeros((n_src, d), dtype=torch.float32, device=grad_out.device)
    grad_out = grad_out.contiguous()
    _T().spmm_backward(indptr, indices, edge_weight, grad_out, X, out, REDUCE[reduce], grad_X)
    return grad_X


def gemm(A1: torch.Tensor, W1: torch.Tensor, A2: Optional[torch.Tensor] = None,
         W2: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None, *,
         relu: bool = False, l2norm: bool = False, sigmoid: bool = False,
         accum: str = "store", out_div: float = 0.0, out: Optional[torch.Tensor] = None,
         a2_deg: Optional[torch.Tensor] = None, a2_mode: int = _lib.A2_NONE,
         attn_vec: Optional[torch.Tensor] = None,
         attn_state: Optional[torch.Tensor] = None,
         bias_nonempty: Optional[torch.Tensor] = None,
         row_norm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a2/a3/a4: out (accum)= epi(A1 W1ᵀ + T(A2) W2ᵀ + bias [+ bias_nonempty where
    a2_deg > 0]).  W are nn.Linear weights [N, K].  row_norm [M] (with l2norm, N <=
    GEMM_ROW_N): receives each row's norm before the normalisation (training)."""
    T = _T()
    _dev(A1, "A1", torch.float32)
    _dev(W1, "W1", torch.float32)
    M, K1 = A1.shape
    N = W1.shape[0]
    if W1.shape[1] != K1:
        raise ValueError(f"W1 shape {tuple(W1.shape)} does not match A1 K={K1}")
    W1 = W1.detach().contiguous()
    _rowmajor(A1, "A1")
    if A2 is not None:
        _dev(A2, "A2", torch.float32)
        _dev(W2, "W2", torch.float32)
        if A2.shape[0] != M or W2.shape[0] != N or W2.shape[1] != A2.shape[1]:
            raise ValueError("A2/W2 shape mismatch")
        _rowmajor(A2, "A2")
        W2 = W2.detach().contiguous()
    if bias is not None:
        _dev(bias, "bias", torch.float32)
        bias = bias.detach().contiguous()
    if a2_mode != _lib.A2_NONE or bias_nonempty is not None:
        _dev(a2_deg, "a2_deg", torch.int32)
    if bias_nonempty is not None:
        _dev(bias_nonempty, "bias_nonempty", torch.float32)
        bias_nonempty = bias_nonempty.detach().contiguous()
    epi = (_lib.EPI_RELU if relu else 0) | (_lib.EPI_L2NORM if l2norm else 0) | (
        _lib.EPI_SIGMOID if sigmoid else 0)
    if out is None:
        if accum not in ("store", "attn_first"):
            raise ValueError("accumulating gemm needs an out tensor")
        out = torch.empty((M, N), dtype=torch.float32, device=A1.device)
    else:
        _dev(out, "out", torch.float32)
        if tuple(out.shape) != (M, N):
            raise ValueError(f"out must be [{M}, {N}]")
    _rowmajor(out, "out")
    av, ast = _attn_args(accum, attn_vec, attn_state, M, N)
    if row_norm is not None:
        _dev(row_norm, "row_norm", torch.float32)
        if not l2norm or N > GEMM_ROW_N or row_norm.numel() != M or not row_norm.is_contiguous():
            raise ValueError(f"row_norm needs l2norm, N <= {GEMM_ROW_N} and a contiguous [{M}]")
    if N > GEMM_ROW_N and (l2norm or av is not None):
        # the row norm / attention score needs the whole row: GEMM (bias, ReLU, sigmoid)
        # into a scratch table, then one row-epilogue pass into out
        z = gemm(A1, W1, A2, W2, bias, relu=relu, sigmoid=sigmoid, a2_deg=a2_deg,
                 a2_mode=a2_mode, bias_nonempty=bias_nonempty)
        T.row_epilogue(z, int(l2norm), ACCUM[accum], float(out_div), av, ast, out)
        return out
    T.gemm(A1, W1, A2, W2, a2_deg, a2_mode, bias, bias_nonempty, epi, ACCUM[accum],
           float(out_div), av, ast, out, row_norm)
    return out


FUSED_D = 128  # gnnrec_spmm_project_f32 handles d_neigh = d_self = out = 128
GEMM_ROW_N = 256  # widest output row gnnrec_gemm_f32 normalises / attends in one block


def can_spmm_project(indptr, X, H, W_self, W_neigh, split: Optional[int] = DEFAULT_SPLIT,
                     avg_deg: Optional[float] = None, gemm_overlaps: bool = False) -> bool:
    """True when a fused aggregation+projection kernel applies (shapes, alignment, no
    heavy rows, GPU tensors).  avg_deg: edges per row to judge
    the degree threshold by (default: this CSR's own).  gemm_overlaps: the caller can run
    an unfused projection GEMM on a second stream under other HBM-bound work (the sharded
    pass) — then low-degree CSRs, whose fused kernel is the MFMA one, stay unfused: the
    overlapped GEMM costs less than the MFMA kernel's extra time over the bare gather
    (C5 bought-by: 13.1 ms fused vs 7.6 ms gather + a 7.1 ms GEMM on the side stream)."""
    D = FUSED_D
    if not ((X.is_cuda or X.is_meta) and (H.is_cuda or H.is_meta) and X.dim() == 2
            and H.dim() == 2):
        return False
    if X.shape[1] != D or H.shape[1] != D or tuple(W_self.shape) != (D, D) or \
            tuple(W_neigh.shape) != (D, D):
        return False
    if X.dtype != torch.float32 or H.dtype != torch.float32:
        return False
    for t in (X, H):
        if t.stride(1) != 1 or t.stride(0) % 4:
            return False
        # 16-B aligned rows; torch.compile's fake tensors have no address (there the
        # library's own alignment check is what refuses a misaligned view, loudly)
        if not torch.compiler.is_compiling() and t.data_ptr() % 16:
            return False
    if split and split_plan(indptr, split) is not None:
        return False
    # below FUSED_MIN_DEG edges per row the VALU kernel's per-row weight reads bound it and
    # the MFMA variant takes the relation (C5 bought-by, 10 edges/row: VALU-fused 18.0 ms,
    # MFMA-fused 13.1 ms, spmm 7.6 + GEMM 7.1 ms back to back); GNNREC_FUSED_MFMA=0 keeps
    # aggregation + GEMM there
    if os.environ.get("GNNREC_FUSED_MFMA", "1") == "0" or gemm_overlaps:
        return fused_variant(indptr, avg_deg) == "valu"
    return True


def fused_preprojects(indptr, X, H, reduce: str, avg_deg: Optional[float] = None) -> bool:
    """A fused launch that can_spmm_project accepted runs the pre-projected form: the MFMA
    variant, a linear reduce and a source table at most half the destination count."""
    return fused_variant(indptr, avg_deg) == "mfma" and preproject_pays(
        X.shape[0], indptr.numel() - 1, reduce)


FUSED_MIN_DEG = 24


def fused_variant(indptr, avg_deg: Optional[float] = None) -> str:
    """'valu' (gnnrec_spmm_project_f32: weights in LDS, read once per 2 rows — bound by
    the gather from FUSED_MIN_DEG edges per row up) or 'mfma' (gnnrec_spmm_project_mfma_f32:
    32-row tiles through fp32 MFMA, weights read once per 32 rows — low degrees).  avg_deg:
    the edges per row to decide by (the sharded pass passes the GLOBAL average so every
    rank picks the same kernel); default this CSR's own (spmm_project's `variant` forces
    one)."""
    if avg_deg is None:
        n = indptr.numel() - 1
        avg_deg = _nnz(indptr) / n if n else float(FUSED_MIN_DEG)
    return "valu" if avg_deg >= FUSED_MIN_DEG else "mfma"


def _nnz(indptr: torch.Tensor) -> int:
    """indptr[-1] as a host int, read back once per CSR (cached on the tensor)."""
    v = getattr(indptr, "_gnnrec_nnz", None)
    if v is None:
        v = int(indptr[-1].item())
        try:
            indptr._gnnrec_nnz = v
        except AttributeError:  # pragma: no cover
            pass
    return v


def _wkey(W: torch.Tensor):
    return (W._version, W.data_ptr(), getattr(W, "_gnnrec_epoch", 0))


def invalidate_weight_cache(*modules_or_tensors) -> None:
    """Drop the transposed / packed weight copies the fused kernels keep on weight tensors.
    They are rebuilt when a weight's version counter moves (every in-place op through the
    autograd-visible tensor: optimizer steps, `with torch.no_grad(): W.copy_(...)`); a write
    through `W.data` (EMA or custom update code) does not move it — call this afterwards
    with the modules or tensors written."""
    for m in modules_or_tensors:
        ts = m.parameters() if isinstance(m, torch.nn.Module) else [m]
        for W in ts:
            try:
                W._gnnrec_epoch = getattr(W, "_gnnrec_epoch", 0) + 1
            except (AttributeError, RuntimeError):  # pragma: no cover
                pass


def _cached_on(W: torch.Tensor, attr: str, key, make):
    """A derived copy of weight W kept as W.<attr>, rebuilt when `key` changes.  Handed to
    another stream than the one that made it, the consumer first waits for its making and
    the copy is record_stream-ed there (so replacing it never frees memory a side-stream
    kernel is still reading)."""
    if torch.cuda.is_current_stream_capturing():
        # inside a captured step (gnnrec.capture): the copy is made by the graph on every
        # replay, after the captured optimizer step changed W — never a stale cached one
        return make()
    hit = getattr(W, attr, None)
    cur = torch.cuda.current_stream(W.device)
    if hit is None or hit[0] != key:
        ev = torch.cuda.Event()
        hit = (key, make(), ev, cur.cuda_stream)
        ev.record(cur)
        try:
            setattr(W, attr, hit)
        except (AttributeError, RuntimeError):  # pragma: no cover
            pass
    elif hit[3] != cur.cuda_stream:  # made on another stream: ordered after its copy
        cur.wait_event(hit[2])
        hit[1].record_stream(cur)
    return hit[1]


def _transposed(W: torch.Tensor) -> torch.Tensor:
    """Wᵀ (k-major, contiguous) of a fused kernel's weight, kept on the weight tensor and
    rebuilt only when the weight changes (its version counter, an optimizer step, or
    invalidate_weight_cache) — not a transpose-copy kernel per launch inside the pass (C4:
    two per layer before the fused launch, profiles/r02f_c4_timeline.txt)."""
    if torch.compiler.is_compiling() or not W.is_cuda:
        return W.detach().t().contiguous()
    return _cached_on(W, "_gnnrec_wt", _wkey(W), lambda: W.detach().t().contiguous())


def _packed4(Ws_a, Wn_a, Ws_b, Wn_b) -> torch.Tensor:
    """[W_self,aᵀ | W_neigh,aᵀ | W_self,bᵀ | W_neigh,bᵀ] as one contiguous [4, d, d] k-major
    array (gnnrec_spmm_pair_f32's WT4), cached on W_self,a like _transposed."""
    Ws = (Ws_a, Wn_a, Ws_b, Wn_b)

    def make():
        return torch.stack([W.detach().t() for W in Ws]).contiguous()

    if torch.compiler.is_compiling() or not Ws_a.is_cuda:
        return make()
    return _cached_on(Ws_a, "_gnnrec_wt4", tuple(_wkey(W) for W in Ws), make)


def spmm_project(indptr, indices, X, H, W_self, W_neigh, reduce: str = "mean",
                 edge_weight: Optional[torch.Tensor] = None, relu: bool = True,
                 l2norm: bool = False, accum: str = "store", out_div: float = 0.0,
                 out: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
                 bias_nonempty: Optional[torch.Tensor] = None,
                 attn_vec: Optional[torch.Tensor] = None,
                 attn_state: Optional[torch.Tensor] = None,
                 avg_deg: Optional[float] = None, variant: Optional[str] = None) -> torch.Tensor:
    """a1+a3 fused: out (accum)= epi(H W_selfᵀ + reduce_e X[src_e] W_neighᵀ + bias
    + [deg > 0]·bias_nonempty), d = 128.  variant 'valu' | 'mfma' (default: fused_variant
    of avg_deg) picks the kernel; both give the same aggregate bits, the projection's
    fp32 summation order differs.

    W_neigh None: X holds pre-projected source rows (preproject(X, W_neigh)) and the
    neighbour term is reduce_e X[src_e] itself (sum / mean only; the mfma kernel, which
    then runs only the self half on the MFMA).  The same value up to fp32 rounding: the
    projection is applied before the (linear) reduction instead of after it."""
    _dev(indptr, "indptr", torch.int64)
    _dev(indices, "indices", torch.int32)
    _dev(X, "X", torch.float32)
    _dev(H, "H", torch.float32)
    n_dst = indptr.numel() - 1
    if H.shape[0] < n_dst:
        raise ValueError(f"H has {H.shape[0]} rows, the CSR {n_dst} destinations")
    if edge_weight is not None:
        _dev(edge_weight, "edge_weight", torch.float32)
        edge_weight = edge_weight.contiguous()
    D = FUSED_D
    if out is None:
        if accum not in ("store", "attn_first"):
            raise ValueError("accumulating spmm_project needs an out tensor")
        out = torch.empty((n_dst, D), dtype=torch.float32, device=X.device)
    else:
        _dev(out, "out", torch.float32)
        if tuple(out.shape) != (n_dst, D):
            raise ValueError(f"out must be [{n_dst}, {D}], got {tuple(out.shape)}")
    if tuple(W_self.shape) != (D, D) or (W_neigh is not None
                                         and tuple(W_neigh.shape) != (D, D)):
        raise ValueError(f"spmm_project needs {D}x{D} weights")
    if W_neigh is None:
        if reduce not in ("sum", "mean"):
            raise ValueError("pre-projected source rows (W_neigh None) need reduce sum or mean")
        if variant not in (None, "mfma"):
            raise ValueError("pre-projected source rows (W_neigh None) run on the mfma kernel")
        variant = "mfma"
    WsT = _transposed(W_self)
    WnT = None if W_neigh is None else _transposed(W_neigh)
    for t, name in ((bias, "bias"), (bias_nonempty, "bias_nonempty")):
        if t is not None:
            _dev(t, name, torch.float32)
            if t.numel() != D:
                raise ValueError(f"{name} must have {D} entries")
    bias = None if bias is None else bias.detach().contiguous()
    bias_nonempty = None if bias_nonempty is None else bias_nonempty.detach().contiguous()
    av, ast = _attn_args(accum, attn_vec, attn_state, n_dst, D)
    epi = (_lib.EPI_RELU if relu else 0) | (_lib.EPI_L2NORM if l2norm else 0)
    variant = variant or fused_variant(indptr, avg_deg)
    if variant not in ("valu", "mfma"):
        raise ValueError(f"spmm_project variant must be 'valu' or 'mfma', not {variant!r}")
    _rowmajor(X, "X")
    _rowmajor(H, "H")
    _rowmajor(out, "out")
    _T().spmm_project(indptr, indices, edge_weight, X, H, WsT, WnT, bias, bias_nonempty,
                      REDUCE[reduce], epi, ACCUM[accum], float(out_div), av, ast,
                      variant == "mfma", out)
    return out


def spmm_project2(rel_a, rel_b, H, W_self_a, W_self_b, bias_a=None, bias_b=None, *,
                  relu: bool = True, l2norm: bool = False, combine: str = "add",
                  out_div: float = 0.0, out: Optional[torch.Tensor] = None,
                  attn_vec: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Two pre-projected relations into one destination type in one launch
    (gnnrec_spmm_project2_f32): out = combine(epi(H W_self_aᵀ + agg_a + bias_a
    [+ bias_nonempty_a]), epi(... b ...)) / out_div.  rel_r = (indptr, indices, Y,
    reduce, edge_weight, bias_nonempty) with Y = preproject(X_r, W_neigh_r); reduce sum
    or mean; combine 'add' (HeteroGraphConv sum, mean with out_div=2), 'max', or
    'attention' with attn_vec [d] (softmax over the two relations of attn_vec·y_r)."""
    D = FUSED_D
    args = []
    n_dst = rel_a[0].numel() - 1
    # the relation with at most half the other's edges (host counts only: no readback) reads
    # its source rows non-temporally, leaving the Infinity Cache to the busier table
    # (GNNREC_SRC_STREAM; C5: bought-by's 100M edges beside clicked-by's 400M)
    ea, eb = (getattr(r[0], "_gnnrec_nnz", None) for r in (rel_a, rel_b))
    stream = None
    if ea is not None and eb is not None and rel_a[4] is None and rel_b[4] is None:
        stream = "b" if 2 * eb <= ea else "a" if 2 * ea <= eb else None
    for name, (indptr, indices, Y, reduce, ew, bne) in (("a", rel_a), ("b", rel_b)):
        _dev(indptr, f"indptr_{name}", torch.int64)
        _dev(indices, f"indices_{name}", torch.int32)
        _dev(Y, f"Y{name}", torch.float32)
        _rowmajor(Y, f"Y{name}")
        if reduce not in ("sum", "mean"):
            raise ValueError("spmm_project2: pre-projected relations reduce by sum or mean")
        if indptr.numel() - 1 != n_dst:
            raise ValueError("spmm_project2: the relations' row counts differ")
        if ew is not None:
            _dev(ew, f"ew_{name}", torch.float32)
            ew = ew.contiguous()
        if bne is not None:
            _dev(bne, f"bias_nonempty_{name}", torch.float32)
            bne = bne.detach().contiguous()
        args += [indptr, indices, ew, Y,
                 REDUCE[reduce] | (_lib.SRC_STREAM if stream == name else 0), bne]
    _dev(H, "H", torch.float32)
    _rowmajor(H, "H")
    if combine not in ("add", "max", "attention"):
        raise ValueError(f"spmm_project2: combine must be 'add', 'max' or 'attention', "
                         f"not {combine!r}")
    if (combine == "attention") != (attn_vec is not None):
        raise ValueError("spmm_project2: attn_vec goes with combine='attention'")
    if attn_vec is not None:
        _dev(attn_vec, "attn_vec", torch.float32)
        if attn_vec.numel() != D:
            raise ValueError(f"attn_vec must have {D} entries")
        attn_vec = attn_vec.detach().contiguous()
    for W in (W_self_a, W_self_b):
        if tuple(W.shape) != (D, D):
            raise ValueError(f"spmm_project2 needs {D}x{D} weights")
    if out is None:
        out = torch.empty((n_dst, D), dtype=torch.float32, device=H.device)
    else:
        _dev(out, "out", torch.float32)
        _rowmajor(out, "out")
    bias_a = None if bias_a is None else bias_a.detach().contiguous()
    bias_b = None if bias_b is None else bias_b.detach().contiguous()
    epi = (_lib.EPI_RELU if relu else 0) | (_lib.EPI_L2NORM if l2norm else 0)
    _T().spmm_project2(*args, H, _transposed(W_self_a), _transposed(W_self_b), bias_a, bias_b,
                       epi,
                       ACCUM["attn_last" if combine == "attention" else combine], attn_vec,
                       float(out_div), out)
    return out


def spmm_pair(rel_a, rel_b, X, H, W_self_a, W_neigh_a, W_self_b, W_neigh_b, bias_a=None,
              bias_b=None, *, relu: bool = True, l2norm: bool = False, combine: str = "add",
              out_div: float = 0.0, out: Optional[torch.Tensor] = None,
              attn_vec: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Two relations gathering from ONE source table X into one destination type, all four
    projections in the launch (gnnrec_spmm_pair_f32, MFMA epilogue): out = combine(
    epi(H W_self_aᵀ + agg_a W_neigh_aᵀ + bias_a [+ bias_nonempty_a]), epi(... b ...)) /
    out_div.  rel_r = (indptr, indices, reduce, edge_weight, bias_nonempty), reduce sum or
    mean; combine as spmm_project2.  Unlike spmm_project2 nothing is pre-projected: the
    gathered working set is X alone; the projections run on the fp32 MFMA."""
    D = FUSED_D
    n_dst = rel_a[0].numel() - 1
    args = []
    for name, (indptr, indices, reduce, ew, bne), b in (("a", rel_a, bias_a), ("b", rel_b, bias_b)):
        _dev(indptr, f"indptr_{name}", torch.int64)
        _dev(indices, f"indices_{name}", torch.int32)
        if reduce not in ("sum", "mean"):
            raise ValueError("spmm_pair: both relations reduce by sum or mean")
        if indptr.numel() - 1 != n_dst:
            raise ValueError("spmm_pair: the relations' row counts differ")
        if ew is not None:
            _dev(ew, f"ew_{name}", torch.float32)
            ew = ew.contiguous()
        if bne is not None:
            _dev(bne, f"bias_nonempty_{name}", torch.float32)
            bne = bne.detach().contiguous()
        if b is not None:
            b = b.detach().contiguous()
        args += [indptr, indices, ew, REDUCE[reduce], b, bne]
    _dev(X, "X", torch.float32)
    _rowmajor(X, "X")
    _dev(H, "H", torch.float32)
    _rowmajor(H, "H")
    if X.shape[1] != D or H.shape[1] != D:
        raise ValueError(f"spmm_pair needs d = {D}")
    if combine not in ("add", "max", "attention"):
        raise ValueError(f"spmm_pair: combine must be 'add', 'max' or 'attention', "
                         f"not {combine!r}")
    if (combine == "attention") != (attn_vec is not None):
        raise ValueError("spmm_pair: attn_vec goes with combine='attention'")
    if attn_vec is not None:
        _dev(attn_vec, "attn_vec", torch.float32)
        if attn_vec.numel() != D:
            raise ValueError(f"attn_vec must have {D} entries")
        attn_vec = attn_vec.detach().contiguous()
    for W in (W_self_a, W_neigh_a, W_self_b, W_neigh_b):
        if tuple(W.shape) != (D, D):
            raise ValueError(f"spmm_pair needs {D}x{D} weights")
    if out is None:
        out = torch.empty((n_dst, D), dtype=torch.float32, device=H.device)
    else:
        _dev(out, "out", torch.float32)
        _rowmajor(out, "out")
    epi = (_lib.EPI_RELU if relu else 0) | (_lib.EPI_L2NORM if l2norm else 0)
    WT4 = _packed4(W_self_a, W_neigh_a, W_self_b, W_neigh_b)
    _T().spmm_pair(*args, X, H, WT4, epi,
                   ACCUM["attn_last" if combine == "attention" else combine], attn_vec,
                   float(out_div), out)
    return out


def preproject_pays(n_src: int, n_dst: int, reduce: str) -> bool:
    """Project a low-degree relation's source rows ahead of the reduction (spmm_project
    with W_neigh=None) when the reduction is linear and the source type has at most half
    as many rows as the destination: the MFMA then runs the self half only (C5 bought-by,
    1M items -> 10M users: fused 13.0 -> 10.6 ms + 0.38 ms for the 1M-row projection)."""
    return reduce in ("sum", "mean") and 2 * n_src <= n_dst


def preproject(X: torch.Tensor, W_neigh: torch.Tensor,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Y = X W_neighᵀ: a relation's source rows projected ahead of its (linear) reduction,
    for spmm_project(..., W_neigh=None).  Worth it where the source type has fewer rows
    than the destination (C5 item -> user: 1M projected rows instead of 10M aggregates)."""
    return gemm(X, W_neigh, out=out)


def gemm_tn(A: torch.Tensor, B: torch.Tensor, out: Optional[torch.Tensor] = None,
            accumulate: bool = False, colsum: Optional[torch.Tensor] = None,
            row_ptr: Optional[torch.Tensor] = None) -> torch.Tensor:
    """f2 weight gradient: out [M,N] (+)= Aᵀ B for A [K,M], B [K,N] (dW = dYᵀ X); with
    colsum [M], also colsum (+)= Σ_k A[k] (the bias gradient) from the same pass — over the
    rows k with row_ptr[k+1] > row_ptr[k] only when row_ptr (an int64 [K+1] indptr) is given.

    Deterministic split-K MFMA (gnnrec_gemm_tn_bias_rows_f32)."""
    T = _T()
    _dev(A, "A", torch.float32)
    _dev(B, "B", torch.float32)
    K, M = A.shape
    if B.shape[0] != K:
        raise ValueError(f"gemm_tn: A {tuple(A.shape)} and B {tuple(B.shape)} differ in K")
    N = B.shape[1]
    _rowmajor(A, "A")
    _rowmajor(B, "B")
    if out is None:
        if accumulate:
            raise ValueError("accumulating gemm_tn needs an out tensor")
        out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    else:
        _dev(out, "out", torch.float32)
        if tuple(out.shape) != (M, N):
            raise ValueError(f"out must be [{M}, {N}]")
    if colsum is not None:
        _dev(colsum, "colsum", torch.float32)
        if colsum.numel() != M or not colsum.is_contiguous():
            raise ValueError(f"colsum must be a contiguous [{M}] tensor")
    _rowmajor(out, "out")
    nbytes = T.gemm_tn_workspace_bytes(K, M, N)
    ws = torch.empty(max(1, nbytes // 4), dtype=torch.float32, device=A.device)
    if row_ptr is not None:
        _dev(row_ptr, "row_ptr", torch.int64)
        if colsum is None or row_ptr.numel() != K + 1:
            raise ValueError(f"row_ptr must be a [{K + 1}] indptr beside colsum")
        row_ptr = row_ptr.contiguous()
    T.gemm_tn(A, B, colsum, bool(accumulate), out, ws, row_ptr)
    return out


def act_backward_normed(z: torch.Tensor, row_norm: torch.Tensor, gz: torch.Tensor,
                        relu: bool = True) -> torch.Tensor:
    """f2: gradient through relu?+L2 norm from the normalised output z and the row norms
    gemm(..., l2norm=True, row_norm=...) wrote (gnnrec_act_backward_normed_f32)."""
    _dev(z, "z", torch.float32)
    _dev(gz, "gz", torch.float32)
    _dev(row_norm, "row_norm", torch.float32)
    n, d = z.shape
    if tuple(gz.shape) != (n, d) or row_norm.numel() != n:
        raise ValueError("act_backward_normed: shape mismatch")
    gu = torch.empty((n, d), dtype=torch.float32, device=z.device)
    _T().act_backward_normed(z, row_norm.contiguous(), gz, bool(relu), gu)
    return gu


def act_backward(u: torch.Tensor, gz: torch.Tensor, relu: bool, l2norm: bool,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """f2: gradient through z = norm?(relu?(u)) (zero-guarded row norm) for pre-activation u."""
    _dev(u, "u", torch.float32)
    _dev(gz, "gz", torch.float32)
    if gz.shape != u.shape:
        raise ValueError("act_backward: u and gz shapes differ")
    n, d = u.shape
    gz = gz.contiguous()
    if out is None:
        out = torch.empty_like(u)
    flags = (_lib.EPI_RELU if relu else 0) | (_lib.EPI_L2NORM if l2norm else 0)
    _T().act_backward(u, gz, flags, out)
    return out


class LstmPlan:
    """Degree-descending visiting order of a CSR's rows and the running-row count of
    every step (one host readback of the degree histogram, cached on the indptr)."""

    def __init__(self, indptr: torch.Tensor):
        deg = indptr[1:] - indptr[:-1]
        self.order = torch.argsort(deg, descending=True, stable=True)
        hist = torch.bincount(deg, minlength=1).tolist()
        n = indptr.numel() - 1
        running, steps = n - hist[0], []
        for t in range(len(hist) - 1):
            steps.append(running)
            running -= hist[t + 1]
        self.n_active = steps  # n_active[t] = #rows with in-degree > t
        self.n_rows = steps[0] if steps else 0

    @classmethod
    def of(cls, indptr):
        p = getattr(indptr, "_gnnrec_lstm_plan", None)
        if p is None:
            p = cls(indptr)
            indptr._gnnrec_lstm_plan = p
        return p


def lstm_aggregate(indptr, indices, X, W_ih, W_hh, b_ih, b_hh,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """f4: per destination, nn.LSTM over its in-neighbour rows of X in CSR (edge) order ->
    final hidden state [n_dst, d]; 0 for zero in-degree (ConvLayer._lstm_reducer)."""
    T = _T()
    _dev(indptr, "indptr", torch.int64)
    _dev(indices, "indices", torch.int32)
    d = W_hh.shape[1]
    n_dst = indptr.numel() - 1
    plan = LstmPlan.of(indptr)
    P = gemm(X.contiguous(), W_ih.detach(), bias=(b_ih + b_hh).detach())  # [N_src, 4d]
    if out is None:
        out = torch.zeros((n_dst, d), dtype=torch.float32, device=X.device)
    else:
        out.zero_()
    if plan.n_rows == 0:
        return out
    h = [torch.zeros((plan.n_rows, d), dtype=torch.float32, device=X.device),
         torch.empty((plan.n_rows, d), dtype=torch.float32, device=X.device)]
    c = torch.zeros((plan.n_rows, d), dtype=torch.float32, device=X.device)
    WT = W_hh.detach().t().contiguous()
    for t, n_act in enumerate(plan.n_active):
        T.lstm_step(P, indptr, indices, plan.order, t, n_act, h[t % 2], h[(t + 1) % 2], c, WT,
                    out)
    return out


def lstm_aggregate_train(indptr, indices, X, W_ih, W_hh, b_ih, b_hh):
    """lstm_aggregate keeping what the backward needs: every step's hidden and cell rows and
    pre-activation gates in a step-major packing (step t: rows order[0..n_t) at slots
    [off[t], off[t] + n_t)).  -> (out [n_dst, d], state for lstm_aggregate_backward)."""
    T = _T()
    _dev(indptr, "indptr", torch.int64)
    _dev(indices, "indices", torch.int32)
    d = W_hh.shape[1]
    n_dst = indptr.numel() - 1
    plan = LstmPlan.of(indptr)
    dev = X.device
    P = gemm(X.contiguous(), W_ih.detach(), bias=(b_ih + b_hh).detach())  # [N_src, 4d]
    out = torch.zeros((n_dst, d), dtype=torch.float32, device=dev)
    steps = plan.n_active
    off = [0]
    for n in steps:
        off.append(off[-1] + n)
    n_slots = off[-1]
    H = torch.empty((n_slots, d), dtype=torch.float32, device=dev)
    C = torch.empty((n_slots, d), dtype=torch.float32, device=dev)
    Z = torch.empty((n_slots, 4 * d), dtype=torch.float32, device=dev)
    WT = W_hh.detach().t().contiguous()
    h0 = torch.zeros((plan.n_rows, d), dtype=torch.float32, device=dev)
    for t, n in enumerate(steps):
        o, q = off[t], (off[t - 1] if t else 0)
        T.lstm_step_save(P, indptr, indices, plan.order, t, n, h0[:n] if t == 0 else H[q:q + n],
                         H[o:o + n], None if t == 0 else C[q:q + n], C[o:o + n], Z[o:o + n], WT,
                         out)
    return out, (plan, off, H, C, Z, WT)


def lstm_aggregate_backward(indptr, indices, X, W_ih, state, g, need_x: bool = True):
    """Backward through time of lstm_aggregate_train on the HIP kernels: per step (t
    descending) the gate Jacobian (gnnrec_lstm_backward_step_f32) and dh_{t-1} = dz·W_hh (a
    GEMM); then dW_hh = Σ_t dz_tᵀ h_{t-1} (one split-K GEMM over the slots, h_{t-1} rows
    gathered to the slots' order), dP = dz summed per source row (the slots' CSR by source,
    one spmm), dX = dP·W_ih, dW_ih = dPᵀ X and db = Σ dP (the same split-K pass).
    -> (dX or None, dW_ih, dW_hh, db)."""
    T = _T()
    plan, off, H, C, Z, WT = state
    steps = plan.n_active
    d = WT.shape[0]
    dev = Z.device
    n_slots = off[-1]
    n_src = X.shape[0]
    if n_slots == 0:
        z = torch.zeros
        return (z(X.shape, device=dev) if need_x else None, z(W_ih.shape, device=dev),
                z((4 * d, d), device=dev), z(4 * d, device=dev))
    g = g.contiguous()
    dZ = torch.empty((n_slots, 4 * d), dtype=torch.float32, device=dev)
    dc = [torch.empty((plan.n_rows, d), dtype=torch.float32, device=dev) for _ in range(2)]
    dh_next = dc_next = None
    n_next = 0
    for t in reversed(range(len(steps))):
        n, o = steps[t], off[t]
        q = off[t - 1] if t else 0
        dcp = dc[t % 2][:n]
        T.lstm_backward_step(Z[o:o + n], C[o:o + n], C[q:q + n] if t else None, dh_next,
                             dc_next, n_next, g, plan.order, n, dZ[o:o + n], dcp)
        if t:
            dh_next = gemm(dZ[o:o + n], WT)  # dz · W_hh
            dc_next, n_next = dcp, n
    src = torch.empty(n_slots, dtype=torch.int64, device=dev)
    prev = torch.empty(n_slots, dtype=torch.int64, device=dev)
    T.lstm_slots(indptr, indices, plan.order,
                 torch.tensor(off[:-1], dtype=torch.int64, device=dev), n_slots, src, prev)
    if len(steps) > 1:
        dW_hh = gemm_tn(dZ[off[1]:], gather_rows(H, prev[off[1]:]))
    else:
        dW_hh = torch.zeros((4 * d, d), dtype=torch.float32, device=dev)
    slots = torch.arange(n_slots, dtype=torch.int64, device=dev)
    ip, ix, _ = csr_build(slots, src, n_src)
    dP = spmm(ip, ix, dZ, "sum")
    db = torch.empty(4 * d, dtype=torch.float32, device=dev)
    dW_ih = gemm_tn(dP, X.detach().contiguous(), colsum=db)
    dX = gemm(dP, W_ih.detach().t().contiguous()) if need_x else None
    return dX, dW_ih, dW_hh, db


def gather_rows(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """a10: src[idx] along dim 0 for a device tensor of any dtype whose rows are contiguous
    (node features into blocks[0].srcdata, edge data into blocks)."""
    _dev(idx, "idx", torch.int64)
    if not (src.is_cuda or src.is_meta):
        raise ValueError("src: expected a device tensor (there is no CPU path)")
    if src.dim() == 0:
        raise ValueError("src: expected at least one dimension")
    row = src[0] if src.shape[0] else src.new_empty(src.shape[1:])
    if not (row.is_contiguous() and (src.dim() == 1 or src.stride(0) >= row.numel())):
        src = src.contiguous()
    out = torch.empty((idx.numel(),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    _T().gather_rows(src, idx.contiguous(), out)
    return out


def sddmm_cos(src: torch.Tensor, dst: torch.Tensor, Hs: torch.Tensor,
              Hd: torch.Tensor) -> torch.Tensor:
    """a7: cosine of the L2-normalised endpoint rows, one value per edge -> [E]."""
    _dev(src, "src", torch.int64)
    _dev(dst, "dst", torch.int64)
    _dev(Hs, "Hs", torch.float32)
    _dev(Hd, "Hd", torch.float32)
    E = src.numel()
    if dst.numel() != E:
        raise ValueError("src/dst length mismatch")
    if Hs.shape[1] != Hd.shape[1]:
        raise ValueError("endpoint feature sizes differ")
    out = torch.empty(E, dtype=torch.float32, device=Hs.device)
    _rowmajor(Hs, "Hs")
    _rowmajor(Hd, "Hd")
    _T().sddmm_cos(src.contiguous(), dst.contiguous(), Hs, Hd, out)
    return out


def cos_grouped_ok(Hs: torch.Tensor, Hd: torch.Tensor) -> bool:
    """Can gnnrec_sddmm_cos_grouped_f32 score these tables (d % 4 == 0, d <= 256, 16-B rows)?"""
    d = Hs.shape[1]
    return (Hs.is_cuda and d % 4 == 0 and d <= 256 and Hs.dim() == 2 and Hd.dim() == 2 and
            Hs.stride(1) == 1 and Hd.stride(1) == 1 and Hs.stride(0) % 4 == 0 and
            Hd.stride(0) % 4 == 0 and Hs.data_ptr() % 16 == 0 and Hd.data_ptr() % 16 == 0)


def sddmm_cos_grouped(src_g: torch.Tensor, first: Optional[torch.Tensor], K: int,
                      dst: torch.Tensor, Hs: torch.Tensor, Hd: torch.Tensor):
    """a7 for the pair graphs of negative_sampler.Uniform(K): group g's positive edge
    (src_g[g], first[g]) and its K negatives (src_g[g], dst[g K + j]) -> (positive scores [G]
    (None without `first`), negative scores [G K]); bitwise sddmm_cos of the expanded lists."""
    for t, n in ((src_g, "src_g"), (dst, "dst")):
        _dev(t, n, torch.int64)
    if first is not None:
        _dev(first, "first", torch.int64)
    _dev(Hs, "Hs", torch.float32)
    _dev(Hd, "Hd", torch.float32)
    G = src_g.numel()
    out_first = torch.empty(G if first is not None else 0, dtype=torch.float32, device=Hs.device)
    out = torch.empty(G * int(K), dtype=torch.float32, device=Hs.device)
    _T().sddmm_cos_grouped(src_g.contiguous(), None if first is None else first.contiguous(),
                           int(K), dst.contiguous(), Hs, Hd, out_first, out)
    return (out_first if first is not None else None), out


def sddmm_cos_backward(src: torch.Tensor, dst: torch.Tensor, Hs: torch.Tensor, Hd: torch.Tensor,
                       grad: torch.Tensor, need_src: bool = True, need_dst: bool = True,
                       groups: int = 0, K: int = 0):
    """f2: gradients of sddmm_cos w.r.t. Hs and Hd given dL/dcos [E] -> (gHs|None, gHd|None),
    one library call (key sort, planned weighted gather, normalisation Jacobian).
    groups > 0: the edges are [groups positives | groups x K negatives] with each negative's
    source its positive's (negative_sampler.Uniform): the source side sorts only the group
    keys (gnnrec_sddmm_cos_backward_grouped_f32), and src may be the positives' sources
    alone (groups entries; the only ones read)."""
    T = _T()
    _dev(src, "src", torch.int64)
    _dev(dst, "dst", torch.int64)
    _dev(Hs, "Hs", torch.float32)
    _dev(Hd, "Hd", torch.float32)
    _dev(grad, "grad", torch.float32)
    E, d = dst.numel(), Hs.shape[1]
    if not (src.numel() == E or (groups and src.numel() == groups)) or grad.numel() != E:
        raise ValueError("sddmm_cos_backward: src/dst/grad length mismatch")
    if Hd.shape[1] != d:
        raise ValueError("endpoint feature sizes differ")
    n_s, n_d = Hs.shape[0], Hd.shape[0]
    gHs = torch.empty((n_s, d), dtype=torch.float32, device=Hs.device) if need_src else None
    gHd = torch.empty((n_d, d), dtype=torch.float32, device=Hs.device) if need_dst else None
    if groups and not (groups * (K + 1) == E and d % 4 == 0 and d <= 256 and
                       Hs.stride(0) % 4 == 0 and Hd.stride(0) % 4 == 0 and
                       Hs.data_ptr() % 16 == 0 and Hd.data_ptr() % 16 == 0):
        if groups and src.numel() == groups and groups * (K + 1) == E:
            src = torch.cat([src, src.repeat_interleave(K)])  # the per-edge form's full list
        groups = K = 0  # the layout or the rows do not fit the grouped form
    nbytes = int(T.sddmm_cos_backward_workspace_bytes(E, n_s, n_d, d, groups, K))
    ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=Hs.device)
    T.sddmm_cos_backward(src.contiguous(), dst.contiguous(), Hs, Hd, grad.contiguous(), gHs, gHd,
                         ws, groups, K)
    return gHs, gHd


def margin_loss(parts, delta: float, flat: bool = False):
    """f2: max_margin_loss forward + unscaled gradients for a list of etype parts
    [(pos [E], neg [E*K], K, mask|None, recency|None)] -> (loss 0-d tensor, N_total,
    [(g_pos, g_neg)]).  Gradients are d(sum of scores)/d(score); the loss is the mean.
    They are views of one buffer, in part order (pos_0, neg_0, pos_1, ...); flat: that
    buffer is returned as well."""
    T = _T()
    dev = parts[0][0].device
    # an etype without positive edges (the pair graphs' other etypes) adds nothing: no
    # launch and no partial for it, unless every etype is empty (the NaN mean below)
    skip = any(p[0].numel() for p in parts)
    blocks = [0 if skip and p[0].numel() == 0 else int(T.margin_loss_blocks(p[0].numel()))
              for p in parts]
    partial = torch.empty(sum(blocks), dtype=torch.float32, device=dev)
    gflat = torch.empty(sum(p[0].numel() + p[1].numel() for p in parts), dtype=torch.float32,
                        device=dev)
    grads, off, total, goff = [], 0, 0, 0
    for (pos, neg, K, mask, rec), nb in zip(parts, blocks):
        _dev(pos, "pos_score", torch.float32)
        _dev(neg, "neg_score", torch.float32)
        n_pos = pos.numel()
        if neg.numel() != n_pos * K:
            raise RuntimeError(f"shape '[-1, {K}]' is invalid for input of size {neg.numel()}")
        if mask is not None:
            mask = mask.to(device=dev, dtype=torch.float32).contiguous()
            if mask.numel() != neg.numel():
                raise ValueError("negative_mask must have one value per negative score")
        if rec is not None:
            rec = rec.to(dev).reshape(-1)
            if rec.dtype not in (torch.int64, torch.float32):
                rec = rec.float()
            rec = rec.contiguous()
            if rec.numel() != n_pos:
                raise ValueError("recency must have one value per positive edge")
        g_pos = gflat.narrow(0, goff, n_pos).view(pos.shape)
        g_neg = gflat.narrow(0, goff + n_pos, neg.numel()).view(neg.shape)
        goff += n_pos + neg.numel()
        if nb == 0:
            grads.append((g_pos, g_neg))
            continue
        T.margin_loss(pos.contiguous(), neg.contiguous(), K, float(delta), mask, rec, g_pos,
                      g_neg, partial[off:off + nb])
        grads.append((g_pos, g_neg))
        off += nb
        total += neg.numel()
    loss = torch.empty((), dtype=torch.float32, device=dev)
    T.sum_scaled(partial, 1.0 / total if total else float('nan'), loss)
    return (loss, total, grads, gflat) if flat else (loss, total, grads)


def edge_mlp(src: torch.Tensor, dst: torch.Tensor, P: torch.Tensor, Q: torch.Tensor,
             W2: torch.Tensor, b2: torch.Tensor, w3: torch.Tensor, b3: torch.Tensor) -> torch.Tensor:
    """a8 tail: sigmoid(w3·relu(W2·relu(P[src]+Q[dst]) + b2) + b3) -> [E]."""
    for t, n in ((P, "P"), (Q, "Q"), (W2, "W2"), (b2, "b2"), (w3, "w3"), (b3, "b3")):
        _dev(t, n, torch.float32)
    _dev(src, "src", torch.int64)
    _dev(dst, "dst", torch.int64)
    if P.shape[1] != 128 or Q.shape[1] != 128 or tuple(W2.shape) != (32, 128):
        raise ValueError("edge_mlp expects the reference's 128/32 hidden sizes")
    P, Q, W2 = P.contiguous(), Q.contiguous(), W2.detach().contiguous()
    E = src.numel()
    out = torch.empty(E, dtype=torch.float32, device=P.device)
    _T().edge_mlp(src.contiguous(), dst.contiguous(), P, Q, W2, b2.detach().contiguous(),
                  w3.detach().contiguous(), b3.detach().contiguous(), out)
    return out


def edge_mlp_grouped(src_g: torch.Tensor, first: Optional[torch.Tensor], K: int,
                     dst: torch.Tensor, P: torch.Tensor, Q: torch.Tensor, W2: torch.Tensor,
                     b2: torch.Tensor, w3: torch.Tensor, b3: torch.Tensor):
    """a8 tail for the pair graphs of negative_sampler.Uniform(K), grouped as
    sddmm_cos_grouped: group g's positive edge (src_g[g], first[g]) and its K negatives
    (src_g[g], dst[g K + j]) -> (positive scores [G] (None without `first`), negative scores
    [G K]); edge_mlp's scores of the expanded lists."""
    for t, n in ((P, "P"), (Q, "Q"), (W2, "W2"), (b2, "b2"), (w3, "w3"), (b3, "b3")):
        _dev(t, n, torch.float32)
    for t, n in ((src_g, "src_g"), (dst, "dst")):
        _dev(t, n, torch.int64)
    if first is not None:
        _dev(first, "first", torch.int64)
    if P.shape[1] != 128 or Q.shape[1] != 128 or tuple(W2.shape) != (32, 128):
        raise ValueError("edge_mlp expects the reference's 128/32 hidden sizes")
    P, Q, W2 = P.contiguous(), Q.contiguous(), W2.detach().contiguous()
    G = src_g.numel()
    out_first = torch.empty(G if first is not None else 0, dtype=torch.float32, device=P.device)
    out = torch.empty(G * int(K), dtype=torch.float32, device=P.device)
    _T().edge_mlp_grouped(src_g.contiguous(), None if first is None else first.contiguous(),
                          int(K), dst.contiguous(), P, Q, W2, b2.detach().contiguous(),
                          w3.detach().contiguous(), b3.detach().contiguous(), out_first, out)
    return (out_first if first is not None else None), out


def synth_edges(seed: int, e0: int, n: int, n_u: int, n_i: int, device,
                zipf_cdf: Optional[torch.Tensor] = None):
    """Counter-hash bipartite edges [e0, e0+n) -> (u int32 [n], i int32 [n])."""
    u = torch.empty(n, dtype=torch.int32, device=device)
    i = torch.empty(n, dtype=torch.int32, device=device)
    if zipf_cdf is not None:
        _dev(zipf_cdf, "zipf_cdf", torch.float64)
    _T().synth_edges(_lib.i64(seed), e0, n_u, n_i, zipf_cdf, u, i)
    return u, i


def exclusive_scan(x: torch.Tensor) -> torch.Tensor:
    """[n] int32/int64 -> [n+1] int64 exclusive prefix sums (last = total)."""
    T = _T()
    _dev(x, "x")
    if x.dtype not in (torch.int64, torch.int32):
        raise ValueError("exclusive_scan supports int32/int64")
    n = x.numel()
    out = torch.empty(n + 1, dtype=torch.int64, device=x.device)
    ws = torch.empty(max(1, (T.scan_workspace_bytes(n) + 7) // 8), dtype=torch.int64,
                     device=x.device)
    T.exclusive_scan(x.contiguous(), out, ws)
    return out


def sample_count(indptr, eids, seeds, fanout: int, seed_key: int = 0,
                 excluded: Optional[torch.Tensor] = None,
                 excluded_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a9 phase 1: per-seed sampled in-edge counts -> out_indptr [n_seeds+1] (device).
    excluded_rows (uint8 per dst node, optional): nonzero exactly on the dst nodes of the
    excluded eids — the other seeds skip the eid checks (same counts)."""
    for t, n in ((indptr, "indptr"), (eids, "eids"), (seeds, "seeds")):
        _dev(t, n, torch.int64)
    for t, n in ((excluded, "excluded"), (excluded_rows, "excluded_rows")):
        if t is not None:
            _dev(t, n, torch.uint8)
    n = seeds.numel()
    fan = -1 if fanout is None or fanout < 0 else int(fanout)
    counts = torch.empty(n, dtype=torch.int64, device=seeds.device)
    _T().sample_count(indptr, eids, excluded, seeds, fan, _lib.i64(seed_key), counts,
                      excluded_rows)
    return exclusive_scan(counts)


def sample_fill(indptr, indices, eids, seeds, fanout: int, seed_key: int, out_indptr,
                total: int, excluded: Optional[torch.Tensor] = None,
                excluded_rows: Optional[torch.Tensor] = None):
    """a9 phase 2: copy the sampled edges at out_indptr offsets -> (src ids, eids).

    indices: the CSR's int32 source ids (graph.in_csr); outputs are int64."""
    _dev(indices, "indices", torch.int32)
    n = seeds.numel()
    fan = -1 if fanout is None or fanout < 0 else int(fanout)
    out_src = torch.empty(total, dtype=torch.int64, device=seeds.device)
    out_eid = torch.empty(total, dtype=torch.int64, device=seeds.device)
    _T().sample_fill(indptr, indices, eids, excluded, seeds, fan, _lib.i64(seed_key), out_indptr,
                     out_src, out_eid, excluded_rows)
    return out_src, out_eid


def sample_neighbors(indptr, indices, eids, seeds, fanout: int, seed_key: int = 0,
                     excluded: Optional[torch.Tensor] = None,
                     excluded_rows: Optional[torch.Tensor] = None):
    """a9: in-edges of `seeds` (all, or `fanout` without replacement), minus excluded eids.

    indices is the CSR's int32 source-id array; returns (out_indptr [n_seeds+1],
    src global ids int64 [E'], eids [E'])."""
    out_indptr = sample_count(indptr, eids, seeds, fanout, seed_key, excluded, excluded_rows)
    total = int(out_indptr[-1].item())  # size readback
    out_src, out_eid = sample_fill(indptr, indices, eids, seeds, fanout, seed_key, out_indptr,
                                   total, excluded, excluded_rows)
    return out_indptr, out_src, out_eid


def sample_layer(indptrs, indices, eids, masks, src_type, dst_type, fanouts, keys, seeds,
                 prefix_pos, marks, mask_rows=None):
    """a9, one block layer in one call (gnnrec::sample_layer): sampled in-edges of every
    relation's seeds + the to_block relabel of every node type, two host size reads.
    mask_rows: per relation the excluded_rows flags of sample_count (or None).
    -> ([out_indptr], [local src int32], [eids], [src node ids per type], [edge counts])."""
    for t in list(indptrs) + list(eids) + list(seeds) + list(prefix_pos):
        _dev(t, "sample_layer operand", torch.int64)
    fans = [-1 if f is None or f < 0 else int(f) for f in fanouts]
    rows = list(mask_rows) if mask_rows is not None else [None] * len(masks)
    return _T().sample_layer(list(indptrs), list(indices), list(eids), list(masks), rows,
                             list(src_type), list(dst_type), fans, [_lib.i64(k) for k in keys],
                             list(seeds), list(prefix_pos), list(marks))


SB_MAX_RELS, SB_MAX_TYPES, SB_MAX_STEPS, SB_MAX_FANOUT = 8, 4, 4, 64
GATHER_MAX_JOBS = 16


class SampleScratch:
    """Per-node-type state of the fused sampler (gnnrec_sample_blocks, include/gnnrec.h):
    `pos` (two arrays of stamped seed positions, used alternately, never cleared), two
    new-source bitmaps and their word ranks, new-source and seed byte marks (two each).  `stamp` advances by steps + 1 per call; before it would wrap, `pos` is zeroed
    and the count restarts (one memset per ~4e9 sampled layers)."""

    def __init__(self, n_nodes: int, device):
        w = (n_nodes + 63) // 64
        self.n_nodes = n_nodes
        self.pos = torch.zeros(2 * n_nodes, dtype=torch.int64, device=device)
        self.bits = torch.zeros(2 * w, dtype=torch.int64, device=device)
        self.word_rank = torch.empty(w + 1, dtype=torch.int64, device=device)
        # two new-source mark arrays, then two seed mark arrays (each pair used alternately)
        self.marks = torch.zeros(4 * 64 * w, dtype=torch.uint8, device=device)


def sample_blocks(indptrs, indices, eids, src_type, dst_type, excl, n_nodes, seeds, scratch,
                  fanouts, keys, stamp, static_shapes=False, sizes_out=None, node_cap_hint=None,
                  overflow=None, edge_tables=(), node_tables=(), edge_recs=()):
    """a9, every block of one bounded-fanout sample_blocks call (gnnrec::sample_blocks,
    1 + 3L launches, one host size read).  fanouts / keys: [step][relation] (step 0 = the
    output block); excl: per relation None or (eids, coo_dst, mask, rows).
    -> per step: ([out_indptr], [local src int32], [eids]) per relation, [src node ids] per
    type, and the sizes (node counts rows -1..L-1 x types, then edge counts).
    static_shapes: every output at its capacity, no host read (the -1-padded layout of
    include/gnnrec.h); the sizes are then the capacities (seed caps, node caps, edge caps).
    sizes_out (int64 device tensor of the sizes' length): the exact outputs at their
    capacities and the sizes left there, not read back — the caller queues work sized by
    them on the device (gather_rows_batch's n_dev) before it reads them itself; the returned
    sizes are the capacities then too.  node_cap_hint ([step][type], static): tighter node
    capacities than the provable ones; a batch that does not fit sets `overflow` (int64
    device flag) and must be discarded or redone.
    edge_tables [(table, relation)] / node_tables [(table, node type)]: the block data (a10),
    gathered inside the call — every step's edge data at its edge ids, the input block's
    (the last step's) node rows at its source ids — returned as a third value in that order
    (step-major for the edge tables).  edge_recs: per relation the packed {eid << 32 | src}
    records of its CSR (HeteroGraph.edge_records), or empty (the index / eid arrays)."""
    steps, R = len(fanouts), len(indptrs)
    ex = [e if e is not None else (None,) * 4 for e in excl]
    o_ip, o_src, o_eid, nodes, sizes, data = _T().sample_blocks(
        list(indptrs), list(indices), list(eids), list(src_type), list(dst_type),
        [e[0] for e in ex], [e[1] for e in ex], [e[2] for e in ex], [e[3] for e in ex],
        list(n_nodes), list(seeds), [s.pos for s in scratch], [s.bits for s in scratch],
        [s.word_rank for s in scratch], [s.marks for s in scratch],
        [int(f) for fs in fanouts for f in fs],
        [_lib.i64(k) for ks in keys for k in ks], steps, int(stamp), bool(static_shapes),
        sizes_out, [int(h) for hs in (node_cap_hint or []) for h in hs], overflow,
        [t for t, _ in edge_tables], [int(r) for _, r in edge_tables],
        [t for t, _ in node_tables], [int(x) for _, x in node_tables], list(edge_recs))
    NT = len(n_nodes)
    out = []
    for s in range(steps):
        out.append(([o_ip[s * R + r] for r in range(R)], [o_src[s * R + r] for r in range(R)],
                    [o_eid[s * R + r] for r in range(R)], [nodes[s * NT + t] for t in range(NT)]))
    return out, sizes, data


class CompactScratch:
    """Per-node-type scratch of compact_ids: two id bitmaps used alternately (the call marks
    one and zeroes the other) and their word ranks."""

    def __init__(self, n_nodes: int, device):
        w = (n_nodes + 63) // 64
        self.n_nodes = n_nodes
        # the two bitmaps, then the scan's ticket and tile flags (GNNREC_COMPACT_SCAN_WS)
        self.bits = torch.zeros(2 * w + 2 + w // 1024, dtype=torch.int64, device=device)
        self.word_rank = torch.empty(w + 1, dtype=torch.int64, device=device)
        self.marks = torch.zeros(2 * 64 * w, dtype=torch.uint8, device=device)
        self.parity = 0


def compact_ids(lists, scratch, caps):
    """a11, DGL's compact_graphs over id lists at static shapes (gnnrec::compact_ids, 3
    launches, no host read): lists = [(ids int64, type index)]; scratch / caps per type.
    -> ([nodes [cap] per type: ascending ids, -1 past the count], [local ids per list],
    count [types] on the device)."""
    for ids, _ in lists:
        _dev(ids, "ids", torch.int64)
    parity = scratch[0].parity
    out = _T().compact_ids([ids.contiguous() for ids, _ in lists], [int(t) for _, t in lists],
                           [s.n_nodes for s in scratch], [int(c) for c in caps],
                           [s.bits for s in scratch], [s.word_rank for s in scratch],
                           [s.marks for s in scratch], parity)
    for s in scratch:
        s.parity = 1 - parity
    return out


def copy_batch(src, dst) -> None:
    """a12: dst[j].copy_(src[j]) for contiguous same-shape device tensors, 64 per launch
    (gnnrec_copy_batch); other pairs through torch's copy."""
    a, b = [], []
    for s_, d_ in zip(src, dst):
        if s_.is_contiguous() and d_.is_contiguous() and s_.dtype == d_.dtype and \
                s_.shape == d_.shape:
            a.append(s_)
            b.append(d_)
        else:
            d_.copy_(s_)
    if a:
        _T().copy_batch(a, b)


def gather_rows_batch(jobs, n_dev=None):
    """a10, several gathers in one launch: jobs = [(src, idx)] -> [src[idx]] (any dtype,
    contiguous rows; at most GATHER_MAX_JOBS per launch).  n_dev: per job None or a one-entry
    int64 device tensor — only the first min(n_dev, len(idx)) rows are gathered (the rest of
    the output is left unwritten)."""
    outs = []
    empty = None
    for i in range(0, len(jobs), GATHER_MAX_JOBS):
        part = jobs[i:i + GATHER_MAX_JOBS]
        srcs, idxs, res, cnts = [], [], [], []
        for k, (src, idx) in enumerate(part):
            c = None if n_dev is None else n_dev[i + k]
            if c is None:
                if empty is None:
                    empty = torch.empty(0, dtype=torch.int64, device=idx.device)
                c = empty
            cnts.append(c)
            _dev(idx, "idx", torch.int64)
            if src.dim() == 0:
                raise ValueError("src: expected at least one dimension")
            row = src[0] if src.shape[0] else src.new_empty(src.shape[1:])
            if not (row.is_contiguous() and (src.dim() == 1 or src.stride(0) >= row.numel())):
                src = src.contiguous()
            srcs.append(src)
            idxs.append(idx.contiguous())
            res.append(torch.empty((idx.numel(),) + tuple(src.shape[1:]), dtype=src.dtype,
                                   device=src.device))
        _T().gather_rows_batch(srcs, idxs, res, cnts if n_dev is not None else [])
        outs.extend(res)
    return outs


def edge_batch_pairs(rel_src, rel_dst, src_type, dst_type, batch, neg_order, k, n_nodes,
                     prefix_pos, marks):
    """EdgeDataLoader's batch head in one call (gnnrec::edge_batch_pairs): positive pairs of
    the batch's edges, k uniform negatives per positive (negative_sampler.Uniform's draws),
    and compact_graphs over both, one host size read.
    -> ([node ids per type], [pos src], [pos dst], [neg src], [neg dst]) in local ids."""
    for t in list(rel_src) + list(rel_dst) + list(batch) + list(prefix_pos):
        _dev(t, "edge_batch_pairs operand", torch.int64)
    return _T().edge_batch_pairs(list(rel_src), list(rel_dst), list(src_type), list(dst_type),
                                 list(batch), list(neg_order), int(k), list(n_nodes),
                                 list(prefix_pos), list(marks))


class Relabeler:
    """Per-node-type scratch for to_block relabelling (mark array + prefix map).

    Keeps two arrays of size n_nodes resident on the device (reset after each
    use by touching only the ids that were set).  `relabel` is the one-shot form;
    begin / mark / finish split it so a caller can batch the size readback of
    several node types into one host sync."""

    def __init__(self, n_nodes: int, device):
        self.n_nodes = n_nodes
        self.prefix_pos = torch.full((n_nodes,), -1, dtype=torch.int64, device=device)
        self.mark = torch.zeros(n_nodes, dtype=torch.int32, device=device)

    def begin(self, prefix: torch.Tensor, id_lists):
        """set the prefix map, mark new ids, scan -> rank (device; rank[-1] = n_new)."""
        T = _T()
        T.set_prefix_pos(prefix, self.prefix_pos)
        for ids in id_lists:
            T.mark_ids(ids, self.prefix_pos, self.mark)
        return exclusive_scan(self.mark)

    def finish(self, prefix: torch.Tensor, id_lists, rank: torch.Tensor, n_new: int):
        """compact the new ids, relabel every list, reset the scratch."""
        T = _T()
        n_p = prefix.numel()
        src_nodes = torch.empty(n_p + n_new, dtype=torch.int64, device=prefix.device)
        src_nodes[:n_p] = prefix
        if n_new:
            T.compact_marked(self.mark, rank, src_nodes[n_p:])
        locals_ = []
        for ids in id_lists:
            loc = torch.empty(ids.numel(), dtype=torch.int64, device=prefix.device)
            T.relabel_ids(ids, self.prefix_pos, rank, n_p, loc)
            locals_.append(loc)
        T.clear_prefix_pos(prefix, self.prefix_pos)
        if n_new:
            self.mark.index_fill_(0, src_nodes[n_p:], 0)
        return src_nodes, locals_

    def relabel(self, prefix: torch.Tensor, id_lists):
        """prefix: dst ids [n_p]; id_lists: list of global src id tensors.

        Returns (src_nodes [n_p + n_new] global ids, [local ids per list])."""
        rank = self.begin(prefix, id_lists)
        return self.finish(prefix, id_lists, rank, int(rank[-1].item()))


# load the library at import (outside any torch.compile trace); if it is missing, every op
# raises GnnrecLibraryError when called — there is no fallback
try:
    _lib.torch_ops()
except _lib.GnnrecLibraryError:
    pass
