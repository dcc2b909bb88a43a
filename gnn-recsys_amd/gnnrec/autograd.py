"""Autograd Functions for training through the drop-in modules.

Forward values always come from the HIP kernels (the same launches as the
inference path, so train/eval numerics agree).  Backward of the aggregation is
the HIP transposed scatter (gnnrec_spmm_backward_f32, first-arg-max routing
for max); the projection / linear weight and input gradients are device GEMMs
on the same stream (recompute-and-differentiate for the fused epilogues).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

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
        if ctx.relu:
            gy = gy * (y > 0).to(gy.dtype)
        elif ctx.sigmoid:
            gy = gy * y * (1 - y)
        gx = gy @ W if ctx.needs_input_grad[0] else None
        gW = gy.t() @ x if ctx.needs_input_grad[1] else None
        gb = gy.sum(0) if ctx.has_b and ctx.needs_input_grad[2] else None
        return gx, gW, gb, None, None


class SpmmFn(torch.autograd.Function):
    """agg = reduce_{e in row v} m[src_e] (* w_e); forward = gnnrec_spmm_csr_f32."""

    @staticmethod
    def forward(ctx, m, indptr, indices, ew, reduce: str, n_dst: int):
        out = ops.spmm(indptr, indices, m.contiguous(), reduce, edge_weight=ew)
        ctx.save_for_backward(m, indptr, indices, ew, out)
        ctx.reduce = reduce
        return out

    @staticmethod
    def backward(ctx, g):
        m, indptr, indices, ew, out = ctx.saved_tensors
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        gm = ops.spmm_backward(indptr, indices, g, ctx.reduce, edge_weight=ew,
                               X=m if ctx.reduce == 'max' else None,
                               out=out if ctx.reduce == 'max' else None, n_src=m.shape[0])
        return gm, None, None, None, None, None


class SageProjectFn(torch.autograd.Function):
    """z = norm?(relu(h_self W_selfᵀ + agg W_neighᵀ)); forward = fused gnnrec_gemm_f32."""

    @staticmethod
    def forward(ctx, h_self, agg, Ws, Wn, norm: bool):
        z = ops.gemm(h_self.contiguous(), Ws.detach(), agg.contiguous(), Wn.detach(), relu=True,
                     l2norm=norm)
        ctx.save_for_backward(h_self, agg, Ws, Wn)
        ctx.norm = norm
        return z

    @staticmethod
    def backward(ctx, gz):
        h_self, agg, Ws, Wn = ctx.saved_tensors
        with torch.enable_grad():
            ins = [t.detach().requires_grad_(True) for t in (h_self, agg, Ws, Wn)]
            z = torch.relu(ins[0] @ ins[2].t() + ins[1] @ ins[3].t())
            if ctx.norm:
                n = z.norm(2, 1, keepdim=True)
                z = z / torch.where(n == 0, torch.ones_like(n), n)
            grads = torch.autograd.grad(z, ins, gz, allow_unused=True)
        return tuple(gr if need else None for gr, need in
                     zip(grads, ctx.needs_input_grad[:4])) + (None,)


class CosineFn(torch.autograd.Function):
    """cos_e = <ĥs[src_e], ĥd[dst_e]>; forward = gnnrec_sddmm_cos_f32."""

    @staticmethod
    def forward(ctx, hs, hd, src, dst):
        out = ops.sddmm_cos(src, dst, hs.contiguous(), hd.contiguous())
        ctx.save_for_backward(hs, hd, src, dst)
        return out

    @staticmethod
    def backward(ctx, g):
        hs, hd, src, dst = ctx.saved_tensors
        with torch.enable_grad():
            a = hs.detach().requires_grad_(True)
            b = hd.detach().requires_grad_(True)
            cos = (F.normalize(a, p=2, dim=-1)[src] * F.normalize(b, p=2, dim=-1)[dst]).sum(-1)
            ga, gb = torch.autograd.grad(cos, (a, b), g, allow_unused=True)
        return ga, gb, None, None
