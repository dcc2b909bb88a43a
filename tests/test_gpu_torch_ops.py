"""GPU checks of the torch dispatcher layer (csrc/torch_ops.cpp): the torch.ops.gnnrec ops
called directly match the oracle, and torch.compile(fullgraph=True) of the drop-in
ConvLayer.forward / HeteroGraphConv.forward (eval mode) runs the same HIP kernels with
results bitwise equal to eager (reference call sites: src/model.py:143-208,226-235,384-406)."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"
RTOL, ATOL = 1e-4, 1e-5


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("reduce", ["sum", "mean", "max"])
def test_torch_op_spmm_csr_matches_oracle(reduce):
    from gnnrec import _lib, ops
    T = _lib.torch_ops()
    rng = np.random.default_rng(3)
    n_dst, n_src, d = 700, 300, 64
    dst, src = rng.integers(0, n_dst, 9000), rng.integers(0, n_src, 9000)
    indptr, indices, _ = oracle.csr_from_coo(src, dst, n_dst)
    X = rng.standard_normal((n_src, d)).astype(np.float32)
    out = torch.empty((n_dst, d), device=DEV)
    T.spmm_csr(_t(indptr), _t(indices.astype(np.int32)), None, _t(X), ops.REDUCE[reduce], 0, out)
    ref = oracle.spmm_csr(indptr, indices, X, reduce)
    if reduce == "max":
        assert np.array_equal(out.cpu().numpy(), ref)
    else:
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=RTOL, atol=ATOL)
    with pytest.raises(ValueError, match="out must be"):
        T.spmm_csr(_t(indptr), _t(indices.astype(np.int32)), None, _t(X), 1, 0, out[:-1])


def _graph(n_u, n_i, deg_u, deg_i, seed):
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(seed)
    E = n_u * deg_u
    u, i = rng.integers(0, n_u, E), rng.integers(0, n_i, E)
    edges = {("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u)}
    return HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(t))
                        for ce, (s, t) in edges.items()}, {"user": n_u, "item": n_i}, device=DEV)


@pytest.mark.parametrize("d,agg,deg", [(128, "mean", 40), (128, "mean", 8), (64, "mean_nn", 20),
                                       (128, "pool_nn", 30)])
def test_compiled_convlayer_equals_eager(d, agg, deg):
    """torch.compile(fullgraph=True) of ConvLayer.forward: no graph break, the fused /
    unfused kernels run through torch.ops.gnnrec, outputs bitwise equal to eager."""
    import torch._dynamo
    from gnnrec import nn as gnn
    g = _graph(600, 200, deg, deg, d + deg)
    rel = g.rel_graph(("item", "bought-by", "user"))
    torch.manual_seed(0)
    layer = gnn.ConvLayer((d, d), d, 0.0, agg, True).to(DEV).eval()
    x = (torch.randn(200, d, device=DEV), torch.randn(600, d, device=DEV))
    with torch.no_grad():
        ref = layer(rel, x)  # eager: also caches the CSR's host-side plan on the indptr
        torch._dynamo.reset()
        got = torch.compile(layer, fullgraph=True, backend="aot_eager")(rel, x)
    assert torch.equal(got, ref)


def test_compiled_heterograph_conv_equals_eager():
    import torch._dynamo
    from gnnrec import nn as gnn
    d = 128
    g = _graph(500, 150, 30, 30, 9)
    torch.manual_seed(1)
    conv = gnn.HeteroGraphConv({e: gnn.ConvLayer((d, d), d, 0.0, "mean", True)
                                for e in ("buys", "bought-by")}, aggregate="sum").to(DEV).eval()
    h = {"user": torch.randn(500, d, device=DEV), "item": torch.randn(150, d, device=DEV)}
    with torch.no_grad():
        ref = conv(g, h)
        torch._dynamo.reset()
        got = torch.compile(conv, fullgraph=True, backend="aot_eager")(g, h)
    for nt in ref:
        assert torch.equal(got[nt], ref[nt]), nt
