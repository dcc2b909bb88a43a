"""CPU-side checks of the torch dispatcher layer (csrc/torch_ops.cpp, TORCH_LIBRARY(gnnrec)):
every C-ABI launch entry point has a torch.ops.gnnrec schema, bad shapes raise ValueError
through TORCH_CHECK_VALUE from the Meta kernels, CPU tensors are refused, and
torch.compile(fullgraph=True) traces the drop-in ConvLayer.forward (eval mode) without
graph breaks — on meta tensors, so nothing launches here (the GPU run of the same compiled
module is in tests/test_gpu_torch_ops.py)."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gnnrec.h")

# C-ABI entry points that are not launches of their own (library state, the forms that
# one torch op covers: gemm_f32 / gemm_tn_f32 are gemm_rownorm / gemm_tn_bias without the
# extra output, the i32/i64 scans are one op dispatching on dtype)
NOT_OPS = {"gnnrec_last_error", "gnnrec_gemm_f32", "gnnrec_gemm_tn_f32",
           "gnnrec_exclusive_scan_i32", "gnnrec_exclusive_scan_i64",
           "gnnrec_spmm_project_mfma_f32",
           "gnnrec_sample_blocks_caps"}  # (sample_blocks sizes its outputs with it)
RENAMED = {"gnnrec_gemm_rownorm_f32": "gemm", "gnnrec_gemm_tn_bias_f32": "gemm_tn",
           "gnnrec_gemm_tn_bias_rows_f32": "gemm_tn", "gnnrec_spmm_csr_live_f32": "spmm_csr",
           "gnnrec_spmm_plan_build_live": "spmm_plan_build",
           "gnnrec_spmm_csr_planned_live_f32": "spmm_csr_planned",
           "gnnrec_row_epilogue_f32": "row_epilogue", "gnnrec_add_f32": "add_",
           "gnnrec_tree_sum_f32": "tree_sum_", "gnnrec_spmm_csr_f32": "spmm_csr",
           "gnnrec_spmm_csr_split_f32": "spmm_csr_split",
           "gnnrec_spmm_csr_planned_f32": "spmm_csr_planned", "gnnrec_spmm_csr2_f32": "spmm_csr2",
           "gnnrec_spmm_backward_f32": "spmm_backward",
           "gnnrec_spmm_project_f32": "spmm_project", "gnnrec_sddmm_cos_f32": "sddmm_cos",
           "gnnrec_spmm_project2_f32": "spmm_project2", "gnnrec_spmm_pair_f32": "spmm_pair",
           "gnnrec_sddmm_cos_backward_f32": "sddmm_cos_backward",
           "gnnrec_sddmm_cos_backward_grouped_f32": "sddmm_cos_backward",
           "gnnrec_sddmm_cos_backward_grouped_workspace_bytes":
               "sddmm_cos_backward_workspace_bytes",
           "gnnrec_sddmm_cos_grouped_f32": "sddmm_cos_grouped",
           "gnnrec_edge_mlp_f32": "edge_mlp", "gnnrec_edge_mlp_grouped_f32": "edge_mlp_grouped",
           "gnnrec_act_backward_f32": "act_backward",
           "gnnrec_act_backward_normed_f32": "act_backward_normed",
           "gnnrec_lstm_step_f32": "lstm_step", "gnnrec_topk_rows_f32": "topk_rows",
           "gnnrec_lstm_step_save_f32": "lstm_step_save",
           "gnnrec_lstm_backward_step_f32": "lstm_backward_step",
           "gnnrec_margin_loss_f32": "margin_loss", "gnnrec_sum_scaled_f32": "sum_scaled"}


def _T():
    from gnnrec import _lib
    return _lib.torch_ops()


def _declared():
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(gnnrec_[a-z0-9_]+)\s*\(", txt)))


def test_every_entry_point_has_a_torch_op():
    T = _T()
    missing = []
    for sym in _declared():
        if sym in NOT_OPS:
            continue
        name = RENAMED.get(sym, sym[len("gnnrec_"):])
        try:
            getattr(T, name).default._schema
        except (AttributeError, RuntimeError):
            missing.append((sym, name))
    assert not missing, missing
    assert T.version() >= 1
    # outputs are declared mutable (functionalisation knows what each launch writes)
    s = str(T.spmm_csr.default._schema)
    assert "Tensor(a!) out" in s and s.endswith("-> ()")
    assert "Tensor(a!) out" in str(T.spmm_project.default._schema)


def _meta(*shape, dtype=torch.float32):
    return torch.empty(*shape, dtype=dtype, device="meta")


def test_meta_kernels_check_shapes():
    T = _T()
    ip, ix, X = _meta(6, dtype=torch.int64), _meta(20, dtype=torch.int32), _meta(10, 4)
    T.spmm_csr(ip, ix, None, X, 1, 0, _meta(5, 4))  # fine: nothing launches on meta
    with pytest.raises(ValueError, match="out must be"):
        T.spmm_csr(ip, ix, None, X, 1, 0, _meta(4, 4))
    with pytest.raises(ValueError, match="indices must be Int"):
        T.spmm_csr(ip, _meta(20, dtype=torch.int64), None, X, 1, 0, _meta(5, 4))
    with pytest.raises(ValueError, match="W1"):
        T.gemm(_meta(8, 16), _meta(4, 8), None, None, None, 0, None, None, 0, 0, 0.0, None, None,
               _meta(8, 4), None)
    with pytest.raises(ValueError, match="unit column stride"):
        T.sddmm_cos(_meta(3, dtype=torch.int64), _meta(3, dtype=torch.int64), _meta(4, 8).t(),
                    _meta(8, 4), _meta(3))
    # two pre-projected relations into one type: row counts must agree
    i64, i32 = torch.int64, torch.int32
    ra = (_meta(6, dtype=i64), _meta(20, dtype=i32), None, _meta(9, 128), 1, None)
    rb = (_meta(6, dtype=i64), _meta(7, dtype=i32), None, _meta(9, 128), 0, None)
    W = _meta(128, 128)
    T.spmm_project2(*ra, *rb, _meta(5, 128), W, W, None, None, 3, 1, None, 0.0, _meta(5, 128))
    with pytest.raises(ValueError, match="row counts differ"):
        T.spmm_project2(*ra, _meta(7, dtype=i64), *rb[1:], _meta(5, 128), W, W, None, None, 3, 1,
                        None, 0.0, _meta(5, 128))
    with pytest.raises(ValueError, match="out must be"):
        T.spmm_project2(*ra, *rb, _meta(5, 128), W, W, None, None, 3, 1, None, 0.0,
                        _meta(4, 128))


def test_cpu_tensors_are_refused():
    T = _T()
    with pytest.raises(ValueError, match="HIP device tensor"):
        T.spmm_csr(torch.zeros(3, dtype=torch.int64), torch.zeros(0, dtype=torch.int32), None,
                   torch.zeros(2, 4), 1, 0, torch.zeros(2, 4))
    from gnnrec import ops
    with pytest.raises(ValueError, match="HIP device tensor"):
        ops.spmm(torch.zeros(3, dtype=torch.int64), torch.zeros(0, dtype=torch.int32),
                 torch.zeros(2, 4))


def _meta_rel(n_src, n_dst, E):
    from gnnrec import ops
    from gnnrec.graph import RelGraph
    indptr = _meta(n_dst + 1, dtype=torch.int64)
    indptr._gnnrec_nnz = E  # what csr_build / the sampler record on a real CSR
    indptr._gnnrec_split_plan = (ops.DEFAULT_SPLIT, None)  # no heavy rows
    return RelGraph(("item", "bought-by", "user"), indptr, _meta(E, dtype=torch.int32), n_src,
                    n_dst)


@pytest.mark.parametrize("d,agg,n_src,deg", [(128, "mean", 50, 30), (64, "mean_nn", 50, 30),
                                             (128, "pool_nn", 50, 30), (128, "mean", 15, 10)])
def test_compile_convlayer_forward_fullgraph(d, agg, n_src, deg):
    """torch.compile(fullgraph=True) of the drop-in ConvLayer.forward in eval mode: every
    launch is a torch.ops.gnnrec op with a meta kernel, nothing breaks the graph (the last
    case: a small source table at 10 edges/row, projected before the reduction)."""
    import torch._dynamo
    from gnnrec import _lib
    from gnnrec import nn as gnn
    _lib.torch_ops()  # the registration loads on first use: not inside the traced region
    torch._dynamo.reset()
    layer = gnn.ConvLayer((d, d), d, 0.0, agg, True).eval().to("meta")
    g = _meta_rel(n_src, 40, 40 * deg)
    x = (_meta(n_src, d), _meta(40, d))
    compiled = torch.compile(layer, fullgraph=True, backend="aot_eager")
    with torch.no_grad():
        z = compiled(g, x)
    assert tuple(z.shape) == (40, d) and z.device.type == "meta"
    ops_seen = set()

    def backend(gm, example_inputs):
        for n in gm.graph.nodes:
            if n.op == "call_function" and "gnnrec" in str(n.target):
                ops_seen.add(str(n.target).split(".")[1])
        return gm.forward
    torch._dynamo.reset()
    with torch.no_grad():
        torch.compile(layer, fullgraph=True, backend=backend)(g, x)
    want = {"spmm_project"} if d == 128 else {"spmm_csr", "gemm"}  # fused at d = 128
    if agg != "mean" or n_src * 2 <= 40:  # fc_preagg on the sources / their pre-projection
        want.add("gemm")  # fc_preagg + ReLU on the source table
    assert want <= ops_seen, ops_seen


def test_compile_heterograph_conv_fullgraph():
    """HeteroGraphConv.forward (relation loop, accumulate modes into one output) traces
    as one graph too: the fused launches accumulate into the destination buffer."""
    import torch._dynamo
    from gnnrec import nn as gnn, ops
    from gnnrec.graph import HeteroGraph
    d, E = 128, 500 * 30
    i64 = torch.int64
    g = HeteroGraph({("user", "buys", "item"): (_meta(E, dtype=i64), _meta(E, dtype=i64)),
                     ("item", "bought-by", "user"): (_meta(E, dtype=i64), _meta(E, dtype=i64))},
                    {"user": 500, "item": 150}, device="meta")
    for ce, n in ((("user", "buys", "item"), 150), (("item", "bought-by", "user"), 500)):
        ip = _meta(n + 1, dtype=i64)
        ip._gnnrec_nnz, ip._gnnrec_split_plan = E, (ops.DEFAULT_SPLIT, None)
        g._csr[ce] = (ip, _meta(E, dtype=torch.int32), _meta(E, dtype=i64))
    conv = gnn.HeteroGraphConv({e: gnn.ConvLayer((d, d), d, 0.0, "mean", True)
                                for e in ("buys", "bought-by")}, aggregate="sum").to("meta").eval()
    torch._dynamo.reset()
    with torch.no_grad():
        out = torch.compile(conv, fullgraph=True, backend="aot_eager")(
            g, {"user": _meta(500, d), "item": _meta(150, d)})
    assert tuple(out["user"].shape) == (500, d) and tuple(out["item"].shape) == (150, d)


def test_sage_rel_ops_meta_shapes():
    """The fused training relation ops (gnnrec/autograd.py SageRelFn) return the forward's
    (z, agg, row norms) and the backward's four gradients with the right shapes on meta
    tensors, and refuse a max reduce."""
    T = _T()
    M, n_src, E, d, N = 5, 9, 20, 8, 6
    ip, ix = _meta(M + 1, dtype=torch.int64), _meta(E, dtype=torch.int32)
    m, hs, Ws, Wn = _meta(n_src, d), _meta(7, d), _meta(N, d), _meta(N, d)
    z, agg, nrm = T.sage_rel_forward(m, hs, M, Ws, Wn, ip, ix, None, 1, True)
    assert tuple(z.shape) == (M, N) and tuple(agg.shape) == (M, d) and tuple(nrm.shape) == (M,)
    g = T.sage_rel_backward(z, z, nrm, hs, agg, Ws, Wn, ip, ix, None, 1, n_src, E, True, 15)
    assert [tuple(t.shape) for t in g] == [(7, d), (n_src, d), (N, d), (N, d), (0,), (0,)]
    # a folded NodeEmbedding's biases: their gradients when asked for (need bits 16, 32)
    b = _meta(N)
    z, agg, nrm = T.sage_rel_forward(m, hs, M, Ws, Wn, ip, ix, None, 1, True, b, b)
    g = T.sage_rel_backward(z, z, nrm, hs, agg, Ws, Wn, ip, ix, None, 1, n_src, E, True, 12 | 48)
    assert [tuple(t.shape) for t in g] == [(0,), (0,), (N, d), (N, d), (N,), (N,)]
    with pytest.raises(ValueError, match="biases"):
        T.sage_rel_forward(m, hs, M, Ws, Wn, ip, ix, None, 1, True, _meta(N + 1), None)
    with pytest.raises(ValueError, match="sum or mean"):
        T.sage_rel_forward(m, hs, M, Ws, Wn, ip, ix, None, 2, True)
