"""CPU-side checks of the product: the C-ABI library loads and exports every
symbol include/gnnrec.h declares (no compute without a GPU), argument
validation fails loudly, and there is no silent CPU path."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gnnrec.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gnnrec_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_hot_path_entry_points():
    syms = declared_symbols()
    for s in ("gnnrec_spmm_csr_f32", "gnnrec_gemm_f32", "gnnrec_sddmm_cos_f32",
              "gnnrec_edge_mlp_f32", "gnnrec_sample_count", "gnnrec_sample_fill",
              "gnnrec_synth_edges", "gnnrec_last_error", "gnnrec_version"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from gnnrec import _lib
    lib = _lib.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes table covers exactly the header
    assert sorted(_lib.SIGNATURES) == declared_symbols()
    assert lib.gnnrec_version() >= 1


def test_argument_validation_without_a_gpu():
    """Shape/enum errors are reported through gnnrec_last_error before any launch."""
    from gnnrec import _lib
    lib = _lib.load()
    rc = lib.gnnrec_spmm_csr_f32(None, None, None, None, 4, 3, 4, 7, 0, None, 4, None)
    assert rc == _lib.OK + 1
    assert b"unknown reduce" in lib.gnnrec_last_error()
    rc = lib.gnnrec_gemm_f32(None, 4, 4, None, None, 1, 0, None, None, 0, None, None, 10, 300,
                             _lib.EPI_L2NORM, 0, 0.0, None, None, ctypes.c_void_p(16), 300, None)
    assert rc != 0 and b"A1" in lib.gnnrec_last_error()
    rc = lib.gnnrec_gemm_f32(None, 4, 0, None, None, 1, 0, None, None, 0, None, None, 10, 8, 0,
                             _lib.ACC_ATTN, 0.0, None, None, ctypes.c_void_p(16), 8, None)
    assert rc != 0 and b"attention" in lib.gnnrec_last_error()
    # the deterministic tree's fold: 2, 4 or 8 tables, 16-B aligned
    parts = (ctypes.c_void_p * 3)(16, 32, 48)
    rc = lib.gnnrec_tree_sum_f32(parts, 3, 8, ctypes.c_void_p(16), None)
    assert rc != 0 and b"n_parts=3" in lib.gnnrec_last_error()
    parts = (ctypes.c_void_p * 2)(16, 36)
    rc = lib.gnnrec_tree_sum_f32(parts, 2, 8, ctypes.c_void_p(16), None)
    assert rc != 0 and b"aligned" in lib.gnnrec_last_error()
    # a device row count (static blocks) drives sum / mean gathers only
    rc = lib.gnnrec_spmm_csr_live_f32(ctypes.c_void_p(16), ctypes.c_void_p(16), None,
                                      ctypes.c_void_p(16), 4, 3, 4, _lib.REDUCE_MAX, 0,
                                      ctypes.c_void_p(16), 4, ctypes.c_void_p(16), None)
    assert rc != 0 and b"sum or mean" in lib.gnnrec_last_error()
    rc = lib.gnnrec_gemm_tn_bias_rows_f32(None, 4, None, 4, -1, 4, 4, None, 4, None, None, 0,
                                          None, None)
    assert rc != 0 and b"negative size" in lib.gnnrec_last_error()
    # empty problems are no-ops that succeed without touching memory
    assert lib.gnnrec_spmm_csr_f32(None, None, None, None, 4, 0, 4, 1, 0, None, 4, None) == 0
    assert lib.gnnrec_tree_sum_f32(parts, 2, 0, None, None) == 0


def test_ops_refuse_cpu_tensors():
    from gnnrec import ops
    x = torch.zeros(3, 4)
    with pytest.raises(ValueError, match="no CPU path"):
        ops.spmm(torch.zeros(4, dtype=torch.int64), torch.zeros(0, dtype=torch.int32), x)
    with pytest.raises(ValueError, match="no CPU path"):
        ops.gemm(x, torch.zeros(2, 4))


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    from gnnrec import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "_load_error", None)
    with pytest.raises(_lib.GnnrecLibraryError):
        _lib.load()
    # monkeypatch restores the loaded handle; no reload (it would drop the op registration
    # handle, and a later torch.compile test would then trace the loader)


def test_modules_keep_reference_state_dict_layout():
    from gnnrec import nn as gnn
    from gnnrec.synth import GraphMeta
    meta = GraphMeta([("user", "buys", "item"), ("item", "bought-by", "user")], ["item", "user"])
    m = gnn.ConvModel(meta, 3, {"user": 4, "item": 6, "hidden": 16, "out": 8}, True, 0.0,
                      "mean_nn", "nn", "sum", True)
    keys = set(m.state_dict())
    assert "user_embed.proj_feats.weight" in keys and "item_embed.proj_feats.bias" in keys
    assert "layers.0.mods.buys.fc_self.weight" in keys
    assert "layers.1.mods.bought-by.fc_preagg.weight" in keys
    assert "pred_fn.layer_nn.hidden_1.weight" in keys and "pred_fn.layer_nn.output.bias" in keys
    with pytest.raises(KeyError):
        gnn.ConvModel(meta, 2, {"user": 4, "item": 6, "hidden": 16, "out": 8}, pred="dot")


def test_lstm_aggregators_follow_the_reference():
    """'lstm' builds an nn.LSTM with the reference's state_dict keys; 'lstm_edge' never
    builds one (src/model.py:103-104) and fails on the attribute in forward, as the
    reference does; LSTM step validation runs before any launch."""
    from gnnrec import _lib
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    layer = gnn.ConvLayer((6, 5), 8, 0.0, "lstm", True)
    assert {"lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0",
            "lstm.bias_hh_l0"} <= set(layer.state_dict())
    g = HeteroGraph({("user", "buys", "item"): (torch.tensor([0, 1]), torch.tensor([1, 0]))},
                    {"user": 2, "item": 2})
    with pytest.raises(AttributeError, match="lstm"):
        gnn.ConvLayer((6, 5), 8, 0.0, "lstm_edge", True)(
            g.rel_graph(("user", "buys", "item")), (torch.zeros(2, 6), torch.zeros(2, 5)))
    lib = _lib.load()
    rc = lib.gnnrec_lstm_step_f32(None, 4, None, None, None, 0, 1, None, None, None, 1000, None,
                                  None, 1000, None)
    assert rc != 0 and b"hidden size" in lib.gnnrec_last_error()
