"""Stream ordering of the sharded pass at ONE rank, where the replicated type's tree +
projection GEMMs run on the side stream under the partitioned type's launch
(ShardedFullGraphPass._owned_on_side) and later layers read their output on BOTH streams.

A delay kernel is queued ahead of every side-stream task (runner.side_delay_us): a read on
the main stream that is not ordered after the side stream's write then reads the table
before it is written, and the outputs differ from the single-stream order
(GNNREC_OWNED_SIDE=0), which must be reproduced bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(n_layers, two_rel, seed=3):
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(seed)
    n_u, n_i, E, d = 4000, 600, 120000, 128  # 30 / 200 edges per user / item row: fused paths
    u, i = rng.integers(0, n_u, E), rng.integers(0, n_i, E)
    rels = {("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u)}
    if two_rel:  # C5's shape: a second relation per destination type
        Ec = E // 3
        uc, ic = rng.integers(0, n_u, Ec), rng.integers(0, n_i, Ec)
        rels[("user", "clicks", "item")] = (uc, ic)
        rels[("item", "clicked-by", "user")] = (ic, uc)
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(t)) for ce, (s, t) in rels.items()},
                    {"user": n_u, "item": n_i}, device="cuda")
    feats = {"user": torch.from_numpy(rng.standard_normal((n_u, d)).astype(np.float32)).cuda(),
             "item": torch.from_numpy(rng.standard_normal((n_i, d)).astype(np.float32)).cuda()}
    torch.manual_seed(0)
    model = gnn.ConvModel(g, n_layers, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0,
                          "mean", "cos", "sum", True).cuda().eval()
    return g, feats, model


def _run(g, feats, model, det, delay_us, passes=1):
    from gnnrec.dist import Exchange
    from gnnrec.inference import GraphShard, ShardedFullGraphPass
    sh = GraphShard.from_graph(g, 0, 1, "user", device="cuda", segments=8)
    runner = ShardedFullGraphPass(model, sh, Exchange(), deterministic=det)
    runner.side_delay_us = delay_us
    x = sh.local_features(feats)
    outs = []
    for _ in range(passes):
        out = runner.run(x)
        outs.append({nt: t.clone() for nt, t in out.items()})
    torch.cuda.synchronize()
    return outs, runner


@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("two_rel", [False, True])
def test_side_stream_tables_are_waited_for_on_main(monkeypatch, det, two_rel):
    """3 conv layers (n_layers=4 with the embedding): layers 2 and 3 read the item table
    that the previous layer's side-stream GEMM wrote, on the side stream (tree + GEMM of
    this layer) and on main (the item->user launch).  With 20 ms of delay ahead of every
    side task, the outputs equal the single-stream order bitwise, pass after pass."""
    g, feats, model = _graph(4, two_rel)
    monkeypatch.setenv("GNNREC_OWNED_SIDE", "0")
    ref, _ = _run(g, feats, model, det, 0)
    monkeypatch.setenv("GNNREC_OWNED_SIDE", "1")
    outs, runner = _run(g, feats, model, det, 20000, passes=3)
    assert runner._owned_side
    for k, out in enumerate(outs):
        for nt in ref[0]:
            assert torch.equal(out[nt], ref[0][nt]), f"pass {k}: {nt} differs from one stream"
