"""Randomised end-to-end parity: many seeded (graph, model) configurations through the
full-graph pass — module path and the one-rank sharded driver — against the oracle.
Covers the fused / unfused / folded dispatch decisions, every aggregator, every hetero
mode, heavy rows, zero-degree rows, d in {16, 64, 128} (d=128 with dense and sparse
relations so both the fused and the GEMM path run).  Embeddings within 1e-4 (rtol)."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

AGGS = ["mean", "mean_nn", "pool_nn", "mean_edge", "mean_nn_edge", "pool_nn_edge"]
HETS = ["sum", "mean", "max", "attention"]


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    d = int(rng.choice([16, 64, 128, 128]))
    n_u, n_i = int(rng.integers(50, 900)), int(rng.integers(20, 400))
    dense = rng.random() < 0.5
    E_b = int(rng.integers(30, 40) * n_u) if dense else int(rng.integers(1, 8) * n_u)
    E_c = int(rng.integers(0, 3) * n_u)
    edges, occ = {}, {}
    for (f, r), E in ((("buys", "bought-by"), E_b), (("clicks", "clicked-by"), E_c)):
        u = rng.integers(0, n_u, E)
        if rng.random() < 0.3 and E:  # a heavy item
            i = np.where(rng.random(E) < 0.4, 0, rng.integers(0, n_i, E))
        else:
            i = rng.integers(0, n_i, E)
        o = rng.integers(1, 9, E)
        edges[("user", f, "item")] = (u, i)
        edges[("item", r, "user")] = (i, u)
        occ[("user", f, "item")] = o
        occ[("item", r, "user")] = o
    agg = AGGS[seed % len(AGGS)]
    het = HETS[(seed // len(AGGS)) % len(HETS)]
    emb = bool(rng.random() < 0.7)
    norm = bool(rng.random() < 0.8)
    n_layers = int(rng.choice([2, 3]))
    return rng, d, {"user": n_u, "item": n_i}, edges, occ, agg, het, emb, norm, n_layers


@pytest.mark.parametrize("seed", range(96))
def test_random_configurations_match_oracle(seed):
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    from gnnrec.inference import GraphShard, ShardedFullGraphPass, full_graph_embeddings
    rng, d, nn_, edges, occ, agg, het, emb, norm, n_layers = _case(seed)
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(t)) for ce, (s, t) in edges.items()},
                    nn_, device="cuda")
    for ce, o in occ.items():
        g.edges[ce].data["occurrence"] = torch.from_numpy(o).cuda()
    feats = {nt: rng.standard_normal((n, d)).astype(np.float32) for nt, n in nn_.items()}
    for nt, f in feats.items():
        g.nodes[nt].data["features"] = torch.from_numpy(f).cuda()
    torch.manual_seed(seed)
    model = gnn.ConvModel(g, n_layers, {"user": d, "item": d, "hidden": d, "out": d}, norm, 0.0,
                          agg, "cos", het, emb).cuda().eval()
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    ref = oracle.model_full_graph(oracle.Graph(nn_, edges, occ), feats, sd, agg, het, norm, emb)
    h1 = full_graph_embeddings(g, model)
    shard = GraphShard.from_graph(g, 0, 1, "user", device="cuda")
    h2 = ShardedFullGraphPass(model, shard).run(shard.local_features(g.ndata["features"]))
    # the bench's form: 8 source-range tiles (heavy rows chunked per TILE_SPLIT), the fixed
    # tree of deterministic mode for sum/mean reducers, in-place tile accumulation for max
    tiles = GraphShard.from_graph(g, 0, 1, "user", device="cuda", segments=8)
    h3 = ShardedFullGraphPass(model, tiles, deterministic=True).run(
        tiles.local_features(g.ndata["features"]))
    for nt in ref:
        scale = max(1.0, float(np.abs(ref[nt]).max()))
        for h in (h1, h2, h3):
            got = h[nt][: ref[nt].shape[0]].cpu().numpy()
            np.testing.assert_allclose(got, ref[nt], rtol=1e-4, atol=1e-5 * scale,
                                       err_msg=f"{nt} d={d} agg={agg} het={het} emb={emb}")


@pytest.mark.parametrize("seed", range(8))
def test_random_training_steps_layer_node_matches_relation_nodes(monkeypatch, seed):
    """Randomised training steps over sampled blocks: the whole layer as one autograd node
    (gnnrec.autograd.HeteroSageFn, GNNREC_TRAIN_LAYER=1) against one node per relation
    (=0): the same loss bits, parameter gradients within fp32 reassociation (a table's
    gradient sums up to four relation parts in the node's own order).  Aggregators with and
    without fc_preagg / edge weights, the max / LSTM-free hetero modes, one or two
    relations per node type, with and without the embedding; and the first layer with the
    NodeEmbedding folded into it (GNNREC_TRAIN_FOLD=1) within fp32 reassociation."""
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    rng = np.random.default_rng(5000 + seed)
    d = int(rng.choice([16, 64, 128]))
    n_u, n_i = int(rng.integers(200, 2000)), int(rng.integers(50, 500))
    two = bool(rng.random() < 0.5)
    rels = {}
    for f, r, share in (("buys", "bought-by", 1.0), ("clicks", "clicked-by", 0.5))[:2 if two else 1]:
        E = int(n_u * rng.integers(3, 20) * share)
        u, i = rng.integers(0, n_u, E), rng.integers(0, n_i, E)
        rels[("user", f, "item")] = (u, i)
        rels[("item", r, "user")] = (i, u)
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(t)) for ce, (s, t) in rels.items()},
                    {"user": n_u, "item": n_i}, device="cuda")
    for ce, (s, _) in rels.items():
        g.edges[ce].data["occurrence"] = torch.from_numpy(rng.integers(1, 9, s.size)).cuda()
    g.nodes["user"].data["features"] = torch.randn(n_u, d, device="cuda")
    g.nodes["item"].data["features"] = torch.randn(n_i, d, device="cuda")
    agg = ["mean", "mean_nn", "mean_edge", "mean_nn_edge"][seed % 4]
    het = ["sum", "mean"][(seed // 4) % 2]
    emb = bool(rng.random() < 0.7)
    torch.manual_seed(seed)
    model = gnn.ConvModel(g, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0, agg,
                          "cos", het, emb).cuda()
    buys = ("user", "buys", "item")
    K = int(rng.integers(1, 6))
    loader = EdgeDataLoader(g, {buys: torch.arange(min(600, len(rels[buys][0])))},
                            MultiLayerNeighborSampler([int(rng.integers(2, 8))] * 2),
                            exclude="reverse_types",
                            reverse_etypes={"buys": "bought-by", "bought-by": "buys",
                                            "clicks": "clicked-by", "clicked-by": "clicks"},
                            negative_sampler=negative_sampler.Uniform(K), batch_size=128)
    _, pos_g, neg_g, blocks = next(iter(loader))
    res = {}
    # layer node vs relation nodes, both embedding then aggregating (GNNREC_TRAIN_FOLD=0: the
    # bitwise comparison below); then the first layer with the NodeEmbedding folded in
    for layer, fold in (("1", "0"), ("0", "0"), ("fold", "1")):
        monkeypatch.setenv("GNNREC_TRAIN_LAYER", "0" if layer == "0" else "1")
        monkeypatch.setenv("GNNREC_TRAIN_FOLD", fold)
        model.zero_grad()
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, emb)
        loss = gnn.max_margin_loss(ps, ns, 0.266, K)
        loss.backward()
        res[layer] = (loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()
                                      if p.grad is not None})
    assert torch.equal(res["1"][0], res["0"][0])
    assert res["1"][1].keys() == res["0"][1].keys() and len(res["1"][1]) > 0
    for n in res["1"][1]:
        if two:
            torch.testing.assert_close(res["1"][1][n], res["0"][1][n], rtol=1e-5, atol=1e-6,
                                       msg=n)
        else:  # one relation per type: every table gradient is a single add either way
            assert torch.equal(res["1"][1][n], res["0"][1][n]), n
    # the fold: the same layer up to fp32 reassociation (W_s (W_e x) = (W_s W_e) x)
    torch.testing.assert_close(res["fold"][0], res["1"][0], rtol=1e-5, atol=1e-6)
    assert res["fold"][1].keys() == res["1"][1].keys()
    for n in res["1"][1]:
        torch.testing.assert_close(res["fold"][1][n], res["1"][1][n], rtol=1e-4, atol=2e-6,
                                   msg=n)
