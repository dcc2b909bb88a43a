"""Every BASELINE.json config at its full size on the GPU, against the CPU oracle.

  C1  1k users x 1k items, 10k click edges, n_layers=2 + NodeEmbedding (one 'mean' conv
      layer), d=32, EdgeDataLoader batch 1024 x K=10 negatives: a whole training epoch,
      every batch's scores and loss against oracle.model_blocks + cosine + max_margin_loss
      (reference src/train/run.py:89-138, src/model.py:415-533).
  C2  1M users x 100k items, 50M edges per direction: the in-CSR of both relations
      bit-exact against oracle.csr_from_coo, the fanout-[10,10] sampler bit-exact against
      oracle.sample_neighbors + to_block_relabel for 2560 seeds, a 2-layer d=64 forward on
      those blocks, and two training steps (reference src/sampling.py:153-241).
  C3  the same graph, mean_nn d=128 + cosine head on 1024 pos x 2500 neg: scores and loss
      (n_layers=3: two conv layers, the reference's convention with embedding_layer; and
      n_layers=4: three conv layers).
  C4/C5  the 500M-edge full-graph pass (bench.py's workload; C5 = 80 % clicks / 20 % buys,
      4 relations, hetero sum and the build-defined attention; C4 with Zipf-1.0 items): every
      layer of the sharded pass checked on a 1/32 slice of each node type + 1000 random rows
      (+ the 100 heaviest items under Zipf) — the layer's GPU inputs for the
      sampled rows' in-neighbourhoods go through oracle.hetero_conv and must give the GPU's
      outputs.  The neighbour lists come from re-generating the edge stream (synth_edges,
      bit-exact to the oracle's generator) and filtering it, not from the product's CSR.

Tolerance: rtol 1e-4, atol 1e-5 (north star); sampled index sets and CSRs bit-exact."""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-4, 1e-5
DEV = "cuda"
BUYS = ("user", "buys", "item")
BOUGHT = ("item", "bought-by", "user")
CLICKS = ("user", "clicks", "item")
CLICKED = ("item", "clicked-by", "user")
REV = {"buys": "bought-by", "bought-by": "buys", "clicks": "clicked-by", "clicked-by": "clicks"}


def _np(t):
    return t.detach().cpu().numpy()


def _oracle_blocks(blocks, occurrence=None):
    return [oracle.BlockGraph({ce: tuple(_np(t) for t in b._rels[ce]) for ce in b.canonical_etypes},
                              {nt: b.number_of_dst_nodes(nt) for nt in b.ntypes}, occurrence)
            for b in blocks]


def _sd(model):
    return {k: _np(v) for k, v in model.state_dict().items()}


def _check_step(model, blocks, pos_g, neg_g, agg, hagg, K, delta=0.266, recency=None,
                neg_mask=None):
    """One training-step forward + loss on the GPU vs the oracle on the same blocks and
    weights; returns the GPU loss (graph attached) for the caller's backward."""
    from gnnrec import nn as gnn
    h, ps, ns = model(blocks, dict(blocks[0].srcdata["features"]), pos_g, neg_g, True)
    kw = {}
    if recency is not None:
        kw.update(use_recency=True, recency_scores=recency)
    if neg_mask is not None:
        kw.update(remove_false_negative=True, negative_mask=neg_mask)
    loss = gnn.max_margin_loss(ps, ns, delta, K, **kw)
    sd = _sd(model)
    feats = {nt: _np(v) for nt, v in blocks[0].srcdata["features"].items()}
    rh = oracle.model_blocks(_oracle_blocks(blocks), feats, sd, agg, hagg, True, True)
    for nt in rh:
        np.testing.assert_allclose(_np(h[nt]), rh[nt], rtol=RTOL, atol=ATOL)
    pos = {ce: tuple(_np(t) for t in pos_g.all_edges(etype=ce)) for ce in pos_g.canonical_etypes}
    neg = {ce: tuple(_np(t) for t in neg_g.all_edges(etype=ce)) for ce in neg_g.canonical_etypes}
    rps, rns = oracle.cosine_prediction(pos, rh), oracle.cosine_prediction(neg, rh)
    assert set(rps) == set(ps) and set(rns) == set(ns)
    for ce in rps:
        np.testing.assert_allclose(_np(ps[ce]), rps[ce], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(_np(ns[ce]), rns[ce], rtol=RTOL, atol=ATOL)
    rl = oracle.max_margin_loss(
        rps, rns, delta, K, use_recency=recency is not None,
        recency=None if recency is None else {ce: _np(v) for ce, v in recency.items()},
        remove_false_negative=neg_mask is not None,
        mask=None if neg_mask is None else {ce: _np(v) for ce, v in neg_mask.items()})
    np.testing.assert_allclose(float(loss), rl, rtol=RTOL, atol=ATOL)
    return loss


# ------------------------------------------------------------------------- C1 ---
def test_c1_training_epoch_matches_oracle():
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph, NID
    from gnnrec.sampling import EdgeDataLoader, MultiLayerFullNeighborSampler, negative_sampler
    n_u, n_i, E, K = 1000, 1000, 10_000, 10
    u, i = oracle.synth_edges(11, 0, E, n_u, n_i)
    u, i = u.astype(np.int64), i.astype(np.int64)
    edges = {CLICKS: (u, i), CLICKED: (i, u)}
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d)) for ce, (s, d) in edges.items()},
                    {"user": n_u, "item": n_i}, device=DEV)
    rng = np.random.default_rng(1)
    # reference-shaped binary node features (src/builder.py:426-431,444-450): user 2, item 4
    g.nodes["user"].data["features"] = torch.from_numpy(
        rng.integers(0, 2, (n_u, 2)).astype(np.float32)).to(DEV)
    g.nodes["item"].data["features"] = torch.from_numpy(
        rng.integers(0, 2, (n_i, 4)).astype(np.float32)).to(DEV)
    g.edges[CLICKS].data["recency"] = torch.from_numpy(rng.integers(1, 30, E)).to(DEV)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 2, {"user": 2, "item": 4, "hidden": 32, "out": 32}, True, 0.0,
                          "mean", "cos", "sum", True).to(DEV).train()
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    loader = EdgeDataLoader(g, {CLICKS: torch.arange(E)}, MultiLayerFullNeighborSampler(1),
                            exclude="reverse_types", reverse_etypes=REV,
                            negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                            shuffle=True)
    pairs = set(zip(u.tolist(), i.tolist()))
    n = 0
    for _, pos_g, neg_g, blocks in loader:
        # negative mask as reference run.py:92-101: has_edges_between on global ids
        nids = neg_g.ndata[NID]
        ns_, nd_ = neg_g.all_edges(etype=CLICKS)
        gs, gd = nids["user"][ns_], nids["item"][nd_]
        mask = g.has_edges_between(gs, gd, etype=CLICKS).float()
        np.testing.assert_array_equal(
            _np(mask), np.array([(a, b) in pairs for a, b in zip(_np(gs), _np(gd))], np.float32))
        masks = {ce: (mask if ce == CLICKS else torch.zeros(0, device=DEV))
                 for ce in pos_g.canonical_etypes}
        rec = {ce: pos_g.edata["recency"][ce] for ce in pos_g.canonical_etypes
               if "recency" in pos_g._edata[ce]}
        loss = _check_step(model, blocks, pos_g, neg_g, "mean", "sum", K, recency=rec,
                           neg_mask=masks)
        opt.zero_grad()
        loss.backward()
        opt.step()
        n += 1
    assert n == len(loader) == 10


# ---------------------------------------------------------------------- C2/C3 ---
@pytest.fixture(scope="module")
def c2_graph():
    from gnnrec import ops
    from gnnrec.graph import HeteroGraph
    n_u, n_i, E = 1_000_000, 100_000, 50_000_000
    u, i = ops.synth_edges(11, 0, E, n_u, n_i, DEV)
    u, i = u.long(), i.long()
    g = HeteroGraph({BUYS: (u, i), BOUGHT: (i, u)}, {"user": n_u, "item": n_i}, device=DEV)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(0)
    g.edges["buys"].data["recency"] = torch.randint(1, 30, (E,), device=DEV, generator=gen)
    feats = {d: {"user": torch.randn(n_u, d, generator=gen, device=DEV),
                 "item": torch.randn(n_i, d, generator=gen, device=DEV)} for d in (64, 128)}
    yield g, feats
    del g, feats
    torch.cuda.empty_cache()


def _set_feats(g, feats):
    for nt, x in feats.items():
        g.nodes[nt].data["features"] = x


def test_c2_csr_and_fanout_sampler_bit_exact(c2_graph):
    from gnnrec import nn as gnn
    from gnnrec.graph import NID
    from gnnrec.sampling import MultiLayerNeighborSampler, _mix
    g, feats = c2_graph
    _set_feats(g, feats[64])
    # the device CSR (row f3) against the oracle's stable COO -> CSR
    csr = {}
    for ce in g.canonical_etypes:
        s, d = g.all_edges(etype=ce)
        ref = oracle.csr_from_coo(_np(s), _np(d), g.num_nodes(ce[2]))
        got = [_np(t) for t in g.in_csr(ce)]
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)
        csr[ce] = ref
    gen = torch.Generator(device=DEV)
    gen.manual_seed(9)
    seeds = {"user": torch.randperm(1_000_000, device=DEV, generator=gen)[:2048],
             "item": torch.randperm(100_000, device=DEV, generator=gen)[:512]}
    sampler = MultiLayerNeighborSampler([10, 10], seed=7)
    blocks = sampler.sample_blocks(g, seeds)
    calls = sampler._calls
    cur = {nt: _np(v) for nt, v in seeds.items()}
    empty = np.zeros(0, np.int64)
    for block_id in reversed(range(2)):
        b = blocks[block_id]
        src_lists = {}
        for r_idx, ce in enumerate(g.canonical_etypes):
            ip, ix, e = csr[ce]
            key = _mix(sampler.seed, calls, block_id, r_idx)
            oip, osrc, oe = oracle.sample_neighbors(ip, ix, e, cur.get(ce[2], empty), 10, key)
            gip, gloc, ge = (_np(t) for t in b._rels[ce])
            np.testing.assert_array_equal(gip, oip)
            np.testing.assert_array_equal(ge, oe)
            np.testing.assert_array_equal(_np(b.srcdata[NID][ce[0]])[gloc], osrc)
            assert (np.diff(oip) <= 10).all()
            src_lists.setdefault(ce[0], []).append((ce, osrc, gloc))
        nxt = {}
        for nt in ("user", "item"):
            pref = cur.get(nt, empty)
            lists = src_lists.get(nt, [])
            nodes, locs = oracle.to_block_relabel(pref, [x[1] for x in lists])
            np.testing.assert_array_equal(_np(b.srcdata[NID][nt]), nodes)
            for (_, _, gloc), loc in zip(lists, locs):
                np.testing.assert_array_equal(gloc, loc)
            assert b.number_of_dst_nodes(nt) == pref.size
            if nodes.size:
                nxt[nt] = nodes
        cur = nxt
    # a 2-layer 'mean' d=64 forward on those blocks (n_layers=3 with NodeEmbedding)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(DEV).eval()
    with torch.no_grad():
        h = model.get_repr(blocks, model.embed(dict(blocks[0].srcdata["features"])))
    rh = oracle.model_blocks(_oracle_blocks(blocks),
                             {nt: _np(v) for nt, v in blocks[0].srcdata["features"].items()},
                             _sd(model), "mean", "sum", True, True)
    assert set(h) == set(rh)
    for nt in rh:
        assert rh[nt].shape[0] == seeds[nt].numel()
        np.testing.assert_allclose(_np(h[nt]), rh[nt], rtol=RTOL, atol=ATOL)


def _edge_loader(g, fanouts, K):
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    return EdgeDataLoader(g, {BUYS: torch.arange(g.num_edges(BUYS))},
                          MultiLayerNeighborSampler(fanouts, seed=3), exclude="reverse_types",
                          reverse_etypes=REV, negative_sampler=negative_sampler.Uniform(K),
                          batch_size=1024, shuffle=True)


def test_c2_training_steps_match_oracle(c2_graph):
    from gnnrec import nn as gnn
    g, feats = c2_graph
    _set_feats(g, feats[64])
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(DEV).train()
    opt = torch.optim.Adam(model.parameters(), lr=0.005)
    K = 10
    it = iter(_edge_loader(g, [10, 10], K))
    for _ in range(2):
        _, pos_g, neg_g, blocks = next(it)
        rec = {BUYS: pos_g.edata["recency"][BUYS]}
        loss = _check_step(model, blocks, pos_g, neg_g, "mean", "sum", K, recency=rec)
        opt.zero_grad()
        loss.backward()
        opt.step()


def test_c2_k2500_default_fold_gradients_match_unfolded(c2_graph, monkeypatch):
    """C2 at the reference's K = 2500: the first block has ~960k source rows, above
    FOLD_MIN_SRC_ROWS, so the DEFAULT mode (GNNREC_TRAIN_FOLD unset = 'auto') folds the
    NodeEmbeddings into the first layer — (W_s W_e) x instead of W_s (W_e x).  Its loss and
    every parameter gradient against the unfolded order (embed every source row, aggregate,
    project; src/model.py:10-24, 143-148, 226-235) on the same blocks: fp32-reassociation
    close (rtol 1e-4, the north star's tolerance), not bitwise."""
    from gnnrec import nn as gnn
    g, feats = c2_graph
    _set_feats(g, feats[64])
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(DEV).train()
    K = 2500
    _, pos_g, neg_g, blocks = next(iter(_edge_loader(g, [10, 10], K)))
    n_src = sum(blocks[0].number_of_src_nodes(nt) for nt in blocks[0].ntypes)
    assert n_src >= gnn.FOLD_MIN_SRC_ROWS, n_src
    res = {}
    for mode in ("auto", "0"):
        if mode == "auto":
            monkeypatch.delenv("GNNREC_TRAIN_FOLD", raising=False)
        else:
            monkeypatch.setenv("GNNREC_TRAIN_FOLD", "0")
        model.zero_grad()
        folded = model._folded_first_layer(blocks, blocks[0].srcdata["features"]) is not None
        assert folded == (mode == "auto")
        model.zero_grad()
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, {BUYS: pos_g.edata["recency"][BUYS]})
        loss.backward()
        res[mode] = (loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()
                                     if p.grad is not None})
    assert res["auto"][1].keys() == res["0"][1].keys()
    torch.testing.assert_close(res["auto"][0], res["0"][0], rtol=1e-4, atol=1e-7)
    for n in res["auto"][1]:
        torch.testing.assert_close(res["auto"][1][n], res["0"][1][n], rtol=1e-4, atol=1e-6,
                                   msg=n)


def _real_blocks(blocks):
    """A static batch's blocks cut to their real rows for the oracle: the real destination
    rows come first (the seeds), their edges are the CSR prefix [0, indptr[n_real]) and point
    only at the real source rows (the sampler's static-shape contract, include/gnnrec.h)."""
    out = []
    for b in blocks:
        n_dst = {nt: int(b._live[("dst", nt)]) for nt in b.ntypes}
        rels = {}
        for ce in b.canonical_etypes:
            ip, loc, eid = (_np(t) for t in b._rels[ce])
            n = n_dst[ce[2]]
            e = int(ip[n])
            n_src = int(b._live[("src", ce[0])])
            assert (loc[:e] < n_src).all() and (eid[:e] >= 0).all()
            rels[ce] = (ip[:n + 1].copy(), loc[:e].copy(), eid[:e].copy())
        out.append(oracle.BlockGraph(rels, n_dst))
    return out


@pytest.mark.parametrize("K,caps", [(10, "provable"), (2500, "auto")])
def test_c2_captured_static_steps_match_oracle(c2_graph, K, caps):
    """The path bench.py's captured minibatch numbers run (bench.captured_step): the C2 graph,
    EdgeDataLoader(static_shapes=True) with its sampling thread — padding rows, dump rows of
    <= 2048 edges, learned capacities at K = 2500 — and CapturedTrainStep (hipGraph replay,
    the first-layer fold forced on).  For three replayed steps, the step's forward embeddings
    (real rows), positive / negative scores and loss against oracle.model_blocks +
    cosine_prediction + max_margin_loss on the batch's real rows, with the weights the step
    started from (reference src/train/run.py:89-138, src/sampling.py:153-165).  The fold
    reassociates fp32 products (W_s W_e) x: rtol 1e-4, the north star's tolerance."""
    from gnnrec import nn as gnn
    from gnnrec import ops
    from gnnrec.capture import CapturedTrainStep
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    g, feats = c2_graph
    _set_feats(g, feats[64])
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(DEV)
    model.train_fold = "1"
    opt = torch.optim.Adam(model.parameters(), lr=0.005, fused=True)
    captured = {}

    def loss_fn(m, batch):
        _, pos_g, neg_g, blocks = batch
        h, ps, ns = m(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        if torch.cuda.is_current_stream_capturing():  # the graph's own output tensors
            captured["out"] = (h, ps, ns)
        return gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])

    step = CapturedTrainStep(model, opt, loss_fn, warmup=2)
    el = EdgeDataLoader(g, {BUYS: torch.arange(g.num_edges(BUYS))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes=REV, negative_sampler=negative_sampler.Uniform(K),
                        batch_size=1024, shuffle=True, num_workers=2, static_shapes=True,
                        static_caps=caps)
    el.sampler.first_transposes_below = 0
    before = ops.plan_overflows()
    checked = 0
    for batch in el:
        sd = _sd(model)  # the weights this step starts from
        r0 = step.replays
        loss = step(batch)
        if step.replays == r0:
            continue
        torch.cuda.synchronize()
        _, pos_g, neg_g, blocks = batch
        assert pos_g.static and all(b.static for b in blocks)
        h, ps, ns = captured["out"]
        rb = _real_blocks(blocks)
        n_src0 = {nt: int(blocks[0]._live[("src", nt)]) for nt in blocks[0].ntypes}
        x = {nt: _np(v)[:n_src0[nt]] for nt, v in blocks[0].srcdata["features"].items()}
        rh = oracle.model_blocks(rb, x, sd, "mean", "sum", True, True)
        for nt in rh:
            n = rh[nt].shape[0]
            assert n == int(blocks[-1]._live[("dst", nt)])
            np.testing.assert_allclose(_np(h[nt])[:n], rh[nt], rtol=RTOL, atol=ATOL,
                                       err_msg=f"replay {checked}: {nt} embeddings")
        pos = {ce: tuple(_np(t) for t in pos_g.all_edges(etype=ce)) for ce in pos_g.canonical_etypes}
        neg = {ce: tuple(_np(t) for t in neg_g.all_edges(etype=ce)) for ce in neg_g.canonical_etypes}
        rps, rns = oracle.cosine_prediction(pos, rh), oracle.cosine_prediction(neg, rh)
        for ce in rps:
            np.testing.assert_allclose(_np(ps[ce]), rps[ce], rtol=RTOL, atol=ATOL)
            np.testing.assert_allclose(_np(ns[ce]), rns[ce], rtol=RTOL, atol=ATOL)
        rec = {ce: _np(v) for ce, v in pos_g.edata["recency"].items()}
        rl = oracle.max_margin_loss(rps, rns, 0.266, K, use_recency=True, recency=rec)
        np.testing.assert_allclose(float(loss), rl, rtol=RTOL, atol=ATOL)
        print(f"  K={K} replay {checked}: loss {float(loss):.6f} (oracle {rl:.6f}), "
              f"{sum(v.shape[0] for v in rh.values())} output rows", flush=True)
        checked += 1
        if checked == 3:
            break
    assert checked == 3 and step.captures == 1
    assert ops.plan_overflows() == before
    del el


@pytest.mark.parametrize("n_layers", [3, 4])
def test_c3_mean_nn_cosine_1024x2500_matches_oracle(c2_graph, n_layers):
    from gnnrec import nn as gnn
    g, feats = c2_graph
    _set_feats(g, feats[128])
    torch.manual_seed(0)
    model = gnn.ConvModel(g, n_layers, {"user": 128, "item": 128, "hidden": 128, "out": 128},
                          True, 0.0, "mean_nn", "cos", "sum", True).to(DEV).train()
    K = 2500
    _, pos_g, neg_g, blocks = next(iter(_edge_loader(g, [10] * (n_layers - 1), K)))
    assert pos_g.num_edges(BUYS) == 1024 and neg_g.num_edges(BUYS) == 1024 * K
    loss = _check_step(model, blocks, pos_g, neg_g, "mean_nn", "sum", K)
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all()
               for n, p in model.named_parameters() if "pred_fn" not in n)


# ---------------------------------------------------------------------- C4/C5 ---
N_U, N_I, N_E, D = 10_000_000, 1_000_000, 500_000_000, 128
SPLITS = {"c4": (("buys", "bought-by", 1.0),),
          "c5": (("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2))}


def _neighbour_lists(split, rows_u, rows_i, chunk=1 << 26, cdf=None):
    """In-edges (eid order) of the sampled user rows (relations item -> user) and item rows
    (user -> item), from the regenerated edge stream: {ce: (indptr, src global, eids)}.
    cdf: the item Zipf CDF of a skewed stream (bench --zipf)."""
    from gnnrec import ops
    from gnnrec.synth import relation_pairs
    pairs = relation_pairs(split)
    sel = {}
    for rows, n in ((rows_u, N_U), (rows_i, N_I)):  # membership tables of the sampled rows
        m = torch.zeros(n, dtype=torch.bool, device=DEV)
        m[rows] = True
        sel[n] = m
    bounds = [0]
    for _, _, frac in pairs:
        bounds.append(min(N_E, bounds[-1] + int(round(frac * N_E))))
    bounds[-1] = N_E
    out = {}
    for (fwd, rev, _), lo, hi in zip(pairs, bounds[:-1], bounds[1:]):
        acc = {fwd: ([], [], []), rev: ([], [], [])}
        for e0 in range(lo, hi, chunk):
            n = min(chunk, hi - e0)
            u, i = ops.synth_edges(11, e0, n, N_U, N_I, DEV, cdf)
            u, i = u.long(), i.long()
            for ce, dst, src, rows in ((rev, u, i, rows_u), (fwd, i, u, rows_i)):
                m = torch.nonzero(sel[N_U if rows is rows_u else N_I][dst]).squeeze(1)
                acc[ce][0].append(torch.searchsorted(rows, dst[m]))
                acc[ce][1].append(src[m])
                acc[ce][2].append(m + (e0 - lo))
        for ce, (d, s, e) in acc.items():
            d, s, e = (_np(torch.cat(x)) for x in (d, s, e))
            ip, _, order = oracle.csr_from_coo_c(np.zeros_like(d), d, (rows_u if ce == rev
                                                                      else rows_i).numel())
            out[ce] = (ip, s[order], e[order])
    return out


def _layer_rows_vs_oracle(model, layer_idx, h_in, h_out, lists, rows, hetero, raw_feats=None):
    """Layer `layer_idx`'s outputs of the sampled rows against oracle.hetero_conv over their
    in-neighbourhoods, fed with the layer's GPU inputs (NodeEmbedding applied on the CPU for
    the first layer, whose GPU inputs are the raw features folded into the kernels)."""
    sd = _sd(model)
    _, layers, _ = oracle.split_state_dict(sd)
    lw = layers[layer_idx]

    def rows_of(nt, ids):
        x = _np(h_in[nt][torch.from_numpy(ids).to(DEV)])
        return oracle.embed_inputs({nt: x}, sd)[nt] if raw_feats else x

    for T, S in (("user", "item"), ("item", "user")):
        ces = [ce for ce in lists if ce[2] == T]
        # the sampled rows' distinct sources and every edge's position among them (on the
        # device: ~190M edges under Zipf, where numpy's unique + searchsorted take minutes)
        allsrc = torch.from_numpy(np.concatenate([lists[ce][1] for ce in ces])).to(DEV)
        uq, inv = torch.unique(allsrc, return_inverse=True)
        uniq, inv = _np(uq), _np(inv.to(torch.int32))
        del allsrc, uq
        rels, o = {}, 0
        for ce in ces:
            n = lists[ce][1].size
            rels[ce] = (lists[ce][0], inv[o:o + n], lists[ce][2])
            o += n
        print(f"  layer {layer_idx} {T}: {rows[T].size} rows, {o} in-edges, {uniq.size} sources",
              flush=True)
        blk = oracle.BlockGraph(rels, {T: rows[T].size})
        ref = oracle.hetero_conv(blk, {S: rows_of(S, uniq)}, lw, "mean", True, hetero,
                                 {T: rows_of(T, rows[T])})[T]
        got = _np(h_out[T][torch.from_numpy(rows[T]).to(DEV)])
        np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL, err_msg=f"layer {layer_idx} {T}")


@pytest.fixture(scope="module", params=["c4", "c5", "c4zipf"])
def full_shard(request):
    """The full-size shard plus the rows checked against the oracle: a contiguous slice
    per node type — 1/32 of the users (312,500: the slice bench.cpu_baseline times) and
    1/16 of the items (62,500: at least 50k rows of each type) — and 1000 random rows;
    with --zipf 1.0 items also the 100 heaviest, whose
    ~180M in-edges (the top item ~35M) run through the chunked heavy-row tiles
    (inference.TILE_SPLIT) and their 16-partial combine."""
    from gnnrec.synth import bipartite_shard, node_features, zipf_cdf
    cfg = request.param
    zipf = 1.0 if cfg == "c4zipf" else 0.0
    split = SPLITS["c5" if cfg == "c5" else "c4"]
    shard = bipartite_shard(N_U, N_I, N_E, 0, 1, torch.device(DEV), split=split, segments=8,
                            zipf_s=zipf)
    feats = {"user": node_features(N_U, D, 0, DEV), "item": node_features(N_I, D, 1, DEV)}
    gen = torch.Generator(device=DEV)
    gen.manual_seed(5)
    rows = {}
    for nt, n in (("user", N_U), ("item", N_I)):
        # (under Zipf the item ids are popularity ranks: the first 1/32 of them hold ~3/4 of
        # the edges, so the item slice is taken from the light end there)
        m = n // 16 if nt == "item" else n // 32
        lo = n - m if zipf and nt == "item" else 0
        pick = [torch.arange(lo, lo + m, device=DEV),
                torch.randperm(n, device=DEV, generator=gen)[:1000]]
        if zipf and nt == "item":
            deg = shard.rels[("user", "buys", "item")].deg_own[:N_I].long()
            pick.append(torch.topk(deg, 100).indices)
        rows[nt] = torch.unique(torch.cat(pick))  # sorted
    cdf = zipf_cdf(N_I, zipf, DEV) if zipf else None
    print(f"[{cfg}] shard built; neighbour lists of {rows['user'].numel()} users and "
          f"{rows['item'].numel()} items", flush=True)
    lists = _neighbour_lists(split, rows["user"], rows["item"], cdf=cdf)
    if zipf:  # the heavy rows really are in the checked set, with their whole in-edge lists
        ip = lists[("user", "buys", "item")][0]
        assert int(np.diff(ip).max()) > 30_000_000
    yield cfg, shard, feats, {nt: _np(v) for nt, v in rows.items()}, lists
    del shard, feats
    torch.cuda.empty_cache()


@pytest.mark.parametrize("hetero", ["sum", "attention"])
def test_full_size_pass_layers_match_oracle(full_shard, hetero):
    from gnnrec import nn as gnn
    from gnnrec.dist import Exchange
    from gnnrec.inference import ShardedFullGraphPass
    from gnnrec.synth import GraphMeta
    config, shard, feats, rows, lists = full_shard
    if config != "c5" and hetero == "attention":
        pytest.skip("C4 has one relation per destination type: attention == identity weights")
    # degree conservation of the product's CSRs: every edge lands in one row
    for ce, rs in shard.rels.items():
        assert int(rs.indptr[-1]) == rs.global_edges
    torch.manual_seed(0)
    meta = GraphMeta(shard.canonical_etypes, ["item", "user"])
    model = gnn.ConvModel(meta, 3, {"user": D, "item": D, "hidden": D, "out": D}, True, 0.0,
                          "mean", "cos", hetero, True).to(DEV).eval()
    runner = ShardedFullGraphPass(model, shard, Exchange(), deterministic=True)
    runner.capture = []
    runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    assert len(runner.capture) == 2
    assert runner.fused or runner.pair_fused, \
        "the C4/C5 pass must run a fused aggregate+project kernel"
    if config == "c5" and hetero == "sum":  # clicked-by + bought-by as one launch
        assert len(runner.pair_fused) == 1
    h1, h2 = runner.capture
    if config == "c4zipf":
        # The Zipf head items have up to ~35M in-edges.  DGL's CPU SpMM (the f32 oracle)
        # keeps ONE sequential fp32 running sum per row: at layer 2 the terms are post-ReLU
        # rows of unit norm, the running sum of a head item reaches ~1e6, whose fp32 ulp
        # (0.06-0.125) exceeds the terms themselves, and the sum stagnates — the
        # reference's own arithmetic is off by up to ~1e-2 there.  The HIP path sums
        # 512-edge chunks and folds the chunk partials, so it is checked against the exact
        # aggregate (double accumulator) at the same 1e-4; the f32 oracle's distance on the
        # head rows is printed beside it.
        with oracle.accumulate_f64():
            _layer_rows_vs_oracle(model, 0, feats, h1, lists, rows, hetero, raw_feats=True)
            _layer_rows_vs_oracle(model, 1, h1, h2, lists, rows, hetero)
        _head_rows_f32_vs_f64(model, h1, h2, lists, rows)
        return
    _layer_rows_vs_oracle(model, 0, feats, h1, lists, rows, hetero, raw_feats=True)
    _layer_rows_vs_oracle(model, 1, h1, h2, lists, rows, hetero)


def _head_rows_f32_vs_f64(model, h1, h2, lists, rows, n_head=20):
    """Layer 2 of the heaviest sampled items three ways — the HIP pass, the f32-sequential
    oracle (DGL's CPU arithmetic) and the double-accumulator oracle — printed, so the
    record shows which side of a Zipf-head mismatch the reference's rounding is on."""
    ce = ("user", "buys", "item")
    ip, src, _ = lists[ce]
    deg = np.diff(ip)
    head = np.argsort(-deg)[:n_head]  # positions in rows['item']
    sub_ip = np.concatenate([[0], np.cumsum(deg[head])]).astype(np.int64)
    sub_src = np.concatenate([src[ip[k]:ip[k + 1]] for k in head])
    uq, inv = torch.unique(torch.from_numpy(sub_src).to(DEV), return_inverse=True)
    x = _np(h1["user"][uq])
    inv = _np(inv.to(torch.int32))
    w = oracle.split_state_dict(_sd(model))[1][1]["buys"]
    ids = rows["item"][head]
    h_self = _np(h1["item"][torch.from_numpy(ids).to(DEV)])
    blk = oracle.BlockGraph({ce: (sub_ip, inv, np.arange(inv.size))}, {"item": head.size})
    z32 = oracle.conv_layer(blk, ce, x, h_self, w, "mean", True)
    with oracle.accumulate_f64():
        z64 = oracle.conv_layer(blk, ce, x, h_self, w, "mean", True)
    got = _np(h2["item"][torch.from_numpy(ids).to(DEV)])
    scale = np.abs(z64).max()
    print(f"  Zipf head items (degrees {deg[head].max()}..{deg[head].min()}): max |HIP - exact| "
          f"= {np.abs(got - z64).max():.2e}, max |f32 oracle - exact| = "
          f"{np.abs(z32 - z64).max():.2e} (outputs up to {scale:.3f})", flush=True)
    np.testing.assert_allclose(got, z64, rtol=RTOL, atol=ATOL)
