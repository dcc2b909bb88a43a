"""GPU tests of the minibatch side (rows a9/a10, f2): block sampler, NodeDataLoader,
EdgeDataLoader (reverse-type exclusion, uniform negatives, compaction) and a
training step through the autograd Functions.

Reference semantics restated from DGL 0.5.2: full-neighbour
blocks are checked as exact index SETS against a Python restatement; the
minibatch embedding loop (reference src/train/run.py:311-349) must equal the
layer-wise full-graph pass when every node has in-degree >= 1 in every relation
(the relation-skip trap of SURVEY §2.3.2 does not bite then)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

BUYS = ("user", "buys", "item")
BOUGHT = ("item", "bought-by", "user")
CLICKS = ("user", "clicks", "item")
CLICKED = ("item", "clicked-by", "user")


def _graph(n_u=60, n_i=40, e_b=400, e_c=500, seed=0, min_deg=True):
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(seed)
    def rel(n):
        s = rng.integers(0, n_u, n)
        d = rng.integers(0, n_i, n)
        if min_deg:  # every user and item appears in every relation
            s[:n_u] = np.arange(n_u)
            d[:n_i] = np.arange(n_i)
        return s, d
    bs, bd = rel(e_b)
    cs, cd = rel(e_c)
    edges = {BUYS: (bs, bd), BOUGHT: (bd, bs), CLICKS: (cs, cd), CLICKED: (cd, cs)}
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d)) for ce, (s, d) in edges.items()},
                    {"user": n_u, "item": n_i}, device=DEV)
    occ_b = torch.from_numpy(rng.integers(1, 9, e_b)).to(DEV)
    occ_c = torch.from_numpy(rng.integers(1, 9, e_c)).to(DEV)
    for ce, o in ((BUYS, occ_b), (BOUGHT, occ_b), (CLICKS, occ_c), (CLICKED, occ_c)):
        g.edges[ce].data["occurrence"] = o
    g.edges[BUYS].data["recency"] = torch.from_numpy(rng.integers(1, 30, e_b)).to(DEV)
    for nt, n, dd in (("user", n_u, 5), ("item", n_i, 6)):
        g.nodes[nt].data["features"] = torch.from_numpy(
            rng.standard_normal((n, dd)).astype(np.float32)).to(DEV)
    return g, edges


def _model(g, agg="mean_nn_edge", hetero="sum", emb=True, n_layers=3, pred="cos"):
    from gnnrec import nn as gnn
    torch.manual_seed(0)
    m = gnn.ConvModel(g, n_layers, {"user": 5, "item": 6, "hidden": 16, "out": 8}, True, 0.0, agg,
                      pred, hetero, emb)
    return m.to(DEV)


def test_full_neighbor_block_sets_match_restatement():
    from gnnrec.graph import NID
    from gnnrec.sampling import MultiLayerFullNeighborSampler
    g, edges = _graph(min_deg=False)
    sampler = MultiLayerFullNeighborSampler(2)
    seeds = {"user": torch.tensor([3, 7, 11], device=DEV), "item": torch.tensor([0, 5], device=DEV)}
    blocks = sampler.sample_blocks(g, seeds)
    assert len(blocks) == 2
    # restatement: in-edges of the seeds, sources = dst prefix + new ids ascending
    cur = {nt: v.cpu().numpy() for nt, v in seeds.items()}
    for b in reversed(blocks):
        for nt in ("user", "item"):
            pref = cur.get(nt, np.zeros(0, np.int64))
            assert b.number_of_dst_nodes(nt) == pref.size
            np.testing.assert_array_equal(b.srcdata[NID][nt][: pref.size].cpu().numpy(), pref)
        new_src = {}
        for ce, (s, d) in edges.items():
            dseeds = cur.get(ce[2], np.zeros(0, np.int64))
            indptr, idx, eids = b._rels[ce]
            ip = indptr.cpu().numpy()
            src_nodes = b.srcdata[NID][ce[0]].cpu().numpy()
            got = set()
            for k, v in enumerate(dseeds):
                loc = idx[ip[k]:ip[k + 1]].cpu().numpy()
                e = eids[ip[k]:ip[k + 1]].cpu().numpy()
                assert (d[e] == v).all() and (s[e] == src_nodes[loc]).all()
                got |= set(e.tolist())
            want = set(np.nonzero(np.isin(d, dseeds))[0].tolist())
            assert got == want, ce
            new_src.setdefault(ce[0], set()).update(s[list(want)].tolist())
        for nt in ("user", "item"):
            pref = cur.get(nt, np.zeros(0, np.int64))
            new = sorted(set(new_src.get(nt, set())) - set(pref.tolist()))
            np.testing.assert_array_equal(b.srcdata[NID][nt][pref.size:].cpu().numpy(), new)
        cur = {nt: b.srcdata[NID][nt].cpu().numpy() for nt in ("user", "item")
               if b.number_of_src_nodes(nt) > 0}


@pytest.mark.parametrize("agg,hetero,pred", [("mean_nn_edge", "sum", "cos"), ("pool_nn", "max", "nn"),
                                             ("mean", "mean", "cos")])
def test_minibatch_embeddings_equal_full_graph_pass(agg, hetero, pred):
    from gnnrec.inference import full_graph_embeddings, get_embeddings
    from gnnrec.sampling import MultiLayerFullNeighborSampler, NodeDataLoader
    g, _ = _graph()
    model = _model(g, agg, hetero, pred=pred).eval()
    full = full_graph_embeddings(g, model)
    loader = NodeDataLoader(g, {"user": torch.arange(60), "item": torch.arange(40)},
                            MultiLayerFullNeighborSampler(2), batch_size=16, shuffle=True)
    y = get_embeddings(g, 8, model, loader, embedding_layer=True)
    for nt in ("user", "item"):
        np.testing.assert_allclose(y[nt].cpu().numpy(), full[nt].cpu().numpy(), rtol=1e-5,
                                   atol=1e-6)


def test_fanout_sampler_structure():
    from gnnrec.sampling import MultiLayerNeighborSampler
    g, edges = _graph(n_u=200, n_i=100, e_b=5000, e_c=5000, min_deg=False)
    sampler = MultiLayerNeighborSampler([3, 2], seed=5)
    seeds = {"user": torch.arange(0, 200, 7, device=DEV)}
    b_last = sampler.sample_blocks(g, seeds)[-1]
    for ce, (s, d) in edges.items():
        if ce[2] != "user":
            continue
        indptr, idx, eids = b_last._rels[ce]
        ip = indptr.cpu().numpy()
        e_all = eids.cpu().numpy()
        for k, v in enumerate(seeds["user"].cpu().numpy()):
            e = e_all[ip[k]:ip[k + 1]]
            assert len(set(e.tolist())) == e.size
            assert (d[e] == v).all()
            assert e.size == min(2, int((d == v).sum()))


def test_edge_loader_exclusion_negatives_and_training_step():
    from gnnrec import nn as gnn
    from gnnrec.graph import EID, NID
    from gnnrec.sampling import EdgeDataLoader, MultiLayerFullNeighborSampler, negative_sampler
    g, edges = _graph()
    K = 4
    loader = EdgeDataLoader(g, {BUYS: torch.arange(400), CLICKS: torch.arange(500)},
                            MultiLayerFullNeighborSampler(2), exclude='reverse_types',
                            reverse_etypes={'buys': 'bought-by', 'bought-by': 'buys',
                                            'clicks': 'clicked-by', 'clicked-by': 'clicks'},
                            negative_sampler=negative_sampler.Uniform(K), batch_size=64,
                            shuffle=True)
    model = _model(g).train()
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    n_batches = 0
    for input_nodes, pos_g, neg_g, blocks in loader:
        n_batches += 1
        # excluded: no block edge is a batch edge or its reverse
        for ce in (BUYS, CLICKS):
            be = pos_g._edata[ce].get(EID)
            if be is None:
                continue
            be = set(be.cpu().tolist())
            for b in blocks:
                for rel in (ce, {BUYS: BOUGHT, CLICKS: CLICKED}[ce]):
                    assert not (set(b._rels[rel][2].cpu().tolist()) & be)
            # positive pairs map back to the batch edges through the compacted ids
            s_l, d_l = pos_g.all_edges(etype=ce)
            s = pos_g.ndata[NID][ce[0]][s_l].cpu().numpy()
            d = pos_g.ndata[NID][ce[2]][d_l].cpu().numpy()
            e = pos_g._edata[ce][EID].cpu().numpy()
            np.testing.assert_array_equal(s, edges[ce][0][e])
            np.testing.assert_array_equal(d, edges[ce][1][e])
            ns, _ = neg_g.all_edges(etype=ce)
            assert ns.numel() == K * len(e)
            np.testing.assert_array_equal(ns.view(-1, K).cpu().numpy(), np.repeat(s_l.cpu().numpy()[:, None], K, 1))
        # seeds of the last block are the pair-graph nodes
        for nt in ("user", "item"):
            np.testing.assert_array_equal(blocks[-1].dstdata[NID][nt].cpu().numpy(),
                                          pos_g.ndata[NID][nt].cpu().numpy())
        h, ps, ns_ = model(blocks, blocks[0].srcdata['features'], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns_, 0.266, K, True, pos_g.edata['recency'])
        opt.zero_grad()
        loss.backward()
        assert all(p.grad is not None and torch.isfinite(p.grad).all()
                   for n, p in model.named_parameters() if 'pred_fn' not in n)
        opt.step()
    assert n_batches == len(loader) == (400 + 500 + 63) // 64


@pytest.mark.parametrize("K", [0, 4])
def test_fused_batch_head_matches_readable_form(K):
    """EdgeDataLoader's batch head as one C++ call (gnnrec::edge_batch_pairs) yields the same
    pair graphs, node ids and blocks bit for bit as find_edges + negative_sampler.Uniform +
    _compact, batch after batch (the same generator draws in the same order)."""
    from gnnrec.graph import NID
    from gnnrec.autograd import _joined
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    g, _ = _graph()

    def epoch(fused):
        torch.manual_seed(11)
        loader = EdgeDataLoader(g, {CLICKS: torch.arange(500), BUYS: torch.arange(400)},
                                MultiLayerNeighborSampler([3, 3], seed=5), exclude='self',
                                negative_sampler=negative_sampler.Uniform(K) if K else None,
                                batch_size=96, shuffle=True)
        assert loader.fused_head
        loader.fused_head = fused
        out = []
        for item in loader:
            pos_g, blocks = item[1], item[-1]
            neg_g = item[2] if K else None
            rec = {nt: pos_g.ndata[NID][nt].cpu() for nt in ("user", "item")}
            for ce in g.canonical_etypes:
                rec[("pos",) + ce] = [t.cpu() for t in pos_g.all_edges(etype=ce)]
                if K:
                    rec[("neg",) + ce] = [t.cpu() for t in neg_g.all_edges(etype=ce)]
                    if fused:  # [positives | negatives] in one buffer per side: joined as a view
                        for pt, nt_ in zip(pos_g.all_edges(etype=ce), neg_g.all_edges(etype=ce)):
                            if pt.numel() and nt_.numel():
                                assert _joined(pt, nt_).data_ptr() == pt.data_ptr(), ce
            rec["b0"] = {nt: blocks[0].srcdata[NID][nt].cpu() for nt in blocks[0].ntypes}
            out.append(rec)
        return out

    a, b = epoch(True), epoch(False)
    assert len(a) == len(b) == -(-900 // 96)
    for ra, rb in zip(a, b):
        assert ra.keys() == rb.keys()
        for key in ra:
            va, vb = ra[key], rb[key]
            if isinstance(va, dict):
                assert all(torch.equal(va[n], vb[n]) for n in va), key
            elif isinstance(va, list):
                assert all(torch.equal(x, y) for x, y in zip(va, vb)), key
            else:
                assert torch.equal(va, vb), key


def test_autograd_matches_torch_reference():
    """Gradients of a ConvModel pass through the HIP-forward autograd Functions equal
    those of a plain torch fp32 restatement of the same math (autograd on torch ops)."""
    from gnnrec.inference import full_graph_embeddings
    g, edges = _graph()
    model = _model(g, "mean_nn_edge", "sum", emb=True).train()
    feats = {nt: g.ndata['features'][nt].clone().requires_grad_(True) for nt in ("user", "item")}
    h = model.embed(feats)
    for layer in model.layers:
        h = layer(g, h)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(7)
    R = {k: torch.randn(v.shape, generator=gen, device=DEV) for k, v in h.items()}
    # a random linear read-out: (unlike sum(z**2)) its gradient is not orthogonal to the
    # normalised rows, so the norm backward is exercised
    loss = sum((v * R[k]).sum() * (i + 1) for i, (k, v) in enumerate(h.items()))
    grads = torch.autograd.grad(loss, list(model.parameters()) + list(feats.values()),
                                allow_unused=True)

    # pure torch restatement
    params = dict(model.named_parameters())
    x = {nt: g.ndata['features'][nt].clone().requires_grad_(True) for nt in ("user", "item")}
    hh = {nt: x[nt] @ params[f"{nt}_embed.proj_feats.weight"].t() + params[f"{nt}_embed.proj_feats.bias"]
          for nt in x}
    for li, layer in enumerate(model.layers):
        out = {}
        for ce in g.canonical_etypes:
            s, d = edges[ce]
            s_t = torch.from_numpy(s).to(DEV)
            d_t = torch.from_numpy(d).to(DEV)
            p = f"layers.{li}.mods.{ce[1]}."
            m = torch.relu(hh[ce[0]] @ params[p + "fc_preagg.weight"].t())
            w = g.edges[ce].data["occurrence"].float()[:, None]
            msg = m[s_t] * w
            agg = torch.zeros(g.num_nodes(ce[2]), m.shape[1], device=DEV).index_add(0, d_t, msg)
            deg = torch.bincount(d_t, minlength=g.num_nodes(ce[2])).clamp(min=1).float()[:, None]
            agg = agg / deg
            z = torch.relu(hh[ce[2]] @ params[p + "fc_self.weight"].t() + agg @ params[p + "fc_neigh.weight"].t())
            n = z.norm(2, 1, keepdim=True)
            z = z / torch.where(n == 0, torch.ones_like(n), n)
            out.setdefault(ce[2], []).append(z)
        hh = {nt: torch.stack(v).sum(0) for nt, v in out.items()}
    loss_ref = sum((hh[k] * R[k]).sum() * (i + 1) for i, k in enumerate(h))
    ref = torch.autograd.grad(loss_ref, list(model.parameters()) + list(x.values()),
                              allow_unused=True)
    np.testing.assert_allclose(loss.item(), loss_ref.item(), rtol=1e-5)
    for (name, _), a, b in zip(list(model.named_parameters()) + [("xu", 0), ("xi", 0)], grads, ref):
        if b is None:
            assert a is None or a.abs().max() == 0, name
            continue
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=2e-4, atol=2e-5,
                                   err_msg=name)


def test_mrr_neg_edges_ranks_positives_among_their_negatives():
    from gnnrec.recs import MRR_neg_edges
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    g, _ = _graph()
    model = _model(g, "mean", "sum", emb=True).eval()
    K = 7
    loader = EdgeDataLoader(g, {("user", "buys", "item"): torch.arange(40)},
                            MultiLayerNeighborSampler([3, 3], seed=3),
                            negative_sampler=negative_sampler.Uniform(K), batch_size=40)
    _, pos_g, neg_g, blocks = next(iter(loader))
    mrr = MRR_neg_edges(model, blocks, pos_g, neg_g, "buys", K)
    with torch.no_grad():
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
    ce = ("user", "buys", "item")
    p = ps[ce].reshape(-1, 1).cpu().numpy()
    n = ns[ce].reshape(-1, K).cpu().numpy()
    ref = np.mean(1.0 / ((n >= p).sum(1) + 1))
    assert 0 < mrr <= 1 and abs(mrr - ref) < 1e-12


def test_reversed_gather_backward_matches_atomic(monkeypatch):
    """The default sum/mean backward (device transpose + gather over the source-major CSR,
    deterministic) == the atomic scatter (GNNREC_SPMM_BWD=atomic), and is bitwise repeatable."""
    from gnnrec.autograd import SpmmFn
    rng = np.random.default_rng(12)
    n_dst, n_src = 300, 200
    deg = rng.integers(0, 30, n_dst)
    indptr = torch.from_numpy(np.concatenate([[0], np.cumsum(deg)])).cuda()
    indices = torch.from_numpy(rng.integers(0, n_src, int(deg.sum())).astype(np.int32)).cuda()
    ew = torch.from_numpy(rng.random(int(deg.sum())).astype(np.float32)).cuda()
    m = torch.randn(n_src, 40, device="cuda")
    g = torch.randn(n_dst, 40, device="cuda")
    for reduce in ("mean", "sum"):
        for w in (None, ew):
            grads = []
            for mode in ("atomic", "gather", "gather"):
                monkeypatch.setenv("GNNREC_SPMM_BWD", mode)
                x = m.clone().requires_grad_(True)
                (SpmmFn.apply(x, indptr, indices, w, reduce, n_dst) * g).sum().backward()
                grads.append(x.grad)
            # atomic order is arbitrary: sums of ~30 terms of size ~1 agree to ~1e-6 absolute
            np.testing.assert_allclose(grads[0].cpu().numpy(), grads[1].cpu().numpy(), rtol=1e-5,
                                       atol=1e-5)
            assert torch.equal(grads[1], grads[2])


def _flat(item):
    from gnnrec.sampling import _tensors
    return [t for t in _tensors(item, []) if t.is_cuda]


@pytest.mark.parametrize("workers", [1, 3])
def test_prefetching_loaders_match_synchronous(workers):
    """num_workers > 0 samples ahead on a second stream: same batches, bit for bit (the
    consumer draws no random numbers), tensors usable on the caller's stream, a training
    step runs on them, and breaking out of the loop early does not hang."""
    from gnnrec import nn as gnn
    from gnnrec.sampling import (EdgeDataLoader, MultiLayerNeighborSampler, NodeDataLoader,
                                 negative_sampler)
    g, _ = _graph()

    def edge_loader(nw):
        torch.manual_seed(7)
        return EdgeDataLoader(g, {BUYS: torch.arange(400), CLICKS: torch.arange(500)},
                              MultiLayerNeighborSampler([3, 2], seed=5),
                              exclude='reverse_types',
                              reverse_etypes={'buys': 'bought-by', 'bought-by': 'buys',
                                              'clicks': 'clicked-by', 'clicked-by': 'clicks'},
                              negative_sampler=negative_sampler.Uniform(4), batch_size=64,
                              shuffle=True, num_workers=nw)

    def node_loader(nw):
        torch.manual_seed(8)
        return NodeDataLoader(g, {"user": torch.arange(60), "item": torch.arange(40)},
                              MultiLayerNeighborSampler([3, 2], seed=6), batch_size=16,
                              shuffle=True, num_workers=nw)

    for make in (edge_loader, node_loader):
        ref = [[t.clone() for t in _flat(item)] for item in make(0)]
        got = [[t.clone() for t in _flat(item)] for item in make(workers)]
        assert len(ref) == len(got) > 1
        for a, b in zip(ref, got):
            assert len(a) == len(b)
            for x, y in zip(a, b):
                assert torch.equal(x, y)
    model = _model(g).train()
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    for step, (_, pos_g, neg_g, blocks) in enumerate(edge_loader(workers)):
        _, ps, ns = model(blocks, blocks[0].srcdata['features'], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, 4, True, pos_g.edata['recency'])
        opt.zero_grad()
        loss.backward()
        opt.step()
        assert torch.isfinite(loss)
        if step == 3:
            break  # the sampling thread stops instead of blocking on a full queue


def test_shared_sampler_across_loaders_after_early_exit():
    """The reference hands ONE sampler to all five loaders (src/sampling.py:153-241) and
    main_train.py runs them with num_workers=4: leaving a prefetching edge loader early and
    starting a node loader on the same sampler (same relabel scratch and masks) must give
    the node loader's synchronous blocks bit for bit — the first producer is joined and its
    stream ordered before the second starts."""
    from gnnrec.sampling import (EdgeDataLoader, MultiLayerFullNeighborSampler, NodeDataLoader,
                                 negative_sampler)
    g, _ = _graph(n_u=300, n_i=200, e_b=6000, e_c=6000)

    def node_items(nw, sampler):
        torch.manual_seed(8)
        loader = NodeDataLoader(g, {"user": torch.arange(300), "item": torch.arange(200)},
                                sampler, batch_size=16, shuffle=True, num_workers=nw)
        return [[t.clone() for t in _flat(item)] for item in loader]

    ref = node_items(0, MultiLayerFullNeighborSampler(2))
    shared = MultiLayerFullNeighborSampler(2)
    for _ in range(3):
        el = EdgeDataLoader(g, {BUYS: torch.arange(6000), CLICKS: torch.arange(6000)}, shared,
                            exclude='reverse_types',
                            reverse_etypes={'buys': 'bought-by', 'bought-by': 'buys',
                                            'clicks': 'clicked-by', 'clicked-by': 'clicks'},
                            negative_sampler=negative_sampler.Uniform(4), batch_size=256,
                            shuffle=True, num_workers=4)
        for step, _item in enumerate(el):
            if step == 1:
                break
        got = node_items(3, shared)
        assert len(ref) == len(got)
        for a, b in zip(ref, got):
            assert len(a) == len(b)
            for x, y in zip(a, b):
                assert torch.equal(x, y)


def test_fanout_sampler_is_uniform():
    """the HIP fanout sampler picks every in-edge of a row with equal
    probability — chi-square over in-row positions (2000 users of in-degree 40, fanout 5,
    four sampler seeds), exactly `fanout` distinct in-edges per seed."""
    from scipy.stats import chi2
    from gnnrec.graph import HeteroGraph
    from gnnrec.sampling import MultiLayerNeighborSampler
    n_u, n_i, deg, fan = 2000, 997, 40, 5
    dst = np.repeat(np.arange(n_u), deg)           # edge e = u * deg + j: j-th in-edge of u
    src = np.arange(n_u * deg) % n_i
    g = HeteroGraph({BOUGHT: (torch.from_numpy(src), torch.from_numpy(dst))},
                    {"user": n_u, "item": n_i}, device=DEV)
    counts = np.zeros(deg)
    for seed in range(4):
        b = MultiLayerNeighborSampler([fan], seed=seed).sample_blocks(
            g, {"user": torch.arange(n_u, device=DEV)})[0]
        indptr, _, eids = b._rels[BOUGHT]
        ip, e = indptr.cpu().numpy(), eids.cpu().numpy()
        assert (np.diff(ip) == fan).all()
        for r in range(0, n_u, 97):
            assert len(set(e[ip[r]:ip[r + 1]].tolist())) == fan
        counts += np.bincount(e - np.repeat(np.arange(n_u), fan) * deg, minlength=deg)
    exp = counts.sum() / deg
    assert chi2.sf(float(((counts - exp) ** 2 / exp).sum()), deg - 1) > 1e-4


@pytest.mark.parametrize("fanouts", [None, [3, 2], [{"buys": 2, "bought-by": 4}, 1]])
def test_cpp_sample_layer_equals_python_form(fanouts):
    """gnnrec::sample_layer (the layer issued from C++) builds the same blocks, bit for bit,
    as the op-by-op Python form it replaces: seeds of both types, a type with no seeds,
    exclusion masks, full and fanout sampling, per-relation fanouts."""
    from gnnrec.sampling import MultiLayerFullNeighborSampler, MultiLayerNeighborSampler
    g, edges = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    mk = (lambda: MultiLayerFullNeighborSampler(2)) if fanouts is None else \
        (lambda: MultiLayerNeighborSampler(fanouts, seed=9))
    seed_sets = [{"user": torch.arange(0, 300, 5, device=DEV),
                  "item": torch.tensor([3, 1, 77, 5], device=DEV)},
                 {"item": torch.arange(0, 120, 3, device=DEV)}]
    for seeds in seed_sets:
        for excl in (None, {BUYS: torch.arange(0, 4000, 3, device=DEV)}):
            blocks = []
            for impl in ("_one_block", "_one_block_py"):
                s = mk()
                masks = {}
                if excl:
                    for ce, e in excl.items():
                        m = s._mask(g, ce)
                        m[e] = 1
                        rows = s._mask_rows(g, ce)
                        dst = g.find_edges(e, ce)[1]
                        rows[dst] = 1
                        masks[ce] = (m, e, rows, dst)
                blocks.append(getattr(s, impl)(g, seeds, 1, masks))
            a, b = blocks
            assert a.canonical_etypes == b.canonical_etypes and a._num_dst == b._num_dst
            for nt in a.ntypes:
                assert torch.equal(a._src[nt]["_ID"], b._src[nt]["_ID"]), nt
            for ce in a.canonical_etypes:
                for x, y in zip(a._rels[ce], b._rels[ce]):
                    assert x.dtype == y.dtype and torch.equal(x, y), ce
                assert a._rels[ce][0]._gnnrec_nnz == b._rels[ce][0]._gnnrec_nnz


@pytest.mark.parametrize("agg,hetero,norm", [("mean", "sum", True), ("mean_edge", "mean", True),
                                             ("mean_nn_edge", "sum", False),
                                             ("mean_nn", "attention", True)])
def test_fused_training_relation_equals_two_node_form(monkeypatch, agg, hetero, norm):
    """gnnrec.autograd.SageRelFn (one node and one C++ call each way per relation) gives
    the loss and every parameter gradient of the SpmmFn + SageProjectFn form bit for bit,
    on sampled blocks (dst-prefix self tables) and on the full graph."""
    from gnnrec import nn as gnn
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    monkeypatch.setenv("GNNREC_TRAIN_FOLD", "0")  # bitwise comparisons: embed, then aggregate
    g, _ = _graph()
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 5, "item": 6, "hidden": 16, "out": 8}, norm, 0.0, agg,
                          "cos", hetero, True).to(DEV)
    loader = EdgeDataLoader(g, {BUYS: torch.arange(400)}, MultiLayerNeighborSampler([4, 4]),
                            exclude="reverse_types",
                            reverse_etypes={"buys": "bought-by", "bought-by": "buys",
                                            "clicks": "clicked-by", "clicked-by": "clicks"},
                            negative_sampler=negative_sampler.Uniform(3), batch_size=64)
    _, pos_g, neg_g, blocks = next(iter(loader))

    def grads(fused, full_graph, layer=False):
        monkeypatch.setenv("GNNREC_TRAIN_FUSED", "1" if fused else "0")
        monkeypatch.setenv("GNNREC_TRAIN_LAYER", "1" if layer else "0")
        model.zero_grad()
        if full_graph:
            h = model.embed(g.ndata["features"])
            for layer in model.layers:
                h = layer(g, h)
            loss = sum((v * v).sum() for v in h.values())
        else:
            _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
            loss = gnn.max_margin_loss(ps, ns, 0.266, 3)
        loss.backward()
        return loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()
                               if p.grad is not None}

    for full_graph in (False, True):
        l1, g1 = grads(True, full_graph)
        l0, g0 = grads(False, full_graph)
        assert torch.equal(l1, l0)
        assert g1.keys() == g0.keys() and len(g1) > 0
        for n in g1:
            assert torch.equal(g1[n], g0[n]), n
    # the whole layer as one node (autograd.HeteroSageFn, blocks only): the same forward
    # bits; a table's gradient sums the relations' parts in the node's own order (four
    # parts per table here: not bitwise the autograd engine's order)
    if agg in ("mean", "mean_edge", "mean_nn_edge", "mean_nn") and hetero in ("sum", "mean"):
        l2, g2 = grads(True, False, layer=True)
        l0, g0 = grads(False, False)
        assert torch.equal(l2, l0)
        assert g2.keys() == g0.keys()
        for n in g2:
            torch.testing.assert_close(g2[n], g0[n], rtol=1e-5, atol=1e-6, msg=n)


def test_layer_node_two_relations_bitwise(monkeypatch):
    """C2's shape — one relation into each node type (buys, bought-by) — through the
    one-node layer (autograd.HeteroSageFn): every table gradient is one relation's gather
    plus the other's self part, a single add as in autograd's engine, so loss and every
    parameter gradient equal the per-relation nodes bit for bit."""
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    monkeypatch.setenv("GNNREC_TRAIN_FOLD", "0")  # bitwise comparisons: embed, then aggregate
    rng = np.random.default_rng(21)
    n_u, n_i, E = 3000, 400, 30000
    u, i = rng.integers(0, n_u, E), rng.integers(0, n_i, E)
    g = HeteroGraph({BUYS: (torch.from_numpy(u), torch.from_numpy(i)),
                     BOUGHT: (torch.from_numpy(i), torch.from_numpy(u))},
                    {"user": n_u, "item": n_i}, device=DEV)
    g.nodes["user"].data["features"] = torch.randn(n_u, 64, device=DEV)
    g.nodes["item"].data["features"] = torch.randn(n_i, 64, device=DEV)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(DEV)
    loader = EdgeDataLoader(g, {BUYS: torch.arange(2000)}, MultiLayerNeighborSampler([10, 10]),
                            exclude="reverse_types",
                            reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                            negative_sampler=negative_sampler.Uniform(10), batch_size=256)
    _, pos_g, neg_g, blocks = next(iter(loader))
    res = {}
    for layer in ("1", "0"):
        monkeypatch.setenv("GNNREC_TRAIN_LAYER", layer)
        model.zero_grad()
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, 10)
        loss.backward()
        res[layer] = (loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()
                                      if p.grad is not None})
    assert torch.equal(res["1"][0], res["0"][0])
    assert res["1"][1].keys() == res["0"][1].keys() and len(res["1"][1]) > 0
    for n in res["1"][1]:
        assert torch.equal(res["1"][1][n], res["0"][1][n]), n


@pytest.mark.parametrize("agg,d_in", [("mean", 64), ("mean", 7), ("mean_nn", 64)])
def test_first_layer_embedding_fold_matches_embed_then_aggregate(monkeypatch, agg, d_in):
    """ConvModel folds the NodeEmbeddings into the first training layer (raw features in,
    W_self W_e / W_neigh W_e with W_self b_e on every row and W_neigh b_e only on rows with
    an in-edge): the loss and every parameter gradient — the embeddings' included — equal
    the reference order (embed every source row, aggregate, project; src/model.py:10-24,
    143-148, 226-235, 462-466) within fp32 rounding.  Half the items were never bought and
    come in as negatives, so rows without in-edges (no neighbour bias) are in the blocks; feature widths differing
    from the hidden width (7) fold as well.  mean_nn (fc_preagg, non-linear) does not fold:
    bit-identical to the unfolded run.  The first block's transposes are no longer built."""
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    rng = np.random.default_rng(4)
    n_u, n_i, E = 4000, 500, 30000
    u, i = rng.integers(0, n_u, E), rng.integers(0, n_i // 2, E)  # items >= n_i/2: no edges
    g = HeteroGraph({BUYS: (torch.from_numpy(u), torch.from_numpy(i)),
                     BOUGHT: (torch.from_numpy(i), torch.from_numpy(u))},
                    {"user": n_u, "item": n_i}, device=DEV)
    g.nodes["user"].data["features"] = torch.randn(n_u, d_in, device=DEV)
    g.nodes["item"].data["features"] = torch.randn(n_i, d_in, device=DEV)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": d_in, "item": d_in, "hidden": 64, "out": 64}, True,
                          0.0, agg, "cos", "sum", True).to(DEV)
    loader = EdgeDataLoader(g, {BUYS: torch.arange(3000)}, MultiLayerNeighborSampler([10, 10]),
                            exclude="reverse_types",
                            reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                            negative_sampler=negative_sampler.Uniform(10), batch_size=512)
    _, pos_g, neg_g, blocks = next(iter(loader))
    # rows without in-edges are in the first block (never-bought items, from the negatives)
    deg = [torch.diff(blocks[0]._rels[ce][0]) for ce in blocks[0].canonical_etypes]
    assert any(bool((d == 0).any()) for d in deg)
    res = {}
    sampler = blocks[0]._sampler()
    assert sampler is loader.sampler and sampler.first_transposes_below is None
    for fold in ("1", "0"):
        monkeypatch.setenv("GNNREC_TRAIN_FOLD", fold)
        model.zero_grad()
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, 10)
        loss.backward()
        res[fold] = (loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters()
                                     if p.grad is not None})
        if fold == "1":  # the fold tells the loader's own sampler, nothing process-wide
            assert (sampler.first_transposes_below is None) == (agg != "mean")
    assert res["1"][1].keys() == res["0"][1].keys()
    assert "user_embed.proj_feats.weight" in res["1"][1]
    if agg != "mean":
        assert torch.equal(res["1"][0], res["0"][0])
        for n in res["1"][1]:
            assert torch.equal(res["1"][1][n], res["0"][1][n]), n
        return
    torch.testing.assert_close(res["1"][0], res["0"][0], rtol=1e-5, atol=1e-7)
    for n in res["1"][1]:
        torch.testing.assert_close(res["1"][1][n], res["0"][1][n], rtol=1e-4, atol=1e-6, msg=n)


def _same_blocks(A, B):
    assert len(A) == len(B)
    for a, b in zip(A, B):
        assert a.canonical_etypes == b.canonical_etypes and a._num_dst == b._num_dst
        assert a.ntypes == b.ntypes
        for nt in a.ntypes:
            assert set(a._src[nt]) == set(b._src[nt])
            for k in a._src[nt]:
                assert torch.equal(a._src[nt][k], b._src[nt][k]), (nt, k)
        for ce in a.canonical_etypes:
            for x, y in zip(a._rels[ce], b._rels[ce]):
                assert x.dtype == y.dtype and torch.equal(x, y), ce
            assert a._rels[ce][0]._gnnrec_nnz == b._rels[ce][0]._gnnrec_nnz
            assert set(a._edata[ce]) == set(b._edata[ce])
            for k in a._edata[ce]:
                assert torch.equal(a._edata[ce][k], b._edata[ce][k]), (ce, k)
            assert set(a._t) == set(b._t)
            if ce in a._t:
                for x, y in zip(a._t[ce], b._t[ce]):
                    assert torch.equal(x, y), ce


@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("fanouts", [[3, 2], [{"buys": 2, "bought-by": 4, "clicks": 0,
                                               "clicked-by": 64}, 1], [10, 10, 5], [1]])
def test_fused_sample_blocks_equal_per_layer_path(fanouts, packed):
    """gnnrec_sample_blocks (every block of a call: 1 + 3L launches, one host read) builds the
    blocks of the per-layer path bit for bit — local ids, eids, node lists, edge data, input
    features and the training transposes — over consecutive calls (the stamped seed positions
    and the alternating bitmaps carried from call to call), seeds of one or both types,
    fanouts 0 / above the degree / per relation, and reverse-type exclusion, whose flags are
    cleared again.  packed: the CSR read as packed {eid, src} records (HeteroGraph
    .edge_records, the default) or as the index and eid arrays."""
    from gnnrec.sampling import MultiLayerNeighborSampler
    g, edges = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    fused = MultiLayerNeighborSampler(fanouts, seed=9)
    fused.packed = packed
    if packed:
        assert len(fused._edge_recs(g, list(g.canonical_etypes))) == len(g.canonical_etypes)
    layer = MultiLayerNeighborSampler(fanouts, seed=9)
    layer.fused = False
    assert fused._fused_ok(g) and not layer._fused_ok(g)
    rng = np.random.default_rng(3)
    cases = [({"user": torch.arange(0, 300, 5, device=DEV),
               "item": torch.tensor([3, 1, 77, 5], device=DEV)}, None),
             ({"item": torch.arange(0, 120, 3, device=DEV)},
              {BUYS: torch.arange(0, 4000, 3, device=DEV),
               BOUGHT: torch.arange(0, 4000, 3, device=DEV)}),
             ({"user": torch.from_numpy(rng.permutation(300)[:50]).to(DEV)},
              {CLICKS: torch.from_numpy(rng.integers(0, 3000, 700)).to(DEV)}),
             ({"user": torch.tensor([299], device=DEV), "item": torch.tensor([0], device=DEV)},
              None)]
    for rep in range(2):
        for seeds, excl in cases:
            a = fused.sample_blocks(g, seeds, excl, transposes=rep == 1)
            b = layer.sample_blocks(g, seeds, excl, transposes=rep == 1)
            _same_blocks(a, b)
    for key, m in fused._exclude_masks.items():
        assert int(m.sum()) == 0, key  # the last finalize cleared every exclusion flag


def test_fused_sampler_stamp_restart():
    """Near the end of the 32-bit stamp range the positions are zeroed and the stamps restart:
    the blocks stay those of the per-layer path."""
    from gnnrec.sampling import MultiLayerNeighborSampler
    g, _ = _graph(n_u=200, n_i=100, e_b=3000, e_c=2000, min_deg=False)
    fused = MultiLayerNeighborSampler([4, 3], seed=2)
    layer = MultiLayerNeighborSampler([4, 3], seed=2)
    layer.fused = False
    seeds = {"user": torch.arange(0, 200, 3, device=DEV)}
    _same_blocks(fused.sample_blocks(g, seeds), layer.sample_blocks(g, seeds))
    fused._stamp = (1 << 32) - 6
    for _ in range(3):
        _same_blocks(fused.sample_blocks(g, seeds), layer.sample_blocks(g, seeds))
    assert fused._stamp < 100


def test_gather_rows_batch_equals_single_gathers():
    from gnnrec import ops
    gen = torch.Generator(device=DEV)
    gen.manual_seed(0)
    srcs = [torch.randint(0, 1 << 40, (1000,), device=DEV, generator=gen),          # 8-B rows
            torch.randn(500, 64, device=DEV, generator=gen),                         # 256-B rows
            torch.randint(0, 255, (300, 7), device=DEV, generator=gen).to(torch.uint8),  # 7 B
            torch.randn(400, 12, device=DEV, generator=gen)[:, :6],                  # strided rows
            torch.randn(10, 3, device=DEV, generator=gen).to(torch.float64),
            torch.zeros(0, 4, device=DEV)]
    idxs = [torch.randint(0, max(s.shape[0], 1), (n,), device=DEV, generator=gen)
            for s, n in zip(srcs, (777, 4096, 33, 1000, 5, 0))]
    jobs = list(zip(srcs, idxs)) * 3  # 18 jobs: more than one launch's worth
    got = ops.gather_rows_batch(jobs)
    for (s, i), o in zip(jobs, got):
        assert torch.equal(o, s[i]), (s.shape, s.dtype)


def test_fused_sampler_repeated_seeds_keep_their_first_position():
    """A seed listed twice (DGL's to_block hash map keeps its first insertion): the fused
    sampler's stamped positions are written by atomicMax of ~position, so every edge whose
    source is that id points at its FIRST position, deterministically, at every step."""
    from gnnrec.graph import NID
    from gnnrec.sampling import MultiLayerNeighborSampler
    g, edges = _graph(n_u=200, n_i=100, e_b=4000, e_c=3000, min_deg=False)
    s = MultiLayerNeighborSampler([4, 3], seed=3)
    seeds = {"user": torch.tensor([5, 9, 5, 17, 9, 5], device=DEV),
             "item": torch.tensor([2, 2, 40], device=DEV)}
    runs = [s.sample_blocks(g, seeds) for _ in range(3)]
    for blocks in runs:
        for b in blocks:
            for ce in b.canonical_etypes:
                ip, loc, eid = (t.cpu().numpy() for t in b._rels[ce])
                src_nodes = b.srcdata[NID][ce[0]].cpu().numpy()
                n_p = b.number_of_dst_nodes(ce[0])
                first = {}
                for k, v in enumerate(src_nodes[:n_p].tolist()):
                    first.setdefault(v, k)
                s_all = edges[ce][0]
                for q in range(loc.size):
                    gid = int(s_all[eid[q]])
                    assert src_nodes[loc[q]] == gid
                    if gid in first:
                        assert loc[q] == first[gid], (ce, gid, loc[q], first[gid])
