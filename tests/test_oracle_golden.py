"""Pin the CPU oracle (oracle/oracle.py + oracle.c) to golden vectors produced by
the reference's own src/model.py (tests/golden/make_golden.py).

Tolerance: fp32 end to end on both sides; reductions run in different orders
(DGL-shim index_add vs the oracle's sequential CSR loop), so we require
|a-b| <= 1e-5 + 1e-5·|b| — two orders tighter than the north-star 1e-4."""
import numpy as np
import pytest

import golden_io
from oracle import oracle

RTOL, ATOL = 1e-5, 1e-5

CASES = golden_io.manifest()
CONV = sorted(k for k, v in CASES.items() if v["kind"] == "convlayer")
MODEL = sorted(k for k, v in CASES.items() if v["kind"] == "model")


def test_manifest_covers_every_aggregator_and_hetero_mode():
    aggs = {CASES[k]["aggregator_type"] for k in CONV}
    assert aggs == {"mean", "mean_nn", "pool_nn", "mean_edge", "mean_nn_edge", "pool_nn_edge",
                    "lstm"}
    assert {CASES[k]["aggregator_hetero"] for k in MODEL} == {"sum", "mean", "max"}
    assert {CASES[k]["pred"] for k in MODEL} == {"cos", "nn"}


@pytest.mark.parametrize("name", CONV)
def test_conv_layer_matches_reference(name):
    meta = CASES[name]
    a = golden_io.load(name)
    num_nodes, edges, occ = golden_io.graph_parts(a)
    g = oracle.Graph(num_nodes, edges, occ)
    ce = tuple(meta["etype"])
    z = oracle.conv_layer(g, ce, a["x_neigh"], a["x_self"], golden_io.state_dict(a),
                          meta["aggregator_type"], meta["norm"])
    np.testing.assert_allclose(z, a["out"], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("name", MODEL)
def test_full_graph_model_matches_reference(name):
    meta = CASES[name]
    a = golden_io.load(name)
    num_nodes, edges, occ = golden_io.graph_parts(a)
    g = oracle.Graph(num_nodes, edges, occ)
    feats = {k[5:]: v for k, v in a.items() if k.startswith("feat/")}
    sd = golden_io.state_dict(a)
    h = oracle.model_full_graph(g, feats, sd, meta["aggregator_type"], meta["aggregator_hetero"],
                                meta["norm"], meta["embedding_layer"])
    ref_h = {k[2:]: v for k, v in a.items() if k.startswith("h/")}
    assert set(h) == set(ref_h)
    for nt in ref_h:
        np.testing.assert_allclose(h[nt], ref_h[nt], rtol=RTOL, atol=ATOL)

    # edge-score heads and the loss on the reference's own embeddings
    pos = {ce: ((a["pos/src"], a["pos/dst"]) if ce == ("user", "buys", "item") else
                (np.zeros(0, np.int64), np.zeros(0, np.int64))) for ce in edges}
    neg = {ce: ((a["neg/src"], a["neg/dst"]) if ce == ("user", "buys", "item") else
                (np.zeros(0, np.int64), np.zeros(0, np.int64))) for ce in edges}
    if meta["pred"] == "cos":
        ps, ns = oracle.cosine_prediction(pos, ref_h), oracle.cosine_prediction(neg, ref_h)
    else:
        _, _, p = oracle.split_state_dict(sd)
        p = {k[len("layer_nn."):]: v for k, v in p.items()}
        ps, ns = oracle.predicting_module(pos, ref_h, p), oracle.predicting_module(neg, ref_h, p)
    ref_ps = golden_io.by_etype(a, "pos_score")
    ref_ns = golden_io.by_etype(a, "neg_score")
    assert set(ps) == set(ref_ps) and set(ns) == set(ref_ns)
    for ce in ref_ps:
        np.testing.assert_allclose(ps[ce], ref_ps[ce], rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(ns[ce], ref_ns[ce], rtol=RTOL, atol=ATOL)
    mask = golden_io.by_etype(a, "mask")
    rec = {("user", "buys", "item"): a["recency"]}
    loss = oracle.max_margin_loss(ref_ps, ref_ns, meta["delta"], meta["neg_sample_size"],
                                  use_recency=True, recency=rec, remove_false_negative=True,
                                  mask=mask)
    np.testing.assert_allclose(loss, a["loss"], rtol=RTOL, atol=ATOL)


def test_relation_skip_case_present():
    """The het_skip fixture has an empty relation; the reference skips it."""
    a = golden_io.load("model_het_mean_sum_skip")
    _, edges, _ = golden_io.graph_parts(a)
    assert edges[("sport", "includes", "sport")][0].size == 0


def test_unknown_aggregator_raises_keyerror():
    g = oracle.Graph({"user": 2, "item": 2}, {("user", "buys", "item"): ([0], [1])})
    w = {"fc_self.weight": np.zeros((3, 2), np.float32), "fc_neigh.weight": np.zeros((3, 2), np.float32)}
    with pytest.raises(KeyError):
        oracle.conv_layer(g, ("user", "buys", "item"), np.zeros((2, 2), np.float32),
                          np.zeros((2, 2), np.float32), w, "median", True)


def test_lstm_edge_fails_like_the_reference():
    """reference ConvLayer builds self.lstm only for 'lstm' (src/model.py:103-104): its
    'lstm_edge' forward fails on the missing attribute."""
    a = golden_io.load(CONV[0])
    num_nodes, edges, occ = golden_io.graph_parts(a)
    g = oracle.Graph(num_nodes, edges, occ)
    with pytest.raises(AttributeError):
        oracle.conv_layer(g, ("user", "buys", "item"), a["x_neigh"], a["x_self"], {},
                          "lstm_edge", True)


def _position_chi2(counts):
    from scipy.stats import chi2
    exp = counts.sum() / counts.size
    stat = float(((counts - exp) ** 2 / exp).sum())
    return chi2.sf(stat, counts.size - 1)


def test_fanout_sampler_restatement_is_uniform():
    """the fanout sampler (Floyd's algorithm over a counter hash; the HIP
    sampler is bit-exact to this restatement, tests/test_gpu_sampling.py) picks every
    in-edge of a row with equal probability: chi-square over in-row positions, 2000 rows
    of degree 40, fanout 5, four sampler keys; and exactly `fanout` distinct edges per row."""
    n_rows, deg, fan = 2000, 40, 5
    indptr = np.arange(n_rows + 1, dtype=np.int64) * deg
    indices = np.arange(n_rows * deg, dtype=np.int64) % 997
    eids = np.arange(n_rows * deg, dtype=np.int64)
    counts = np.zeros(deg)
    for key in range(4):
        ip, _, eid = oracle.sample_neighbors(indptr, indices, eids, np.arange(n_rows), fan, key=key)
        assert (np.diff(ip) == fan).all()
        rows = np.repeat(np.arange(n_rows), fan)
        assert all(len(set(eid[ip[r]:ip[r + 1]].tolist())) == fan for r in range(0, n_rows, 97))
        counts += np.bincount(eid - rows * deg, minlength=deg)
    assert _position_chi2(counts) > 1e-4


def _full_blocks(g, n_blocks):
    """the reference's golden run passes the full graph as every block (make_golden.py:176)"""
    rels = {ce: g.csr(ce) for ce in g.canonical_etypes}
    return [oracle.BlockGraph(rels, g.num_nodes, g.occurrence) for _ in range(n_blocks)]


@pytest.mark.parametrize("name", MODEL)
def test_model_blocks_on_full_blocks_matches_reference(name):
    """oracle.model_blocks (get_repr over blocks, dst-prefix slicing) with the full graph as
    every block, as the golden run feeds the reference, reproduces the reference's h."""
    meta = CASES[name]
    a = golden_io.load(name)
    num_nodes, edges, occ = golden_io.graph_parts(a)
    g = oracle.Graph(num_nodes, edges, occ)
    feats = {k[5:]: v for k, v in a.items() if k.startswith("feat/")}
    sd = golden_io.state_dict(a)
    n_blocks = meta["n_layers"] - 1 if meta["embedding_layer"] else meta["n_layers"]
    h = oracle.model_blocks(_full_blocks(g, n_blocks), feats, sd, meta["aggregator_type"],
                            meta["aggregator_hetero"], meta["norm"], meta["embedding_layer"])
    ref_h = {k[2:]: v for k, v in a.items() if k.startswith("h/")}
    assert set(h) == set(ref_h)
    for nt in ref_h:
        np.testing.assert_allclose(h[nt], ref_h[nt], rtol=RTOL, atol=ATOL)


def test_model_blocks_prefix_block_equals_full_graph_rows():
    """A one-layer block over a seed subset (full in-neighbourhoods, sources = dst prefix +
    new ids ascending) gives the seeds' rows of the one-layer full-graph model."""
    name = next(k for k in MODEL if CASES[k]["aggregator_type"] == "mean_nn_edge")
    meta = CASES[name]
    a = golden_io.load(name)
    num_nodes, edges, occ = golden_io.graph_parts(a)
    g = oracle.Graph(num_nodes, edges, occ)
    feats = {k[5:]: v for k, v in a.items() if k.startswith("feat/")}
    sd = {k: v for k, v in golden_io.state_dict(a).items() if not k.startswith("layers.1")
          and not k.startswith("layers.2")}
    full = oracle.model_full_graph(g, feats, sd, meta["aggregator_type"],
                                   meta["aggregator_hetero"], meta["norm"],
                                   meta["embedding_layer"])
    rng = np.random.default_rng(0)
    seeds = {nt: np.sort(rng.choice(n, max(1, n // 3), replace=False))
             for nt, n in num_nodes.items() if n > 0}
    rels, picked = {}, {}
    for ce in g.canonical_etypes:
        ip, ix, e = g.csr(ce)
        s = seeds.get(ce[2], np.zeros(0, np.int64))
        oip, osrc, oe = oracle.sample_neighbors(ip, ix, e, s, -1)
        rels[ce] = [oip, osrc, oe]
        picked.setdefault(ce[0], []).append(ce)
    src_feats = {}
    for nt in num_nodes:
        pref = seeds.get(nt, np.zeros(0, np.int64))
        nodes, locs = oracle.to_block_relabel(pref, [rels[ce][1] for ce in picked.get(nt, [])])
        for ce, loc in zip(picked.get(nt, []), locs):
            rels[ce][1] = loc
        if nodes.size:
            src_feats[nt] = feats[nt][nodes]
    blk = oracle.BlockGraph({ce: tuple(r) for ce, r in rels.items()},
                            {nt: v.size for nt, v in seeds.items()}, occ)
    h = oracle.model_blocks([blk], src_feats, sd, meta["aggregator_type"],
                            meta["aggregator_hetero"], meta["norm"], meta["embedding_layer"])
    for nt, v in seeds.items():
        if nt in full:
            np.testing.assert_allclose(h[nt], full[nt][v], rtol=RTOL, atol=ATOL)


@pytest.mark.parametrize("E,n_dst", [(0, 5), (1, 1), (1000, 7), (200_000, 50_000),
                                     (3_000_000, 1000)])
def test_csr_from_coo_c_equals_numpy_restatement(E, n_dst):
    """oracle.c's parallel counting sort (large graphs, CPU baseline, row f3's checker)
    gives the numpy stable-argsort CSR bit for bit, empty rows included."""
    rng = np.random.default_rng(E)
    src = rng.integers(0, 1 << 30, E)
    dst = rng.integers(0, n_dst, E) if E else np.zeros(0, np.int64)
    for a, b in zip(oracle.csr_from_coo_c(src, dst, n_dst), oracle.csr_from_coo(src, dst, n_dst)):
        np.testing.assert_array_equal(a, b)
