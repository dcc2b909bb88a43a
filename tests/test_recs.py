"""Row f1: recommendation top-k + metrics vs the reference's own src/metrics.py
(golden vectors from tests/golden/make_golden.py).  Recommendation lists must
match item for item, metrics exactly.

Ties: the generator keeps only seeds whose ranked lists have no two consecutive
entries within 1e-5 relative (1e-6 for the MLP head at k = 100; the gap reached is
in MANIFEST.json), and stores the reference's own rating vectors (`scores`).  A list
may differ from the fixture only by swapping items whose stored ratings are within
that gap of each other — a near-tie that fp32 rounding on another host or device may
order either way — which `_assert_same_ranking` checks from the stored scores."""
import numpy as np
import pytest
import torch

import golden_io

CASES = sorted(k for k, v in golden_io.manifest().items() if v["kind"] == "recs")


class _G:
    def __init__(self, n_items, pop, device="cpu"):
        self._n = n_items
        self.ndata = {"popularity": {"item": torch.from_numpy(pop).to(device)}}

    def num_nodes(self, nt):
        return self._n


def _assert_same_ranking(got, ref, scores, tol, msg):
    """got == ref item for item, except swaps among items whose reference ratings are
    within `tol` relative of each other."""
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, msg
    bad = np.nonzero(got != ref)[0]
    if bad.size == 0:
        return
    assert sorted(got[bad].tolist()) == sorted(ref[bad].tolist()), msg
    for j in bad:
        a, b = float(scores[got[j]]), float(scores[ref[j]])
        assert abs(a - b) <= tol * max(abs(a), abs(b)), f"{msg}: rank {j} {got[j]} vs {ref[j]}"


@pytest.mark.parametrize("name", CASES)
def test_fixture_scores_rank_to_fixture_recs(name):
    """The stored reference ratings, ranked (already-bought removed), give the fixture's
    lists exactly, and no two consecutive ranks are closer than the manifest's gap: the
    fixtures hold no near-tie whose order depends on rounding."""
    from gnnrec.recs import create_ground_truth
    meta = golden_io.manifest()[name]
    a = golden_io.load(name)
    already = create_ground_truth(a["bought/u"], a["bought/i"])
    for u, s, ref in zip(a["user_ids"], a["scores"], a["recs"]):
        bought = set(already[int(u)])
        order = [j for j in np.argsort(-s.astype(np.float64), kind="stable") if j not in bought]
        np.testing.assert_array_equal(order[: meta["k"]], ref[ref >= 0], err_msg=f"user {u}")
        v = s[order[: meta["k"] + 1]].astype(np.float64)
        gaps = (v[:-1] - v[1:]) / np.abs(v[:-1])
        assert gaps.min() >= meta["min_rel_gap_required"], (u, gaps.min())


@pytest.mark.parametrize("name", CASES)
def test_recs_to_metrics_matches_reference(name):
    from gnnrec.recs import create_ground_truth, recs_to_metrics
    a = golden_io.load(name)
    recs = {int(u): r[r >= 0] for u, r in zip(a["user_ids"], a["recs"])}
    gt = create_ground_truth(a["gt/u"], a["gt/i"])
    got = recs_to_metrics(recs, gt, _G(a["h/item"].shape[0], a["popularity"]))
    np.testing.assert_allclose(got, a["metrics"], rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_get_recs_matches_reference(name):
    from gnnrec.nn import PredictingLayer
    from gnnrec.recs import create_ground_truth, get_recs
    meta = golden_io.manifest()[name]
    a = golden_io.load(name)
    dev = "cuda"
    h = {"user": torch.from_numpy(a["h/user"]).to(dev), "item": torch.from_numpy(a["h/item"]).to(dev)}
    model = type("M", (), {})()
    model.pred_fn = type("P", (), {})()
    pl = PredictingLayer(meta["embed_dim"])
    pl.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in a.items() if k.startswith("w/")})
    model.pred_fn.layer_nn = pl.to(dev).eval()
    already = create_ground_truth(a["bought/u"], a["bought/i"])
    with torch.no_grad():
        recs = get_recs(_G(a["h/item"].shape[0], a["popularity"], dev), h, model, meta["embed_dim"],
                        meta["k"], a["user_ids"].tolist(), already, True, True, None, meta["pred"],
                        meta["use_popularity"], meta["weight_popularity"], batch_size=7)
    for u, ref, s in zip(a["user_ids"], a["recs"], a["scores"]):
        ref = ref[ref >= 0]
        _assert_same_ranking(recs[int(u)], ref, s, meta["min_rel_gap_required"], f"user {u}")
        assert not set(recs[int(u)].tolist()) & set(already[int(u)])


@pytest.mark.gpu
def test_topk_rows_edge_cases():
    from gnnrec.recs import topk_rows
    rng = np.random.default_rng(0)
    S = rng.standard_normal((5, 3000)).astype(np.float32)
    S[1, 10] = S[1, 20] = 100.0  # tie -> lower column first
    ex_ptr = torch.tensor([0, 0, 1, 3001, 3001, 3001], device="cuda")
    ex = np.concatenate([[20], np.arange(3000)]).astype(np.int64)  # row 2 excludes everything
    vals, idx = topk_rows(torch.from_numpy(S).cuda(), 16, ex_ptr, torch.from_numpy(ex).cuda())
    idx = idx.cpu().numpy()
    for r in (0, 3, 4):
        ref = np.lexsort((np.arange(3000), -S[r]))[:16]
        np.testing.assert_array_equal(idx[r], ref)
    assert idx[1][0] == 10 and 20 not in idx[1]
    assert (idx[2] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [64, 65, 100, 200, 3000, 3010])
def test_topk_rows_beyond_one_pass(k):
    """k > 64 runs in passes of 64 (each keeps only columns after the previous pass's
    last result): the same order as a full (score desc, column asc) sort, ties across a
    pass boundary included, exclusions honoured, rows that run out padded with -1."""
    from gnnrec.recs import topk_rows
    rng = np.random.default_rng(k)
    S = rng.integers(-40, 40, (4, 3000)).astype(np.float32)  # many ties
    ex_ptr = torch.tensor([0, 0, 500, 500, 500], device="cuda")
    ex = rng.choice(3000, 500, replace=False).astype(np.int64)
    vals, idx = topk_rows(torch.from_numpy(S).cuda(), k, ex_ptr, torch.from_numpy(ex).cuda())
    idx, vals = idx.cpu().numpy(), vals.cpu().numpy()
    for r in range(4):
        cols = np.arange(3000)
        if r == 1:
            cols = np.setdiff1d(cols, ex)
        ref = cols[np.lexsort((cols, -S[r, cols]))][:k]
        np.testing.assert_array_equal(idx[r, : ref.size], ref)
        np.testing.assert_array_equal(vals[r, : ref.size], S[r, ref])
        assert (idx[r, ref.size:] == -1).all()


@pytest.mark.gpu
def test_inference_ondemand_end_to_end(tmp_path):
    """graph file -> ConvModel -> full-graph embeddings -> top-k, vs the oracle composition."""
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    from gnnrec.inference import inference_ondemand
    from gnnrec.io import save_graphs
    from oracle import oracle
    rng = np.random.default_rng(3)
    n_u, n_i, E = 120, 80, 900
    u, i = rng.integers(0, n_u, E), rng.integers(0, n_i, E)
    edges = {("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u)}
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d)) for ce, (s, d) in edges.items()},
                    {"user": n_u, "item": n_i})
    feats = {"user": rng.standard_normal((n_u, 5)).astype(np.float32),
             "item": rng.standard_normal((n_i, 6)).astype(np.float32)}
    for nt, f in feats.items():
        g.nodes[nt].data["features"] = torch.from_numpy(f)
    path = str(tmp_path / "g.bin")
    save_graphs(path, [g])
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 5, "item": 6, "hidden": 32, "out": 16}, True, 0.0,
                          "mean_nn", "cos", "sum", True).cuda()
    recs, h = inference_ondemand(path, model, user_ids=[0, 5, 7], k=5)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    ref = oracle.model_full_graph(oracle.Graph({"user": n_u, "item": n_i}, edges), feats, sd,
                                  "mean_nn", "sum", True, True)
    for nt in ref:
        np.testing.assert_allclose(h[nt].cpu().numpy(), ref[nt], rtol=1e-4, atol=1e-5)
    iu = ref["item"] / np.maximum(np.linalg.norm(ref["item"], axis=1, keepdims=True), 1e-12)
    for user in (0, 5, 7):
        hu = ref["user"][user] / max(np.linalg.norm(ref["user"][user]), 1e-12)
        scores = iu @ hu
        bought = set(i[u == user].tolist())
        order = [j for j in np.argsort(-scores, kind="stable") if j not in bought][:5]
        np.testing.assert_array_equal(recs[user], order)
