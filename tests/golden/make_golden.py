"""Generate golden vectors by running the reference's own model code.

TEST INFRASTRUCTURE.  Runs ONLY in the build container, where the read-only
reference is mounted at /root/reference; skips cleanly elsewhere (the GPU box
has no reference).  It imports /root/reference/src/model.py UNMODIFIED, with
tests/golden/dgl_shim.py registered as `dgl` (DGL 0.5.2 is not installable
offline), runs the reference's ConvLayer / ConvModel / CosinePrediction /
PredictingModule / max_margin_loss on small seeded synthetic heterographs, and
writes inputs + state_dict + outputs as .npz fixtures next to this script.
No reference source is copied: only numbers are stored.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("GNNREC_REFERENCE", "/root/reference")

USER_ITEM = ("user", "item")
ONLY: list = []  # name filters from the command line (empty: write every case)


def _write(name, arrs):
    if not ONLY or any(o in name for o in ONLY):
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)


def load_reference_model():
    sys.dont_write_bytecode = True  # never write into the read-only reference tree
    sys.path.insert(0, HERE)
    import dgl_shim  # noqa: E402

    dgl_shim.install()
    spec = importlib.util.spec_from_file_location("ref_model", os.path.join(REF, "src", "model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, dgl_shim


def make_graph(rng, num_nodes, rel_sizes, zero_rels=()):
    """Reverse relations share the forward relation's eid order (utils_data.py:205-238)."""
    edges = {}
    occ = {}
    pairs = [(("user", "buys", "item"), ("item", "bought-by", "user")),
             (("user", "clicks", "item"), ("item", "clicked-by", "user")),
             (("item", "utilized-for", "sport"), ("sport", "utilizes", "item")),
             (("user", "practices", "sport"), ("sport", "practiced-by", "user")),
             (("sport", "belongs-to", "sport"), ("sport", "includes", "sport"))]
    for fwd, rev in pairs:
        if fwd[1] not in rel_sizes:
            continue
        n = rel_sizes[fwd[1]]
        s = rng.integers(0, num_nodes[fwd[0]], n)
        d = rng.integers(0, num_nodes[fwd[2]], n)
        o = rng.integers(1, 9, n)
        edges[fwd] = (s, d)
        occ[fwd] = o
        if rev[1] in zero_rels:
            edges[rev] = (np.zeros(0, np.int64), np.zeros(0, np.int64))
            occ[rev] = np.zeros(0, np.int64)
        else:
            edges[rev] = (d, s)
            occ[rev] = o
    return edges, occ


def to_shim(dgl_shim, edges, occ, num_nodes):
    g = dgl_shim.HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d))
                              for ce, (s, d) in edges.items()}, num_nodes)
    for ce in edges:
        if ce[0] in USER_ITEM and ce[2] in USER_ITEM:
            g._edata[ce]["occurrence"] = torch.from_numpy(occ[ce])
    return g


def etype_key(ce):
    return "__".join(ce)


def save_graph(arrs, edges, occ, num_nodes, prefix="g"):
    for nt, n in num_nodes.items():
        arrs[f"{prefix}/num_nodes/{nt}"] = np.array(n, np.int64)
    for ce, (s, d) in edges.items():
        k = etype_key(ce)
        arrs[f"{prefix}/src/{k}"] = s.astype(np.int64)
        arrs[f"{prefix}/dst/{k}"] = d.astype(np.int64)
        arrs[f"{prefix}/occurrence/{k}"] = occ[ce].astype(np.int64)


def gen_convlayer_cases(ref, dgl_shim, manifest):
    rng = np.random.default_rng(11)
    num_nodes = {"user": 37, "item": 29, "sport": 5}
    edges, occ = make_graph(rng, num_nodes, {"buys": 180, "practices": 20})
    g = to_shim(dgl_shim, edges, occ, num_nodes)
    dims = {"user": 5, "item": 6, "sport": 3}
    feats = {nt: rng.standard_normal((n, dims[nt])).astype(np.float32) for nt, n in num_nodes.items()}
    for ce in (("user", "buys", "item"), ("item", "bought-by", "user"),
               ("user", "practices", "sport")):
        for agg in ("mean", "mean_nn", "pool_nn", "mean_edge", "mean_nn_edge", "pool_nn_edge",
                    "lstm"):
            for norm in (True, False):
                torch.manual_seed(7)
                layer = ref.ConvLayer((dims[ce[0]], dims[ce[2]]), 12, 0.0, agg, norm)
                layer.eval()
                with torch.no_grad():
                    z = layer(g[ce], (torch.from_numpy(feats[ce[0]]), torch.from_numpy(feats[ce[2]])))
                name = f"convlayer_{ce[1]}_{agg}_{'norm' if norm else 'nonorm'}"
                arrs = {"x_neigh": feats[ce[0]], "x_self": feats[ce[2]], "out": z.numpy()}
                for k, v in layer.state_dict().items():
                    arrs[f"w/{k}"] = v.numpy()
                save_graph(arrs, edges, occ, num_nodes)
                _write(name, arrs)
                manifest[name] = {"kind": "convlayer", "etype": list(ce), "aggregator_type": agg,
                                  "norm": norm, "out_feats": 12}


def gen_model_cases(ref, dgl_shim, manifest):
    cases = [
        # (name, graph kind, agg, hetero, embedding_layer, n_layers, pred, norm)
        ("model_bip_mean_sum_emb", "bip", "mean", "sum", True, 3, "cos", True),
        ("model_bip_meannn_sum_noemb", "bip", "mean_nn", "sum", False, 3, "cos", True),
        ("model_bip_poolnn_max_noemb_nn", "bip", "pool_nn", "max", False, 2, "nn", True),
        ("model_het_meannnedge_mean_emb", "het", "mean_nn_edge", "mean", True, 3, "cos", True),
        ("model_het_pooledge_sum_noemb_nn", "het", "pool_nn_edge", "sum", False, 2, "nn", False),
        ("model_het_meanedge_max_emb", "het", "mean_edge", "max", True, 2, "cos", True),
        ("model_het_mean_sum_skip", "het_skip", "mean", "sum", False, 3, "cos", True),
        ("model_bip_lstm_sum_emb", "bip", "lstm", "sum", True, 3, "cos", True),
        ("model_het_lstm_mean_noemb_nn", "het", "lstm", "mean", False, 2, "nn", True),
    ]
    for case_no, (name, kind, agg, hagg, emb, n_layers, pred, norm) in enumerate(cases):
        rng = np.random.default_rng(1234 + case_no)
        if kind == "bip":
            num_nodes = {"user": 41, "item": 23}
            edges, occ = make_graph(rng, num_nodes, {"buys": 160})
            dims = {"user": 5, "item": 6}
        else:
            num_nodes = {"user": 43, "item": 31, "sport": 6}
            edges, occ = make_graph(rng, num_nodes, {"buys": 120, "clicks": 150, "utilized-for": 40,
                                                     "practices": 30, "belongs-to": 8},
                                    zero_rels=("includes",) if kind == "het_skip" else ())
            dims = {"user": 5, "item": 6, "sport": 3}
        g = to_shim(dgl_shim, edges, occ, num_nodes)
        dim_dict = dict(dims)
        dim_dict.update({"hidden": 16, "out": 8})
        torch.manual_seed(3)
        model = ref.ConvModel(g, n_layers, dim_dict, norm, 0.0, agg, pred, hagg, emb)
        model.eval()
        feats = {nt: rng.standard_normal((n, dims[nt])).astype(np.float32)
                 for nt, n in num_nodes.items()}
        # pair graphs on the full node sets (pos: first 16 buys edges; neg: K per positive)
        K = 5
        bs, bd = edges[("user", "buys", "item")]
        pos_s, pos_d = bs[:16], bd[:16]
        neg_s = np.repeat(pos_s, K)
        neg_d = rng.integers(0, num_nodes["item"], neg_s.size)
        empty = (np.zeros(0, np.int64), np.zeros(0, np.int64))
        pos_edges = {ce: ((pos_s, pos_d) if ce == ("user", "buys", "item") else empty)
                     for ce in edges}
        neg_edges = {ce: ((neg_s, neg_d) if ce == ("user", "buys", "item") else empty)
                     for ce in edges}
        pos_g = dgl_shim.HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d))
                                      for ce, (s, d) in pos_edges.items()}, num_nodes)
        neg_g = dgl_shim.HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d))
                                      for ce, (s, d) in neg_edges.items()}, num_nodes)
        n_blocks = n_layers - 1 if emb else n_layers
        with torch.no_grad():
            h_in = {nt: torch.from_numpy(v) for nt, v in feats.items()}
            h, pos_score, neg_score = model([g] * n_blocks, dict(h_in), pos_g, neg_g, emb)
            recency = {("user", "buys", "item"): torch.from_numpy(
                rng.integers(1, 30, pos_s.size).astype(np.int64))}
            mask = {ce: torch.from_numpy((rng.random(neg_edges[ce][0].size) < 0.1)
                                         .astype(np.float32)) for ce in pos_score}
            loss = ref.max_margin_loss(pos_score, neg_score, 0.266, K, use_recency=True,
                                       recency_scores=recency, remove_false_negative=True,
                                       negative_mask=mask)
        arrs = {}
        save_graph(arrs, edges, occ, num_nodes)
        for nt, v in feats.items():
            arrs[f"feat/{nt}"] = v
        for nt, v in h.items():
            arrs[f"h/{nt}"] = v.numpy()
        for k, v in model.state_dict().items():
            arrs[f"w/{k}"] = v.numpy()
        arrs["pos/src"], arrs["pos/dst"] = pos_s, pos_d
        arrs["neg/src"], arrs["neg/dst"] = neg_s, neg_d
        for ce, v in pos_score.items():
            arrs[f"pos_score/{etype_key(ce)}"] = v.numpy()
        for ce, v in neg_score.items():
            arrs[f"neg_score/{etype_key(ce)}"] = v.numpy()
        arrs["recency"] = recency[("user", "buys", "item")].numpy()
        for ce, v in mask.items():
            arrs[f"mask/{etype_key(ce)}"] = v.numpy()
        arrs["loss"] = np.array(loss.item(), np.float32)
        _write(name, arrs)
        manifest[name] = {"kind": "model", "aggregator_type": agg, "aggregator_hetero": hagg,
                          "embedding_layer": emb, "n_layers": n_layers, "pred": pred,
                          "norm": norm, "dim_dict": dim_dict, "neg_sample_size": K,
                          "delta": 0.266, "canonical_etypes": [list(ce) for ce in edges]}


class _StubGraph:
    """What reference src/metrics.py reads from g: num_nodes('item'), ndata['popularity']."""

    def __init__(self, n_items, popularity):
        self._n = n_items
        self.ndata = {"popularity": {"item": torch.from_numpy(popularity)}}

    def num_nodes(self, nt):
        assert nt == "item"
        return self._n


def _ref_scores(ref_metrics, g, hu, hi, model, d, user_ids, pred, pop, wpop):
    """Each user's rating vector exactly as reference src/metrics.py:55-72 forms it (the
    same torch modules, the reference's own softmax), before its argsort."""
    out = []
    with torch.no_grad():
        for user in user_ids:
            ue = torch.from_numpy(hu)[user]
            rpt = torch.cat(hi.shape[0] * [ue]).reshape(-1, d)
            if pred == "cos":
                r = torch.nn.CosineSimilarity(dim=1, eps=1e-6)(rpt, torch.from_numpy(hi))
            else:
                r = model.pred_fn.layer_nn(torch.cat((rpt, torch.from_numpy(hi)), 1))
            r = r.cpu().numpy().reshape(hi.shape[0])
            if pop:
                r = np.add(ref_metrics.softmax(r), g.ndata["popularity"]["item"].numpy() * wpop)
            out.append(r)
    return out


def _min_rel_gap(s, bought, k):
    """Smallest relative gap between consecutive entries of the ranked list, through the
    k/k+1 boundary, already-bought items removed."""
    order = [j for j in np.argsort(-s, kind="stable") if j not in set(bought)][: k + 1]
    v = s[order].astype(np.float64)
    gaps = (v[:-1] - v[1:]) / np.maximum(np.abs(v[:-1]), 1e-30)
    return float(gaps.min()) if gaps.size else np.inf


def gen_metrics_cases(ref, manifest):
    """Reference src/metrics.py get_recs / recs_to_metrics (imported unmodified)."""
    import importlib
    sys.path.insert(0, REF)
    ref_metrics = importlib.import_module("src.metrics")
    # k=100 (> the 64 results of one top-k pass): the reference's --k is unbounded
    cases = [("recs_cos", "cos", False, 10), ("recs_cos_pop", "cos", True, 10),
             ("recs_nn", "nn", False, 10), ("recs_cos_k100", "cos", False, 100),
             ("recs_nn_k100", "nn", False, 100)]
    for case_no, (name, pred, pop, k) in enumerate(cases):
        # tie-robust fixtures: a seed is kept only if no two consecutive entries of any
        # user's ranked list (through rank k, already-bought removed) are within `need`
        # relative — the reference's argsort (quicksort, unstable) and fp32 rounding on
        # another host or device would otherwise order a near-tie either way.  1e-5; the
        # MLP head's k = 100 case 1e-6 (2000 gaps between sigmoid outputs: a 1e-5-free seed
        # is a 1-in-20000 event) — still ~16 ulp at 0.5, beyond a dot product's rounding
        need = 1e-6 if (pred == "nn" and k == 100) else 1e-5
        for attempt in range(200):
            rng = np.random.default_rng(500 + case_no + 1000 * attempt)
            n_u, n_i, d = 40, 300, 16
            hu = rng.standard_normal((n_u, d)).astype(np.float32)
            hi = rng.standard_normal((n_i, d)).astype(np.float32)
            popularity = rng.random(n_i).astype(np.float32)
            bu = rng.integers(0, n_u, 400)
            bi = rng.integers(0, n_i, 400)
            already = ref_metrics.create_ground_truth(bu, bi)
            user_ids = list(range(0, n_u, 2))
            torch.manual_seed(9)
            model = type("M", (), {})()
            model.pred_fn = type("P", (), {})()
            model.pred_fn.layer_nn = ref.PredictingLayer(d)
            model.pred_fn.layer_nn.eval()
            g = _StubGraph(n_i, popularity)
            scores = _ref_scores(ref_metrics, g, hu, hi, model, d, user_ids, pred, pop, 0.5)
            gap = min(_min_rel_gap(s, already[u], k) for u, s in zip(user_ids, scores))
            if gap >= need:
                break
        else:
            raise RuntimeError(f"{name}: no tie-free seed in 200 attempts")
        with torch.no_grad():
            recs = ref_metrics.get_recs(g, {"user": torch.from_numpy(hu), "item": torch.from_numpy(hi)},
                                        model, d, k, user_ids, already, True, False, None, pred,
                                        pop, 0.5)
        gu = rng.integers(0, n_u, 120)
        gi = rng.integers(0, n_i, 120)
        gt = ref_metrics.create_ground_truth(gu, gi)
        recs_gt = {u: v for u, v in recs.items()}
        for u in recs_gt:
            gt[u]  # defaultdict: materialise every user key, as the reference does
        prec, rec, cov = ref_metrics.recs_to_metrics(recs_gt, gt, g)
        arrs = {"h/user": hu, "h/item": hi, "popularity": popularity, "bought/u": bu,
                "bought/i": bi, "user_ids": np.array(user_ids, np.int64),
                "recs": np.stack([np.pad(np.asarray(recs[u], np.int64), (0, k - len(recs[u])),
                                         constant_values=-1) for u in user_ids]),
                "gt/u": gu, "gt/i": gi, "scores": np.stack(scores).astype(np.float32),
                "metrics": np.array([prec, rec, cov], np.float64)}
        for kk, v in model.pred_fn.layer_nn.state_dict().items():
            arrs[f"w/{kk}"] = v.numpy()
        _write(name, arrs)
        manifest[name] = {"kind": "recs", "pred": pred, "use_popularity": pop,
                          "weight_popularity": 0.5, "k": k, "embed_dim": d,
                          "seed_attempt": attempt, "min_rel_gap": float(gap),
                          "min_rel_gap_required": need}


def main():
    """python make_golden.py [substring ...]: regenerate every case, or only the cases whose
    name contains one of the substrings (the others keep their files and manifest entries)."""
    if not os.path.exists(os.path.join(REF, "src", "model.py")):
        print(f"reference not found at {REF}: skipping golden generation")
        return 0
    ref, dgl_shim = load_reference_model()
    only = sys.argv[1:]
    ONLY[:] = only
    manifest = {}
    gen_convlayer_cases(ref, dgl_shim, manifest)
    gen_model_cases(ref, dgl_shim, manifest)
    gen_metrics_cases(ref, manifest)
    if only:
        # cases outside the filter keep their files and manifest entries
        old = json.load(open(os.path.join(HERE, "MANIFEST.json")))["cases"]
        for name in list(manifest):
            if not any(o in name for o in only):
                manifest[name] = old.get(name, manifest[name])
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference_files": ["src/model.py", "src/metrics.py"],
                   "torch": torch.__version__, "cases": manifest}, f, indent=1, sort_keys=True)
    print(f"wrote {len(manifest)} golden cases to {HERE}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
