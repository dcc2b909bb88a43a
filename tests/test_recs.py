"""Row f1: recommendation top-k + metrics vs the reference's own src/metrics.py
(golden vectors from tests/golden/make_golden.py).  Recommendation lists must
match item for item (ties are broken by column index; the goldens contain no
exact ties), metrics exactly."""
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
    for u, ref in zip(a["user_ids"], a["recs"]):
        ref = ref[ref >= 0]
        np.testing.assert_array_equal(recs[int(u)], ref, err_msg=f"user {u}")
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
