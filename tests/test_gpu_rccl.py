"""RCCL itself, on the one GPU a gpurun box gives: an nccl process group of world size 1,
and the sharded full-graph pass driven through an Exchange that issues every collective
anyway (force_collectives=True: no world-size-1 shortcut, the pass's multi-rank schedule).

So `reduce_scatter_tensor`, `all_to_all_single` (both async, waited by `work.wait()` on the
consuming stream), `all_gather_into_tensor`, the all-gather-as-all-to-all form and the
`all_reduce` of max_scalar run on RCCL before the driver's 8-GPU bench does — and every
output must equal the no-group one-rank pass: bitwise in deterministic mode (the same
per-segment tree at any world size), to the north-star 1e-4 in fast mode (where the one-rank
pass fuses the item side that the multi-rank schedule exchanges as partials).

Each case runs in ONE spawned process (a default process group per process)."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _build(d, two_rel):
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(1)
    n_u, n_i, E = 3000, 700, 100000
    u, i = rng.integers(0, n_u, E), rng.integers(0, n_i, E)
    rels = {("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u)}
    if two_rel:
        uc, ic = rng.integers(0, n_u, E // 3), rng.integers(0, n_i, E // 3)
        rels[("user", "clicks", "item")] = (uc, ic)
        rels[("item", "clicked-by", "user")] = (ic, uc)
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(t)) for ce, (s, t) in rels.items()},
                    {"user": n_u, "item": n_i}, device="cuda")
    feats = {"user": torch.from_numpy(rng.standard_normal((n_u, d)).astype(np.float32)).cuda(),
             "item": torch.from_numpy(rng.standard_normal((n_i, d)).astype(np.float32)).cuda()}
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0, "mean",
                          "cos", "sum", True).cuda().eval()
    return g, feats, model


def _worker(port, d, two_rel, det, ag_mode, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["GNNREC_ALLGATHER"] = ag_mode
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from gnnrec.dist import Exchange, RecordingExchange
        from gnnrec.inference import GraphShard, ShardedFullGraphPass
        g, feats, model = _build(d, two_rel)
        seg = 8 if det else None
        sh = GraphShard.from_graph(g, 0, 1, "user", device="cuda", segments=seg)
        x = sh.local_features(feats)
        base_ex = Exchange()
        assert not base_ex.multi and base_ex._rccl
        ref = ShardedFullGraphPass(model, sh, base_ex, deterministic=det).run(x)
        ref = {nt: t.clone() for nt, t in ref.items()}
        ex = Exchange(force_collectives=True)
        rec = RecordingExchange(ex)
        runner = ShardedFullGraphPass(model, sh, rec, deterministic=det)
        outs = []
        for rep in (True, False, True):  # back to back: scratch reuse across passes
            o = runner.run(x, replicate_output=rep)
            outs.append({nt: t.clone() for nt, t in o.items()})
        torch.cuda.synchronize()
        kinds = sorted({c[0] for c in rec.calls})
        m = ex.max_scalar(3.5, dev)
        q.put(("ok", ex.path, kinds, m,
               {nt: t.cpu().numpy() for nt, t in ref.items()},
               [{nt: t.cpu().numpy() for nt, t in o.items()} for o in outs]))
    except BaseException as exc:  # surfaced in the test
        q.put(("error", repr(exc)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("d,two_rel,det,ag_mode", [
    (128, False, True, "rccl"),    # C4 shape: tiles + fixed tree + all_to_all + all-gather
    (128, True, True, "a2a"),      # C5 shape (pair launch), all-gather as all-to-all
    (32, False, False, "rccl"),    # fast mode: reduce-scatter of the item partials
])
def test_rccl_world_size_one_matches_no_group_pass(d, two_rel, det, ag_mode):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), d, two_rel, det, ag_mode, q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=120)
    assert res[0] == "ok", res
    _, path, kinds, m, ref, outs = res
    assert p.exitcode == 0
    assert path == "rccl", path
    want = {"all_gather", "all_to_all"} if det else {"all_gather", "reduce_scatter"}
    assert want <= set(kinds), kinds
    assert m == 3.5
    n_i = 700
    for o in outs:
        for nt in ("user", "item"):
            a, b = o[nt][:n_i] if nt == "item" else o[nt], ref[nt][:n_i] if nt == "item" else ref[nt]
            if det:
                assert np.array_equal(a, b), f"{nt}: RCCL pass differs from the no-group pass"
            else:
                np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
