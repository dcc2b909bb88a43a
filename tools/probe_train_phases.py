"""C3 training step split into phases (sampling, forward, loss, backward, optimizer), with
the block shapes of one batch.  GPU box:  python tools/probe_train_phases.py"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from bench_minibatch import c2_graph  # noqa: E402
from gnnrec import nn as gnn  # noqa: E402
from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler  # noqa


def main():
    dev = torch.device("cuda")
    g = c2_graph(128, dev)
    K = 2500
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 128, "item": 128, "hidden": 128, "out": 128}, True,
                          0.0, "mean_nn", "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005)
    el = EdgeDataLoader(g, {("user", "buys", "item"): torch.arange(50_000_000)},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True)
    it = iter(el)
    ph = {k: 0.0 for k in ("sample", "forward", "loss", "backward", "optim")}

    def t():
        torch.cuda.synchronize()
        return time.perf_counter()

    shapes = None
    n = int(os.environ.get("STEPS", "10"))
    for s in range(n + 3):
        t0 = t()
        _, pos_g, neg_g, blocks = next(it)
        t1 = t()
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        t2 = t()
        loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
        t3 = t()
        opt.zero_grad()
        loss.backward()
        t4 = t()
        opt.step()
        t5 = t()
        if s >= 3:
            for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4)):
                ph[k] += v * 1e3 / n
        if shapes is None:
            shapes = [{"src": {nt: b.number_of_src_nodes(nt) for nt in ("user", "item")},
                       "dst": {nt: b.number_of_dst_nodes(nt) for nt in ("user", "item")},
                       "edges": {ce[1]: b.num_edges(ce) for ce in b.canonical_etypes}}
                      for b in blocks]
    ph["total"] = sum(ph.values())
    # whole steps without phase syncs, synchronous loader vs sampling ahead on a side stream
    free = {}
    for nw in (0, 2):
        el.num_workers = nw
        it2 = iter(el)

        def step():
            _, pos_g, neg_g, blocks = next(it2)
            _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
            loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
            opt.zero_grad()
            loss.backward()
            opt.step()
            return loss.item()
        for _ in range(3):
            step()
        t0 = t()
        for _ in range(n):
            step()
        free[f"num_workers={nw}"] = (t() - t0) * 1e3 / n
        del it2
    print(json.dumps({"ms": ph, "step_ms": free, "blocks": shapes}, indent=1))


if __name__ == "__main__":
    main()
