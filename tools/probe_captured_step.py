"""C2 training step, eager (num_workers=2) against captured (static-shape batches replayed
from a hipGraph), at K = 10 and the reference's K = 2500 — bench.captured_step and the
eager loop of bench.minibatch_step without the rooflines.

    python tools/probe_captured_step.py [--captured-only] [K ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def eager(g, dev, K, steps, warmup):
    from gnnrec import nn as gnn
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    buys = ("user", "buys", "item")
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005, fused=True)
    el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, num_workers=2)
    it = iter(el)

    def step():
        _, pos_g, neg_g, blocks = next(it)
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    return {"ms_per_step": round(ms, 3), "loss": float(loss.detach())}


def main():
    from gnnrec.synth import minibatch_graph
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    only = "--captured-only" in sys.argv
    Ks = [int(k) for k in sys.argv[1:] if not k.startswith("--")] or [10, 2500]
    for K in Ks:
        steps = 100 if K <= 10 else 40
        rec = {"K": K}
        if not only:
            rec["eager_num_workers2"] = eager(g, dev, K, steps, 5)
        rec["captured_num_workers2"] = bench.captured_step(g, dev, K, steps, 5)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
