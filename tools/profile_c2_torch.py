"""Host-time breakdown of the C2 training step with torch.profiler (CPU activity only):
every autograd node's backward and every dispatcher op, both threads (the autograd engine
runs the backward on its own thread, which cProfile does not see).

    python tools/profile_c2_torch.py [K] [num_workers]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench_minibatch import BUYS, c2_graph  # noqa: E402
from gnnrec import nn as gnn  # noqa: E402
from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    dev = torch.device("cuda")
    g = c2_graph(64, dev)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005)
    el = EdgeDataLoader(g, {BUYS: torch.arange(50_000_000)}, MultiLayerNeighborSampler([10, 10]),
                        exclude="reverse_types", reverse_etypes={"buys": "bought-by",
                                                                  "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, num_workers=nw)
    it = iter(el)

    def step():
        _, pos_g, neg_g, blocks = next(it)
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    n = 20
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(n):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=45))


if __name__ == "__main__":
    main()
