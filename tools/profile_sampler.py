"""Where does a C2 fanout-[10,10] sampler batch / a C3 training step spend its time?
(torch.profiler, GPU box)

    python tools/profile_sampler.py [--train]
"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from bench_minibatch import c2_graph  # noqa: E402
from gnnrec.sampling import MultiLayerNeighborSampler, NodeDataLoader  # noqa: E402


def train():
    from gnnrec import nn as gnn
    from gnnrec.sampling import EdgeDataLoader, negative_sampler
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

    def step():
        _, pos_g, neg_g, blocks = next(it)
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss.item()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(5):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=45))
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=30))


def main():
    if "--train" in sys.argv:
        return train()
    dev = torch.device("cuda")
    g = c2_graph(64, dev)
    loader = NodeDataLoader(g, {"user": torch.arange(1_000_000), "item": torch.arange(100_000)},
                            MultiLayerNeighborSampler([10, 10], seed=1), batch_size=1024,
                            shuffle=True)
    it = iter(loader)
    for _ in range(3):
        next(it)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        next(it)
    torch.cuda.synchronize()
    print(f"ms/batch {(time.perf_counter() - t) / 20 * 1e3:.3f}")
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            next(it)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=40))
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))


if __name__ == "__main__":
    main()
