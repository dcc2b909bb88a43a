"""Host-side profile (cProfile) of the C2 minibatch step's phases: where the Python/ATen
dispatch time of the EdgeDataLoader batch and of forward/backward goes.

    python tools/profile_c2_host.py [sample|step]
"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench_minibatch import BUYS, c2_graph  # noqa: E402
from gnnrec import nn as gnn  # noqa: E402
from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler  # noqa: E402


def main(what):
    dev = torch.device("cuda")
    g = c2_graph(64, dev)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005)
    el = EdgeDataLoader(g, {BUYS: torch.arange(50_000_000)}, MultiLayerNeighborSampler([10, 10]),
                        exclude="reverse_types", reverse_etypes={"buys": "bought-by",
                                                                  "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(10), batch_size=1024,
                        shuffle=True)
    it = iter(el)

    def step():
        _, pos_g, neg_g, blocks = next(it)
        if what == "sample":
            return
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, 10, True, pos_g.edata["recency"])
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(10):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "sample")
