"""The eager C2 training loop (bench.py minibatch's K{K}_num_workers2 form: EdgeDataLoader
with the sampling thread, exact shapes, fold 'auto'), N timed steps after 5 warm-up — for
a kernel-stats difference between two N (tools/kstats_diff.py): the step's kernel budget
loader included.

    python tools/probe_eager_step.py [K] [N] [num_workers]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnn-recsys_amd"))
import torch  # noqa: E402


def main():
    from gnnrec import nn as gnn
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    from gnnrec.synth import minibatch_graph
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    nw = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    buys = ("user", "buys", "item")
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005, fused=True)
    el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
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
        return loss

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)  # trace markers (tools/rocpd_timeline.py)
    t = time.perf_counter()
    for _ in range(N):
        loss = step()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print(json.dumps({"K": K, "steps": N, "ms_per_step": (time.perf_counter() - t) / N * 1e3,
                      "loss": float(loss)}))
    del it, el


if __name__ == "__main__":
    main()
