"""The captured C2 training step's graph alone: after a few batches through
CapturedTrainStep, replay the graph N times with nothing else on the GPU, so that a
`rocprofv3 --kernel-trace --stats` of this script is the replay's own kernel budget
(totals / N per step).

    python tools/probe_replay.py [K] [N] [caps: provable | auto]
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
    from gnnrec.capture import CapturedTrainStep
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    from gnnrec.synth import minibatch_graph
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    caps = sys.argv[3] if len(sys.argv) > 3 else "provable"
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    buys = ("user", "buys", "item")
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    model.train_fold = "1"
    opt = torch.optim.Adam(model.parameters(), lr=0.005, fused=True)

    def loss_fn(m, batch):
        _, pos_g, neg_g, blocks = batch
        _, ps, ns = m(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        return gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])

    el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, static_shapes=True, static_caps=caps)
    el.sampler.first_transposes_below = 0
    step = CapturedTrainStep(model, opt, loss_fn, warmup=2)
    it = iter(el)
    for _ in range(5 + (el.STATIC_LEARN if caps == "auto" else 0)):
        step(next(it))
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)  # trace marker (tools/rocpd_timeline.py, rocpd_sequence.py)
    t = time.perf_counter()
    for _ in range(N):
        step.graph.replay()
    host = time.perf_counter() - t
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    # host time of the replay calls alone (a launch that waits for the previous replay shows
    # here as the GPU time per replay)
    print(json.dumps({"K": K, "caps": caps, "replays": N, "ms_per_replay": (time.perf_counter() - t) / N * 1e3,
                      "host_ms_per_replay_call": host / N * 1e3}))


if __name__ == "__main__":
    main()
