"""The captured C2 training loop (bench.captured_step's loop: EdgeDataLoader(static_shapes,
num_workers=2) -> CapturedTrainStep), its timed steps bracketed by torch.cuda._sleep marker
kernels, for a kernel trace whose steady state tools/rocpd_timeline.py measures.

    python tools/probe_captured_loop.py [K] [steps] [switch_interval_s | 0] [num_workers]
        [provable | auto]
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
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    if len(sys.argv) > 3 and float(sys.argv[3]) > 0:  # the thread switch interval (s), A/B
        sys.setswitchinterval(float(sys.argv[3]))
    nw = int(sys.argv[4]) if len(sys.argv) > 4 else 2  # the loader's sampling thread(s)
    caps = sys.argv[5] if len(sys.argv) > 5 else "provable"  # EdgeDataLoader static_caps
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

    step = CapturedTrainStep(model, opt, loss_fn, warmup=2)
    el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, num_workers=nw, static_shapes=True,
                        static_caps=caps)
    el.sampler.first_transposes_below = 0
    it = iter(el)
    for _ in range(5):
        step(next(it))
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step(next(it))
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(json.dumps({"K": K, "steps": steps, "ms_per_step": round(ms, 4),
                      "switch_interval": sys.getswitchinterval(), "num_workers": nw,
                      "static_caps": caps, "redone": el.static_redone,
                      "replays": step.replays, "loss": float(loss)}))
    del it, el


if __name__ == "__main__":
    main()
