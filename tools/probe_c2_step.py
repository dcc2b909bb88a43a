"""C2 training step split into host time and GPU time (is the step launch-bound?).

Times 20 steps of the C2 shape (2 conv layers 'mean' d=64, fanout [10,10], 1024 pos x 10
neg, cosine head, Adam) and counts the kernels one step launches (torch profiler-free: a
rocprofv3 --kernel-trace of this script gives the per-kernel split).

    python tools/probe_c2_step.py [K] [num_workers] [d] [aggregator]

d=128 aggregator=mean_nn K=2500 is the C3 step (BASELINE configs[2]).

GNNREC_SWITCH_INTERVAL=<s>: sys.setswitchinterval for the run (the GIL hand-over period
between the training thread and a prefetching sampler thread).
GNNREC_FUSED_HEAD=0: the loader's batch head in its Python form (find_edges + Uniform +
_compact) instead of the one gnnrec::edge_batch_pairs call.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench_minibatch import BUYS, c2_graph  # noqa: E402
from gnnrec import nn as gnn  # noqa: E402
from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    nw = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    if os.environ.get("GNNREC_SWITCH_INTERVAL"):
        sys.setswitchinterval(float(os.environ["GNNREC_SWITCH_INTERVAL"]))
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    agg = sys.argv[4] if len(sys.argv) > 4 else "mean"
    dev = torch.device("cuda")
    g = c2_graph(d, dev)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0,
                          agg, "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005,
                           fused=os.environ.get('GNNREC_BENCH_ADAM_FUSED') != '0')
    el = EdgeDataLoader(g, {BUYS: torch.arange(50_000_000)}, MultiLayerNeighborSampler([10, 10]),
                        exclude="reverse_types", reverse_etypes={"buys": "bought-by",
                                                                  "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, num_workers=nw)
    el.fused_head = el.fused_head and os.environ.get("GNNREC_FUSED_HEAD", "1") != "0"
    it = iter(el)
    phases = {"sample": 0.0, "forward": 0.0, "backward": 0.0, "optim": 0.0}

    def step(timed):
        t0 = time.perf_counter()
        _, pos_g, neg_g, blocks = next(it)
        t1 = time.perf_counter()
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
        t2 = time.perf_counter()
        opt.zero_grad()
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        if timed:  # host-side (launch) time per phase; the GPU runs behind
            for k, a, b in (("sample", t0, t1), ("forward", t1, t2), ("backward", t2, t3),
                            ("optim", t3, t4)):
                phases[k] += (b - a) * 1e3
        return loss

    for _ in range(3):
        step(False).item()
    torch.cuda.synchronize()
    n = int(os.environ.get("GNNREC_PROBE_STEPS", "20"))
    t = time.perf_counter()
    for _ in range(n):
        step(True)
    host = (time.perf_counter() - t) * 1e3 / n
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) * 1e3 / n
    print({"K": K, "d": d, "aggregator": agg, "num_workers": nw, "fused_head": el.fused_head, "switch_interval": sys.getswitchinterval(),
           "wall_ms_per_step": wall, "host_ms_per_step": host,
           "host_phase_ms": {k: v / n for k, v in phases.items()}}, flush=True)


if __name__ == "__main__":
    main()
