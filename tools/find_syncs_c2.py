"""Where does a C2 training step synchronise the host with the GPU?  Runs steps under
torch.cuda.set_sync_debug_mode('warn') and prints each synchronising call site once.

    python tools/find_syncs_c2.py
"""
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench_minibatch import BUYS, c2_graph  # noqa: E402
from gnnrec import nn as gnn  # noqa: E402
from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler  # noqa: E402


def main():
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
        _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        loss = gnn.max_margin_loss(ps, ns, 0.266, 10, True, pos_g.edata["recency"])
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    seen = {}

    def show(message, category, filename, lineno, file=None, line=None):
        stack = [f for f in traceback.extract_stack()[:-1] if "gnnrec" in f.filename
                 or "tools" in f.filename]
        key = tuple((os.path.basename(f.filename), f.lineno) for f in stack[-3:])
        seen[key] = seen.get(key, 0) + 1

    warnings.showwarning = show
    torch.cuda.set_sync_debug_mode("warn")
    for _ in range(5):
        step()
    torch.cuda.set_sync_debug_mode(0)
    for k, n in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(n / 5, "per step:", " <- ".join(f"{f}:{ln}" for f, ln in reversed(k)))


if __name__ == "__main__":
    main()
