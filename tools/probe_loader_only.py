"""The static-shape C2 loader alone (EdgeDataLoader(static_shapes=True), one thread, first-
block transposes skipped as under the fold): N batches, for a kernel-stats difference
between two N (tools/kstats_diff.py) — the loader's per-batch kernel budget.

    python tools/probe_loader_only.py [K] [N] [caps: provable | auto] [packed: 1 | 0]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import sampling  # noqa: E402


def main():
    from gnnrec.synth import minibatch_graph
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    buys = ("user", "buys", "item")
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    caps = sys.argv[3] if len(sys.argv) > 3 else "provable"
    packed = (sys.argv[4] if len(sys.argv) > 4 else "1") == "1"
    el = sampling.EdgeDataLoader(
        g, {buys: torch.arange(g.num_edges(buys))},
        sampling.MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
        negative_sampler=sampling.negative_sampler.Uniform(K), batch_size=1024,
        shuffle=True, static_shapes=True, static_caps=caps)
    el.sampler.first_transposes_below = 0
    el.sampler.packed = packed
    it = iter(el)
    for _ in range(3 + (el.STATIC_LEARN if caps == "auto" else 0)):
        next(it)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        next(it)
    torch.cuda.synchronize()
    print(json.dumps({"K": K, "batches": n, "caps": caps, "packed": packed,
                      "ms_per_batch": (time.perf_counter() - t) / n * 1e3}))


if __name__ == "__main__":
    main()
