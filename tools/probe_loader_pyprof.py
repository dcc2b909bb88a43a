"""Host time of the static C2 loader's Python per batch (cProfile over N batches of
EdgeDataLoader(static_shapes=True), one thread, first-block transposes skipped as under
the fold): where the sampling thread's ~1 ms per K = 10 batch goes.
    python tools/probe_loader_pyprof.py [K] [N]"""
import cProfile
import io
import os
import pstats
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
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    el = sampling.EdgeDataLoader(
        g, {buys: torch.arange(g.num_edges(buys))},
        sampling.MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
        negative_sampler=sampling.negative_sampler.Uniform(K), batch_size=1024,
        shuffle=True, static_shapes=True, static_caps="provable" if K <= 100 else "auto")
    el.sampler.first_transposes_below = 0
    it = iter(el)
    for _ in range(5):
        next(it)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    for _ in range(n):
        next(it)
    pr.disable()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / n * 1e3
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(f"ms per batch (under cProfile): {wall:.3f}")
    print(s.getvalue())


if __name__ == "__main__":
    main()
