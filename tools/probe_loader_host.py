"""Host cost of the static-shape C2 loader (EdgeDataLoader(static_shapes=True), no sampling
thread, no synchronisation between batches): batches per second when nothing else runs, and
a cProfile of the same loop (top functions by own time and by cumulative time).

    python tools/probe_loader_host.py [K] [n_batches]
"""
import cProfile
import io
import json
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
        shuffle=True, static_shapes=True)
    el.sampler.first_transposes_below = 0
    it = iter(el)
    for _ in range(5):
        next(it)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        next(it)
    host = (time.perf_counter() - t) / n * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / n * 1e3
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        next(it)
    pr.disable()
    torch.cuda.synchronize()
    print(json.dumps({"K": K, "batches": n, "host_ms_per_batch": round(host, 4),
                      "wall_ms_per_batch": round(wall, 4)}), flush=True)
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(45)
        print(s.getvalue(), flush=True)
    del it, el
    # the captured step with the sampling thread: how long the training loop waits for
    # the loader's queue per step
    waits = []

    class TimedQueue(sampling.queue.Queue):
        def get(self, *a, **kw):
            t0 = time.perf_counter()
            r = super().get(*a, **kw)
            waits.append(time.perf_counter() - t0)
            return r

    sampling.queue.Queue = TimedQueue
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    rec = bench.captured_step(g, dev, K, 100, 5)
    w = waits[-100:]
    rec["queue_wait_ms_per_step"] = round(sum(w) / len(w) * 1e3, 4)
    print(json.dumps(rec), flush=True)
    # the training thread's own host time, by function (the loader thread is not profiled)
    pr = cProfile.Profile()
    pr.enable()
    bench.captured_step(g, dev, K, 300, 5)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
