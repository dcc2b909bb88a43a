"""Where a static-shape C2 batch's time goes (EdgeDataLoader(static_shapes=True), one
thread, synchronised after every phase): the batch head (pairs, negatives, compaction), the
sampler, the block data gathers and transposes — against the exact loader's batch, at K = 10
and K = 2500.

    python tools/probe_static_loader.py [K ...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops, sampling  # noqa: E402


def main():
    from gnnrec.synth import minibatch_graph
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    buys = ("user", "buys", "item")
    Ks = [int(k) for k in sys.argv[1:]] or [10, 2500]
    timers = {}

    def wrap(obj, name):
        f = getattr(obj, name)

        def w(*a, **kw):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f(*a, **kw)
            torch.cuda.synchronize()
            timers[name] = timers.get(name, 0.0) + time.perf_counter() - t
            return r
        setattr(obj, name, w)

    wrap(ops, "compact_ids")
    wrap(ops, "sample_blocks")
    wrap(ops, "gather_rows_batch")
    wrap(ops, "edge_batch_pairs")
    wrap(sampling, "_add_transposes")
    for K in Ks:
        for static in (False, True):
            el = sampling.EdgeDataLoader(
                g, {buys: torch.arange(g.num_edges(buys))},
                sampling.MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                negative_sampler=sampling.negative_sampler.Uniform(K), batch_size=1024,
                shuffle=True, static_shapes=static)
            it = iter(el)
            for _ in range(3):
                next(it)
            timers.clear()
            n = 10
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(n):
                item = next(it)
            torch.cuda.synchronize()
            tot = (time.perf_counter() - t) / n * 1e3
            blocks = item[-1]
            rec = {"K": K, "static": static, "ms_per_batch": round(tot, 3),
                   "phase_ms": {k: round(v / n * 1e3, 3) for k, v in timers.items()},
                   "src_rows_block0": {nt: blocks[0].number_of_src_nodes(nt) for nt in blocks[0].ntypes},
                   "edges": [sum(b.num_edges(ce) for ce in b.canonical_etypes) for b in blocks]}
            print(json.dumps(rec), flush=True)
            del it, el


if __name__ == "__main__":
    main()
