"""C2 block sampler, fused (gnnrec_sample_blocks) against the per-layer path, alternating on
one box: wall ms per sample_blocks call (1024 user + 1024 item seeds, fanout [10,10], the
bench's minibatch_rooflines shape) and bitwise equality of the blocks.

    python tools/sampler_ab.py [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402


def main():
    from gnnrec.sampling import MultiLayerNeighborSampler
    from gnnrec.synth import minibatch_graph
    from test_gpu_sampling import _same_blocks
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    g = minibatch_graph(64, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    # distinct seeds (the per-layer path's prefix map is racy for repeated seeds; the fused
    # one keeps the first position)
    seeds = [{"user": torch.randperm(g.num_nodes("user"), device=dev, generator=gen)[:1024],
              "item": torch.randperm(g.num_nodes("item"), device=dev, generator=gen)[:1024]}
             for _ in range(reps)]
    fused = MultiLayerNeighborSampler([10, 10], seed=4)
    layer = MultiLayerNeighborSampler([10, 10], seed=4)
    layer.fused = False
    for k in range(3):
        _same_blocks(fused.sample_blocks(g, seeds[k]), layer.sample_blocks(g, seeds[k]))
    out = {}
    for rnd in range(2):
        for name, s in (("fused", fused), ("per_layer", layer)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for sd in seeds:
                s.sample_blocks(g, sd)
            torch.cuda.synchronize()
            out.setdefault(name, []).append(round((time.perf_counter() - t0) / reps * 1e3, 4))
    print(json.dumps({"ms_per_call": out, "reps": reps, "bitwise": True}), flush=True)


if __name__ == "__main__":
    main()
