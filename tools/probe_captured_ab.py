"""The bench's captured C2 step (bench.captured_step: EdgeDataLoader(static_shapes=True)
with its sampling thread + CapturedTrainStep) with the static blocks' data gathered lazily
inside the graph (the default) and by the sampler call, alternating, same process:
    python tools/probe_captured_ab.py [K] [steps] [rounds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from gnnrec import sampling  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    from gnnrec.synth import minibatch_graph
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    caps = "auto" if K > 100 else "provable"
    res = {"K": K, "steps": steps, "lazy": [], "eager_gather": []}
    orig = sampling.BlockSampler.__init__

    for _ in range(rounds):
        for lazy in (True, False):
            def init(self, *a, **kw):
                orig(self, *a, **kw)
                self.lazy_static_data = lazy
            sampling.BlockSampler.__init__ = init
            try:
                r = bench.captured_step(g, dev, K, steps, 5, caps=caps)
            finally:
                sampling.BlockSampler.__init__ = orig
            res["lazy" if lazy else "eager_gather"].append(
                (r["ms_per_step"], r.get("gpu_ms_per_replay")))
            print(json.dumps({"lazy": lazy, **{k: r[k] for k in ("ms_per_step", "gpu_ms_per_replay")}}),
                  file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
