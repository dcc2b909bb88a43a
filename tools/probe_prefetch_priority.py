"""The bench's captured C2 step (bench.captured_step) with the loader's sampling stream at
normal and at high priority (sampling._Prefetch.priority 0 / -1), alternating, same process:
    python tools/probe_prefetch_priority.py [K] [steps] [rounds]"""
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
    res = {"K": K, "steps": steps, "priority_0": [], "priority_-1": []}
    for _ in range(rounds):
        for prio in (0, -1):
            sampling._Prefetch.priority = prio
            r = bench.captured_step(g, dev, K, steps, 5, caps=caps)
            res[f"priority_{prio}"].append(r["ms_per_step"])
            print(json.dumps({"priority": prio, "ms_per_step": r["ms_per_step"]}), file=sys.stderr,
                  flush=True)
    sampling._Prefetch.priority = 0
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
