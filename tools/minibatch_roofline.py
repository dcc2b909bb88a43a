"""The §8d d3/d4 rooflines of the minibatch kernels alone (bench.minibatch_rooflines): the
C2 block sampler, the C3 cosine head and the C3 edge-MLP head, so that a
`rocprofv3 --kernel-trace --stats` of this script gives their per-kernel averages without
the training step's launches of the same kernels at other shapes.

    python tools/minibatch_roofline.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    print(json.dumps(bench.minibatch_rooflines(torch.device("cuda", 0), reps=reps)), flush=True)
