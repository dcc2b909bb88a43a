"""Exclusive scans of the sampler's sizes (int32 marks, int64 counts), HIP-event time per call
and a check against torch.cumsum:  python tools/micro/scan_one.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
g = torch.Generator(device="cuda")
g.manual_seed(0)
for dt in (torch.int32, torch.int64):
    for n in (5000, 102_400, 323_000, 1_000_000, 4_000_000):
        x = torch.randint(0, 3, (n,), device="cuda", generator=g, dtype=dt)
        ref = torch.cat([torch.zeros(1, dtype=torch.int64, device="cuda"), x.long().cumsum(0)])
        out = ops.exclusive_scan(x)
        assert torch.equal(out, ref), (dt, n)
        for _ in range(5):
            ops.exclusive_scan(x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            ops.exclusive_scan(x)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        byt = n * (x.element_size() + 8)
        print(f"{str(dt):12s} n={n:>9d}: {us:7.2f} us/call  {byt / us / 1e3:7.1f} GB/s", flush=True)
