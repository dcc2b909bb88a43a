"""Partial-table add (gnnrec_add_f32) vs torch.add on a [1M, 128] fp32 table.

    python tools/bench_add.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


a = torch.randn(1_000_000, 128, device="cuda")
b = torch.randn_like(a)
ref = a + b
ops.add_(a.clone(), b)
c = a.clone()
assert torch.equal(ops.add_(c, b), ref)
ms = t(lambda: ops.add_(a, b))
mt = t(lambda: torch.add(a, b, out=a))
print(f"gnnrec_add_f32 {ms:.3f} ms ({3 * a.numel() * 4 / ms / 1e9:.2f} TB/s), "
      f"torch {mt:.3f} ms ({3 * a.numel() * 4 / mt / 1e9:.2f} TB/s)")
