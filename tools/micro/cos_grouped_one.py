"""The grouped cosine launch at C3's shape (1024 positives x K negatives, d = 128, 100k
item rows), timed with HIP events:
    python tools/micro/cos_grouped_one.py [K] [d] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
d = int(sys.argv[2]) if len(sys.argv) > 2 else 128
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
g = torch.Generator(device="cuda")
g.manual_seed(0)
G, n_u, n_i = 1024, 1024, 100000
Hs = torch.randn(n_u, d, device="cuda", generator=g)
Hd = torch.randn(n_i, d, device="cuda", generator=g)
ps = torch.randint(0, n_u, (G,), device="cuda", generator=g)
pd = torch.randint(0, n_i, (G,), device="cuda", generator=g)
nd = torch.randint(0, n_i, (G * K,), device="cuda", generator=g)
for _ in range(3):
    ops.sddmm_cos_grouped(ps, pd, K, nd, Hs, Hd)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    ops.sddmm_cos_grouped(ps, pd, K, nd, Hs, Hd)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(f"cos_grouped G={G} K={K} d={d}: {ms * 1e3:.1f} us "
      f"{G * (K + 1) * (4 * d + 8) / ms / 1e9:.2f} TB/s (rows + ids)", flush=True)
