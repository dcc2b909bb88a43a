"""The grouped cosine backward at C2's K = 2500 head (1024 positives x K negatives, d = 64,
100k item rows), timed with HIP events, and a digest of its gradients (to compare two builds):
    python tools/micro/cos_bwd_grouped_one.py [K] [d] [reps]"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
d = int(sys.argv[2]) if len(sys.argv) > 2 else 64
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
g = torch.Generator(device="cuda")
g.manual_seed(0)
G, n_u, n_i = 1024, 1024, 100000
Hs = torch.randn(n_u, d, device="cuda", generator=g)
Hd = torch.randn(n_i, d, device="cuda", generator=g)
ps = torch.randint(0, n_u, (G,), device="cuda", generator=g)
dst = torch.randint(0, n_i, (G * (K + 1),), device="cuda", generator=g)
grad = torch.randn(G * (K + 1), device="cuda", generator=g)


def run():
    return ops.sddmm_cos_backward(ps, dst, Hs, Hd, grad, groups=G, K=K)


for _ in range(3):
    run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    out = run()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
h = hashlib.md5(b"".join(t.cpu().numpy().tobytes() for t in out)).hexdigest()[:16]
print(f"cos_backward_grouped G={G} K={K} d={d}: {ms * 1e3:.1f} us (both sides), grads {h}",
      flush=True)
