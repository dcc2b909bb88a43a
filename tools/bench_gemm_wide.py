import os, sys, json
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "gnn-recsys_amd"))
import torch
from gnnrec import ops
def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
res = {}
for M, K, N in [(1_000_000, 128, 256), (1_000_000, 128, 512), (2_560_000, 256, 128), (1_000_000, 256, 256)]:
    A = torch.randn(M, K, device="cuda"); W = torch.randn(N, K, device="cuda")
    ms = t(lambda: ops.gemm(A, W))
    res[f"M={M} K={K} N={N}"] = {"ms": ms, "TFs": 2 * M * K * N / ms / 1e9}
print(json.dumps(res))
