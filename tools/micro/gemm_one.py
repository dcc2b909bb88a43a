"""One GEMM shape, a few launches (for rocprofv3 passes): M K N [reps]."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

M, K, N = (int(x) for x in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
A = torch.randn(M, K, device="cuda")
W = torch.randn(N, K, device="cuda")
for _ in range(reps):
    ops.gemm(A, W)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    ops.gemm(A, W)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(f"M={M} K={K} N={N}: {ms:.3f} ms {2 * M * K * N / ms / 1e9:.1f} TF/s")
