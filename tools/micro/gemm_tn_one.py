"""One weight-gradient shape C[M,N] = A[K,M]^T B[K,N], timed with HIP events:
    python tools/micro/gemm_tn_one.py K M N [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

K, M, N = (int(x) for x in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
A = torch.randn(K, M, device="cuda")
B = torch.randn(K, N, device="cuda")
for _ in range(3):
    ops.gemm_tn(A, B)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    ops.gemm_tn(A, B)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(f"gemm_tn K={K} M={M} N={N}: {ms * 1e3:.1f} us {K * (M + N) * 4 / ms / 1e9:.2f} TB/s", flush=True)
