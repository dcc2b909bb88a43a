"""One GEMM shape, a few launches (for rocprofv3 passes): M K N [reps] [form].

form 'one' (default): out = A·Wᵀ, K deep.  form 'sage': the sharded pass's owned-row
projection — [h_self | partial / deg]·[W_self | W_neigh]ᵀ, K/2 + K/2 deep, ReLU, row L2 norm,
the partial divided by the global in-degree in the operand load (GNNREC_A2_DIV_DEG)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import _lib, ops  # noqa: E402

M, K, N = (int(x) for x in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
form = sys.argv[5] if len(sys.argv) > 5 else "one"
if form == "sage":
    H = torch.randn(M, K // 2, device="cuda")
    P = torch.randn(M, K // 2, device="cuda")
    deg = torch.randint(0, 1000, (M,), device="cuda", dtype=torch.int32)
    Ws, Wn = torch.randn(N, K // 2, device="cuda"), torch.randn(N, K // 2, device="cuda")

    def run():
        ops.gemm(H, Ws, P, Wn, relu=True, l2norm=True, a2_deg=deg, a2_mode=_lib.A2_DIV_DEG)
else:
    A = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda")

    def run():
        ops.gemm(A, W)
for _ in range(reps):
    run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    run()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(f"M={M} K={K} N={N} {form}: {ms:.3f} ms {2 * M * K * N / ms / 1e9:.1f} TF/s")
