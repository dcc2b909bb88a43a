"""Weight-gradient GEMM (dW = dYᵀ X) at training shapes: HIP split-K vs torch (hipBLASLt).

    python tools/bench_wgrad.py
"""
import json
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


def main():
    res = {}
    for K, M, N in [(730_000, 128, 128), (100_000, 128, 128), (730_000, 256, 128),
                    (10_000_000, 128, 128)]:
        A = torch.randn(K, M, device="cuda")
        B = torch.randn(K, N, device="cuda")
        out = torch.empty(M, N, device="cuda")
        th = t(lambda: ops.gemm_tn(A, B, out=out))
        tt = t(lambda: torch.mm(A.t(), B, out=out))
        fl = 2.0 * K * M * N
        res[f"K={K} M={M} N={N}"] = {"hip_ms": th, "hip_TFs": fl / th / 1e9,
                                     "torch_ms": tt, "torch_TFs": fl / tt / 1e9,
                                     "hip_GBs": 4.0 * K * (M + N) / th / 1e6}
        del A, B
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
