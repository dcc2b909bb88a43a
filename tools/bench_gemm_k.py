"""GEMM rate vs K at fixed M x N (is the short-K prologue/epilogue the loss?).

    python tools/bench_gemm_k.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402


def t(fn, reps=10):
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
    for M, K in [(862_000, 128), (2_000_000, 128), (2_000_000, 256), (500_000, 1024),
                 (125_000, 4096)]:
        A = torch.randn(M, K, device="cuda")
        W = torch.randn(128, K, device="cuda")
        ms = t(lambda: ops.gemm(A, W))
        ms_n = t(lambda: ops.gemm(A, W, relu=True, l2norm=True))
        res[f"M={M} K={K} N=128"] = {"ms": ms, "TFs": 2 * M * K * 128 / ms / 1e9,
                                     "TFs_relu_l2": 2 * M * K * 128 / ms_n / 1e9}
        if K == 256:  # the SAGE projection form: two K=128 operands
            A1, A2 = A[:, :128], A[:, 128:]
            W1, W2 = W[:, :128].contiguous(), W[:, 128:].contiguous()
            ms2 = t(lambda: ops.gemm(A1, W1, A2, W2, relu=True, l2norm=True))
            res[f"M={M} K=128+128 N=128 relu l2"] = {"ms": ms2,
                                                     "TFs": 2 * M * K * 128 / ms2 / 1e9}
        del A
    res["GNNREC_GEMM_BK16"] = os.environ.get("GNNREC_GEMM_BK16", "0")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
