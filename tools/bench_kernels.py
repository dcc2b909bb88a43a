"""Per-kernel timing on C4 shapes (HIP events, interleaved repetitions in one process).

    python tools/bench_kernels.py [--only gemm|spmm|heads]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402
from gnnrec.graph import build_csr  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--zipf", type=float, default=1.0)
    args = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    if args.only in ("", "gemm"):
        M, d = 10_000_000, 128
        A1 = torch.randn(M, d, device=dev)
        A2 = torch.randn(M, d, device=dev)
        W1 = torch.randn(d, d, device=dev) * 0.1
        W2 = torch.randn(d, d, device=dev) * 0.1
        b = torch.randn(d, device=dev)
        out = torch.empty(M, d, device=dev)
        med, mn = timeit(lambda: ops.gemm(A1, W1, A2, W2, relu=True, l2norm=True, out=out))
        fl = 2 * M * 2 * d * d
        res["gemm_sage_10Mx256x128"] = {"ms": med, "min_ms": mn, "TFLOPs": fl / med / 1e9,
                                        "GBs": 4 * M * (3 * d) / med / 1e6}
        med, mn = timeit(lambda: ops.gemm(A1, W1, bias=b, out=out))
        res["gemm_embed_10Mx128x128"] = {"ms": med, "min_ms": mn, "TFLOPs": 2 * M * d * d / med / 1e9,
                                         "GBs": 4 * M * (2 * d) / med / 1e6}
        th = torch.matmul
        med, mn = timeit(lambda: th(A1, W1.t(), out=out))
        res["torch_matmul_fp32_10Mx128x128"] = {"ms": med, "TFLOPs": 2 * M * d * d / med / 1e9}
        del A1, A2, out
    if args.only in ("", "spmm"):
        n_u, n_i, E, d = 10_000_000, 1_000_000, 500_000_000, 128
        for zipf in (0.0, args.zipf):
            cdf = None
            if zipf > 0:
                w = 1.0 / torch.arange(1, n_i + 1, dtype=torch.float64, device=dev) ** zipf
                cdf = torch.cumsum(w, 0)
                cdf /= cdf[-1].clone()
            u, i = ops.synth_edges(11, 0, E, n_u, n_i, dev, cdf)
            ip_i, ix_i, _ = build_csr(u.long(), i.long(), n_i)   # user -> item (dst item)
            ip_u, ix_u, _ = build_csr(i.long(), u.long(), n_u)   # item -> user (dst user)
            del u, i
            Xu = torch.randn(n_u, d, device=dev)
            Xi = torch.randn(n_i, d, device=dev)
            oi = torch.empty(n_i, d, device=dev)
            ou = torch.empty(n_u, d, device=dev)
            tag = f"zipf{zipf:g}"
            for name, fn, by in (
                    ("user->item sum", lambda: ops.spmm(ip_i, ix_i, Xu, "sum", out=oi),
                     E * (4 * d + 4) + n_i * (8 + 4 * d)),
                    ("item->user mean", lambda: ops.spmm(ip_u, ix_u, Xi, "mean", out=ou),
                     E * (4 * d + 4) + n_u * (8 + 4 * d))):
                med, mn = timeit(fn, reps=5)
                res[f"spmm {name} {tag}"] = {"ms": med, "min_ms": mn, "TBs_alg": by / med / 1e9,
                                             "Gedges": E / med / 1e6}
            if zipf > 0:
                med, _ = timeit(lambda: ops.spmm(ip_i, ix_i, Xu, "sum", out=oi, split=None), reps=2,
                                warm=1)
                res[f"spmm user->item sum {tag} NO split"] = {"ms": med}
            del ip_i, ix_i, ip_u, ix_u, Xu, Xi, oi, ou
            torch.cuda.empty_cache()
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
