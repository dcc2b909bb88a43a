"""Aggregation backward (atomic scatter vs device transpose + gather) on a sampled-block shape: 730k dst rows x fanout 10
into 1.1M source rows, d=128 (the first block of a C3 training step).

    python tools/bench_spmm_bwd.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402


def t(fn, reps=5):
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
    dev = torch.device("cuda")
    n_dst, n_src, fan, d = 730_000, 1_100_000, 10, 128
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    indptr = torch.arange(0, (n_dst + 1) * fan, fan, device=dev, dtype=torch.int64)
    idx = torch.randint(0, n_src, (n_dst * fan,), device=dev, generator=gen, dtype=torch.int32)
    G = torch.randn(n_dst, d, device=dev, generator=gen)
    X = torch.randn(n_src, d, device=dev, generator=gen)
    res = {}
    for reduce in ("mean", "max"):
        Y = ops.spmm(indptr, idx, X, reduce)
        gX = torch.zeros(n_src, d, device=dev)
        ms = t(lambda: ops.spmm_backward(indptr, idx, G, reduce, None, X=X, out=Y, grad_X=gX))
        E = n_dst * fan
        res[reduce] = {"atomic_ms": ms, "edges": E, "G_atomics_per_s": E * d / ms / 1e6}
        if reduce == "mean":
            tt = t(lambda: ops.csr_transpose(indptr, idx, n_src, mean=True))
            ip_t, ix_t, w_t = ops.csr_transpose(indptr, idx, n_src, mean=True)
            tg = t(lambda: ops.spmm(ip_t, ix_t, G, "sum", edge_weight=w_t))
            res[reduce].update({"transpose_ms": tt, "gather_ms": tg, "transpose_gather_ms": tt + tg})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
