"""Quick GPU probe: load libgnnrec.so next to torch and run each kernel once
against torch fp32 references (developer tool; the real tests live in tests/)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402


def csr_random(n_dst, n_src, avg_deg, g):
    deg = torch.randint(0, 2 * avg_deg + 1, (n_dst,), generator=g)
    indptr = torch.zeros(n_dst + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(deg, 0)
    E = int(indptr[-1])
    idx = torch.randint(0, n_src, (E,), generator=g, dtype=torch.int64)
    return indptr, idx


def ref_spmm(indptr, idx, X, reduce, w=None):
    n_dst = indptr.numel() - 1
    out = torch.zeros(n_dst, X.shape[1], dtype=torch.float64)
    Xd = X.double()
    for v in range(n_dst):
        a, b = int(indptr[v]), int(indptr[v + 1])
        if b == a:
            continue
        m = Xd[idx[a:b]]
        if w is not None:
            m = m * w[a:b].double()[:, None]
        if reduce == "max":
            out[v] = m.max(0).values
        elif reduce == "mean":
            out[v] = m.sum(0) / (b - a)
        else:
            out[v] = m.sum(0)
    return out


def main():
    dev = torch.device("cuda")
    print("device:", torch.cuda.get_device_name(0), flush=True)
    g = torch.Generator().manual_seed(0)
    ok = True
    for d in (128, 64, 32, 100, 7, 256, 300):
        for reduce in ("mean", "max", "sum"):
            for weighted in (False, True):
                indptr, idx = csr_random(300, 500, 9, g)
                X = torch.randn(500, d, generator=g)
                w = torch.rand(idx.numel(), generator=g) * 4 if weighted else None
                out = ops.spmm(indptr.to(dev), idx.to(torch.int32).to(dev), X.to(dev), reduce,
                               edge_weight=None if w is None else w.to(dev))
                ref = ref_spmm(indptr, idx, X, reduce, w)
                err = ((out.cpu().double() - ref).abs().max() / (ref.abs().max() + 1e-30)).item()
                if err > 1e-5:
                    ok = False
                print(f"spmm d={d} {reduce} w={weighted}: rel err {err:.2e}", flush=True)
    for (M, K1, K2, N) in ((1000, 128, 128, 128), (777, 64, 64, 64), (300, 4, 256, 256),
                           (513, 2, 0, 32), (129, 128, 0, 1)):
        A1 = torch.randn(M, K1, generator=g)
        W1 = torch.randn(N, K1, generator=g) * 0.1
        A2 = torch.randn(M, K2, generator=g) if K2 else None
        W2 = torch.randn(N, K2, generator=g) * 0.1 if K2 else None
        b = torch.randn(N, generator=g)
        z = A1.double() @ W1.double().T + b.double()
        if K2:
            z = z + A2.double() @ W2.double().T
        z = torch.relu(z)
        nrm = z.norm(dim=1, keepdim=True)
        zr = z / torch.where(nrm == 0, torch.ones_like(nrm), nrm)
        out = ops.gemm(A1.to(dev), W1.to(dev), None if A2 is None else A2.to(dev),
                       None if W2 is None else W2.to(dev), b.to(dev), relu=True, l2norm=N <= 256)
        err = ((out.cpu().double() - zr).abs().max()).item()
        if err > 1e-5:
            ok = False
        print(f"gemm M={M} K1={K1} K2={K2} N={N}: max abs err {err:.2e}", flush=True)
    # timing of a C4-like relation slice
    n_dst, n_src, deg, d = 1_000_000, 10_000_000, 50, 128
    indptr = torch.arange(0, (n_dst + 1) * deg, deg, dtype=torch.int64, device=dev)
    idx = torch.randint(0, n_src, (n_dst * deg,), dtype=torch.int32, device=dev)
    X = torch.randn(n_src, d, device=dev)
    out = torch.empty(n_dst, d, device=dev)
    for _ in range(3):
        ops.spmm(indptr, idx, X, "mean", out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 10
    for _ in range(reps):
        ops.spmm(indptr, idx, X, "mean", out=out)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    E = n_dst * deg
    bytes_ = E * (d * 4 + 4) + n_dst * (8 + d * 4)
    print(f"spmm 1M x deg50 d128 from 10M table: {t*1e3:.2f} ms, {E/t/1e9:.2f} Gedges/s, "
          f"{bytes_/t/1e12:.2f} TB/s algorithmic", flush=True)
    print("ALL OK" if ok else "MISMATCH", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
