"""Per-relation timing of the fused aggregate+project launches on the C5 graph
(80 % clicks / 20 % buys): which launch is slow and why.

    python tools/probe_c5.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402
from gnnrec.synth import bipartite_shard  # noqa: E402


def t(fn, reps=3):
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
    split = (("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2))
    sh = bipartite_shard(10_000_000, 1_000_000, 500_000_000, 0, 1, dev, split=split)
    d = 128
    X = {"user": torch.randn(10_000_000, d, device=dev), "item": torch.randn(1_000_000, d, device=dev)}
    W = torch.randn(d, d, device=dev) * 0.1
    only = os.environ.get("PROBE_REL")  # e.g. bought-by
    for ce, rs in sh.rels.items():
        if only and ce[1] != only:
            continue
        n = rs.indptr.numel() - 1
        deg = (rs.indptr[1:] - rs.indptr[:-1])
        out = torch.empty(n, d, device=dev)
        E = int(rs.indptr[-1])
        res = {}
        for v in [v for v in os.environ.get("PROBE_VARIANTS", "valu,mfma,pre").split(",")
                  if v in ("valu", "mfma")]:
            res[v] = t(lambda: ops.spmm_project(rs.indptr, rs.indices, X[ce[0]], X[ce[2]][:n], W,
                                                W, "mean", None, relu=True, l2norm=True, out=out,
                                                variant=v))
        if "pre" in os.environ.get("PROBE_VARIANTS", "valu,mfma,pre").split(","):
            # pre-projected source rows: the fused launch runs the self half on the MFMA
            Y = ops.preproject(X[ce[0]], W)
            res["pre"] = t(lambda: ops.spmm_project(rs.indptr, rs.indices, Y, X[ce[2]][:n], W,
                                                    None, "mean", None, relu=True, l2norm=True,
                                                    out=out))
            res["preproj"] = t(lambda: ops.preproject(X[ce[0]], W, out=Y))
            del Y
        agg = ops.spmm(rs.indptr, rs.indices, X[ce[0]], "mean")
        res["spmm"] = t(lambda: ops.spmm(rs.indptr, rs.indices, X[ce[0]], "mean", out=agg))
        res["gemm"] = t(lambda: ops.gemm(X[ce[2]][:n], W, agg, W, relu=True, l2norm=True,
                                         out=out))
        alg = E * 516 + n * 1032  # fused: per edge row + index, per row indptr + self + out
        print(f"{ce}: rows {n} edges {E} deg max {int(deg.max())} mean {E / n:.1f} | "
              + " ".join(f"{k} {ms:.2f} ms" for k, ms in res.items())
              + " | fused " + ", ".join(f"{v} {alg / res[v] / 1e9:.2f} TB/s" for v in
                                         ("valu", "mfma", "pre") if v in res)
              + " (algorithmic) | split_plan "
              f"{'yes' if ops.split_plan(rs.indptr) is not None else 'no'}", flush=True)


def dual():
    """C5's two item->user relations (clicked-by 40 edges/row, bought-by 10) as one
    pre-projected launch (ops.spmm_project2) vs the pass's two launches."""
    dev = torch.device("cuda")
    split = (("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2))
    sh = bipartite_shard(10_000_000, 1_000_000, 500_000_000, 0, 1, dev, split=split)
    d = 128
    Xu, Xi = torch.randn(10_000_000, d, device=dev), torch.randn(1_000_000, d, device=dev)
    W = [torch.randn(d, d, device=dev) * 0.1 for _ in range(4)]
    ra, rb = sh.rels[("item", "clicked-by", "user")], sh.rels[("item", "bought-by", "user")]
    Ya, Yb = ops.preproject(Xi, W[1]), ops.preproject(Xi, W[3])
    out = torch.empty(10_000_000, d, device=dev)
    res = {}
    res["dual"] = t(lambda: ops.spmm_project2((ra.indptr, ra.indices, Ya, "mean", None, None),
                                              (rb.indptr, rb.indices, Yb, "mean", None, None),
                                              Xu, W[0], W[2], relu=True, l2norm=True,
                                              out=out))

    def two():
        ops.spmm_project(ra.indptr, ra.indices, Xi, Xu, W[0], W[1], "mean", None, relu=True,
                         l2norm=True, out=out)
        ops.spmm_project(rb.indptr, rb.indices, Yb, Xu, W[2], None, "mean", None, relu=True,
                         l2norm=True, accum="add", out=out)
    res["two"] = t(two)
    E = int(ra.indptr[-1]) + int(rb.indptr[-1])
    alg = E * 516 + 10_000_000 * (16 + 1024)
    print("user side (clicked-by + bought-by): " + " ".join(f"{k} {v:.2f} ms" for k, v in
                                                             res.items())
          + f" | dual {alg / res['dual'] / 1e9:.2f} TB/s (algorithmic)", flush=True)


if __name__ == "__main__":
    if os.environ.get("PROBE_DUAL") == "1":
        dual()
        sys.exit(0)
    main()
