"""Do the HBM-bound aggregation and the MFMA-bound projection GEMM co-run on two streams?

Times spmm alone, GEMM alone, and both launched on separate streams (C4 item->user shape).
    GNNREC_SPMM_BLOCKS_PER_CU=4 python tools/overlap_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402
from gnnrec.graph import build_csr  # noqa: E402


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
    n_u, n_i, E, d = 10_000_000, 1_000_000, 500_000_000, 128
    u, i = ops.synth_edges(11, 0, E, n_u, n_i, dev)
    ip, ix, _ = build_csr(i.long(), u.long(), n_u)
    del u, i
    Xi = torch.randn(n_i, d, device=dev)
    agg = torch.empty(n_u, d, device=dev)
    A1 = torch.randn(n_u, d, device=dev)
    A2 = torch.randn(n_u, d, device=dev)
    W = torch.randn(d, d, device=dev) * 0.1
    out = torch.empty(n_u, d, device=dev)
    side = torch.cuda.Stream()

    def spmm():
        ops.spmm(ip, ix, Xi, "mean", out=agg)

    def gemm():
        ops.gemm(A1, W, A2, W, relu=True, l2norm=True, out=out)

    def both():
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            gemm()
        spmm()
        torch.cuda.current_stream().wait_stream(side)

    ts, tg, tb = t(spmm), t(gemm), t(both)
    print(f"blocks/CU={os.environ.get('GNNREC_SPMM_BLOCKS_PER_CU', '8')}: spmm {ts:.2f} ms, "
          f"gemm {tg:.2f} ms, both {tb:.2f} ms (serial sum {ts + tg:.2f}, hidden "
          f"{ts + tg - tb:.2f} ms)", flush=True)


if __name__ == "__main__":
    main()
