"""How fast does the gather+aggregate run when the gathered table fits the Infinity Cache?

Same edge count and destination rows, source tables of different sizes (uniform random
sources).  Decides whether a source-chunked (cache-blocked) schedule can beat the
plain pull over a 5 GB table.

    python tools/probe_table_size.py
"""
import json
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
    d = 128
    res = {}
    for n_dst, E in ((100_000, 50_000_000), (1_000_000, 50_000_000)):
        dst = torch.randint(0, n_dst, (E,), device=dev)
        for n_src in (16_384, 65_536, 131_072, 262_144, 524_288, 1_000_000, 10_000_000):
            src = torch.randint(0, n_src, (E,), device=dev)
            ip, ix, _ = build_csr(src, dst, n_dst)
            X = torch.randn(n_src, d, device=dev)
            out = torch.empty(n_dst, d, device=dev)
            ms = t(lambda: ops.spmm(ip, ix, X, "sum", out=out))
            by = E * (d * 4 + 4) + n_dst * (8 + d * 4)
            res[f"dst={n_dst} src={n_src} ({n_src * d * 4 / 2**20:.0f} MiB)"] = {
                "ms": ms, "TBs_alg": by / ms / 1e9}
            print(json.dumps(res, indent=1), flush=True)
            del src, ip, ix, X, out
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
