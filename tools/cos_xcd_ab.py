"""Grouped cosine at BASELINE configs[2]'s (C3) head shape — 1024 sources x 2500 negatives,
d = 128, a 100k-row item table (51 MB) — over the XCD-slice pass counts
(GNNREC_COS_XCD_PASSES: 0 = the unsliced kernel), and d = 64 (C2's 25.6 MB table): HIP-event
time per launch and a bitwise check against the per-edge kernel.

    python tools/cos_xcd_ab.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    for d in (128, 64):
        n_u, n_i, K = 1024, 100_000, 2500
        Hs = torch.randn(n_u, d, device=dev, generator=gen)
        Hd = torch.randn(n_i, d, device=dev, generator=gen)
        ps = torch.arange(n_u, device=dev)
        pd = torch.randint(0, n_i, (n_u,), device=dev, generator=gen)
        nd = torch.randint(0, n_i, (n_u * K,), device=dev, generator=gen)
        ref = ops.sddmm_cos(torch.cat([ps, ps.repeat_interleave(K)]), torch.cat([pd, nd]), Hs, Hd)
        res = {"d": d, "table_MB": n_i * d * 4 / 1e6}
        for passes in ("0", "1", "2", "3", "4", "6"):
            os.environ["GNNREC_COS_XCD_PASSES"] = passes
            a, b = ops.sddmm_cos_grouped(ps, pd, K, nd, Hs, Hd)
            same = bool(torch.equal(a, ref[:n_u]) and torch.equal(b, ref[n_u:]))
            for _ in range(3):
                ops.sddmm_cos_grouped(ps, pd, K, nd, Hs, Hd)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                ops.sddmm_cos_grouped(ps, pd, K, nd, Hs, Hd)
            e.record()
            e.synchronize()
            res[f"passes{passes}"] = {"ms": round(s.elapsed_time(e) / 50, 4), "bitwise": same}
        os.environ.pop("GNNREC_COS_XCD_PASSES")
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
