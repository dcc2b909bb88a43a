"""Per-rank compute of the sharded C4/C5 pass at P ranks, EVERY rank, measured on one GPU.

For each P and each rank r < P: builds rank r's shard of the P-way partition exactly as
bench.py does at P ranks (its users' edges in 8/P source tiles, the replicated item table,
degree-balanced user ranges), then runs the bench's pass (deterministic mode, the P > 1
row schedule: 16 CUs reserved + row queue) with gnnrec.dist.ComputeOnlyExchange(P, r) —
the same kernels and launch order, no bytes moved — and times it.  The max over ranks is
the compute floor of a P-GPU pass; the collectives come on top, partly hidden.

Projection per P (written with the measurements):
  comm_bytes   bytes one rank sends per pass: per layer an all-to-all of the item partials
               ((P-1)/P of the padded table) and, except after the last layer, an all-gather
               of the projected item rows ((P-1) own blocks);
  comm_ms      comm_bytes over 7 xGMI links x 153 GB/s (MI355X_MICROARCH.md; the ideal
               all-to-all: every peer on its own link) — a floor, RCCL reaches less;
  projected_ms max rank compute + comm_ms (no overlap: the pessimistic end) and
               max(compute, comm) (full overlap), with the speedups over P = 1.

    python tools/probe_rank_work.py [--config c4|c5] [--out FILE] [P ...]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import nn as gnn  # noqa: E402
from gnnrec.dist import ComputeOnlyExchange  # noqa: E402
from gnnrec.inference import RESERVE_CUS, ShardedFullGraphPass  # noqa: E402
from gnnrec.synth import GraphMeta, bipartite_shard, node_features  # noqa: E402

XGMI_GBS = 7 * 153.0
LINK_FRACTIONS = (1.0, 0.5, 0.35, 0.25)  # of the links' peak an RCCL exchange may reach


def rank_ms(P, r, split, dev, reps=3):
    n_u, n_i, E, d = 10_000_000, 1_000_000, 500_000_000, 128
    t_build = time.perf_counter()
    sh = bipartite_shard(n_u, n_i, E, r, P, dev, split=split, segments=8)
    feats = {"user": node_features(n_u, d, 0, dev, slice(sh.p_lo, sh.p_hi)),
             "item": torch.zeros((sh.padded_rows("item"), d), device=dev)}
    feats["item"][:n_i] = node_features(n_i, d, 1, dev)
    t_build = time.perf_counter() - t_build
    torch.manual_seed(0)
    meta = GraphMeta(sh.canonical_etypes, ["item", "user"])
    model = gnn.ConvModel(meta, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev).eval()
    conc = (RESERVE_CUS, True) if P > 1 else None  # what the pass picks at P ranks
    runner = ShardedFullGraphPass(model, sh, ComputeOnlyExchange(P, r), deterministic=True,
                                  concurrency=conc)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    for _ in range(2):
        runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / reps * 1e3
    rec = {"rank": r, "compute_ms": round(ms, 3), "local_edges": sh.local_edge_count(),
           "users": [sh.p_lo, sh.p_hi], "build_s": round(t_build, 1)}
    S = sh.padded_rows("item") // P
    del sh, feats, runner, model
    torch.cuda.empty_cache()
    return rec, S


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ps", nargs="*", type=int, default=[1, 2, 4, 8])
    ap.add_argument("--config", choices=["c4", "c5"], default="c4")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    split = ((("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2)) if a.config == "c5"
             else (("buys", "bought-by", 1.0),))
    dev = torch.device("cuda")
    d, layers = 128, 2
    res = {"config": a.config, "device": torch.cuda.get_device_name(dev),
           "schedule": f"P > 1: {RESERVE_CUS} CUs reserved + row queue (the bench's default)",
           "per_P": {}}
    for P in a.ps:
        ranks = []
        for r in range(P):
            rec, S = rank_ms(P, r, split, dev)
            ranks.append(rec)
            print(json.dumps({"P": P, **rec}), file=sys.stderr, flush=True)
        comp = max(x["compute_ms"] for x in ranks)
        tbl = P * S * d * 4  # padded item table, fp32
        n_rep = len(split)  # item partial tables exchanged per layer (one per relation into items)
        a2a = layers * n_rep * tbl * (P - 1) // P
        ag = (layers - 1) * (P - 1) * S * d * 4
        comm_b = a2a + ag
        comm_ms = comm_b / (XGMI_GBS * 1e9) * 1e3
        res["per_P"][str(P)] = {
            "ranks": ranks, "max_compute_ms": comp,
            "imbalance": comp / (sum(x["compute_ms"] for x in ranks) / P),
            "comm_bytes_per_rank": comm_b, "comm_ms_floor": round(comm_ms, 3),
            "projected_ms_no_overlap": round(comp + comm_ms, 3),
            "projected_ms_full_overlap": round(max(comp, comm_ms), 3),
            # RCCL's all-to-all reaching half the links' rate, nothing overlapped
            "projected_ms_half_rate_no_overlap": round(comp + 2 * comm_ms, 3),
            # the exchange priced at a stated fraction of the 7 x 153 GB/s link peak, nothing
            # overlapped (the pass overlaps the partial exchange with the item->user launch,
            # so these are upper bounds on the pass time at that rate)
            "projected_ms_by_link_fraction_no_overlap": {
                str(f): round(comp + comm_ms / f, 3) for f in LINK_FRACTIONS}}
        print(json.dumps({"P": P, **{k: v for k, v in res["per_P"][str(P)].items()
                                     if k != "ranks"}}), flush=True)
    if "1" in res["per_P"]:
        base = res["per_P"]["1"]["max_compute_ms"]
        for P, v in res["per_P"].items():
            v["speedup_no_overlap"] = round(base / v["projected_ms_no_overlap"], 2)
            v["speedup_full_overlap"] = round(base / v["projected_ms_full_overlap"], 2)
            v["speedup_half_rate_no_overlap"] = round(
                base / v["projected_ms_half_rate_no_overlap"], 2)
            v["speedup_by_link_fraction_no_overlap"] = {
                f: round(base / ms, 2) for f, ms in v["projected_ms_by_link_fraction_no_overlap"].items()}
    out = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(out)
    print(out, flush=True)


if __name__ == "__main__":
    main()
