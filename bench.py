"""bench.py — edges aggregated/s of the full-graph inference embedding pass.

BASELINE.json metric: "edges aggregated/sec, full-graph embed pass, d=128, at
1/2/4/8 MI355X".  Workload (BASELINE.json configs[3], "C4"): 10M users x 1M
items, 500M user->item edges (+ the 500M reverse item->user edges), ConvModel
with NodeEmbedding + L=2 ConvLayers (n_layers=3, embedding_layer=True),
aggregator 'mean', hetero 'sum', norm=True, d=128 fp32 (reference
src/model.py:330-421 driven as src/train/run.py:311-349 with a full-neighbour
sampler).  Synthetic graph (counter-hash generator, seed 11), N(0,1) features
(seed 0) and xavier weights (torch.manual_seed(0)) — no dataset exists offline.

A step = one full pass over the whole graph: embed + 2 layers x 2 relations.
edges aggregated per step = L x sum_r |E_r| = 2 x (500M + 500M) = 2e9.
Multi-GPU: one process per GPU (torchrun), users partitioned, edges follow
their user; per layer one reduce-scatter + one all-gather of the 1M-row item
table over RCCL; per-GPU work shrinks with N at fixed total graph.

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=500_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--zipf", type=float, default=0.0, help="item Zipf exponent (0 = uniform)")
    ap.add_argument("--aggregator", default="mean")
    ap.add_argument("--config", choices=["c4", "c5"], default="c4",
                    help="c5: the C4 graph split 80%% clicks / 20%% buys -> 4 relations")
    ap.add_argument("--hetero", choices=["sum", "mean", "max", "attention"], default="sum")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--mode", choices=["deterministic", "fast"], default="deterministic",
                    help="deterministic: outputs bitwise equal at 1/2/4/8 GPUs (fixed segment "
                         "tree + all-to-all); fast: tiles accumulated in place + reduce-scatter")
    ap.add_argument("--segments", type=int, default=8,
                    help="source-range tiles of the user->item relation (0: none; "
                         "deterministic mode needs a power of two divisible by the GPU count)")
    ap.add_argument("--concurrency", default="auto",
                    help="row-kernel schedule: 'auto' (static at one rank; 16 CUs reserved + "
                         "work queue beside RCCL at several) or 'R,Q' (R reserved CUs, Q=1 queue)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-scale", type=float, default=0.1,
                    help="fraction of the graph used for the bounded CPU-baseline sample")
    return ap.parse_args()


class EventTimers:
    """HIP-event timing of tagged kernel launches on the current stream."""

    def __init__(self):
        self.events = {}
        self.enabled = False

    @contextlib.contextmanager
    def __call__(self, tag):
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self.events.setdefault(tag, []).append((s, e))

    def mean_ms(self, tag):
        ev = self.events.get(tag, [])
        if not ev:
            return float("nan"), 0
        return sum(s.elapsed_time(e) for s, e in ev) / len(ev), len(ev)


KERNELS = {
    "spmm_project": ("spmm_project_kernel", "gnnrec spmm_project_kernel (gather + segmented "
                     "mean + fused SAGE projection, ReLU, L2 norm)"),
    "spmm_tile": ("spmm_csr_kernel", "gnnrec spmm_csr_kernel (gather + segmented sum of one "
                  "source-range tile, accumulated in place)"),
    "spmm": ("spmm_csr_kernel", "gnnrec spmm_csr_kernel (gather + segmented mean)"),
}


def launch_bytes(shard, d, fused, deterministic):
    """Algorithmic bytes per layer and launches per layer of each aggregation kernel tag
    (SURVEY §8d row d4): per edge d*4 (fp32 source row) + 4 (int32 index); per dst row 8
    (int64 indptr) + d*4 (write), + d*4 for the h_self row when the projection is fused
    into the launch, + d*4 for the partial read back when a tile accumulates in place."""
    out = {}
    for ce, rs in shard.rels.items():
        if ce in fused:
            tag, b, n = "spmm_project", rs.local_edges * (d * 4 + 4) + rs.n_rows * (8 + 8 * d), 1
        elif rs.segs is not None:
            tag, b, n = "spmm_tile", 0, len(rs.segs)
            for j, (ip, ix, _) in enumerate(rs.segs):
                acc = (j % 2 == 1) if deterministic else j > 0
                b += ix.numel() * (d * 4 + 4) + rs.n_rows * (8 + 4 * d * (2 if acc else 1))
        else:
            tag, b, n = "spmm", rs.local_edges * (d * 4 + 4) + rs.n_rows * (8 + 4 * d), 1
        tb, tn = out.get(tag, (0, 0))
        out[tag] = (tb + b, tn + n)
    return out


def pmc_traffic(args, world, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (FETCH_SIZE x2 for gfx950's half-counted wide reads + WRITE_SIZE, KB -> B), for
    the default single-GPU C4 workload they were collected on; None otherwise."""
    import csv
    default = (args.users, args.items, args.edges, args.dim, args.zipf, args.aggregator,
               args.config, args.mode, args.segments) == (10_000_000, 1_000_000, 500_000_000,
                                                          128, 0.0, "mean", "c4",
                                                          "deterministic", 8)
    f = os.path.join(ROOT, "profiles", "r01_c4_pmc_fetch.csv")
    w = os.path.join(ROOT, "profiles", "r01_c4_pmc_write.csv")
    if world != 1 or not default or not (os.path.exists(f) and os.path.exists(w)):
        return None
    tot, n = 0.0, 0
    for path, scale in ((f, 2.0), (w, 1.0)):
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                tot += float(r["Counter_Value"]) * 1024 * scale
                n += scale == 2.0
    return tot / n if n else None


def cpu_baseline(args, d):
    """Bounded sample of the same workload on the host cores: the oracle's C/OpenMP
    restatement of DGL 0.5's CPU SpMM + numpy fp32 GEMMs (kind 'port')."""
    import numpy as np

    sys.path.insert(0, ROOT)
    from oracle import oracle

    U = max(1000, int(args.users * args.cpu_scale))
    I = max(100, int(args.items * args.cpu_scale))
    E = max(1000, int(args.edges * args.cpu_scale))
    u, i = oracle.synth_edges(11, 0, E, U, I)
    g = oracle.Graph({"user": U, "item": I},
                     {("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u)})
    for ce in g.canonical_etypes:
        g.csr(ce)
    rng = np.random.default_rng(0)
    feats = {"user": rng.standard_normal((U, d), dtype=np.float32),
             "item": rng.standard_normal((I, d), dtype=np.float32)}
    torch.manual_seed(0)
    sd = {}
    for nt in ("user", "item"):
        lin = torch.nn.Linear(d, d)
        sd[f"{nt}_embed.proj_feats.weight"] = lin.weight.detach().numpy()
        sd[f"{nt}_embed.proj_feats.bias"] = lin.bias.detach().numpy()
    for layer in range(2):
        for rel in ("buys", "bought-by"):
            for w in ("fc_self", "fc_neigh"):
                t = torch.empty(d, d)
                torch.nn.init.xavier_uniform_(t, gain=torch.nn.init.calculate_gain("relu"))
                sd[f"layers.{layer}.mods.{rel}.{w}.weight"] = t.numpy()
    reps, t_tot = 0, 0.0
    while reps < 2 or (t_tot < 10.0 and reps < 5):
        t0 = time.perf_counter()
        oracle.model_full_graph(g, feats, sd, args.aggregator, "sum", True, True)
        t_tot += time.perf_counter() - t0
        reps += 1
    edges = 2 * 2 * E
    return {"value": edges * reps / t_tot, "unit": "edges/s", "cores": oracle.num_threads(),
            "kind": "port",
            "sample": f"{U} users x {I} items x {E} edges ({args.cpu_scale:g} of the workload, "
                      f"same mean degrees), same model, {reps} passes, {t_tot:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = local_rank % max(1, torch.cuda.device_count())  # rehearsals may share one GPU
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if world > 1:
        # RCCL over xGMI; GNNREC_DIST_BACKEND=gloo rehearses several ranks on one GPU
        backend = os.environ.get("GNNREC_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from gnnrec import nn as gnn
    from gnnrec.dist import Exchange
    from gnnrec.inference import ShardedFullGraphPass
    from gnnrec.synth import GraphMeta, bipartite_shard, node_features

    d = args.dim
    split = ((("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2)) if args.config == "c5"
             else (("buys", "bought-by", 1.0),))
    segments = args.segments or None
    det = args.mode == "deterministic"
    if det and (segments is None or segments % world or segments & (segments - 1)):
        det = False  # the fixed tree needs a power-of-two segment count divisible by P
    if segments is not None and segments < world:
        segments = None
    shard = bipartite_shard(args.users, args.items, args.edges, rank, world, dev,
                            zipf_s=args.zipf, split=split, segments=segments)
    feats = {"user": node_features(args.users, d, 0, dev, slice(shard.p_lo, shard.p_hi)),
             "item": torch.zeros((shard.padded_rows("item"), d), device=dev)}
    feats["item"][: args.items] = node_features(args.items, d, 1, dev)
    torch.manual_seed(0)
    meta = GraphMeta(shard.canonical_etypes, ["item", "user"])
    model = gnn.ConvModel(meta, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0,
                          args.aggregator, "cos", args.hetero, True).to(dev).eval()
    ex = Exchange()
    conc = None
    if args.concurrency != "auto":
        r, q = args.concurrency.split(",")
        conc = (int(r), bool(int(q)))
    runner = ShardedFullGraphPass(model, shard, ex, overlap=not args.no_overlap,
                                  deterministic=det, concurrency=conc)
    timers = EventTimers()
    runner.timers = timers
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        out = runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timers.enabled = True
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = ex.max_scalar(elapsed, dev)
    del out

    edges_per_step = 2 * sum(rs.global_edges for rs in shard.rels.values())  # L=2 layers
    value = edges_per_step * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3
    # roofline of the aggregation kernels: the fused gather+projection launch when the pass
    # has one (C4: the user side, ~half the pass), else the busiest tag; the other
    # aggregation kernel (C4: the item side's source-range tiles) is reported beside it
    per_tag = launch_bytes(shard, d, runner.fused, det)
    ran = [t for t in per_tag if timers.mean_ms(t)[1]]

    def line(t):
        ms, n = timers.mean_ms(t)
        b = per_tag[t][0] / per_tag[t][1]  # bytes per layer / launches per layer
        return ms, n, b, b / (ms * 1e-3) / 1e9

    tag = "spmm_project" if "spmm_project" in ran else max(
        ran, key=lambda t: timers.mean_ms(t)[0] * timers.mean_ms(t)[1]) if ran else "spmm"
    spmm_ms, n_launch, bytes_per_launch, achieved = line(tag) if ran else (None, 0, None, None)
    others = {t: dict(zip(("launch_ms", "launches_timed", "bytes_per_launch", "achieved"),
                          line(t)), kernel=KERNELS[t][1]) for t in ran if t != tag}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        try:
            cpu = cpu_baseline(args, d)
        except Exception as exc:  # the baseline never masks the GPU result
            cpu = {"value": None, "unit": "edges/s", "cores": None, "kind": "port",
                   "sample": f"failed: {exc!r}"}

    if rank == 0:
        rec = {
            "metric": "edges aggregated/sec, full-graph embed pass, d=128",
            "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (counter-hash graph seed 11, N(0,1) features, xavier weights)",
            "config": {"workload": (args.config.upper() if (args.users, args.items, args.edges) ==
                                    (10_000_000, 1_000_000, 500_000_000) else "custom")
                                   + f" full-graph embed pass: {args.users} users x {args.items} "
                                   f"items, {args.edges} edges/direction"
                                   + (" (80% clicks / 20% buys, 4 relations)"
                                      if args.config == "c5" else "")
                                   + f", NodeEmbedding + L=2 ConvLayer '{args.aggregator}', "
                                     f"hetero {args.hetero}, norm, d={d}"
                                   + (f", item zipf s={args.zipf}" if args.zipf else "")
                                   + (f", {shard.segments} source tiles" if shard.segments
                                      else "")
                                   + (", deterministic (bitwise equal at 1/2/4/8 GPUs)" if det
                                      else ""),
                       "edges_per_step": edges_per_step, "parallelism": f"graph{world}",
                       "output": "partitioned (each rank keeps the user and item rows it owns)",
                       "overlap": not args.no_overlap,
                       "row_schedule": ("static" if not runner.concurrency or
                                        not runner.concurrency[1] else "queue")
                                       + (f", {runner.concurrency[0]} CUs reserved"
                                          if runner.concurrency and runner.concurrency[0]
                                          else "")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": pmc_traffic(args, world, KERNELS[tag][0]),
                         "kernel": KERNELS[tag][1],
                         "bytes_per_launch": bytes_per_launch, "launch_ms": spmm_ms,
                         "launches_timed": n_launch,
                         "other_kernels": {t: dict(o, frac=o["achieved"] / HBM_PEAK_GBS)
                                           for t, o in others.items()}},
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
