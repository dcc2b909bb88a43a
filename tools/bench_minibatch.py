"""Minibatch-side measurements on the BASELINE.json C2/C3 shapes (rows a7/a8/a9).

C2: 1M users x 100k items, 50M edges per direction, d=64, 2-layer, fanout [10,10],
    node batch 1024  -> GPU block sampler throughput (sampled edges/s, batches/s)
C3: same graph, d=128, n_layers=3 mean_nn (+NodeEmbedding: 2 conv layers), cosine head,
    edge batch 1024 x 2500 negatives -> heads kernels (GB/s) and one training step.
CPU comparison: the oracle's C sampler (single thread, same algorithm) on the same seeds.

    python tools/bench_minibatch.py [--batches 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gnnrec import nn as gnn, ops  # noqa: E402
from gnnrec.graph import HeteroGraph  # noqa: E402
from gnnrec.sampling import (EdgeDataLoader, MultiLayerFullNeighborSampler,  # noqa: E402
                             MultiLayerNeighborSampler, NodeDataLoader, negative_sampler)

BUYS = ("user", "buys", "item")
BOUGHT = ("item", "bought-by", "user")


def sync_time(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t, r


def c2_graph(d, dev, n_u=1_000_000, n_i=100_000, E=50_000_000):
    from gnnrec.synth import minibatch_graph
    return minibatch_graph(d, dev, n_u, n_i, E)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    res = {}

    # ---- C2: fanout [10,10] block sampling, node batch 1024 -------------------------------
    g = c2_graph(64, dev)
    sampler = MultiLayerNeighborSampler([10, 10], seed=1)
    loader = NodeDataLoader(g, {"user": torch.arange(1_000_000), "item": torch.arange(100_000)},
                            sampler, batch_size=1024, shuffle=True)
    it = iter(loader)
    next(it)  # warm-up (relabel scratch, plans)
    n_edges = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.batches):
        _, _, blocks = next(it)
        n_edges += sum(b.num_edges(ce) for b in blocks for ce in b.canonical_etypes)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["C2 sampler fanout[10,10] batch1024"] = {
        "batches_per_s": args.batches / dt, "sampled_edges_per_s": n_edges / dt,
        "ms_per_batch": dt / args.batches * 1e3, "edges_per_batch": n_edges / args.batches}
    # CPU oracle sampler on the same CSR and the same seeds (one layer, single thread)
    from oracle import oracle
    indptr, indices, eids = [t.cpu().numpy().astype(np.int64) for t in g.in_csr_global(BOUGHT)]
    seeds = np.random.default_rng(0).choice(1_000_000, 1024 * 8, replace=False).astype(np.int64)
    t = time.perf_counter()
    _, s_cpu, _ = oracle.sample_neighbors(indptr, indices, eids, seeds, 10, 7)
    t_cpu = time.perf_counter() - t
    tg, (ip_g, s_g, _) = sync_time(lambda: ops.sample_neighbors(
        *g.in_csr_global(BOUGHT), torch.from_numpy(seeds).to(dev), 10, 7))
    assert np.array_equal(s_g.cpu().numpy(), s_cpu)
    res["one-layer fanout-10 sampling, 8192 seeds"] = {
        "gpu_ms": tg * 1e3, "cpu_oracle_ms_1thread": t_cpu * 1e3, "bit_exact": True}

    # ---- full-neighbour block (the reference inference loader: batch 128) -----------------
    fl = NodeDataLoader(g, {"user": torch.arange(1_000_000)}, MultiLayerFullNeighborSampler(2),
                        batch_size=128, shuffle=True)
    it = iter(fl)
    next(it)
    n_edges = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        _, _, blocks = next(it)
        n_edges += sum(b.num_edges(ce) for b in blocks for ce in b.canonical_etypes)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res["C2 full-neighbour 2-layer blocks, batch 128"] = {
        "ms_per_batch": dt / 5 * 1e3, "edges_per_batch": n_edges / 5,
        "sampled_edges_per_s": n_edges / dt}
    # ---- f4: LSTM reducer on a fanout-10 block (C2 shape: 10k seeds x 10, d=64) -----------
    from gnnrec.graph import build_csr
    for n_dst, fan, d in ((10_240, 10, 64), (100_000, 10, 128)):
        dst = torch.arange(n_dst, device=dev).repeat_interleave(fan)
        src = torch.randint(0, 1_000_000, (dst.numel(),), device=dev)
        ip, ix, _ = build_csr(src, dst, n_dst)
        X = torch.randn(1_000_000, d, device=dev)
        W_ih, W_hh = torch.randn(4 * d, d, device=dev) * 0.1, torch.randn(4 * d, d, device=dev) * 0.1
        b = torch.zeros(4 * d, device=dev)
        ops.lstm_aggregate(ip, ix, X, W_ih, W_hh, b, b)
        tl, _ = sync_time(lambda: [ops.lstm_aggregate(ip, ix, X, W_ih, W_hh, b, b)
                                   for _ in range(5)])
        tl /= 5
        fl = 2.0 * dst.numel() * d * 4 * d + 2.0 * X.shape[0] * d * 4 * d
        res[f"LSTM reducer {n_dst} dst x {fan} steps, d={d} (incl. input-projection GEMM)"] = {
            "ms": tl * 1e3, "TFLOPs": fl / tl / 1e12}
        del X
    del g, loader, fl, it, blocks
    torch.cuda.empty_cache()

    # ---- C2: one training step (2 conv layers 'mean', d=64, fanout [10,10], cosine head) --
    def train_steps(g, model, K, label):
        opt = torch.optim.Adam(model.parameters(), lr=0.005)
        el = EdgeDataLoader(g, {BUYS: torch.arange(50_000_000)},
                            MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                            reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                            negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                            shuffle=True)
        for nw in (0, 2):  # num_workers=2: the next batches are sampled on a second stream
            el.num_workers = nw
            it = iter(el)

            def step():
                _, pos_g, neg_g, blocks = next(it)
                _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
                loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
                opt.zero_grad()
                loss.backward()
                opt.step()
                return loss.item()

            for _ in range(2):
                step()
            ts, _ = sync_time(lambda: [step() for _ in range(10)])
            res[f"{label}, num_workers={nw}"] = {"ms_per_step": ts / 10 * 1e3,
                                                 "pos_edges_per_s": 1024 * 10 / ts}
            del it

    g = c2_graph(64, dev)
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    for K in (10, 2500):
        train_steps(g, model, K, f"C2 training step (fanout [10,10], 1024 pos x {K} neg, "
                                 f"mean d=64)")
    del g, model
    torch.cuda.empty_cache()

    # ---- C3: heads kernels + one training step --------------------------------------------
    g = c2_graph(128, dev)
    E_pos, K = 1024, 2500
    hs = torch.randn(1_000_000, 128, device=dev)
    hd = torch.randn(100_000, 128, device=dev)
    src = torch.randint(0, 1_000_000, (E_pos,), device=dev).repeat_interleave(K)
    dst = torch.randint(0, 100_000, (E_pos * K,), device=dev)
    for _ in range(2):
        ops.sddmm_cos(src, dst, hs, hd)
    tc, _ = sync_time(lambda: [ops.sddmm_cos(src, dst, hs, hd) for _ in range(10)])
    tc /= 10
    by = src.numel() * (2 * 128 * 4 + 16 + 4)
    res["C3 cosine head 1024x2500 edges"] = {"ms": tc * 1e3, "GBs_alg": by / tc / 1e9,
                                             "Gedges_per_s": src.numel() / tc / 1e9}
    torch.manual_seed(0)
    pl = gnn.PredictingLayer(128).to(dev).eval()
    with torch.no_grad():
        pl.score_edges(hs, hd, src, dst)
        tm, _ = sync_time(lambda: [pl.score_edges(hs, hd, src, dst) for _ in range(5)])
    tm /= 5
    res["C3 MLP head 1024x2500 edges (incl. per-node P/Q GEMMs)"] = {
        "ms": tm * 1e3, "Gedges_per_s": src.numel() / tm / 1e9}

    model = gnn.ConvModel(g, 3, {"user": 128, "item": 128, "hidden": 128, "out": 128}, True,
                          0.0, "mean_nn", "cos", "sum", True).to(dev)
    train_steps(g, model, K, "C3 training step (fanout [10,10], 1024 pos x 2500 neg, mean_nn d=128)")
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
