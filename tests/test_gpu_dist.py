"""Two ranks on ONE GPU (gloo transport, HIP kernels for all arithmetic): the sharded
full-graph pass must reproduce the single-process GPU pass.  (RCCL itself needs
one GPU per rank; the collectives' nccl forms run in the driver's multi-GPU bench.)

The ranks exchange through gnnrec.dist.AsyncEmulatedExchange: every collective is issued
async and returns a work handle, its input is read late on a copy-in stream behind a delay
kernel and its output lands late on a copy-out stream — the ordering RCCL imposes — so the
pass's waits (inference.py: the owner's work.wait() before the projection, the pending
all-gather waited by _get, scratch reuse across passes) are exercised, not bypassed."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _build(agg, hetero, d=32, two_rel=False):
    from gnnrec import nn as gnn
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(0)
    n_u, n_i, E = 3000, 700, (40000 if d == 32 else 100000)  # d=128: >= 24 edges/row, fused
    u = rng.integers(0, n_u, E)
    i = rng.integers(0, n_i, E)
    rels = {("user", "buys", "item"): (u, i), ("item", "bought-by", "user"): (i, u)}
    if hetero == "attention" or two_rel:  # a second relation per dst type (sparser)
        Ec = E // 3
        uc, ic = rng.integers(0, n_u, Ec), rng.integers(0, n_i, Ec)
        rels[("user", "clicks", "item")] = (uc, ic)
        rels[("item", "clicked-by", "user")] = (ic, uc)
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(t)) for ce, (s, t) in rels.items()},
                    {"user": n_u, "item": n_i}, device="cuda")
    for ce, (s, _) in rels.items():
        g.edges[ce].data["occurrence"] = torch.from_numpy(rng.integers(1, 9, s.size)).cuda()
    feats = {"user": torch.from_numpy(rng.standard_normal((n_u, d)).astype(np.float32)).cuda(),
             "item": torch.from_numpy(rng.standard_normal((n_i, d)).astype(np.float32)).cuda()}
    torch.manual_seed(0)
    hidden = 64 if d == 32 else d  # d = 128: every layer takes the fused aggregate+project path
    model = gnn.ConvModel(g, 3, {"user": d, "item": d, "hidden": hidden, "out": d}, True, 0.0, agg,
                          "cos", hetero, True).cuda().eval()
    return g, feats, model


def _async_exchange():
    from gnnrec.dist import AsyncEmulatedExchange
    return AsyncEmulatedExchange(delay_us=2000)


def _worker(rank, world, port, agg, hetero, d, q, segments=None, det=None, two_rel=False,
            passes=2):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gnnrec.inference import GraphShard, ShardedFullGraphPass, gather_partitioned
        g, feats, model = _build(agg, hetero, d, two_rel)
        ex = _async_exchange()
        sh = GraphShard.from_graph(g, rank, world, "user", device="cuda", segments=segments)
        det = segments is not None if det is None else det
        runner = ShardedFullGraphPass(model, sh, ex, deterministic=det)
        x = sh.local_features(feats)
        res = []
        for _ in range(passes):  # back to back: the scratch tables are reused across passes
            out = runner.run(x)
            res.append((out["user"].clone(), out["item"][:700].clone()))
        assert ex.works_issued >= 2 * passes and ex.sync_calls == 0, \
            (ex.works_issued, ex.sync_calls)
        for u, i in res[1:]:
            assert torch.equal(u, res[0][0]) and torch.equal(i, res[0][1]), "passes differ"
        if two_rel and hetero != "attention":  # both item->user relations in one launch
            assert len(runner.pair_fused) == 1, runner.pair_fused
        users = gather_partitioned(sh, res[0][0], ex)
        q.put((rank, users.cpu().numpy(), res[0][1].cpu().numpy()))
        ex.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("agg,hetero,d", [("mean", "sum", 32), ("pool_nn_edge", "max", 32),
                                          ("mean", "sum", 128), ("pool_nn", "mean", 128),
                                          ("mean", "attention", 128), ("mean_edge", "attention", 32),
                                          ("lstm", "sum", 32)])  # item rows: full_in_rows
def test_two_ranks_one_gpu_match_single_process(agg, hetero, d):
    import torch.multiprocessing as mp
    from gnnrec.inference import full_graph_embeddings
    g, feats, model = _build(agg, hetero, d)
    with torch.no_grad():
        ref = full_graph_embeddings(g, model, feats)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, agg, hetero, d, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for _, users, items in res:
        np.testing.assert_allclose(users, ref["user"].cpu().numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(items, ref["item"].cpu().numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("agg,hetero,d", [("mean", "sum", 128), ("mean_edge", "attention", 32)])
def test_deterministic_mode_bitwise_across_world_sizes(agg, hetero, d):
    """with segments=8 the outputs are bitwise identical at P = 1, 2, 4 and 8
    (the replicated type's sums are the same per-segment partials folded in the same tree
    whatever the rank count; every kernel choice is made from global sizes)."""
    import torch.multiprocessing as mp
    from gnnrec.dist import Exchange
    from gnnrec.inference import GraphShard, ShardedFullGraphPass, full_graph_embeddings
    g, feats, model = _build(agg, hetero, d)
    with torch.no_grad():
        ref = full_graph_embeddings(g, model, feats)
    sh = GraphShard.from_graph(g, 0, 1, "user", device="cuda", segments=8)
    one = ShardedFullGraphPass(model, sh, Exchange(), deterministic=True).run(
        sh.local_features(feats))
    base = (one["user"].cpu().numpy(), one["item"][:700].cpu().numpy())
    np.testing.assert_allclose(base[0], ref["user"].cpu().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(base[1], ref["item"].cpu().numpy(), rtol=1e-4, atol=1e-5)
    ctx = mp.get_context("spawn")
    for world in (2, 4, 8):  # 8 ranks sharing the one GPU: HIP kernels, emulated RCCL
        q = ctx.Queue()
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, agg, hetero, d, q, 8))
                 for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        for rank, users, items in res:
            assert np.array_equal(users, base[0]), f"P={world} rank {rank}: users differ"
            assert np.array_equal(items, base[1]), f"P={world} rank {rank}: items differ"


@pytest.mark.parametrize("hetero", ["sum", "mean"])
def test_deterministic_pair_launch_bitwise_across_world_sizes(hetero):
    """Two item->user relations (the C5 shape, small) run as ONE pre-projected
    spmm_project2 launch on every rank — the choice is made from the global user count —
    so deterministic mode stays bitwise identical at P = 1, 2, 4 and 8."""
    import torch.multiprocessing as mp
    from gnnrec.dist import Exchange
    from gnnrec.inference import GraphShard, ShardedFullGraphPass, full_graph_embeddings
    g, feats, model = _build("mean", hetero, 128, two_rel=True)
    with torch.no_grad():
        ref = full_graph_embeddings(g, model, feats)
    sh = GraphShard.from_graph(g, 0, 1, "user", device="cuda", segments=8)
    runner = ShardedFullGraphPass(model, sh, Exchange(), deterministic=True)
    one = runner.run(sh.local_features(feats))
    assert len(runner.pair_fused) == 1
    base = (one["user"].cpu().numpy(), one["item"][:700].cpu().numpy())
    np.testing.assert_allclose(base[0], ref["user"].cpu().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(base[1], ref["item"].cpu().numpy(), rtol=1e-4, atol=1e-5)
    ctx = mp.get_context("spawn")
    for world in (2, 4, 8):
        q = ctx.Queue()
        port = _port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, "mean", hetero, 128, q, 8, None,
                                                   True)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        for rank, users, items in res:
            assert np.array_equal(users, base[0]), f"P={world} rank {rank}: users differ"
            assert np.array_equal(items, base[1]), f"P={world} rank {rank}: items differ"


@pytest.mark.parametrize("agg,hetero,d", [("mean", "sum", 128), ("mean_nn", "attention", 128),
                                          ("pool_nn", "max", 32)])
def test_source_tiles_match_single_process(agg, hetero, d):
    """Source-range tiles (segments=8, default mode): the user->item relation is gathered
    tile by tile into one partial (GNNREC_SPMM_ACCUM), with the NodeEmbedding folded into
    the GEMM (bias on non-empty rows) — at one rank and at two."""
    import torch.multiprocessing as mp
    from gnnrec.dist import Exchange
    from gnnrec.inference import GraphShard, ShardedFullGraphPass, full_graph_embeddings
    g, feats, model = _build(agg, hetero, d)
    with torch.no_grad():
        ref = full_graph_embeddings(g, model, feats)
    sh = GraphShard.from_graph(g, 0, 1, "user", device="cuda", segments=8)
    runner = ShardedFullGraphPass(model, sh, Exchange())
    one = runner.run(sh.local_features(feats))
    if agg == "mean" and d == 128:
        assert runner._fold == {} and "user" in runner._folded_types
    np.testing.assert_allclose(one["user"].cpu().numpy(), ref["user"].cpu().numpy(), rtol=1e-4,
                               atol=1e-5)
    np.testing.assert_allclose(one["item"][:700].cpu().numpy(), ref["item"].cpu().numpy(),
                               rtol=1e-4, atol=1e-5)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, agg, hetero, d, q, 8, False))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for _, users, items in res:
        np.testing.assert_allclose(users, ref["user"].cpu().numpy(), rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(items, ref["item"].cpu().numpy(), rtol=1e-4, atol=1e-5)


def _digest(t):
    """Bit-pattern checksum of a large table, on the device: Σ v_i·(2i+1) and Σ v_i·(2i+1)²
    (mod 2^64) over the int32 views v_i — any single changed bit changes both sums."""
    v = t.contiguous().view(torch.int32).reshape(-1).to(torch.int64)
    w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) * 2 + 1
    return int((v * w).sum()), int((v * (w * w)).sum()), v.numel()


def _c4_pass(rank, world, users, items, edges, split=None, ex=None, passes=1):
    """The bench's default pass (deterministic, 8 source tiles, partitioned output) on this
    rank's shard: (own user range, user digest, own item block range, item digest).
    split: C5's relation split (4 relations; the item->user pair runs as one launch).
    passes: back-to-back runs (scratch reuse across passes); every one must give the same
    digests."""
    from gnnrec import nn as gnn
    from gnnrec.dist import Exchange
    from gnnrec.inference import ShardedFullGraphPass
    from gnnrec.synth import GraphMeta, bipartite_shard, node_features
    dev, d = torch.device("cuda", 0), 128
    kw = {} if split is None else {"split": split}
    sh = bipartite_shard(users, items, edges, rank, world, dev, segments=8, **kw)
    feats = {"user": node_features(users, d, 0, dev, slice(sh.p_lo, sh.p_hi)),
             "item": torch.zeros((sh.padded_rows("item"), d), device=dev)}
    feats["item"][:items] = node_features(items, d, 1, dev)
    torch.manual_seed(0)
    model = gnn.ConvModel(GraphMeta(sh.canonical_etypes, ["item", "user"]), 3,
                          {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0, "mean",
                          "cos", "sum", True).to(dev).eval()
    runner = ShardedFullGraphPass(model, sh, ex if ex is not None else Exchange(),
                                  deterministic=True)
    S = sh.shard_rows["item"]
    lo, hi = rank * S, min((rank + 1) * S, items)
    digs = []
    for _ in range(passes):
        with torch.no_grad():
            out = runner.run(feats, replicate_output=False)
        digs.append((_digest(out["user"]), _digest(out["item"][: hi - lo])))
    assert all(dg == digs[0] for dg in digs), f"rank {rank}: back-to-back passes differ {digs}"
    if split is not None:
        assert len(runner.pair_fused) == 1, runner.pair_fused
    return (sh.p_lo, sh.p_hi, digs[0][0], lo, hi, digs[0][1], out)


def _c4_worker(rank, world, port, q, split=None):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = _async_exchange()
        r = _c4_pass(rank, world, *C4, split=split, ex=ex, passes=3)[:6]
        # per pass: layer 1 all-to-all + all-gather, layer 2 all-to-all (partitioned output)
        assert ex.works_issued >= 3 * 3 and ex.sync_calls == 0, (ex.works_issued, ex.sync_calls)
        q.put((rank,) + r)
        ex.close()
    finally:
        dist.destroy_process_group()


C5_SPLIT = (("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2))


C4 = (10_000_000, 1_000_000, 500_000_000)


def test_c4_full_size_pass_bitwise_at_two_ranks():
    """SURVEY §8e at BASELINE.json's full C4 size (10M users x 1M items x 500M edges per
    direction, d=128, the bench's default deterministic pass): at P = 2 (gloo
    transport, both ranks on one GPU; more ranks sharing one GPU, each regenerating the
    500M-edge stream and exchanging 512 MB tables through host memory, exceed a test's
    time budget — the small-graph tests above cover P = 4 bitwise, and 8 on CPU gloo) every rank produces exactly the bits of its user range
    and item block that the single-process pass produces (device checksum of every owned
    table)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    res = []
    for world in (2,):
        q, port = ctx.Queue(), _port()
        procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
        try:
            for p in procs:
                p.start()
            res += [(world,) + q.get(timeout=240) for _ in range(world)]
            for p in procs:
                p.join(timeout=30)
                assert p.exitcode == 0
        finally:
            for p in procs:  # the workers this test started, if a failure left them running
                if p.is_alive():
                    p.kill()
    out = _c4_pass(0, 1, *C4)[6]
    for world, rank, ulo, uhi, udig, ilo, ihi, idig in res:
        assert _digest(out["user"][ulo:uhi]) == udig, f"P={world} rank {rank}: user rows differ"
        assert _digest(out["item"][ilo:ihi]) == idig, f"P={world} rank {rank}: item rows differ"


def test_c5_full_size_pass_bitwise_at_two_ranks():
    """The same at C5 (the C4 graph split 80/20 into clicks and buys, four relations): the
    item->user pair runs as one pre-projected launch on every rank, decided from the global
    user count, so the two ranks reproduce the single-process bits."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q, port, world = ctx.Queue(), _port(), 2
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q, C5_SPLIT))
             for r in range(world)]
    try:
        for p in procs:
            p.start()
        res = [q.get(timeout=240) for _ in range(world)]
        for p in procs:
            p.join(timeout=30)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    out = _c4_pass(0, 1, *C4, split=C5_SPLIT)[6]
    for rank, ulo, uhi, udig, ilo, ihi, idig in res:
        assert _digest(out["user"][ulo:uhi]) == udig, f"rank {rank}: user rows differ"
        assert _digest(out["item"][ilo:ihi]) == idig, f"rank {rank}: item rows differ"


def _emulation_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gnnrec.dist import AsyncEmulatedExchange
        # ordered by events, not by a delay outrunning the other rank's kernels on the
        # shared GPU: the gate holds the copy-in until the event recorded after the early
        # read, and the copy-out follows the copy-in
        ex = AsyncEmulatedExchange(delay_us=0)
        own = torch.full((4, 8), float(rank + 1), device="cuda")
        out = torch.full((8, 8), -1.0, device="cuda")
        ex.gate()
        _, work = ex.all_gather_rows(own, out, async_op=True)
        own.fill_(7.0)  # the collective reads its input late: this write races it
        early = out.clone()  # no wait: the output has not landed yet
        after = torch.cuda.Event()
        after.record()
        ex.release(after)
        work.wait()
        late = out.clone()
        full = torch.arange(16.0, device="cuda").view(8, 2) * (rank + 1)
        blocks, work = ex.all_to_all_rows(full, async_op=True)
        work.wait()
        # the all-gather as an all-to-all of the own block x P (GNNREC_ALLGATHER=a2a)
        ex.ag_mode = "a2a"
        own2 = torch.full((4, 8), float(rank + 1), device="cuda")
        out2 = torch.full((8, 8), -1.0, device="cuda")
        _, work = ex.all_gather_rows(own2, out2, async_op=True)
        work.wait()
        want = torch.cat([torch.full((4, 8), float(r + 1), device="cuda") for r in range(world)])
        assert torch.equal(out2, want)
        q.put((rank, early.cpu().numpy(), late.cpu().numpy(), blocks.cpu().numpy()))
        ex.close()
    finally:
        dist.destroy_process_group()


def test_async_emulation_lands_late_and_reads_late():
    """The emulation does what makes it a test of the pass's ordering: a reader that skips
    work.wait() sees the output before it lands, and the input is read when the collective
    runs, not when it is issued — as under RCCL.  Ordered by events (AsyncEmulatedExchange
    .gate/release), so the assertions do not depend on a delay beating another process's
    kernels."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q, port = ctx.Queue(), _port()
    procs = [ctx.Process(target=_emulation_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, early, late, blocks in res:
        assert (early == -1).all(), "the output landed before the delay ran out"
        assert (late == 7.0).all(), "the input was read before the collective ran"
        for src in range(2):  # block `rank` of every rank's table, in source-rank order
            want = np.arange(16.0).reshape(8, 2)[rank * 4:(rank + 1) * 4] * (src + 1)
            np.testing.assert_array_equal(blocks[src], want)
