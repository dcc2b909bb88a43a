"""Multi-process (world_size 2 and 4, gloo on CPU) tests of the sharded full-graph
pass: partition, reduce-scatter / all-gather exchange, relation-skip and hetero
aggregation, checked against the single-process oracle on the SAME graph.

The per-rank arithmetic runs on the oracle backend (tests/oracle_ops.py); the
code under test is gnnrec.inference.{GraphShard, ShardedFullGraphPass} and
gnnrec.dist.Exchange exactly as used on the GPUs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import golden_io
from oracle import oracle


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ops
        from gnnrec import nn as gnn
        from gnnrec.dist import AsyncEmulatedExchange, Exchange
        from gnnrec.graph import HeteroGraph
        from gnnrec.inference import GraphShard, ShardedFullGraphPass, gather_partitioned

        case, _, xk = case.partition("~")  # "~sync": the synchronous gloo Exchange
        case, _, det = case.partition("#")  # "#det": deterministic segment mode, "#seg": tiles
        seg, part, det = det == "seg", det == "part", det == "det"
        case, _, hetero = case.partition("@")  # "@attention": build-defined hetero mode
        meta = dict(golden_io.manifest()[case])
        if hetero:
            meta["aggregator_hetero"] = hetero
        a = golden_io.load(case)
        num_nodes, edges, occ = golden_io.graph_parts(a)
        g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d)) for ce, (s, d) in
                         edges.items()}, num_nodes)
        for ce, o in occ.items():
            if ce[0] in ("user", "item") and ce[2] in ("user", "item"):
                g._edata[ce]["occurrence"] = torch.from_numpy(o)
        model = gnn.ConvModel(g, meta["n_layers"], meta["dim_dict"], meta["norm"], 0.0,
                              meta["aggregator_type"], meta["pred"], meta["aggregator_hetero"],
                              meta["embedding_layer"])
        model.load_state_dict({k: torch.from_numpy(v) for k, v in golden_io.state_dict(a).items()},
                              strict=not hetero)
        _set_attention(model)
        model.eval()
        # default: every collective async with a real work handle (gloo's own async works),
        # as RCCL issues them; "~sync": the blocking emulation
        # "~a2a": the synchronous Exchange with the all-gather as an all-to-all
        # "~force": the Exchange issuing every collective at world size 1 too (the
        # multi-rank schedule of the pass on one rank; its RCCL form: test_gpu_rccl.py)
        ex = (Exchange(force_collectives=True) if xk == "force" else
              Exchange() if xk in ("sync", "a2a") else AsyncEmulatedExchange())
        if xk == "a2a":
            ex.ag_mode = "a2a"
        shard = GraphShard.from_graph(g, rank, world, "user", device="cpu",
                                      segments=8 if (det or seg) else None)
        feats = {k[5:]: torch.from_numpy(v) for k, v in a.items() if k.startswith("feat/")}
        p = ShardedFullGraphPass(model, shard, ex, ops_backend=oracle_ops, deterministic=bool(det))
        out = p.run(shard.local_features(feats), replicate_output=not part)
        if xk == "force":
            assert ex.multi and ex.path == "emulated", ex.path
        if not xk and world > 1:  # the pass asked for every collective async
            assert ex.works_issued > 0 and ex.sync_calls == 0, (ex.works_issued, ex.sync_calls)
        users = gather_partitioned(shard, out["user"], ex)
        res = {"user": users.numpy()}
        for nt in out:
            if nt != "user":
                if part:  # each rank holds its own row block: assemble them here to compare
                    full = torch.empty((shard.padded_rows(nt), out[nt].shape[1]))
                    ex.all_gather_rows(out[nt].contiguous(), full)
                    res[nt] = full[: num_nodes[nt]].numpy()
                else:
                    res[nt] = out[nt][: num_nodes[nt]].numpy()
        q.put((rank, res, shard.local_edge_count(), shard.global_edge_count()))
    finally:
        dist.destroy_process_group()


def _set_attention(model):
    """Deterministic attention vectors (the goldens have none: the mode is build-defined)."""
    with torch.no_grad():
        for i, layer in enumerate(model.layers):
            if getattr(layer, "attn", None) is not None:
                for nt, p in layer.attn.items():
                    p.copy_(torch.linspace(-1.0, 1.0, p.numel()) * (i + 1) * (1 if nt == "user" else -1))


def _run(case, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(results, key=lambda r: r[0])


@pytest.mark.parametrize("case,world", [
    ("model_bip_mean_sum_emb", 2),
    ("model_bip_mean_sum_emb~sync", 2),
    ("model_het_meanedge_max_emb~a2a", 4),
    ("model_het_meannnedge_mean_emb", 2),
    ("model_het_pooledge_sum_noemb_nn", 2),
    ("model_het_meanedge_max_emb", 4),
    ("model_het_mean_sum_skip", 2),
    ("model_bip_poolnn_max_noemb_nn", 8),  # 41 users over 8 ranks: ragged and tiny shards
    ("model_het_meannnedge_mean_emb@attention", 2),
    ("model_het_mean_sum_skip@attention", 4),
    ("model_bip_mean_sum_emb#det", 1),
    ("model_het_meannnedge_mean_emb#det", 2),
    ("model_het_mean_sum_skip@attention#det", 4),
    ("model_het_meanedge_max_emb#det", 8),
    ("model_het_meanedge_max_emb#det~sync", 4),
    ("model_het_meannnedge_mean_emb#seg", 1),
    ("model_het_meanedge_max_emb#seg", 2),
    ("model_het_mean_sum_skip#part", 4),
    # the LSTM reducer at P > 1: the owner of a block of item rows runs it over their every
    # in-edge from the all-gathered user table (GraphShard.full_in_rows)
    ("model_bip_lstm_sum_emb", 2),
    ("model_het_lstm_mean_noemb_nn", 4),
    ("model_bip_lstm_sum_emb#det", 2),
    # one rank through the multi-rank schedule (every collective issued, none shortcut)
    ("model_bip_mean_sum_emb#det~force", 1),
    ("model_het_meanedge_max_emb~force", 1),
    ("model_het_mean_sum_skip#part~force", 1),
])
def test_sharded_pass_matches_single_process_oracle(case, world):
    """(#det: the deterministic segment mode, segments=8: per-segment partials folded in a
    fixed tree and exchanged all-to-all; its bitwise independence of the world size is
    checked on the GPU, tests/test_gpu_dist.py, where the arithmetic is the product's.)"""
    name, _, hetero = case.split("~")[0].split("#")[0].partition("@")
    meta = dict(golden_io.manifest()[name])
    a = golden_io.load(name)
    num_nodes, edges, occ = golden_io.graph_parts(a)
    g = oracle.Graph(num_nodes, edges, occ)
    feats = {k[5:]: v for k, v in a.items() if k.startswith("feat/")}
    sd = golden_io.state_dict(a)
    if hetero:
        meta["aggregator_hetero"] = hetero
        from gnnrec import nn as gnn
        from gnnrec.synth import GraphMeta
        m = gnn.ConvModel(GraphMeta(list(edges), sorted(num_nodes)), meta["n_layers"],
                          meta["dim_dict"], meta["norm"], 0.0, meta["aggregator_type"],
                          meta["pred"], hetero, meta["embedding_layer"])
        _set_attention(m)
        sd = dict(sd, **{k: v.detach().numpy() for k, v in m.state_dict().items() if ".attn." in k})
    ref = oracle.model_full_graph(g, feats, sd, meta["aggregator_type"],
                                  meta["aggregator_hetero"], meta["norm"], meta["embedding_layer"])
    results = _run(case, world)
    # every rank holds the same replicated tables and the same assembled user table
    for rank, res, local_e, global_e in results:
        assert set(res) == set(ref)
        for nt in ref:
            np.testing.assert_allclose(res[nt], ref[nt], rtol=1e-5, atol=1e-5,
                                       err_msg=f"rank {rank} {nt}")
    # edges are partitioned: every edge aggregated by exactly one rank
    assert sum(r[2] for r in results) == results[0][3]
    # and the golden (the reference's own output) agrees too
    if hetero:
        return  # attention is build-defined: no reference output to compare with
    for nt in ref:
        np.testing.assert_allclose(results[0][1][nt], a["h/" + nt], rtol=1e-5, atol=1e-5)


def _ag_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gnnrec.dist import Exchange, RecordingExchange
        ex = Exchange()
        own = torch.arange(6 * 3, dtype=torch.float32).view(6, 3) + 100 * rank
        res = {}
        for mode in ("rccl", "a2a"):
            ex.ag_mode = mode
            out = torch.full((6 * world, 3), -1.0)
            got, work = ex.all_gather_rows(own, out, async_op=True)
            if work is not None:
                work.wait()
            res[mode] = got.numpy().copy()  # numpy: pickled by value (a tensor's shared
            # memory would be gone once this process exits)
        ex.ag_mode = "rccl"
        rec = RecordingExchange(ex)
        rec.all_gather_rows(own, torch.empty(6 * world, 3))
        kinds = rec.replay_by_kind(torch.device("cpu"), reps=1)
        both = rec.replay_ms_by_allgather(torch.device("cpu"), reps=1)
        assert ex.ag_mode == "rccl" and sorted(both) == ["a2a", "rccl"]
        q.put((rank, res, sorted(kinds)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_all_gather_as_all_to_all(world):
    """Exchange.ag_mode 'a2a' (GNNREC_ALLGATHER): the all-gather as an all-to-all of the own
    block replicated P times gives the all-gather's table, and the multi-GPU diagnostics
    replay the all-gathers in both forms."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ag_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = torch.cat([torch.arange(18, dtype=torch.float32).view(6, 3) + 100 * r
                      for r in range(world)]).numpy()
    for _, res, kinds in results:
        np.testing.assert_array_equal(res["rccl"], want)
        np.testing.assert_array_equal(res["a2a"], want)
        assert kinds == ["all_gather", "all_gather_a2a"]
