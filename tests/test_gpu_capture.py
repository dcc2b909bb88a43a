"""GPU tests of the static-shape minibatch path and the captured training step (row f2,
reference src/train/run.py:104-160 per EdgeDataLoader batch).

Static blocks (BlockSampler static shapes, include/gnnrec.h) must hold exactly the exact
blocks' rows for every real node — the same edges, eids and source ids, local ids aside —
with padding only in padding rows; the static batch head must give the exact pair graphs;
and a step over a static batch, eager or replayed from a hipGraph, must train the model as
the exact batch does (fp32 tolerance: the padded GEMMs sum over more rows)."""
import copy

import numpy as np
import pytest
import torch

from test_gpu_sampling import BOUGHT, BUYS, CLICKED, CLICKS, DEV, _graph, _model

pytestmark = pytest.mark.gpu

REV = {'buys': 'bought-by', 'bought-by': 'buys', 'clicks': 'clicked-by',
       'clicked-by': 'clicks'}


def _rows(block, ce):
    """dst global id -> [(src global id, eid)] of every row, and the padding rows' edges."""
    from gnnrec.graph import NID
    ip, loc, eid = (t.cpu().numpy() for t in block._rels[ce])
    src = block.srcdata[NID][ce[0]].cpu().numpy()
    dst = block.dstdata[NID][ce[2]].cpu().numpy()
    assert dst.size == block.number_of_dst_nodes(ce[2])
    real, pad = {}, []
    for i, v in enumerate(dst.tolist()):
        edges = [(int(src[loc[e]]), int(eid[e])) for e in range(ip[i], ip[i + 1])]
        if v >= 0:
            real[v] = edges
        else:
            pad += edges
    return real, pad, ip


@pytest.mark.parametrize("fanouts", [[4, 3], [{"buys": 2, "bought-by": 5, "clicks": 0,
                                               "clicked-by": 64}, 1]])
def test_static_blocks_hold_the_exact_rows(fanouts):
    from gnnrec.graph import NID
    from gnnrec.sampling import MultiLayerNeighborSampler
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    exact = MultiLayerNeighborSampler(fanouts, seed=4)
    stat = MultiLayerNeighborSampler(fanouts, seed=4)
    users = torch.arange(3, 300, 7, device=DEV)
    items = torch.tensor([5, 1, 77, 9], device=DEV)
    pad = torch.full((6,), -1, dtype=torch.int64, device=DEV)
    excl = {BUYS: torch.arange(0, 4000, 5, device=DEV), BOUGHT: torch.arange(0, 4000, 5, device=DEV)}
    for rep in range(2):
        a = exact.sample_blocks(g, {"user": users, "item": items}, excl, transposes=True)
        b = stat.sample_blocks(g, {"user": torch.cat([users, pad]), "item": torch.cat([items, pad])},
                               excl, transposes=True, static_shapes=True)
        assert all(x.static for x in b) and not any(x.static for x in a)
        for ba, bb in zip(a, b):
            for nt in bb.ntypes:
                # source list: the exact one (the seeds, then the new sources, at the same
                # positions), then -1 — the padding-edge source slot and the next block's
                # dump row last; destinations: the seed slots, -1 at padding and dump rows
                sa = ba.srcdata[NID][nt].cpu().numpy()
                sb = bb.srcdata[NID][nt].cpu().numpy()
                np.testing.assert_array_equal(sb[:sa.size], sa)
                assert (sb[sa.size:] == -1).all() and sb.size >= sa.size + 2
                da = ba.dstdata[NID][nt].cpu().numpy()
                db = bb.dstdata[NID][nt].cpu().numpy()
                np.testing.assert_array_equal(db[:da.size], da)
                assert (db[da.size:] == -1).all() and db[-1] == -1
            for ce in bb.canonical_etypes:  # dump rows: runs of at most 2048 edges
                ip = bb._rels[ce][0]
                assert int((ip[1:] - ip[:-1]).max()) <= 2048
                f = bb._src[nt].get("features")
                if f is not None:
                    assert not f.cpu().numpy()[sb < 0].any()
            for ce in bb.canonical_etypes:
                ra, pa, _ = _rows(ba, ce)
                rb, pb, ipb = _rows(bb, ce)
                assert ra == rb, ce
                assert not pa and all(s == -1 and e == -1 for s, e in pb), ce
                assert ipb[-1] == bb.num_edges(ce) == bb._rels[ce][0]._gnnrec_nnz
                occ = bb._edata[ce].get("occurrence")
                if occ is not None:
                    eid = bb._rels[ce][2].cpu().numpy()
                    assert not occ.cpu().numpy()[eid < 0].any()
            # the layer chain: every block's output rows are the next block's source rows
        for lo, hi in zip(b[:-1], b[1:]):
            for nt in lo.ntypes:
                assert lo.number_of_dst_nodes(nt) == hi.number_of_src_nodes(nt)


def _loader(g, static, K=4, batch=64, n=700, seed=5, fanouts=(4, 3), nw=0, caps="provable"):
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    return EdgeDataLoader(g, {BUYS: torch.arange(n)}, MultiLayerNeighborSampler(list(fanouts), seed=seed),
                          exclude='reverse_types', reverse_etypes=REV,
                          negative_sampler=negative_sampler.Uniform(K), batch_size=batch,
                          shuffle=True, static_shapes=static, num_workers=nw, static_caps=caps)


def test_static_batch_head_gives_the_exact_pair_graphs():
    from gnnrec.graph import NID
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    out = []
    for static in (False, True):
        torch.manual_seed(3)
        out.append(list(_loader(g, static)))
    assert len(out[0]) == len(out[1]) == -(-700 // 64)
    for k, (ia, ib) in enumerate(zip(*out)):
        (_, pa, na, ba), (_, pb, nb, bb) = ia, ib
        last = k == len(out[0]) - 1  # 700 % 64: the partial batch is exact
        assert pb.static == (not last) and all(x.static == (not last) for x in bb)
        for nt in ("user", "item"):
            ida, idb = pa.ndata[NID][nt].cpu().numpy(), pb.ndata[NID][nt].cpu().numpy()
            np.testing.assert_array_equal(idb[:ida.size], ida)
            assert (idb[ida.size:] == -1).all()
            if not last:
                assert int(pb.node_counts[nt]) == ida.size
        for ce in g.canonical_etypes:
            for ga, gb in ((pa, pb), (na, nb)):
                for x, y in zip(ga.all_edges(etype=ce), gb.all_edges(etype=ce)):
                    assert torch.equal(x, y), ce
        assert nb.src_repeats_pos == na.src_repeats_pos == 4


def _loss(K):
    from gnnrec import nn as gnn

    def f(model, batch):
        _, pos_g, neg_g, blocks = batch
        _, ps, ns = model(blocks, blocks[0].srcdata['features'], pos_g, neg_g, True)
        return gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata['recency'])
    return f


def _close(a, b, what, rtol=2e-4, atol=2e-6):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol, msg=what)


@pytest.mark.parametrize("agg,fold,fanouts", [("mean", "0", (4, 3)), ("mean", "1", (4, 3)),
                                              ("mean_nn_edge", "auto", (4, 3)),
                                              ("mean", "0", (64, 64)), ("mean", "1", (64, 64))])
def test_static_step_trains_as_the_exact_step(monkeypatch, agg, fold, fanouts):
    """One step over the static batch and over the exact one: the same loss and gradients
    (fp32 rounding: the weight-gradient GEMMs sum over the padding rows' zeros too).  Fanout
    64 on this graph leaves more than 2048 padding edges per relation: the heavy-row plans of the
    transposed backward gather are built on the device (the dump rows are cut at 2048)."""
    monkeypatch.setenv("GNNREC_TRAIN_FOLD", fold)
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    K = 4
    batches = []
    for static in (False, True):
        torch.manual_seed(3)
        batches.append(next(iter(_loader(g, static, K=K, fanouts=fanouts))))
    for b in batches[1][-1]:  # no row past a heavy-row split, whatever the padding
        for ip, _l, _e in b._rels.values():
            assert int((ip[1:] - ip[:-1]).max()) <= 2048
    base = _model(g, agg=agg).train()
    grads = []
    for batch in batches:
        m = copy.deepcopy(base)
        loss = _loss(K)(m, batch)
        loss.backward()
        grads.append((loss.detach(), {n: p.grad.clone() for n, p in m.named_parameters()
                                      if p.grad is not None}))
    (la, ga), (lb, gb) = grads
    _close(lb, la, "loss")
    assert ga.keys() == gb.keys() and ga
    for n in ga:
        _close(gb[n], ga[n], n)


@pytest.mark.parametrize("nw,fanouts,caps", [(0, (4, 3), "provable"), (2, (4, 3), "provable"),
                                             (0, (64, 64), "provable"), (2, (4, 3), "auto")])
def test_captured_steps_train_as_the_eager_loop(nw, fanouts, caps):
    """CapturedTrainStep over a static loader (warm-up steps, capture, replays, the exact
    partial batch eagerly) against the eager loop over the exact loader: per-step losses and
    the final parameters agree."""
    from gnnrec.capture import CapturedTrainStep
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    K = 4
    base = _model(g, agg="mean").train()
    runs = []
    for captured in (False, True):
        torch.manual_seed(7)
        m = copy.deepcopy(base)
        opt = torch.optim.Adam(m.parameters(), lr=0.01, fused=True)
        step = CapturedTrainStep(m, opt, _loss(K), warmup=1)
        losses = []
        # an epoch and the start of the next: warm-up, capture, replays, the partial batch
        # eagerly, replays again (further on, a hinge of the margin loss flipped by the two
        # runs' fp32 rounding differences moves the losses apart by one term)
        for epoch in range(2):
            for k, batch in enumerate(_loader(g, captured, K=K, fanouts=fanouts, caps=caps,
                                              nw=nw if captured else 0)):
                if epoch == 0 or k < 3:
                    loss = step(batch) if captured else step.eager(batch)
                    losses.append(float(loss.detach()))
        runs.append((losses, m, step))
    (la, ma, _), (lb, mb, st) = runs
    full = 700 // 64
    if caps == "auto":  # each epoch's loader first learns its capacities on 3 exact batches
        assert st.replays == full - 3 - 1 and st.eager_steps == 3 + 1 + 1 + 3
    else:
        assert st.replays == full - 1 + 3 and st.eager_steps == 1 + 1
    np.testing.assert_allclose(lb, la, rtol=1e-4, atol=1e-6)
    for (n, pa), (_, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        _close(pb.detach(), pa.detach(), n, rtol=2e-3, atol=2e-5)


def test_copy_batch_equals_tensor_copies():
    """ops.copy_batch (gnnrec_copy_batch, 64 copies per launch): every dtype and size,
    16-B-aligned and unaligned (offset views), more than one launch's worth, empty ones."""
    from gnnrec import ops
    gen = torch.Generator(device=DEV)
    gen.manual_seed(0)
    src = []
    for k in range(70):
        n = int(torch.randint(0, 5000, (1,), generator=gen, device=DEV))
        base = torch.randint(-1 << 40, 1 << 40, (n + 3,), device=DEV, generator=gen)
        t = [base[:n], base[1:n + 1].to(torch.int32), base[3:].float(), base[:n].to(torch.uint8),
             base[2:n + 2].double()][k % 5]
        src.append(t.contiguous() if k % 3 else t)
    dst = [torch.empty_like(s) for s in src]
    ops.copy_batch(src, dst)
    for s, d in zip(src, dst):
        assert torch.equal(s, d)


def test_learned_caps_shrink_the_blocks_and_overflow_is_redone():
    """static_caps='auto': after 3 exact batches the source lists get learned capacities,
    below the provable ones where a fanout reaches most of a type (items here); a batch that
    outgrows them raises the sampler's overflow flag — memory-safe — and is redone exactly."""
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    prov = [x for x in _loader(g, True, fanouts=(10, 10), caps="provable")]
    auto_l = _loader(g, True, fanouts=(10, 10), caps="auto")
    auto = list(auto_l)
    assert [x[1].static for x in auto[:3]] == [False] * 3 and auto[3][1].static
    rows = lambda item: sum(b.number_of_src_nodes(nt) for b in item[-1] for nt in b.ntypes)  # noqa: E731
    assert rows(auto[3]) <= rows(prov[3])
    tight = _loader(g, True, fanouts=(10, 10), caps="auto")
    tight._node_hint = {(s_, nt): 1 for s_ in range(2) for nt in ("user", "item")}
    item = next(iter(tight))
    assert tight.static_redone == 1 and not item[1].static and not item[-1][0].static
    loss = _loss(4)(_model(g, agg="mean").train(), item)
    assert torch.isfinite(loss)


@pytest.mark.parametrize("planned", [False, True])
def test_live_row_count_gathers_only_the_real_rows(planned):
    """gnnrec_spmm_csr_live_f32 / the planned form: rows below the device count are bitwise
    the plain gather's, rows from it on are empty rows (0) — or left alone under ACCUM — and
    never heavy; a static block's padding and dump rows (sampling static_shapes) so cost no
    gathers."""
    from gnnrec import _lib, ops
    T = ops._T()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(5)
    n_dst, n_src, d = 3000, 700, 64
    deg = torch.randint(0, 12, (n_dst,), device=DEV, generator=gen)
    deg[2500] = 9000  # a heavy row past the live count
    deg[100] = 5000   # and one below it
    ip = torch.zeros(n_dst + 1, dtype=torch.int64, device=DEV)
    ip[1:] = torch.cumsum(deg, 0)
    nnz = int(ip[-1])
    ix = torch.randint(0, n_src, (nnz,), device=DEV, generator=gen).int()
    X = torch.randn(n_src, d, device=DEV, generator=gen)
    live_n = 2200
    live = torch.tensor([live_n], dtype=torch.int64, device=DEV)
    ref = ops.spmm(ip, ix, X, 'mean')

    def run(lv, flags=0, out=None):
        out = torch.full((n_dst, d), 7.0, device=DEV) if out is None else out
        if not planned:
            T.spmm_csr(ip, ix, None, X, ops.REDUCE['mean'], flags, out, lv)
            return out
        split = 2048
        cap_h = min(n_dst, nnz // (split + 1))
        cap_c = nnz // split + cap_h
        plan = torch.empty(3 + 2 * cap_h + cap_c, dtype=torch.int64, device=DEV)
        T.spmm_plan_build(ip, split, cap_h, plan, lv)
        ws = torch.empty(cap_c * d, device=DEV)
        T.spmm_csr_planned(ip, ix, None, X, ops.REDUCE['mean'], flags, split, plan, cap_h,
                           cap_c, out, ws, lv)
        return out

    full = run(None)
    np.testing.assert_allclose(full.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-5)
    out = run(live)
    assert torch.equal(out[:live_n], full[:live_n])
    assert torch.count_nonzero(out[live_n:]) == 0
    acc = torch.ones(n_dst, d, device=DEV)
    run(live, _lib.SPMM_ACCUM, acc)
    assert torch.equal(acc[live_n:], torch.ones_like(acc[live_n:]))
    np.testing.assert_allclose(acc[:live_n].cpu().numpy(), (1 + full[:live_n]).cpu().numpy(),
                               rtol=1e-6, atol=1e-6)
    zero = torch.zeros(1, dtype=torch.int64, device=DEV)
    assert torch.count_nonzero(run(zero)) == 0


@pytest.mark.parametrize("short", ["rows", "chunks"])
def test_overflowed_plan_is_flagged_and_reduces_every_row(short):
    """A device-built heavy-row plan whose capacities are too short for its CSR (a host edge
    count that understates the edges): the build marks the plan overflowed (n_heavy < 0,
    n_chunks = 0), the library's overflow counter rises, and the planned gather reduces every
    row in the row kernel — bitwise the unplanned gather, no row dropped or clipped."""
    from gnnrec import ops
    T = ops._T()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(11)
    n_dst, n_src, d, split = 2000, 500, 64, 2048
    deg = torch.randint(0, 9, (n_dst,), device=DEV, generator=gen)
    deg[[7, 901, 1999]] = torch.tensor([9000, 5000, 20000], device=DEV)  # 3 heavy rows, 18 chunks
    ip = torch.zeros(n_dst + 1, dtype=torch.int64, device=DEV)
    ip[1:] = torch.cumsum(deg, 0)
    nnz = int(ip[-1])
    ix = torch.randint(0, n_src, (nnz,), device=DEV, generator=gen).int()
    X = torch.randn(n_src, d, device=DEV, generator=gen)
    ref = torch.empty(n_dst, d, device=DEV)
    T.spmm_csr(ip, ix, None, X, ops.REDUCE["mean"], 0, ref, None)  # no plan: unsplit rows
    cap_h, cap_c = (1, 64) if short == "rows" else (8, 4)
    plan = torch.empty(3 + 2 * cap_h + cap_c, dtype=torch.int64, device=DEV)
    before = ops.plan_overflows()
    T.spmm_plan_build(ip, split, cap_h, plan, None)
    ws = torch.empty(cap_c * d, device=DEV)
    out = torch.full((n_dst, d), 7.0, device=DEV)
    T.spmm_csr_planned(ip, ix, None, X, ops.REDUCE["mean"], 0, split, plan, cap_h, cap_c, out,
                       ws, None)
    torch.cuda.synchronize()
    assert int(plan[0]) == -3 and int(plan[1]) == 0
    assert ops.plan_overflows() == before + 1
    assert torch.equal(out, ref)
    # a plan with room for its rows is not flagged, and splits the heavy rows as before
    plan = torch.empty(3 + 2 * 8 + 64, dtype=torch.int64, device=DEV)
    T.spmm_plan_build(ip, split, 8, plan, None)
    ws = torch.empty(64 * d, device=DEV)
    T.spmm_csr_planned(ip, ix, None, X, ops.REDUCE["mean"], 0, split, plan, 8, 64, out, ws, None)
    torch.cuda.synchronize()
    assert int(plan[0]) == 3 and int(plan[1]) == 5 + 3 + 10
    assert ops.plan_overflows() == before + 1
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)


def test_static_block_data_is_lazy_until_read():
    """A static batch's block data (node features of the input block, every block's edge
    data) is held as LazyRows: walking the batch for a captured step's inputs
    (sampling._tensors) leaves it unread and unlisted — a captured step that reads it
    gathers it inside its graph from the captured ids — and reading it gives the rows the
    exact gather gives, zero rows at the padding slots."""
    from gnnrec.graph import NID, LazyRows
    from gnnrec.sampling import _tensors
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    batch = next(iter(_loader(g, True)))
    blocks = batch[-1]
    assert all(b.static for b in blocks)
    lazy = [(f, k) for f in blocks[0]._src.values() for k, v in f.lazy_items()
            if isinstance(v, LazyRows)]
    lazy += [(f, k) for b in blocks for f in b._edata.values() for k, v in f.lazy_items()
             if isinstance(v, LazyRows)]
    assert lazy
    listed = {t.data_ptr() for t in _tensors(batch, [])}
    assert all(isinstance(dict.__getitem__(f, k), LazyRows) for f, k in lazy)
    for nt, f in blocks[0]._src.items():
        for k in [k for k, v in f.lazy_items() if isinstance(v, LazyRows)]:
            got = f[k]  # gathered now
            assert got.data_ptr() not in listed
            ids = f[NID]
            table = g.nodes[nt].data[k]
            ref = table[ids.clamp(min=0)] * (ids >= 0).reshape((-1,) + (1,) * (table.dim() - 1))
            assert torch.equal(got, ref.to(got.dtype)), (nt, k)
            assert not isinstance(dict.__getitem__(f, k), LazyRows)
    for b in blocks:
        for ce, f in b._edata.items():
            eid = b._rels[ce][2]
            for k in [k for k, v in f.lazy_items() if isinstance(v, LazyRows)]:
                table = g.edges[ce].data[k]
                ref = table[eid.clamp(min=0)] * (eid >= 0).reshape((-1,) + (1,) * (table.dim() - 1))
                assert torch.equal(f.get(k), ref.to(table.dtype)), (ce, k)


def test_capture_beside_a_sampling_thread_drawing_negatives():
    """A sampling thread drawing negatives from torch's default CUDA generator while the
    training thread captures its step: torch refuses a draw from a non-capturing stream
    during a capture ("Offset increment outside graph capture"), so the capture holds
    sampling.RNG_LOCK and the loaders draw under it — no draw lands in the window."""
    import threading
    from gnnrec.capture import CapturedTrainStep
    from gnnrec.sampling import negative_sampler
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    batches = [b for b in _loader(g, True)][:3]
    stop, errors, draws = threading.Event(), [], [0]

    def draw():
        neg = negative_sampler.Uniform(4)
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                while not stop.is_set():
                    neg(g, {BUYS: torch.arange(64, device=DEV)})
                    draws[0] += 1
        except Exception as e:  # noqa: BLE001 — surfaced below
            errors.append(e)

    t = threading.Thread(target=draw, daemon=True)
    t.start()
    try:
        for _ in range(3):
            m = _model(g, agg="mean").train()
            opt = torch.optim.Adam(m.parameters(), lr=0.01, fused=True)
            step = CapturedTrainStep(m, opt, _loss(4), warmup=1)
            for b in batches:
                step(b)
            assert step.captures == 1 and step.replays >= 1, \
                (step.captures, step.replays, step.eager_steps)
    finally:
        stop.set()
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    assert draws[0] > 0
