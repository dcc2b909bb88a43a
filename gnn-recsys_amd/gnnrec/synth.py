"""Synthetic benchmark graphs of the BASELINE.json shapes, built on the device.

Edge e of the user–item relation is a pure function of (seed, e)
(gnnrec_synth_edges, a counter hash), so each rank regenerates the stream and
keeps the edges of its own users without any graph exchange.
The reverse relation (item -> user, "bought-by") reuses the same edges and eid
order, as reference src/utils_data.py:205-214 builds reverse relations.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import ops
from .inference import GraphShard

BUYS = ("user", "buys", "item")
BOUGHT_BY = ("item", "bought-by", "user")


class GraphMeta:
    """Minimal metagraph for constructing a ConvModel (reference ConvModel only
    reads g.canonical_etypes and g.ntypes, src/model.py:376-406)."""

    def __init__(self, canonical_etypes, ntypes):
        self.canonical_etypes = list(canonical_etypes)
        self.ntypes = list(ntypes)


def zipf_cdf(n: int, s: float, device) -> torch.Tensor:
    w = 1.0 / torch.arange(1, n + 1, dtype=torch.float64, device=device) ** s
    c = torch.cumsum(w, 0)
    return c / c[-1]


def relation_pairs(split):
    """[(fwd canonical etype, reverse canonical etype, fraction)] for user->item relations."""
    return [(("user", rel, "item"), ("item", rev, "user"), frac) for rel, rev, frac in split]


def bipartite_shard(n_users: int, n_items: int, n_edges: int, rank: int, world: int, device,
                    seed: int = 11, zipf_s: float = 0.0, chunk: int = 1 << 26,
                    occurrence: bool = False,
                    split=(("buys", "bought-by", 1.0),),
                    segments: Optional[int] = None, balance: str = "degree") -> GraphShard:
    """This rank's GraphShard of the synthetic user->item graph (+ reverse relations).

    `split` assigns consecutive eid ranges of the generated edge stream to relations
    (e.g. C5: clicks 80 % / buys 20 %); eids are per relation, reverse relations share
    the forward eid order.  balance='degree' partitions users by cumulative in-degree
    (one extra pass over the regenerated edge stream counts it), 'count' by
    user count."""
    dev = torch.device(device)
    pairs = relation_pairs(split)
    etypes = [ce for f, r, _ in pairs for ce in (f, r)]
    cdf = zipf_cdf(n_items, zipf_s, dev) if zipf_s > 0 else None
    weight = None
    if balance == "degree" and (world > 1 or segments is not None):
        # (at one rank too when segmented: the segment ranges must not depend on P)
        # every relation's edges are incident to one user (its reverse lands on it)
        weight = torch.ones(n_users, dtype=torch.int64, device=dev)
        for e0 in range(0, n_edges, chunk):
            u, _ = ops.synth_edges(seed, e0, min(chunk, n_edges - e0), n_users, n_items, dev,
                                   cdf)
            weight += torch.bincount(u, minlength=n_users)
            del u
    elif balance not in ("degree", "count"):
        raise ValueError(f"balance must be 'degree' or 'count', not {balance!r}")
    sh = GraphShard(rank, world, "user", {"user": n_users, "item": n_items}, etypes, dev,
                    segments, weight)
    bounds = [0]
    for _, _, frac in pairs:
        bounds.append(min(n_edges, bounds[-1] + int(round(frac * n_edges))))
    bounds[-1] = n_edges
    for (fwd, rev, _), lo, hi in zip(pairs, bounds[:-1], bounds[1:]):
        keep_u, keep_i, keep_e = [], [], []
        item_deg = torch.zeros(n_items, dtype=torch.int64, device=dev)
        for e0 in range(lo, hi, chunk):
            n = min(chunk, hi - e0)
            u, i = ops.synth_edges(seed, e0, n, n_users, n_items, dev, cdf)
            item_deg += torch.bincount(i, minlength=n_items)
            if world == 1:
                keep_u.append(u)
                keep_i.append(i)
                keep_e.append(torch.arange(e0 - lo, e0 - lo + n, device=dev))
            else:
                m = (u >= sh.p_lo) & (u < sh.p_hi)
                idx = torch.nonzero(m).squeeze(1)
                keep_u.append(u[idx])
                keep_i.append(i[idx])
                keep_e.append(idx + (e0 - lo))
            del u, i
        u = torch.cat(keep_u).to(torch.int64)
        i = torch.cat(keep_i).to(torch.int64)
        eid = torch.cat(keep_e)
        del keep_u, keep_i, keep_e
        w = ((eid % 8) + 1) if occurrence else None  # deterministic 1..8 'occurrence' counts
        sh.add_relation(fwd, u, i, eid, hi - lo, weights=w, dst_global_deg=item_deg)
        sh.add_relation(rev, i, u, eid, hi - lo, weights=w)
        del u, i, eid, w
    return sh


def node_features(n: int, d: int, seed: int, device, rows: Optional[slice] = None) -> torch.Tensor:
    """N(0,1) fp32 features from a seeded device generator (partition-independent:
    every rank draws the full table and keeps its rows)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    x = torch.randn((n, d), generator=gen, device=device, dtype=torch.float32)
    if rows is not None:
        x = x[rows].contiguous()
    return x


def minibatch_graph(d: int, device, n_users: int = 1_000_000, n_items: int = 100_000,
                    n_edges: int = 50_000_000):
    """BASELINE configs[1]/[2]'s graph (C2 / C3): users x items, one buys relation and its
    reverse from the counter-hash edge stream (seed 11), N(0,1) features of width d, a
    'recency' edge field in [1, 30), both in-CSRs built."""
    from . import ops
    from .graph import HeteroGraph
    buys, bought = ("user", "buys", "item"), ("item", "bought-by", "user")
    u, i = ops.synth_edges(11, 0, n_edges, n_users, n_items, device)
    u, i = u.long(), i.long()
    g = HeteroGraph({buys: (u, i), bought: (i, u)}, {"user": n_users, "item": n_items},
                    device=device)
    gen = torch.Generator(device=device)
    gen.manual_seed(0)
    g.nodes["user"].data["features"] = torch.randn(n_users, d, generator=gen, device=device)
    g.nodes["item"].data["features"] = torch.randn(n_items, d, generator=gen, device=device)
    g.edges["buys"].data["recency"] = torch.randint(1, 30, (n_edges,), device=device)
    for ce in (buys, bought):
        g.in_csr(ce)
    return g

