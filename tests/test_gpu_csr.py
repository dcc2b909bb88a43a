"""Row f3: the device COO -> CSR builder (gnnrec_csr_build, the library's stable radix sort
of the dst ids) against the oracle's CSR (numpy stable argsort / oracle.c counting sort),
bit for bit: indptr, the int32 source ids and the int64 edge ids, in-row order = edge id
(DGL's in-CSR of dgl.heterograph, reference src/builder.py:377-383)."""
import time

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(src, dst, n_dst, ref=None):
    from gnnrec import ops
    got = [t.cpu().numpy() for t in ops.csr_build(src, dst, n_dst)]
    if ref is None:
        ref = oracle.csr_from_coo(src.cpu().numpy(), dst.cpu().numpy(), n_dst)
    for a, b, name in zip(got, ref, ("indptr", "indices", "eids")):
        np.testing.assert_array_equal(a, b, err_msg=name)


@pytest.mark.parametrize("E,n_dst", [(0, 1), (0, 9), (1, 1), (5, 1), (5000, 7), (5000, 300),
                                     (2049, 70_000), (100_000, 255), (100_000, 256),
                                     (100_000, 257), (300_000, 65_536), (300_000, 20_000_000),
                                     (100_000, 1024), (100_000, 1025), (300_000, 262_145),
                                     (300_000, 1 << 20), (300_000, (1 << 20) + 1)])
def test_csr_build_matches_oracle(E, n_dst):
    """every digit plan of the radix sort (csrsort.hip radix_plan: 1 pass of 8-10 bits, 2 of
    8 / 9 / 10, 3 of 8 / 9), tile tails (E not a multiple of 2048), empty rows, one row,
    empty relations"""
    g = torch.Generator(device=DEV)
    g.manual_seed(E + n_dst)
    src = torch.randint(0, 1 << 31, (E,), device=DEV, generator=g)
    dst = torch.randint(0, n_dst, (E,), device=DEV, generator=g)
    _check(src, dst, n_dst)


@pytest.mark.parametrize("E,n_dst", [(2_097_151, 100_000), (2_097_152, 100_000),
                                     (2_097_153, 1_100_000)])
def test_csr_build_across_the_tile_size_switch(E, n_dst):
    """The scatter's tile grows from 2048 to 4096 edges at 512 tiles of 4096 (E = 2^21): both
    sides of the switch build the oracle's CSR, bit for bit (9- and 10/11-bit digits)."""
    g = torch.Generator(device=DEV)
    g.manual_seed(E)
    src = torch.randint(0, 1 << 20, (E,), device=DEV, generator=g)
    dst = torch.randint(0, n_dst, (E,), device=DEV, generator=g)
    _check(src, dst, n_dst)


def test_csr_build_skewed_and_sorted_inputs():
    """one heavy row (half of all edges), already-sorted and reverse-sorted dst ids"""
    n, E = 50_000, 1_000_000
    g = torch.Generator(device=DEV)
    g.manual_seed(3)
    src = torch.arange(E, device=DEV)
    dst = torch.randint(0, n, (E,), device=DEV, generator=g)
    dst[::2] = 17
    _check(src, dst, n)
    _check(src, torch.sort(dst).values, n)
    _check(src, torch.sort(dst, descending=True).values, n)


def test_graph_csr_uses_device_builder():
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(0)
    u, i = rng.integers(0, 300, 5000), rng.integers(0, 40, 5000)
    g = HeteroGraph({("user", "buys", "item"): (torch.from_numpy(u), torch.from_numpy(i)),
                     ("item", "bought-by", "user"): (torch.from_numpy(i), torch.from_numpy(u))},
                    {"user": 300, "item": 40}, device=DEV)
    for ce, (s, d, n) in {("user", "buys", "item"): (u, i, 40),
                          ("item", "bought-by", "user"): (i, u, 300)}.items():
        got = [t.cpu().numpy() for t in g.in_csr(ce)]
        for a, b in zip(got, oracle.csr_from_coo(s, d, n)):
            np.testing.assert_array_equal(a, b)


def test_csr_build_c4_size_bit_exact():
    """C4: 500M edges, both relations (10M user rows, 1M item rows), against oracle.c's
    counting sort; prints the device build time."""
    from gnnrec import ops
    n_u, n_i, E = 10_000_000, 1_000_000, 500_000_000
    u, i = ops.synth_edges(11, 0, E, n_u, n_i, DEV)
    u, i = u.long(), i.long()
    hu, hi = u.cpu().numpy(), i.cpu().numpy()
    for src, dst, n_dst, hs, hd in ((i, u, n_u, hi, hu), (u, i, n_i, hu, hi)):
        ops.csr_build(src, dst, n_dst)  # warm-up (workspace allocation)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = ops.csr_build(src, dst, n_dst)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"csr_build {E} edges -> {n_dst} rows: {dt * 1e3:.1f} ms")
        ref = oracle.csr_from_coo_c(hs, hd, n_dst)
        for a, b, name in zip(out, ref, ("indptr", "indices", "eids")):
            np.testing.assert_array_equal(a.cpu().numpy(), b, err_msg=name)
        del out, ref
        torch.cuda.empty_cache()


@pytest.mark.parametrize("n_src,n_dst,E", [(1, 1, 0), (300, 40, 5000), (40, 300, 5000),
                                           (100_000, 2_000, 400_000), (3_000, 90_000, 400_000)])
def test_has_edges_between_matches_oracle(n_src, n_dst, E):
    """K10 (reference src/train/run.py:95-101): the device membership search against the
    oracle's set lookup, bit for bit — true edges, multi-edges, random pairs (mostly
    absent), ids outside the node ranges, one heavy row (a third of the edges)."""
    from gnnrec.graph import HeteroGraph
    rng = np.random.default_rng(E + n_src)
    s = rng.integers(0, n_src, E)
    d = rng.integers(0, n_dst, E)
    if E:
        d[::3] = n_dst // 2
    ce = ("user", "buys", "item")
    g = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d))},
                    {"user": n_src, "item": n_dst}, device=DEV)
    qn = 200_000
    qu = rng.integers(-2, n_src + 2, qn)
    qv = rng.integers(-2, n_dst + 2, qn)
    if E:  # a third of the queries are real edges
        k = rng.integers(0, E, qn // 3)
        qu[: qn // 3], qv[: qn // 3] = s[k], d[k]
    got = g.has_edges_between(torch.from_numpy(qu).to(DEV), torch.from_numpy(qv).to(DEV),
                              etype="buys")
    assert got.dtype == torch.bool and got.device.type == "cuda"
    ref = oracle.has_edges_between(s, d, n_src, n_dst, qu, qv)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
    host = HeteroGraph({ce: (torch.from_numpy(s), torch.from_numpy(d))},
                       {"user": n_src, "item": n_dst})
    np.testing.assert_array_equal(host.has_edges_between(qu, qv).numpy(), ref)
