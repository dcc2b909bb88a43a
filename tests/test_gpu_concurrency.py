"""Row kernels in concurrency mode (gnnrec_set_concurrency): CUs reserved for collective
kernels and rows handed out by the device work queue.  The queue changes which wave
reduces a row, never how — outputs must be bitwise identical to the static schedule,
also when another kernel holds CUs while the launch starts (a collective's footprint,
gnnrec_hold_cus) and after the per-device ring of queue slots wraps around."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _csr(n_dst, n_src, deg_max, seed):
    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, deg_max + 1, (n_dst,), generator=g)
    indptr = torch.zeros(n_dst + 1, dtype=torch.int64)
    torch.cumsum(deg, 0, out=indptr[1:])
    indices = torch.randint(0, n_src, (int(indptr[-1]),), generator=g, dtype=torch.int32)
    return indptr.cuda(), indices.cuda()


@pytest.fixture
def static_mode():
    from gnnrec import ops
    old = ops.get_concurrency()
    ops.set_concurrency(0, False)
    yield
    ops.set_concurrency(*old)


def _both(fn, hold=False):
    """fn() under the static schedule, then under (16 reserved CUs, queue) — with a
    CU-holding kernel launched just before on a side stream when `hold`."""
    from gnnrec import ops
    ref = fn().clone()
    side = torch.cuda.Stream()
    with ops.concurrency(16, True):
        if hold:
            side.wait_stream(torch.cuda.current_stream())
            ops.hold_cus(96, 300, lds_bytes=32768, stream=side)
        out = fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    return ref, out


@pytest.mark.parametrize("d,reduce,weighted", [(128, "mean", False), (128, "max", True),
                                               (64, "sum", False), (32, "mean", True)])
@pytest.mark.parametrize("hold", [False, True])
def test_spmm_queue_bitwise(static_mode, d, reduce, weighted, hold):
    from gnnrec import ops
    n_dst, n_src = 400_000, 40_000  # >= 32 rows per wave: the row kernel takes the queue
    indptr, indices = _csr(n_dst, n_src, 24, 1)
    X = torch.randn(n_src, d, device="cuda")
    ew = torch.rand(indices.numel(), device="cuda") if weighted else None
    q0, _ = ops.rowq_stats()
    ref, out = _both(lambda: ops.spmm(indptr, indices, X, reduce, edge_weight=ew), hold)
    assert ops.rowq_stats()[0] > q0  # the second launch did take the queue
    assert torch.equal(ref, out)
    # accumulate in place (a source-range tile onto the partial of earlier tiles)
    base = torch.randn(n_dst, d, device="cuda")

    def acc():
        o = base.clone()
        ops.spmm(indptr, indices, X, "sum", out=o, accumulate=True)
        return o
    ref, out = _both(acc, hold)
    assert torch.equal(ref, out)


@pytest.mark.parametrize("variant", ["valu", "mfma"])
@pytest.mark.parametrize("accum", ["store", "add", "attn"])
@pytest.mark.parametrize("hold", [False, True])
def test_spmm_project_queue_bitwise(static_mode, accum, hold, variant):
    """(mfma: whole 32-row tiles per ticket, drawn by one wave for the block.)  Row counts
    large enough for the launch to take the queue at 16 reserved CUs (VALU: ≥ 240 blocks ×
    16 waves × 8-row tickets × 4; MFMA: ≥ 480 blocks × 64-row tickets × 4)."""
    from gnnrec import ops
    n_dst, n_src, d = (200_000, 30_000, 128) if variant == "valu" else (300_000, 30_000, 128)
    indptr, indices = _csr(n_dst, n_src, 40 if variant == "valu" else 16, 2)
    X = torch.randn(n_src, d, device="cuda")
    H = torch.randn(n_dst, d, device="cuda")
    Ws, Wn = torch.randn(d, d, device="cuda") * 0.1, torch.randn(d, d, device="cuda") * 0.1
    base = torch.randn(n_dst, d, device="cuda")
    av = torch.randn(d, device="cuda")
    st0 = torch.randn(n_dst, 2, device="cuda")

    def run():
        o = base.clone()
        kw = {}
        if accum == "attn":
            kw = {"attn_vec": av, "attn_state": st0.clone()}
        ops.spmm_project(indptr, indices, X, H, Ws, Wn, "mean", relu=True, l2norm=True,
                         accum=accum, out=o, variant=variant, **kw)
        return o
    q0, _ = ops.rowq_stats()
    ref, out = _both(run, hold)
    assert ops.rowq_stats()[0] > q0  # the concurrent launch did take the queue
    assert torch.equal(ref, out)


def test_queue_ring_wraps(static_mode):
    """More launches than the ring has slots (1024): every slot is reset by the last block
    of its previous launch, so reuse starts from zero."""
    from gnnrec import ops
    n_dst, n_src, d = 300_000, 5_000, 32  # >= 32 rows per wave of the grid: queued
    indptr, indices = _csr(n_dst, n_src, 4, 3)
    X = torch.randn(n_src, d, device="cuda")
    ref = ops.spmm(indptr, indices, X, "sum")
    outs = []
    q0, b0 = ops.rowq_stats()
    with ops.concurrency(0, True):
        for i in range(1100):
            o = ops.spmm(indptr, indices, X, "sum")
            if i % 100 == 99:
                outs.append(o)
    torch.cuda.synchronize()
    q1, b1 = ops.rowq_stats()
    # every launch either ran queued or, when its slot's previous launch was still in
    # flight, statically; fresh slots are always granted
    assert (q1 - q0) + (b1 - b0) == 1100 and q1 - q0 >= 1024
    for o in outs:
        assert torch.equal(ref, o)
