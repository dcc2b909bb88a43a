"""The first-layer fold's weight products (autograd.FoldFn; reference NodeEmbedding folded into
the first ConvLayer: src/model.py:10-24, 226-235) on the library's fp32 MFMA GEMMs: outputs
and every gradient against the cat / matmul / slice form in float64 (torch autograd) and
against that form in fp32 — the vendor-BLAS products FoldFn ran before — at rtol 1e-5."""
import pytest
import torch

from gnnrec import autograd as ag

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _reference(W_e, b_e, Ws):
    A = torch.cat(Ws, 0)
    rows = [W.shape[0] for W in Ws]
    return (*(A @ W_e).split(rows), *(A @ b_e).split(rows))


@pytest.mark.parametrize("d_in,hid,rows", [(64, 64, (64, 64)), (4, 5, (3, 2, 4)),
                                           (2, 64, (64, 64)), (128, 128, (128,))])
def test_fold_products_and_gradients_match_torch(d_in, hid, rows):
    g = torch.Generator(device=DEV).manual_seed(0)
    W_e = torch.randn(hid, d_in, device=DEV, generator=g)
    b_e = torch.randn(hid, device=DEV, generator=g)
    Ws = [torch.randn(r, hid, device=DEV, generator=g) for r in rows]
    # upstream gradients for every product, one of them absent (None counts as zero)
    gouts = [torch.randn(r, d_in, device=DEV, generator=g) for r in rows] + \
            [torch.randn(r, device=DEV, generator=g) for r in rows]
    if len(rows) > 1:
        gouts[0] = None

    def run(fn, dtype):
        leaves = [t.detach().to(dtype).requires_grad_() for t in (W_e, b_e, *Ws)]
        out = fn(leaves[0], leaves[1], leaves[2:])
        pairs = [(o, go.to(dtype)) for o, go in zip(out, gouts) if go is not None]
        torch.autograd.backward([o for o, _ in pairs], [go for _, go in pairs])
        return [o.detach().double() for o in out], [t.grad.double() for t in leaves]

    got_o, got_g = run(lambda w, b, ws: ag.FoldFn.apply(w, b, *ws), torch.float32)
    ref_o, ref_g = run(_reference, torch.float64)
    old_o, old_g = run(_reference, torch.float32)
    for a, b, c in zip(got_o + got_g, ref_o + ref_g, old_o + old_g):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-5)
    out = ag.FoldFn.apply(W_e, b_e, *Ws)
    assert all(o.is_contiguous() for o in out)
