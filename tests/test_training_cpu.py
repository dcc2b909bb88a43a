"""CPU checks of the training step's host-side autograd pieces (no launches): the first-layer
fold's weight products as one node (autograd.FoldFn, reference NodeEmbedding folded into the
first ConvLayer: src/model.py:19-24,226-235) against torch's own gradients, and the
zero-copy join the cosine backward uses for an etype's positive and negative lists."""
import pytest
import torch

from gnnrec import autograd as ag


def test_fold_products_and_gradients_match_torch():
    """FoldFn(W_e, b_e, W_1, .., W_n) = (W_i W_e, W_i b_e) with the gradients of the
    cat / matmul / slice form (double precision: gradcheck)."""
    g = torch.Generator().manual_seed(0)
    W_e = torch.randn(5, 4, dtype=torch.float64, generator=g, requires_grad=True)
    b_e = torch.randn(5, dtype=torch.float64, generator=g, requires_grad=True)
    Ws = [torch.randn(r, 5, dtype=torch.float64, generator=g, requires_grad=True)
          for r in (3, 2, 4)]
    out = ag.FoldFn.apply(W_e, b_e, *Ws)
    for i, W in enumerate(Ws):
        torch.testing.assert_close(out[i], W @ W_e)
        torch.testing.assert_close(out[len(Ws) + i], W @ b_e)
        assert out[i].is_contiguous() and out[len(Ws) + i].is_contiguous()
    assert torch.autograd.gradcheck(lambda *a: ag.FoldFn.apply(*a), (W_e, b_e, *Ws))
    # a product nothing reads (None gradient) counts as zero
    out = ag.FoldFn.apply(W_e, b_e, *Ws)
    (out[0].sum() + out[5].sum()).backward()  # W_1 reaches neither
    assert Ws[1].grad is not None and torch.count_nonzero(Ws[1].grad) == 0


@pytest.mark.parametrize("dtype", [torch.int64, torch.float32])
def test_joined_is_a_view_when_adjacent(dtype):
    buf = torch.arange(10).to(dtype)
    a, b = buf[2:5], buf[5:9]
    j = ag._joined(a, b)
    assert j.data_ptr() == a.data_ptr() and torch.equal(j, torch.cat([a, b]))
    # not adjacent, or not the same storage: a cat
    j = ag._joined(buf[0:2], buf[5:9])
    assert torch.equal(j, torch.cat([buf[0:2], buf[5:9]]))
    other = buf.clone()
    j = ag._joined(buf[2:5], other[5:9])
    assert j.data_ptr() != buf.data_ptr() and torch.equal(j, torch.cat([buf[2:5], other[5:9]]))
