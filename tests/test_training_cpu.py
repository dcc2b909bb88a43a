"""CPU checks of the training step's host-side autograd pieces (no launches): the zero-copy
join the cosine backward uses for an etype's positive and negative lists.  (The first-layer
fold's weight products, autograd.FoldFn, run on the library's GEMMs: tests/test_gpu_fold.py.)"""
import pytest
import torch

from gnnrec import autograd as ag


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
