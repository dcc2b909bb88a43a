"""Host logic of the lazily gathered block data (gnnrec.graph.LazyRows in a _FrameDict): no
GPU — the row gather itself is stubbed; tests/test_gpu_capture.py checks it on the device."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))

from gnnrec.graph import LazyRows, _FrameDict  # noqa: E402
from gnnrec.sampling import _tensors  # noqa: E402


class _Counted(LazyRows):
    """LazyRows whose gather is a host index_select (-1 -> zero row), counting its reads."""
    __slots__ = ("reads",)

    def __init__(self, table, ids):
        super().__init__(table, ids)
        self.reads = 0

    def get(self):
        self.reads += 1
        ok = (self.ids >= 0).to(self.table.dtype).unsqueeze(1)
        return self.table.index_select(0, self.ids.clamp(min=0)) * ok


def _frame():
    table = torch.arange(12, dtype=torch.float32).reshape(6, 2)
    lazy = _Counted(table, torch.tensor([4, -1, 0]))
    return _FrameDict({"_ID": torch.tensor([4, -1, 0]), "features": lazy}), lazy, table


def test_a_lazy_value_is_gathered_once_on_first_read():
    f, lazy, table = _frame()
    want = torch.stack([table[4], torch.zeros(2), table[0]])
    assert torch.equal(f["features"], want)
    assert torch.equal(f["features"], want) and lazy.reads == 1  # replaced by its tensor
    assert not isinstance(dict.__getitem__(f, "features"), LazyRows)


def test_every_read_path_materialises_and_lazy_items_does_not():
    for read in (lambda f: f.get("features"), lambda f: dict(f.items())["features"],
                 lambda f: f.values()[1], lambda f: f.pop("features")):
        f, lazy, _ = _frame()
        assert dict(f.lazy_items())["features"] is lazy and lazy.reads == 0
        assert isinstance(read(f), torch.Tensor) and lazy.reads == 1
    f, _, _ = _frame()
    assert f.get("missing", 7) == 7 and f.pop("missing", 8) == 8


def test_the_capture_input_walk_leaves_lazy_values_unread():
    f, lazy, _ = _frame()
    found = _tensors([f, (f,)], [])
    assert lazy.reads == 0 and all(isinstance(t, torch.Tensor) for t in found)
    assert len(found) == 2  # the two _ID references, no gathered features
