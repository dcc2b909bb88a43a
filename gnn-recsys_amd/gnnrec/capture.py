"""A training step captured once into a hipGraph and replayed per batch (SURVEY §8f row f2,
the reference's train loop src/train/run.py:104-160 — forward, max_margin_loss, backward,
optimizer step — per EdgeDataLoader batch).

The batches come from EdgeDataLoader(static_shapes=True): every full batch has the same
shapes and nothing in the step reads a value back to the host, so the whole step — some
hundreds of kernels, each a few microseconds, whose launches bound the eager step on the
host — is recorded once and re-issued by one hipGraphLaunch.  Per batch the step copies the
batch's tensors into the captured batch's buffers (ops.copy_batch: one launch per 64
tensors, not one blit per tensor) and replays.

    step = CapturedTrainStep(model, opt, lambda m, b: loss_of(m, b))
    for batch in loader:            # loader = EdgeDataLoader(..., static_shapes=True)
        loss = step(batch)          # a device scalar; read it when needed

Eager steps: the first `warmup` static batches (lazy initialisation, the model's and the
sampler's settled choices, e.g. the first-layer fold), and every batch whose structure
differs from the captured one (a final partial batch comes in the exact, non-static form).
A new structure seen on `recapture_after` batches in a row is captured in place of the old
(the batches a prefetching loader built before such a choice settled run eagerly).
The optimizer must keep its step counts on the device (Adam / AdamW with fused=True or
capturable=True); its param groups are switched to capturable at capture.  Between steps
the gradients live in the graph's memory: do not zero or replace them (the graph overwrites
them every replay, as the eager step's zero_grad + backward would).
"""
from __future__ import annotations

import torch

from . import ops
from .sampling import RNG_LOCK, _tensors


def batch_is_static(batch) -> bool:
    """A loader item of EdgeDataLoader(static_shapes=True) at fixed shapes."""
    return any(getattr(x, "static", False) for x in batch[1:-1]) and \
        all(getattr(b, "static", False) for b in batch[-1])


def _signature(tensors):
    return tuple((tuple(t.shape), t.dtype, t.stride(), t.device) for t in tensors)


class CapturedTrainStep:
    """loss_fn(model, batch) -> scalar loss: the step's forward (model + loss)."""

    def __init__(self, model, optimizer, loss_fn, warmup: int = 2, recapture_after: int = 2):
        self.model, self.opt, self.loss_fn = model, optimizer, loss_fn
        self.warmup = int(warmup)
        self.recapture_after = int(recapture_after)
        self._new_sig, self._new_seen = None, 0
        self.captures = 0
        self.graph = None
        self.loss = None
        self._batch = None   # the captured batch: its tensors are the graph's inputs
        self._inputs = None
        self._sig = None
        self.seen = 0
        self.replays = 0
        self.eager_steps = 0

    def eager(self, batch):
        """One ordinary step (the form the graph records)."""
        self.eager_steps += 1
        loss = self.loss_fn(self.model, batch)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        # no reference to the step's autograd graph outlives it: a kept graph keeps its
        # AccumulateGrad nodes (bound to this stream) alive into the capture, whose backward
        # would then accumulate on the wrong stream
        return loss.detach()

    def _capturable(self):
        for group in self.opt.param_groups:
            if "capturable" not in group:
                raise TypeError(f"{type(self.opt).__name__}: no capturable mode to replay in a "
                                "graph (use Adam / AdamW with fused=True or capturable=True)")
            group["capturable"] = True
            for p in group["params"]:
                st = self.opt.state.get(p, {})
                step = st.get("step")
                if torch.is_tensor(step) and step.device != p.device:
                    st["step"] = step.to(p.device)

    def _capture(self, batch, inputs):
        self._capturable()
        # the step's own ops run at least once outside the capture on this batch's shapes
        # (the warm-up steps), so every lazy allocation / library init has happened
        self.opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # a loader's sampling thread draws no negatives while the capture is under way
        # (sampling.RNG_LOCK)
        with RNG_LOCK, torch.cuda.graph(g, capture_error_mode="thread_local"):
            loss = self.loss_fn(self.model, batch)
            loss.backward()
            self.opt.step()
        self.graph, self.loss = g, loss.detach()
        del loss
        self._batch, self._inputs, self._sig = batch, inputs, _signature(inputs)
        self.captures += 1

    def __call__(self, batch):
        if not batch_is_static(batch):
            return self.eager(batch)
        self.seen += 1
        if self.seen <= self.warmup:
            return self.eager(batch)
        inputs = [t for t in _tensors(batch, []) if t.is_cuda]
        sig = None if self.graph is None else _signature(inputs)
        if self.graph is not None and sig != self._sig:
            if sig != self._new_sig:
                self._new_sig, self._new_seen = sig, 0
            self._new_seen += 1
            if self._new_seen < self.recapture_after:
                return self.eager(batch)
            self.graph = None  # the new structure has settled: capture it instead
        self._new_sig, self._new_seen = None, 0
        if self.graph is None:
            self._capture(batch, inputs)  # records only: the replay below runs the step
        else:
            ops.copy_batch(inputs, self._inputs)  # one launch per 64 tensors
        self.graph.replay()
        self.replays += 1
        return self.loss
