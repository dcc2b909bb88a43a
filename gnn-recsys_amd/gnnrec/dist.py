"""Collective exchange for the sharded full-graph pass.

One process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm),
xGMI between the 8 MI355X of a node.  Two collectives per layer and per
replicated node type, both sized by the SMALL side of the bipartite graph:

  reduce-scatter  partial aggregates of the relations whose destination type
                  is replicated (user→item: each rank aggregates the edges of
                  its own users into every item row) -> the item rows it owns;
  all-gather      the item rows each rank projected -> the full item table
                  every rank reads as sources of item→user edges next layer.

Replicated tables are padded to P·S rows (S = ceil(N/P)) so both collectives
are the equal-count RCCL forms.  On gloo (CPU tests) reduce-scatter is
emulated by all_reduce + slice and all-gather by the list form.
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.distributed as dist


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world() -> int:
    return dist.get_world_size() if is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def multi_rank(ex) -> bool:
    """Does the sharded pass run its multi-rank schedule with exchange `ex` (world size > 1,
    or an Exchange forcing its collectives at world size 1)?"""
    return bool(getattr(ex, "multi", ex.ws > 1))


def even_ranges(n: int, parts: int) -> List[int]:
    """Boundaries b[0..parts] of a contiguous, count-balanced split of [0, n)."""
    return [(n * p) // parts for p in range(parts + 1)]


def degree_ranges(weight: torch.Tensor, parts: int) -> List[int]:
    """Boundaries b[0..parts] of a contiguous split of [0, n) balanced by cumulative weight
    ("contiguous global-id ranges balanced by cumulative in-degree"): b[p] is
    the first id whose exclusive prefix weight reaches p·W/parts.  `weight` is a per-node
    int tensor (callers pass in-degree summed over relations + 1, so a row's fixed cost
    counts and zero-degree ranges still split).  Integer arithmetic only: every rank that
    computes it from the same degrees gets the same boundaries."""
    n = int(weight.numel())
    if n == 0 or parts == 1:
        return [0] + [n] * parts if n else [0] * (parts + 1)
    c = torch.cumsum(weight.to(torch.int64), 0)
    W = int(c[-1])
    if W <= 0:
        return even_ranges(n, parts)
    t = torch.tensor([(W * p) // parts for p in range(1, parts)], dtype=torch.int64,
                     device=c.device)
    # exclusive prefix of id j is c[j-1]: first j with c[j-1] >= t is searchsorted(c, t) + 1
    inner = (torch.searchsorted(c, t) + 1).clamp_(max=n).tolist()
    b = [0] + [int(x) for x in inner] + [n]
    for p in range(1, parts + 1):  # monotone even with ties
        b[p] = max(b[p], b[p - 1])
    return b


def padded_shard(n: int, parts: int) -> int:
    """Rows per rank of a replicated table padded to parts·S rows."""
    return (n + parts - 1) // parts if n else 0


class Exchange:
    """reduce-scatter / all-gather of equal row blocks of a [P·S, d] table."""

    def __init__(self, group=None, force_collectives: bool = False):
        self.group = group
        self.ws = world()
        self.rk = rank()
        # force_collectives: issue every collective even at world size 1 (no shortcut), and
        # make the sharded pass take its multi-rank schedule (`multi`) — the RCCL forms
        # then run on a one-GPU box (tests/test_gpu_rccl.py), bitwise the one-rank pass
        self.multi = self.ws > 1 or bool(force_collectives)
        self.backend = dist.get_backend(group) if is_initialized() else None
        # a group created without an explicit backend reports e.g. 'cpu:gloo,cuda:nccl'
        self._rccl = self.backend is not None and "nccl" in str(self.backend)
        self.path = None  # 'rccl' | 'emulated' once the first collective has run
        # all-gather as RCCL's all-gather ('rccl'), or as an all-to-all of the own block
        # replicated P times ('a2a': every peer reached over its own xGMI link at once
        # instead of RCCL's ring schedule — SURVEY §5's ring cap); GNNREC_ALLGATHER
        self.ag_mode = os.environ.get("GNNREC_ALLGATHER", "rccl")
        if self.ag_mode not in ("rccl", "a2a"):
            raise ValueError(f"GNNREC_ALLGATHER={self.ag_mode!r}: 'rccl' or 'a2a'")

    def _fast(self, t: torch.Tensor) -> bool:
        """RCCL's reduce-scatter / all-gather-into / all-to-all for device tensors on an
        nccl (RCCL) group; the gloo emulation otherwise (CPU tests, gloo rehearsals)."""
        fast = self._rccl and t.is_cuda
        if self.path is None:
            self.path = "rccl" if fast else "emulated"
        return fast

    def reduce_scatter_rows(self, full: torch.Tensor, op: str, async_op: bool = False):
        """full [P·S, d] partial on every rank -> (own [S, d], work|None)."""
        if not self.multi:
            return full, None
        S = full.shape[0] // self.ws
        rop = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
        if self._fast(full):
            out = torch.empty((S,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
            work = dist.reduce_scatter_tensor(out, full, op=rop, group=self.group,
                                              async_op=async_op)
            return out, work
        dist.all_reduce(full, op=rop, group=self.group)
        return full[self.rk * S:(self.rk + 1) * S], None

    def all_gather_rows(self, own: torch.Tensor, out: torch.Tensor, async_op: bool = False):
        """own [S, d] -> out [P·S, d] in rank order, returns (out, work|None)."""
        if not self.multi:
            if out.data_ptr() != own.data_ptr():
                out.copy_(own)
            return out, None
        if self.ag_mode == "a2a":
            # block j of every rank's input is its own block: all-to-all delivers rank j's
            # block into slot j everywhere (one local copy of P blocks to stage it)
            self._fast(own)
            src = own.unsqueeze(0).expand((self.ws,) + tuple(own.shape)).contiguous()
            work = dist.all_to_all_single(out, src.view(out.shape), group=self.group,
                                          async_op=async_op)
            return out, work
        if self._fast(own):
            work = dist.all_gather_into_tensor(out, own.contiguous(), group=self.group,
                                               async_op=async_op)
            return out, work
        S = own.shape[0]
        tmp = [torch.empty_like(own) for _ in range(self.ws)]
        dist.all_gather(tmp, own.contiguous(), group=self.group)
        for i, t in enumerate(tmp):
            out[i * S:(i + 1) * S].copy_(t)
        return out, None

    def all_to_all_rows(self, full: torch.Tensor, async_op: bool = False):
        """full [P·S, d] on every rank -> ([P, S, d], work|None): block rk of every rank's
        table, in source-rank order (the deterministic pass folds them in a fixed tree)."""
        S = full.shape[0] // self.ws
        shape = (self.ws, S) + tuple(full.shape[1:])
        if not self.multi:
            return full.view(shape), None
        out = torch.empty_like(full)
        if self._fast(full):
            work = dist.all_to_all_single(out, full.contiguous(), group=self.group,
                                          async_op=async_op)
            return out.view(shape), work
        # gloo (tests): gather every table, keep our block of each
        tmp = [torch.empty_like(full) for _ in range(self.ws)]
        dist.all_gather(tmp, full.contiguous(), group=self.group)
        for i, t in enumerate(tmp):
            out[i * S:(i + 1) * S].copy_(t[self.rk * S:(self.rk + 1) * S])
        return out.view(shape), None

    def all_reduce_(self, t: torch.Tensor, op: str = "sum"):
        if self.multi:
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX,
                            group=self.group)
        return t

    def max_scalar(self, x: float, device) -> float:
        t = torch.tensor([x], dtype=torch.float64, device=device)
        self.all_reduce_(t, "max")
        return float(t.item())


class _StreamWork:
    """The work handle RCCL returns, restated for the emulation: the collective completes
    on its own stream, and wait() makes the CURRENT stream wait for that completion (the
    host blocks only until the transport thread has queued the copy-out, as a torch RCCL
    work's wait() blocks only until the collective is enqueued)."""

    def __init__(self, fut, device):
        self._fut, self._dev = fut, device

    def wait(self, timeout=None):
        ev = self._fut.result()
        torch.cuda.current_stream(self._dev).wait_event(ev)
        return True

    def is_completed(self) -> bool:
        return self._fut.done() and self._fut.result().query()


class AsyncEmulatedExchange(Exchange):
    """The RCCL exchange's asynchrony without RCCL (gloo transport): what a one-GPU box and
    the CPU tests can run of the multi-GPU pass's ordering (the pool gives one GPU per job,
    so RCCL itself only runs in the driver's 8-GPU bench).

    Device tensors: every collective is issued like an async RCCL one —
      * a copy-in stream waits for the issuing stream, runs a delay kernel holding
        `hold_blocks` CUs for `delay_us` µs (gnnrec_hold_cus: a collective kernel's
        residency and latency), then copies the input to pinned host memory — so the input
        is read LATE, and a producer that overwrites it before waiting on the work races;
      * one transport thread (FIFO: the same collective order on every rank) runs the gloo
        collective on the host copies, then queues on a copy-out stream another delay and
        the copy of the result into the device output, and records the completion event;
      * the work's wait() makes the current stream wait for that event — so a reader that
        skips the wait reads the output before it arrives.
    CPU tensors: gloo's own async_op works (a transport thread per group).

    Every collective returns a work (never None): `works_issued` counts them and
    `sync_calls` counts the collectives asked for synchronously (async_op=False)."""

    def __init__(self, group=None, delay_us: int = 500, hold_blocks: int = 16):
        super().__init__(group)
        if self._rccl:
            raise ValueError("AsyncEmulatedExchange emulates RCCL on a gloo group; this group "
                             "is RCCL already: use Exchange")
        self.path = "emulated-async"
        self.delay_us, self.hold_blocks = int(delay_us), int(hold_blocks)
        self.works_issued = 0
        self.sync_calls = 0
        self._streams = None
        self._pool = None
        self._gate = None
        # the transport thread's collectives go through their own gloo group, so they never
        # interleave with collectives the main thread issues on the default one
        self._tgroup = dist.new_group(backend="gloo") if self.ws > 1 else None

    def _fast(self, t):
        return False

    # ---- device tensors: copy-in (main thread) -> gloo (transport thread) -> copy-out ----
    def _dev_setup(self, dev):
        if self._streams is None:
            import concurrent.futures
            self._dev = dev
            self._streams = (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev))
            self._pool = concurrent.futures.ThreadPoolExecutor(
                max_workers=1, thread_name_prefix="gnnrec-exchange",
                initializer=torch.cuda.set_device, initargs=(dev,))

    def _delay(self, stream):
        if self.delay_us > 0:
            from . import ops
            ops.hold_cus(self.hold_blocks, self.delay_us, stream=stream)

    def gate(self):
        """Ordering by events instead of delays (tests of the emulation itself): the
        collectives issued from now until release(event) copy their input in only after
        `event` — recorded by the caller on its stream once it has done whatever must come
        first — and land their output only after that copy-in, so 'the input is read late'
        and 'the output lands late' hold by construction, whatever the box's load."""
        import threading
        self._gate = {"open": threading.Event(), "after": None}

    def release(self, event: torch.cuda.Event):
        g, self._gate = self._gate, None
        g["after"] = event
        g["open"].set()

    def _issue(self, src: torch.Tensor, out: torch.Tensor, transport, async_op: bool):
        """src (device) -> transport(h_in, h_out) on host copies -> out (device)."""
        dev = src.device
        self._dev_setup(dev)
        s_in, s_out = self._streams
        cur = torch.cuda.current_stream(dev)
        h_in = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        gate = self._gate

        def copy_in():
            with torch.cuda.stream(s_in):
                self._delay(s_in)
                h_in.copy_(src, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s_in)
            return ev

        if gate is None:
            s_in.wait_stream(cur)
            ev_in = copy_in()
        else:  # the copy-in is queued by the transport thread once the gate opens
            ev_in = None
            ev_issue = torch.cuda.Event()
            ev_issue.record(cur)
        src.record_stream(s_in)
        out.record_stream(s_out)
        h_out = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)

        def job():
            nonlocal ev_in
            if gate is not None:
                gate["open"].wait()
                s_in.wait_event(ev_issue)
                s_in.wait_event(gate["after"])
                ev_in = copy_in()
            ev_in.synchronize()
            transport(h_in, h_out)
            with torch.cuda.stream(s_out):
                self._delay(s_out)
                out.copy_(h_out, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s_out)
            return ev

        work = _StreamWork(self._pool.submit(job), dev)
        self.works_issued += 1
        if not async_op:
            self.sync_calls += 1
            work.wait()
            return None
        return work

    def reduce_scatter_rows(self, full, op, async_op=False):
        if self.ws == 1:
            return full, None
        S = full.shape[0] // self.ws
        rop = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
        out = torch.empty((S,) + tuple(full.shape[1:]), dtype=full.dtype, device=full.device)
        if full.is_cuda:
            def transport(h_in, h_out):
                dist.reduce_scatter_tensor(h_out, h_in, op=rop, group=self._tgroup)
            return out, self._issue(full, out, transport, async_op)
        work = dist.reduce_scatter_tensor(out, full.contiguous(), op=rop, group=self._tgroup,
                                          async_op=True)
        return out, self._cpu(work, async_op)

    def all_gather_rows(self, own, out, async_op=False):
        if self.ws == 1:
            return super().all_gather_rows(own, out, async_op)
        own = own.contiguous()
        if own.is_cuda:
            if self.ag_mode == "a2a":  # as Exchange's: an all-to-all of the own block x P
                src = own.unsqueeze(0).expand((self.ws,) + tuple(own.shape)).contiguous()

                def transport(h_in, h_out):
                    dist.all_to_all_single(h_out, h_in.view(h_out.shape), group=self._tgroup)
                return out, self._issue(src, out, transport, async_op)

            def transport(h_in, h_out):
                dist.all_gather_into_tensor(h_out, h_in, group=self._tgroup)
            return out, self._issue(own, out, transport, async_op)
        work = dist.all_gather_into_tensor(out, own, group=self._tgroup, async_op=True)
        return out, self._cpu(work, async_op)

    def all_to_all_rows(self, full, async_op=False):
        S = full.shape[0] // self.ws
        shape = (self.ws, S) + tuple(full.shape[1:])
        if self.ws == 1:
            return full.view(shape), None
        full = full.contiguous()
        out = torch.empty_like(full)
        if full.is_cuda:
            def transport(h_in, h_out):
                dist.all_to_all_single(h_out, h_in, group=self._tgroup)
            return out.view(shape), self._issue(full, out, transport, async_op)
        work = dist.all_to_all_single(out, full, group=self._tgroup, async_op=True)
        return out.view(shape), self._cpu(work, async_op)

    def _cpu(self, work, async_op):
        self.works_issued += 1
        if not async_op:
            self.sync_calls += 1
            work.wait()
            return None
        return work

    def all_reduce_(self, t, op="sum"):
        self.drain()
        return super().all_reduce_(t, op)

    def drain(self):
        """Block until every issued device collective has queued its copy-out."""
        if self._pool is not None:
            self._pool.submit(lambda: None).result()

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=True)
            self._pool = None
            self._streams = None


class ComputeOnlyExchange:
    """An Exchange of world size P that moves nothing: each collective returns this rank's
    own data in the right shape.  Runs a rank's share of the pass with the same kernels,
    launch order and concurrency settings as the real one, minus the communication
    (bench.py's per-rank compute time at P > 1; tools/probe_rank_work.py)."""

    def __init__(self, ws: int, rk: int = 0):
        self.ws, self.rk, self.backend, self.group, self.path = ws, rk, None, None, "none"
        self.multi = ws > 1

    def reduce_scatter_rows(self, full, op, async_op=False):
        S = full.shape[0] // self.ws
        return full[self.rk * S:(self.rk + 1) * S], None

    def all_to_all_rows(self, full, async_op=False):
        S = full.shape[0] // self.ws
        return full.view((self.ws, S) + tuple(full.shape[1:])), None

    def all_gather_rows(self, own, out, async_op=False):
        S = own.shape[0]
        out[self.rk * S:(self.rk + 1) * S].copy_(own)
        return out, None

    def all_reduce_(self, t, op="sum"):
        return t

    def max_scalar(self, x, device):
        return x


_M64 = (1 << 64) - 1


def table_digest(t: torch.Tensor, row0: int = 0, chunk: int = 1 << 24):
    """Bit-pattern checksum of rows [row0, row0 + len(t)) of a global fp32/int32 table, on
    the tensor's device: (Σ v_i·(2i+1), Σ v_i·(2i+1)²) mod 2^64 over the int32 views v_i,
    i = the GLOBAL element index.  Any single changed bit changes both sums, and the sums
    are additive over disjoint row ranges, so the digests of every rank's owned rows add
    up (mod 2^64) to the one-process digest of the whole table — a P > 1 run checks its
    bits against P = 1 without moving the tables (bench.py `bitwise_vs_p1`)."""
    t = t.contiguous()
    per_row = t[0].numel() if t.dim() > 1 and t.shape[0] else 1
    v = t.view(torch.int32).reshape(-1)
    acc = torch.zeros(2, dtype=torch.int64, device=t.device)
    for e0 in range(0, v.numel(), chunk):
        blk = v[e0:e0 + chunk].to(torch.int64)
        g0 = row0 * per_row + e0
        w = torch.arange(g0, g0 + blk.numel(), device=t.device, dtype=torch.int64) * 2 + 1
        bw = blk * w
        acc[0] += bw.sum()
        acc[1] += (bw * w).sum()
    s1, s2 = (int(x) for x in acc.tolist())
    return s1 & _M64, s2 & _M64


def digest_add(*ds):
    """Sum of (s1, s2) digests of disjoint row ranges, mod 2^64."""
    return (sum(d[0] for d in ds) & _M64, sum(d[1] for d in ds) & _M64)


class ProgressExchange:
    """Wraps an Exchange and prints one stderr line per collective issued — rank, pass,
    layer, kind, shape — so a multi-GPU run that stops inside a collective names it.  With
    `checked` (the bench's first warm-up pass) every collective is also waited on and the
    device synchronised before the pass goes on, and its completion is printed with its
    time: on first contact with RCCL a stuck collective is then the last 'issued' line
    without its 'done', and the process group's timeout ends the run instead of a silent
    hang.  Everything else is the inner exchange's."""

    def __init__(self, inner, runner=None, stream=None):
        self.inner, self.runner = inner, runner
        self.stream = stream if stream is not None else __import__("sys").stderr
        self.checked = False
        self.pass_no = 0
        self.enabled = True

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def _say(self, msg):
        if self.enabled:
            layer = getattr(self.runner, "_layer_idx", None)
            self.stream.write(f"[gnnrec r{self.inner.rk}] pass {self.pass_no} layer {layer} "
                              f"{msg}\n")  # one write per line (ranks share a stderr)
            self.stream.flush()

    def layer_start(self, i):
        """ShardedFullGraphPass.progress hook: one line per layer."""
        self._say("start")

    def _call(self, kind, t, fn):
        import time
        self._say(f"{kind} {tuple(t.shape)} issued")
        t0 = time.perf_counter()
        res = fn()
        if self.checked:
            work = res[1]
            if work is not None:
                work.wait()
            if t.is_cuda:
                torch.cuda.synchronize(t.device)
            self._say(f"{kind} done in {(time.perf_counter() - t0) * 1e3:.1f} ms")
        return res

    def reduce_scatter_rows(self, full, op, async_op=False):
        return self._call("reduce_scatter", full,
                          lambda: self.inner.reduce_scatter_rows(full, op, async_op))

    def all_to_all_rows(self, full, async_op=False):
        return self._call("all_to_all", full, lambda: self.inner.all_to_all_rows(full, async_op))

    def all_gather_rows(self, own, out, async_op=False):
        return self._call("all_gather", out,
                          lambda: self.inner.all_gather_rows(own, out, async_op))


class RecordingExchange:
    """Wraps an Exchange and records every collective of a pass: (kind, shape, dtype, op)
    plus the bytes this rank sends (all-to-all / reduce-scatter: (P−1)/P of the table;
    all-gather: (P−1)·own).  `replay_ms` times the same collectives alone, back to back,
    on fresh tensors: the communication a pass would cost with nothing to overlap."""

    def __init__(self, inner: Exchange):
        self.inner = inner
        self.ws, self.rk, self.group = inner.ws, inner.rk, inner.group
        self.multi = multi_rank(inner)
        self.backend = inner.backend
        self.calls = []

    @property
    def path(self):
        return self.inner.path

    def _rec(self, kind, t, op=None, sent=0):
        self.calls.append((kind, tuple(t.shape), t.dtype, op, int(sent)))

    def reduce_scatter_rows(self, full, op, async_op=False):
        self._rec("reduce_scatter", full, op,
                  full.numel() * full.element_size() * (self.ws - 1) // self.ws)
        return self.inner.reduce_scatter_rows(full, op, async_op)

    def all_to_all_rows(self, full, async_op=False):
        self._rec("all_to_all", full, None,
                  full.numel() * full.element_size() * (self.ws - 1) // self.ws)
        return self.inner.all_to_all_rows(full, async_op)

    def all_gather_rows(self, own, out, async_op=False):
        self._rec("all_gather", out, None,
                  own.numel() * own.element_size() * (self.ws - 1))
        return self.inner.all_gather_rows(own, out, async_op)

    def all_reduce_(self, t, op="sum"):
        return self.inner.all_reduce_(t, op)

    def max_scalar(self, x, device):
        return self.inner.max_scalar(x, device)

    def bytes_sent(self) -> int:
        return sum(c[4] for c in self.calls)

    def replay_ms(self, device, reps: int = 3) -> float:
        """Mean wall ms of one pass's collectives issued alone (synchronous, in order)."""
        if self.ws == 1 or not self.calls:
            return 0.0
        bufs = []
        for kind, shape, dtype, op, _ in self.calls:
            full = torch.zeros(shape, dtype=dtype, device=device)
            if kind == "all_gather":
                own = full[: shape[0] // self.ws].clone()
                bufs.append((kind, own, full, op))
            else:
                bufs.append((kind, full, None, op))

        def once():
            for kind, a, b, op in bufs:
                if kind == "reduce_scatter":
                    self.inner.reduce_scatter_rows(a, op)
                elif kind == "all_to_all":
                    self.inner.all_to_all_rows(a)
                else:
                    self.inner.all_gather_rows(a, b)

        return self._timed(once, device, reps)

    def replay_by_kind(self, device, reps: int = 3) -> dict:
        """Per collective kind, that kind's calls of one pass replayed alone:
        {kind: {'ms': per call, 'calls': per pass, 'bytes': sent per call, 'busbw_GBs'}}.
        The all-gathers are replayed in both forms ('all_gather' as the pass ran them,
        'all_gather_<other mode>' the alternative of Exchange.ag_mode), so one multi-GPU
        run shows whether RCCL's ring schedule or the direct all-to-all moves them faster."""
        if self.ws == 1 or not self.calls:
            return {}
        out = {}
        for kind in sorted({c[0] for c in self.calls}):
            calls = [c for c in self.calls if c[0] == kind]
            modes = [None]
            if kind == "all_gather" and getattr(self.inner, "ag_mode", None) in ("rccl", "a2a"):
                modes.append("a2a" if self.inner.ag_mode == "rccl" else "rccl")
            for mode in modes:
                sub = RecordingExchange(self.inner)
                sub.calls = calls
                keep = getattr(self.inner, "ag_mode", None)
                if mode is not None:
                    self.inner.ag_mode = mode
                try:
                    ms = sub.replay_ms(device, reps) / len(calls)
                finally:
                    if mode is not None:
                        self.inner.ag_mode = keep
                sent = sum(c[4] for c in calls) / len(calls)
                out[kind if mode is None else f"{kind}_{mode}"] = {
                    "ms": ms, "calls": len(calls), "bytes": int(sent),
                    "busbw_GBs": sent / (ms * 1e-3) / 1e9 if ms > 0 else None}
        return out

    def replay_ms_by_allgather(self, device, reps: int = 3) -> dict:
        """replay_ms with the pass's all-gathers in each form: {'rccl': ms, 'a2a': ms} — the
        communication one pass would cost under either GNNREC_ALLGATHER setting."""
        if self.ws == 1 or not self.calls or not hasattr(self.inner, "ag_mode"):
            return {}
        keep, out = self.inner.ag_mode, {}
        try:
            for mode in ("rccl", "a2a"):
                self.inner.ag_mode = mode
                out[mode] = self.replay_ms(device, reps)
        finally:
            self.inner.ag_mode = keep
        return out

    def _timed(self, once, device, reps):
        import time
        once()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        dist.barrier(group=self.group)
        t0 = time.perf_counter()
        for _ in range(reps):
            once()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        dist.barrier(group=self.group)
        return (time.perf_counter() - t0) / reps * 1e3
