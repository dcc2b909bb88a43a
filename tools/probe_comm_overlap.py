"""Does rank 0's share of the P=8 C4 pass absorb its collectives?  Measured on one GPU.

Rank 0's shard of the 8-way partition runs as in tools/probe_rank_work.py, but every
collective the pass issues (the partial all-to-all, the item all-gather) is replaced by
a kernel with a collective's residency on its own stream: `blocks` workgroups holding
`lds` bytes of LDS for `usec` µs (gnnrec_hold_cus; default 1.5 ms = 448 MB at 300 GB/s
over xGMI, 64 blocks, 32 KiB).  No bytes move, so this prices the CU sharing alone: a
real collective also adds its HBM traffic (0.45 GB read + 0.45 GB written per exchange).
Outputs are not compared here: the local exchange leaves 7/8 of the gathered item table
unwritten (timing only); tests/test_gpu_concurrency.py checks the modes bitwise.

Modes of the aggregation kernels (ops.set_concurrency):
  static      grid-stride rows, every CU (the single-GPU bench mode)
  queue       rows from the device work queue (rowq.hpp), every CU
  queue+rN    the queue, N CUs left free

    python tools/probe_comm_overlap.py [--usec 1500] [--blocks 64] [--lds 32768]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-recsys_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gnnrec import nn as gnn  # noqa: E402
from gnnrec import ops  # noqa: E402
from gnnrec.inference import ShardedFullGraphPass  # noqa: E402
from gnnrec.synth import GraphMeta, bipartite_shard, node_features  # noqa: E402
from probe_rank_work import LocalExchange  # noqa: E402


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class HeldExchange(LocalExchange):
    """LocalExchange whose async collectives hold CUs on a comm stream like RCCL's."""

    def __init__(self, ws, usec, blocks, lds):
        super().__init__(ws)
        self.usec, self.blocks, self.lds = usec, blocks, lds
        self.stream = torch.cuda.Stream()

    def _comm(self):
        self.stream.wait_stream(torch.cuda.current_stream())
        ops.hold_cus(self.blocks, self.usec, lds_bytes=self.lds, stream=self.stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _Work(ev)

    def reduce_scatter_rows(self, full, op, async_op=False):
        own, _ = super().reduce_scatter_rows(full, op)
        return own, self._comm()

    def all_to_all_rows(self, full, async_op=False):
        blocks, _ = super().all_to_all_rows(full)
        return blocks, self._comm()

    def all_gather_rows(self, own, out, async_op=False):
        out, _ = super().all_gather_rows(own, out)
        return out, self._comm()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--usec", type=int, default=1500)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--lds", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    n_u, n_i, E, d, P = 10_000_000, 1_000_000, 500_000_000, 128, args.P
    sh = bipartite_shard(n_u, n_i, E, 0, P, dev, segments=8)
    feats = sh.local_features({"user": node_features(n_u, d, 0, dev),
                               "item": node_features(n_i, d, 1, dev)})
    torch.manual_seed(0)
    meta = GraphMeta(sh.canonical_etypes, ["item", "user"])
    model = gnn.ConvModel(meta, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev).eval()
    modes = {"static": (0, False), "queue": (0, True), "queue+r8": (8, True),
             "queue+r16": (16, True), "queue+r32": (32, True)}
    res = {"P": P, "hold": {"usec": args.usec, "blocks": args.blocks, "lds": args.lds},
           "collectives_per_pass": None, "ms": {}}
    for comm in ("none", "held"):
        for name, conc in modes.items():
            ex = LocalExchange(P) if comm == "none" else HeldExchange(P, args.usec, args.blocks,
                                                                      args.lds)
            runner = ShardedFullGraphPass(model, sh, ex, deterministic=True, concurrency=conc)
            calls = [0]
            if comm == "held":
                inner = ex._comm

                def counted(inner=inner):
                    calls[0] += 1
                    return inner()
                ex._comm = counted
            runner.run(feats, replicate_output=False)
            torch.cuda.synchronize()
            n0 = calls[0]
            runner.run(feats, replicate_output=False)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.reps):
                runner.run(feats, replicate_output=False)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / args.reps * 1e3
            if comm == "held":
                res["collectives_per_pass"] = n0
            res["ms"][f"{comm}/{name}"] = round(ms, 3)
            print(json.dumps(res), flush=True)
    ops.set_concurrency(0, False)


if __name__ == "__main__":
    main()
