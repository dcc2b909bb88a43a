"""bench.py — edges aggregated/s of the full-graph inference embedding pass.

BASELINE.json metric: "edges aggregated/sec, full-graph embed pass, d=128, at
1/2/4/8 MI355X".  Workload (BASELINE.json configs[3], "C4"): 10M users x 1M
items, 500M user->item edges (+ the 500M reverse item->user edges), ConvModel
with NodeEmbedding + L=2 ConvLayers (n_layers=3, embedding_layer=True),
aggregator 'mean', hetero 'sum', norm=True, d=128 fp32 (reference
src/model.py:330-421 driven as src/train/run.py:311-349 with a full-neighbour
sampler).  Synthetic graph (counter-hash generator, seed 11), N(0,1) features
(seed 0) and xavier weights (torch.manual_seed(0)) — no dataset exists offline.

A step = one full pass over the whole graph: embed + 2 layers x 2 relations.
edges aggregated per step = L x sum_r |E_r| = 2 x (500M + 500M) = 2e9.
Multi-GPU: one process per GPU (torchrun), users partitioned, edges follow
their user; per layer one reduce-scatter + one all-gather of the 1M-row item
table over RCCL; per-GPU work shrinks with N at fixed total graph.

Run:  python bench.py [--gpus N --steps K --warmup W]
      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks).  Without a launcher (WORLD_SIZE unset) N > 1 starts N "
                         "rank processes itself (torch.distributed.run as a child); under a "
                         "launcher WORLD_SIZE must equal N (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=500_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--zipf", type=float, default=0.0, help="item Zipf exponent (0 = uniform)")
    ap.add_argument("--aggregator", default="mean")
    ap.add_argument("--config", choices=["c4", "c5"], default="c4",
                    help="c5: the C4 graph split 80%% clicks / 20%% buys -> 4 relations")
    ap.add_argument("--hetero", choices=["sum", "mean", "max", "attention"], default="sum")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--mode", choices=["deterministic", "fast"], default="deterministic",
                    help="deterministic: outputs bitwise equal at 1/2/4/8 GPUs (fixed segment "
                         "tree + all-to-all); fast: tiles accumulated in place + reduce-scatter")
    ap.add_argument("--segments", type=int, default=8,
                    help="source-range tiles of the user->item relation (0: none; "
                         "deterministic mode needs a power of two divisible by the GPU count)")
    ap.add_argument("--concurrency", default="auto",
                    help="row-kernel schedule: 'auto' (static at one rank; 16 CUs reserved + "
                         "work queue beside RCCL at several) or 'R,Q' (R reserved CUs, Q=1 queue)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--minibatch", choices=["auto", "off"], default="auto",
                    help="also time the C2 training step (one GPU; a secondary field)")
    ap.add_argument("--cpu-sample", type=float, default=1 / 32,
                    help="fraction of each relation's destination rows the bounded CPU "
                         "baseline aggregates (over the full-size tables and edge stream)")
    ap.add_argument("--p1-digests", default=os.path.join(ROOT, "profiles", "p1_output_digests.json"),
                    help="committed one-GPU output digests a P > 1 run compares its bits with")
    ap.add_argument("--record-digest", default=None, metavar="PATH",
                    help="(one GPU) add this run's output digest to the digest file PATH")
    ap.add_argument("--allgather", choices=["auto", "rccl", "a2a"], default="auto",
                    help="P > 1: the item tables' all-gather as RCCL's all-gather or as an "
                         "all-to-all of the own block (GNNREC_ALLGATHER); auto: after the "
                         "warm-up, replay the pass's all-gathers both ways and keep the faster "
                         "(the outputs are the same bits either way)")
    ap.add_argument("--pg-timeout", type=float, default=300.0,
                    help="process-group timeout (s): a stuck collective ends the run, named")
    return ap.parse_args(argv) if argv is None else ap.parse_known_args(argv)[0]


class EventTimers:
    """HIP-event timing of tagged kernel launches on the current stream."""

    def __init__(self):
        self.events = {}
        self.enabled = False

    @contextlib.contextmanager
    def __call__(self, tag):
        if not self.enabled:
            yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self.events.setdefault(tag, []).append((s, e))

    def mean_ms(self, tag):
        ev = self.events.get(tag, [])
        if not ev:
            return float("nan"), 0
        return sum(s.elapsed_time(e) for s, e in ev) / len(ev), len(ev)


KERNELS = {
    "spmm_project": ("spmm_project_kernel", "gnnrec spmm_project_kernel (gather + segmented "
                     "mean + fused SAGE projection, ReLU, L2 norm)"),
    "spmm_project_mfma": ("spmm_project_mfma_kernel", "gnnrec spmm_project_mfma_kernel (gather "
                          "+ mean of 32-row tiles, SAGE projection on fp32 MFMA, ReLU, L2 norm)"),
    "spmm_tile": ("spmm_csr_kernel", "gnnrec spmm_csr_kernel (gather + segmented sum of one "
                  "source-range tile, accumulated in place)"),
    "spmm_tile2": ("spmm_csr2_kernel", "gnnrec spmm_csr2_kernel (gather + segmented sums of two "
                   "relations' source-range tiles from one table in one launch)"),
    "spmm": ("spmm_csr_kernel", "gnnrec spmm_csr_kernel (gather + segmented mean)"),
    "spmm_pair": ("spmm_pair_mfma_kernel", "gnnrec spmm_pair_mfma_kernel (two relations' "
                  "gathers + means from ONE source table into 32-row LDS tiles, all four SAGE "
                  "projections on the fp32 MFMA, ReLU, L2 norm, cross-relation combine)"),
    "spmm_project2": ("spmm_project2_pipe_kernel", "gnnrec spmm_project2_pipe_kernel (two "
                      "pre-projected relations' gathers + means into one dst row, both SAGE self "
                      "projections, ReLU, L2 norm, cross-relation sum; next rows' heads "
                      "prefetched)"),
}


def launch_bytes(shard, d, runner, deterministic):
    """Algorithmic bytes per layer and launches per layer of each aggregation kernel tag
    (SURVEY §8d row d4): per edge d*4 (fp32 source row) + 4 (int32 index); per dst row 8
    (int64 indptr) + d*4 (write), + d*4 for the h_self row when the projection is fused
    into the launch, + d*4 for the partial read back when a tile accumulates in place."""
    out = {}
    paired = {c: pair for pair in runner.tile_pairs for c in pair}
    fused2 = {c: pair for pair in getattr(runner, 'pair_fused', ()) for c in pair}
    raw2 = {c for pair in getattr(runner, 'pair_raw', ()) for c in pair}
    for ce, rs in shard.rels.items():
        if ce in fused2:  # one launch for both: their edges, 2 indptr, the h_self row + output
            tag = "spmm_pair" if ce in raw2 else "spmm_project2"
            n = 1 if ce == fused2[ce][0] else 0
            b = rs.local_edges * (d * 4 + 4) + rs.n_rows * (8 + (8 * d if n else 0))
        elif ce in paired:  # both relations' tile bytes, one launch per segment for the pair
            tag, b = "spmm_tile2", 0
            n = len(rs.segs) if ce == paired[ce][0] else 0
            for j, (ip, ix, _) in enumerate(rs.segs):
                acc = (j % 2 == 1) if deterministic else j > 0
                b += ix.numel() * (d * 4 + 4) + rs.n_rows * (8 + 4 * d * (2 if acc else 1))
        elif ce in runner.fused:
            avg = rs.global_edges / max(shard.num_nodes[ce[2]], 1) if deterministic else None
            tag = runner._fused_tag(rs, avg)
            b, n = rs.local_edges * (d * 4 + 4) + rs.n_rows * (8 + 8 * d), 1
        elif rs.segs is not None:
            tag, b, n = "spmm_tile", 0, len(rs.segs)
            for j, (ip, ix, _) in enumerate(rs.segs):
                acc = (j % 2 == 1) if deterministic else j > 0
                b += ix.numel() * (d * 4 + 4) + rs.n_rows * (8 + 4 * d * (2 if acc else 1))
        else:
            tag, b, n = "spmm", rs.local_edges * (d * 4 + 4) + rs.n_rows * (8 + 4 * d), 1
        tb, tn = out.get(tag, (0, 0))
        out[tag] = (tb + b, tn + n)
    return out


CSRC = os.path.join(ROOT, "gnn-recsys_amd", "csrc")


# the sources of the kernels whose HBM traffic the PMC passes measure (the aggregation
# launches and what they include) plus the build flags
PMC_SOURCES = ("spmm.hip", "spmm_project.hip", "spmm_pair_mfma.hip", "gemm.hip", "rowq.hip", "gather.hpp", "rowq.hpp",
               "common.hpp", "Makefile")


def csrc_digest() -> str:
    """sha256 (16 hex) of the sources and build flags the profiled kernels are compiled
    from (PMC_SOURCES): ties a committed PMC profile to the kernels that produced it."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(PMC_SOURCES):
        h.update(f.encode())
        h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()[:16]


def workload_key(args) -> tuple:
    """What a PMC profile's bytes depend on: the graph, the model and the pass mode."""
    return (args.users, args.items, args.edges, args.dim, args.zipf, args.aggregator,
            args.config, args.hetero, args.mode, args.segments)


def default_workload(args) -> bool:
    return workload_key(args) == (10_000_000, 1_000_000, 500_000_000, 128, 0.0, "mean", "c4",
                                  "sum", "deterministic", 8)


def pmc_traffic(args, world):
    """{bench tag: HBM bytes per launch} from the newest committed rocprofv3 PMC passes of
    THIS run's workload (profiles/<tag>_pmc_{fetch,write}.csv + <tag>_pmc_meta.json, whose
    bench_args give the same workload_key: C4 by default, C5 with --config c5, ...):
    FETCH_SIZE x2 (gfx950 counts half the bytes of wide reads) + WRITE_SIZE, KB -> B.  One
    GPU only, and only if the HIP sources hash to the `csrc_sha` the profile was taken
    with; otherwise ({}, reason)."""
    import csv
    import glob
    if world != 1:
        return {}, "not the profiled workload (profiles are single-GPU)"
    mine = workload_key(args)
    def key_of(m):  # a profile whose recorded flags no longer parse is skipped, not fatal
        try:
            return workload_key(parse(json.load(open(m)).get("bench_args", [])))
        except (Exception, SystemExit):
            return None
    metas = [m for m in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_meta.json")))
             if key_of(m) == mine]
    if not metas:
        return {}, "no PMC profile of this workload"
    cur = [m for m in metas if json.load(open(m)).get("csrc_sha") == csrc_digest()]
    if not cur:
        tag = os.path.basename(metas[-1])[: -len("_pmc_meta.json")]
        return {}, (f"stale: {tag} profiled csrc {json.load(open(metas[-1])).get('csrc_sha')}, "
                    f"now {csrc_digest()}")
    metas = cur  # newest profile of these very kernels
    meta = json.load(open(metas[-1]))
    tag = os.path.basename(metas[-1])[: -len("_pmc_meta.json")]
    out = {}
    for t, kernel in meta["kernels"].items():  # bench tag -> kernel-name substring
        tot, n = 0.0, 0
        for kind, scale in (("fetch", 2.0), ("write", 1.0)):
            path = os.path.join(ROOT, "profiles", f"{tag}_pmc_{kind}.csv")
            for r in csv.DictReader(open(path)):
                if kernel in r["Kernel_Name"]:
                    tot += float(r["Counter_Value"]) * 1024 * scale
                    n += kind == "fetch"
        if n:
            out[t] = tot / n
    return out, f"{tag} (csrc {meta['csrc_sha']})"


def bits_digest() -> str:
    """sha256 (16 hex) of every source the pass's output BITS depend on: the HIP/C++
    sources and build flags, the C header and the Python package (kernel choices).  Keys
    the committed one-GPU output digests (--p1-digests) a P > 1 run compares against."""
    import glob
    import hashlib
    h = hashlib.sha256()
    pats = (os.path.join(CSRC, "*.hip"), os.path.join(CSRC, "*.hpp"), os.path.join(CSRC, "*.cpp"),
            os.path.join(CSRC, "Makefile"), os.path.join(ROOT, "include", "*.h"),
            os.path.join(ROOT, "gnn-recsys_amd", "gnnrec", "*.py"))
    for f in sorted(p for pat in pats for p in glob.glob(pat)):
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def _signed64(x: int) -> int:
    return x - (1 << 64) if x >= 1 << 63 else x


def output_digest(args, shard, out, rank, world, dev):
    """{ntype: 32-hex digest} of the pass's whole output — every rank's owned user range and
    item block (gnnrec.dist.table_digest: global-index-weighted sums, additive over ranks),
    summed over the ranks mod 2^64, so the value is P-independent whenever the bits are.
    GNNREC_BENCH_PERTURB_RANK=r flips one bit of rank r's first user row first (the check
    that a wrong rank is caught)."""
    from gnnrec.dist import digest_add, table_digest
    S = shard.shard_rows["item"]
    lo, hi = rank * S, min((rank + 1) * S, args.items)
    u = out["user"]
    pert = os.environ.get("GNNREC_BENCH_PERTURB_RANK")
    if pert is not None and int(pert) == rank:
        u = u.clone()
        u.view(torch.int32).reshape(-1)[:1].bitwise_xor_(1)
    du = table_digest(u, shard.p_lo)
    di = table_digest(out["item"][: hi - lo], lo) if hi > lo else (0, 0)
    if world > 1:
        t = torch.tensor([_signed64(x) for x in du + di], dtype=torch.int64, device=dev)
        allr = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allr, t)
        parts = [[int(x) & ((1 << 64) - 1) for x in a.tolist()] for a in allr]
        du = digest_add(*[p[:2] for p in parts])
        di = digest_add(*[p[2:] for p in parts])
    return {"user": f"{du[0]:016x}{du[1]:016x}", "item": f"{di[0]:016x}{di[1]:016x}"}


def p1_digest_lookup(path, args):
    """The committed one-GPU digest of this workload on these sources, or (None, reason)."""
    try:
        entries = json.load(open(path)).get("entries", [])
    except OSError:
        return None, f"no digest file {os.path.relpath(path, ROOT)}"
    src, wl = bits_digest(), list(workload_key(args))
    same_wl = [e for e in entries if e.get("workload") == wl]
    if not same_wl:
        return None, "no one-GPU digest of this workload"
    for e in same_wl:
        if e.get("sources") == src:
            return e, f"one-GPU run of sources {src} ({e.get('recorded', '?')})"
    return None, (f"stale: one-GPU digests exist for sources "
                  f"{sorted({e.get('sources') for e in same_wl})}, now {src}")


def p1_digest_record(path, args, digest, ms_step):
    try:
        data = json.load(open(path))
    except OSError:
        data = {"about": "bench.py output digests at one GPU (--record-digest), keyed by "
                         "bits_digest() and workload_key(); a P > 1 run reports "
                         "bitwise_vs_p1 against them", "entries": []}
    src, wl = bits_digest(), list(workload_key(args))
    data["entries"] = [e for e in data["entries"]
                       if not (e.get("sources") == src and e.get("workload") == wl)]
    data["entries"].append({"sources": src, "workload": wl, "digest": digest,
                            "ms_per_step": ms_step,
                            "recorded": time.strftime("%Y-%m-%d %H:%M:%S")})
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    json.dump(data, open(path, "w"), indent=1)


class Heartbeat:
    """A stderr line every `period` s naming the phase the rank is in: a multi-GPU run that
    stalls (graph build, first collective, a kernel) says where, long before any timeout."""

    def __init__(self, rank, period=60.0):
        import threading
        self.rank, self.period, self.phase, self.t0 = rank, period, "start", time.time()
        self._stop = threading.Event()
        self._th = threading.Thread(target=self._loop, daemon=True, name="bench-heartbeat")
        self._th.start()

    def _loop(self):
        while not self._stop.wait(self.period):
            self.say(f"alive, in {self.phase}")

    def say(self, msg):  # one write per line: ranks sharing a stderr do not interleave
        sys.stderr.write(f"[bench r{self.rank} +{time.time() - self.t0:.0f}s] {msg}\n")
        sys.stderr.flush()

    def enter(self, phase):
        self.phase = phase
        self.say(phase)

    def stop(self):
        self._stop.set()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, d):
    """The same workload on the host cores, timed on a bounded row sample.

    Full-size inputs — the whole user and item tables (C4: 5.1 GB + 512 MB fp32) and the
    same generated edge stream — and the destination rows [0, f·N) of both relations (f =
    --cpu-sample): every sampled row gathers its full in-neighbourhood from the full table,
    so the cache behaviour is the workload's, not a small graph's.  Timed per pass: the
    NodeEmbedding of f of the nodes, then L=2 ConvLayers 'mean' over both sampled
    relations (hetero sum over one relation per type is the identity).
      kind 'port': the oracle (C/OpenMP restatement of DGL 0.5's CPU SpMM + numpy fp32
        GEMMs, reference src/model.py:143-148,226-235);
      'index_add_value': torch CPU, edge-chunked index_add_ + matmul (the second data point
        SURVEY §8d asks for).
    Rate = sampled edges aggregated / time."""
    import numpy as np

    sys.path.insert(0, ROOT)
    from oracle import oracle

    U, I, E, f = args.users, args.items, args.edges, args.cpu_sample
    Us, Is = max(1, int(U * f)), max(1, int(I * f))
    t_setup = time.perf_counter()
    # sampled CSRs: bought-by rows = users [0, Us) (sources: items), buys rows = items [0, Is)
    su, du, si, di = [], [], [], []
    chunk = 1 << 26
    for e0 in range(0, E, chunk):
        u, i = oracle.synth_edges(11, e0, min(chunk, E - e0), U, I)
        m = u < Us
        su.append(i[m]); du.append(u[m])
        m = i < Is
        si.append(u[m]); di.append(i[m])
    ce_u, ce_i = ("item", "bought-by", "user"), ("user", "buys", "item")
    csr = {ce_u: oracle.csr_from_coo_c(np.concatenate(su), np.concatenate(du), Us),
           ce_i: oracle.csr_from_coo_c(np.concatenate(si), np.concatenate(di), Is)}
    del su, du, si, di
    X = {"user": oracle.fill_f32(1, (U, d)), "item": oracle.fill_f32(2, (I, d))}
    torch.manual_seed(0)
    w = {}
    for rel in ("buys", "bought-by"):
        w[rel] = {}
        for name in ("fc_self.weight", "fc_neigh.weight"):
            t = torch.empty(d, d)
            torch.nn.init.xavier_uniform_(t, gain=torch.nn.init.calculate_gain("relu"))
            w[rel][name] = t.numpy()
    emb = {nt: (oracle.fill_f32(3, (d, d)) * 0.1, oracle.fill_f32(4, (d,))) for nt in X}
    t_setup = time.perf_counter() - t_setup

    class Sample:  # what oracle.conv_layer reads of a graph: the CSR of the relation
        occurrence = {}

        @staticmethod
        def csr(ce):
            return csr[ce]

    edges = sum(int(c[0][-1]) for c in csr.values()) * 2  # L=2 layers
    rows = {"user": Us, "item": Is}

    def port_pass():
        for nt in X:  # the NodeEmbedding share of the sampled rows
            oracle.linear(X[nt][: rows[nt]], *emb[nt])
        for _ in range(2):
            for ce in (ce_u, ce_i):
                oracle.conv_layer(Sample, ce, X[ce[0]], X[ce[2]][: rows[ce[2]]],
                                  w[ce[1]], "mean", True)

    tX = {nt: torch.from_numpy(x) for nt, x in X.items()}
    tcsr = {}
    for ce, (ip, ix, _) in csr.items():
        ipt = torch.from_numpy(ip)
        deg = ipt[1:] - ipt[:-1]
        tcsr[ce] = (torch.repeat_interleave(torch.arange(deg.numel()), deg),
                    torch.from_numpy(ix).long(), deg.clamp(min=1).float().unsqueeze(1))
    tw = {rel: {k: torch.from_numpy(v) for k, v in ww.items()} for rel, ww in w.items()}
    temb = {nt: (torch.from_numpy(a), torch.from_numpy(b)) for nt, (a, b) in emb.items()}

    def torch_pass():
        for nt in tX:
            torch.nn.functional.linear(tX[nt][: rows[nt]], *temb[nt])
        for _ in range(2):
            for ce in (ce_u, ce_i):
                dst, src, deg = tcsr[ce]
                agg = torch.zeros((rows[ce[2]], d))
                for k in range(0, src.numel(), 1 << 22):
                    agg.index_add_(0, dst[k:k + (1 << 22)], tX[ce[0]][src[k:k + (1 << 22)]])
                agg /= deg
                z = torch.relu(tX[ce[2]][: rows[ce[2]]] @ tw[ce[1]]["fc_self.weight"].t()
                               + agg @ tw[ce[1]]["fc_neigh.weight"].t())
                n = z.norm(dim=1, keepdim=True)
                z / torch.where(n == 0, torch.ones_like(n), n)

    def timed(fn, budget=8.0, warm=True):
        if warm:
            fn()  # page faults, thread pools
        reps, tot = 0, 0.0
        while reps < 1 or (tot < budget and reps < 5):
            t0 = time.perf_counter()
            fn()
            tot += time.perf_counter() - t0
            reps += 1
        return edges * reps / tot, reps, tot

    cores = oracle.num_threads()
    torch.set_num_threads(cores)
    port, reps, tot = timed(port_pass)
    alt, _, _ = timed(torch_pass, budget=4.0, warm=False)
    wl = "C4" if default_workload(args) else "custom"
    if args.config == "c5" and (U, I, E) == (10_000_000, 1_000_000, 500_000_000):
        # the sample is the single-relation (C4) form on C5's tables and edge count: the
        # same edges, without C5's 80/20 relation split and second projection per type
        wl = "C5 sizes in the C4 form (one relation per node type)"
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"value": port, "unit": "edges/s", "cores": cores, "kind": "port",
            "cores_affinity": aff, "cores_machine": os.cpu_count(),
            "cores_note": (f"{cores} of the machine's {os.cpu_count()} logical CPUs: {cores} "
                           f"OpenMP threads = the job's CPU lease (OMP_NUM_THREADS="
                           f"{os.environ.get('OMP_NUM_THREADS', 'unset')}; the process may run "
                           f"on {aff} CPUs), not the whole host SURVEY 8(d) d5 names"),
            "cpu_model": cpu_model(), "index_add_value": alt, "config": wl,
            "sample": f"{wl} full-size tables ({U}x{d} + {I}x{d} fp32) and edge stream; dst rows "
                      f"[0,{f:g}N) of both relations = {edges // 2} edges/layer; 2 layers, "
                      f"{reps} passes, {tot:.1f} s (setup {t_setup:.0f} s)"}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def resolve_world(args, env=None):
    """(world size, None) for this process, or (None, N) when this process must start N
    ranks itself.  Decided before anything touches the GPU:
      WORLD_SIZE unset, --gpus N > 1  -> spawn N ranks (the driver or a user ran
                                         `python bench.py --gpus N` without torchrun);
      WORLD_SIZE set                  -> it must equal --gpus when --gpus is given: a
                                         mismatch would print a line whose n_gpus is not
                                         the GPU count asked for, so it is an error."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            raise SystemExit(f"bench.py: --gpus {n}: need at least one GPU")
        return (1, None) if n == 1 else (None, n)
    ws = int(ws)
    if args.gpus is not None and args.gpus != ws:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}: the launcher "
                         f"started {ws} rank(s); refusing to report a {ws}-GPU line as "
                         f"{args.gpus} GPUs")
    return ws, None


def spawn_ranks(n: int, argv) -> int:
    """Start n rank processes of this script with torch.distributed.run (one per GPU, RCCL
    rendezvous on 127.0.0.1) as a CHILD process and return its exit status (non-zero if any
    rank failed).  The ranks inherit stdout, so rank 0's JSON line is this run's output.
    Nothing here initialises the GPU (device_count does not, on this image), so the parent
    never holds a device while its children run."""
    import subprocess
    backend = os.environ.get("GNNREC_DIST_BACKEND", "nccl")
    have = torch.cuda.device_count()
    if backend == "nccl" and have < n:
        sys.stderr.write(f"bench.py: --gpus {n} needs {n} visible GPUs for RCCL, found {have}\n")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    sys.stderr.write(f"[bench] starting {n} ranks: {' '.join(cmd)}\n")
    sys.stderr.flush()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    world, spawn = resolve_world(args)
    if spawn is not None:
        sys.exit(spawn_ranks(spawn, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev_idx = local_rank % max(1, torch.cuda.device_count())  # rehearsals may share one GPU
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    hb = Heartbeat(rank)
    if world > 1:
        # RCCL over xGMI; GNNREC_DIST_BACKEND=gloo rehearses several ranks on one GPU.  An
        # explicit timeout: a collective that never completes ends the run with the
        # watchdog's report (op type, sequence number) instead of a silent hang
        import datetime
        backend = os.environ.get("GNNREC_DIST_BACKEND", "nccl")
        hb.enter(f"init_process_group({backend}, timeout {args.pg_timeout:g} s)")
        tmo = datetime.timedelta(seconds=args.pg_timeout)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)

    from gnnrec import nn as gnn
    from gnnrec.dist import AsyncEmulatedExchange, Exchange, ProgressExchange
    from gnnrec.inference import ShardedFullGraphPass
    from gnnrec.synth import GraphMeta, bipartite_shard, node_features

    d = args.dim
    split = ((("clicks", "clicked-by", 0.8), ("buys", "bought-by", 0.2)) if args.config == "c5"
             else (("buys", "bought-by", 1.0),))
    segments = args.segments or None
    det = args.mode == "deterministic"
    if det and (segments is None or segments % world or segments & (segments - 1)):
        det = False  # the fixed tree needs a power-of-two segment count divisible by P
    if segments is not None and segments < world:
        segments = None
    hb.enter("graph build (edge stream, CSRs, source tiles)")
    shard = bipartite_shard(args.users, args.items, args.edges, rank, world, dev,
                            zipf_s=args.zipf, split=split, segments=segments)
    feats = {"user": node_features(args.users, d, 0, dev, slice(shard.p_lo, shard.p_hi)),
             "item": torch.zeros((shard.padded_rows("item"), d), device=dev)}
    feats["item"][: args.items] = node_features(args.items, d, 1, dev)
    torch.manual_seed(0)
    meta = GraphMeta(shard.canonical_etypes, ["item", "user"])
    model = gnn.ConvModel(meta, 3, {"user": d, "item": d, "hidden": d, "out": d}, True, 0.0,
                          args.aggregator, "cos", args.hetero, True).to(dev).eval()
    # RCCL when the group is nccl; a gloo rehearsal (GNNREC_DIST_BACKEND=gloo) exchanges
    # through the async emulation, so the pass waits on real work handles as under RCCL
    ex = Exchange()
    if world > 1 and not ex._rccl:
        ex = AsyncEmulatedExchange(delay_us=0)
    conc = None
    if args.concurrency != "auto":
        r, q = args.concurrency.split(",")
        conc = (int(r), bool(int(q)))
    runner = ShardedFullGraphPass(model, shard, ex, overlap=not args.no_overlap,
                                  deterministic=det, concurrency=conc)
    pex = None
    if world > 1:  # one stderr line per layer and collective; the first pass checks each
        pex = ProgressExchange(ex, runner)
        runner.ex, runner.progress = pex, pex.layer_start
    timers = EventTimers()
    runner.timers = timers
    torch.cuda.synchronize()
    # the graph build's temporaries (edge streams, CSR sort workspaces: ~20 B per edge) sit in
    # the caching allocator; hand them back so the pass's own tables never meet a full pool
    # (an allocation that finds none frees the whole cache under a device sync: 2 s stalls)
    torch.cuda.empty_cache()
    if os.environ.get("GNNREC_BENCH_MEMINFO"):
        print(f"[bench] allocated {torch.cuda.memory_allocated() / 2**30:.1f} GiB, reserved "
              f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB", file=sys.stderr, flush=True)

    for w in range(args.warmup):
        hb.enter(f"warm-up pass {w}" + (" (every collective waited on)" if pex and w == 0 else ""))
        if pex is not None:
            pex.pass_no, pex.checked = -args.warmup + w, w == 0
        t0 = time.perf_counter()
        out = runner.run(feats, replicate_output=False)
        torch.cuda.synchronize()
        hb.say(f"warm-up pass {w} done in {(time.perf_counter() - t0) * 1e3:.1f} ms")
    if pex is not None:
        # the warm-up passes named every collective; the timed passes run the bare exchange
        # (no per-collective stderr writes inside the measurement) and only the heartbeat
        # says where a stalled rank is
        runner.ex, runner.progress = ex, None
    ag_choice = None
    if world > 1:
        hb.enter("all-gather form")
        ag_choice = choose_allgather(args, runner, ex, feats, dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    hb.enter(f"timed region ({args.steps} passes)")
    timers.enabled = True
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        out = runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    hb.enter(f"timed region done: {elapsed / args.steps * 1e3:.2f} ms per pass on this rank")
    if os.environ.get("GNNREC_BENCH_MEMINFO"):
        print(f"[bench] after the timed passes: allocated "
              f"{torch.cuda.memory_allocated() / 2**30:.1f} GiB, reserved "
              f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB, peak "
              f"{torch.cuda.max_memory_reserved() / 2**30:.1f} GiB, alloc retries "
              f"{torch.cuda.memory_stats().get('num_alloc_retries', 0)}", file=sys.stderr,
              flush=True)
    elapsed = ex.max_scalar(elapsed, dev)
    hb.enter("output digest")
    digest = output_digest(args, shard, out, rank, world, dev)
    del out
    bitwise, digest_src = None, None
    if world > 1:
        if det:
            ref, digest_src = p1_digest_lookup(args.p1_digests, args)
            if ref is not None:
                bitwise = ref["digest"] == digest
        else:
            digest_src = "fast mode: item sums depend on P (not bitwise P-independent)"
    if args.record_digest and world == 1 and rank == 0:
        p1_digest_record(args.record_digest, args, digest, elapsed / args.steps * 1e3)

    edges_per_step = 2 * sum(rs.global_edges for rs in shard.rels.values())  # L=2 layers
    value = edges_per_step * args.steps / elapsed
    ms_step = elapsed / args.steps * 1e3

    # roofline of the aggregation (SURVEY §8d d4 algorithmic bytes ÷ HIP-event time of the
    # launches, timed live on the stream they run on).  Headline: every aggregation launch
    # of a pass COMBINED — their bytes per pass ÷ their summed time per pass — so it cannot
    # flip between two kernels of near-equal share (C4: the user->item source tiles and the
    # fused item->user launch, ~half the pass each); every kernel rides along as flat
    # `<field>_<tag>` keys, and `pass_frac` prices the whole step: aggregation bytes per
    # step ÷ ms_per_step ÷ peak
    per_tag = launch_bytes(shard, d, runner, det)
    stats = {}
    for t in per_tag:
        ms, n = timers.mean_ms(t)
        if n:
            b = per_tag[t][0] / per_tag[t][1]  # bytes per layer / launches per layer
            stats[t] = {"launch_ms": ms, "launches_timed": n, "bytes_per_launch": b,
                        "achieved": b / (ms * 1e-3) / 1e9, "ms_per_pass": ms * n / args.steps,
                        "launches_per_pass": n / args.steps}
    traffic, traffic_src = pmc_traffic(args, world)
    roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None, "traffic": None}
    if stats:
        order = sorted(stats, key=lambda t: -stats[t]["ms_per_pass"])
        bytes_pass = sum(st["bytes_per_launch"] * st["launches_per_pass"] for st in stats.values())
        ms_pass = sum(st["ms_per_pass"] for st in stats.values())
        ach = bytes_pass / (ms_pass * 1e-3) / 1e9
        tr = None
        if traffic and all(t in traffic for t in stats):
            tr = sum(traffic[t] * stats[t]["launches_per_pass"] for t in stats)
        roof.update(achieved=ach, frac=ach / HBM_PEAK_GBS, traffic=tr,
                    kernel="every aggregation launch of one pass: " + " + ".join(
                        f"{stats[t]['launches_per_pass']:g} x {KERNELS[t][0]}" for t in order),
                    unit_of_work="one pass (achieved and traffic: bytes per pass)",
                    bytes_per_pass=bytes_pass, kernel_ms_per_pass=ms_pass,
                    share_of_step=ms_pass / ms_step,
                    pass_frac=bytes_pass / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    dominant=order[0], traffic_src=traffic_src)
        for t in order:
            o = stats[t]
            roof.update({f"frac_{t}": o["achieved"] / HBM_PEAK_GBS, f"achieved_{t}": o["achieved"],
                         f"launch_ms_{t}": o["launch_ms"], f"launches_{t}": o["launches_timed"],
                         f"bytes_per_launch_{t}": o["bytes_per_launch"],
                         f"share_of_step_{t}": o["ms_per_pass"] / ms_step,
                         f"traffic_{t}": traffic.get(t)})

    diag = None
    if world > 1:
        hb.enter("multi-GPU diagnostics (collective replay, per-rank compute)")
        diag = multi_gpu_diagnostics(args, runner, ex, feats, model, shard, det, conc, dev,
                                     ms_step)

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        hb.enter("CPU baseline")
        try:
            cpu = cpu_baseline(args, d)
        except Exception as exc:  # the baseline never masks the GPU result
            cpu = {"value": None, "unit": "edges/s", "cores": None, "kind": "port",
                   "sample": f"failed: {exc!r}"}

    mb = None
    if world == 1 and args.minibatch == "auto":
        hb.enter("minibatch (C2 training step)")
        try:
            mb = minibatch_step(dev)
        except Exception as exc:  # a secondary measurement never masks the metric
            mb = {"error": repr(exc)}

    if rank == 0:
        wl = (args.config.upper() if (args.users, args.items, args.edges) ==
              (10_000_000, 1_000_000, 500_000_000) else "custom")
        cfg = {"workload": f"{wl}: {args.users / 1e6:g}M users x {args.items / 1e6:g}M items, "
                           f"{args.edges / 1e6:g}M edges/dir, embed + 2 SAGE '{args.aggregator}'"
                           f", hetero {args.hetero}, d={d}"
                           + (" (80/20 clicks/buys)" if args.config == "c5" else "")
                           + (f", zipf {args.zipf}" if args.zipf else ""),
               "edges_per_step": edges_per_step, "parallelism": f"graph{world}",
               "mode": ("deterministic (bitwise equal at 1/2/4/8 GPUs)" if det else "fast"),
               "source_tiles": shard.segments or 0, "partition": shard.balance,
               "output": "partitioned (each rank keeps the user and item rows it owns)",
               "overlap": not args.no_overlap,
               "row_schedule": ("static" if not runner.concurrency or
                                not runner.concurrency[1] else "queue")
                               + (f", {runner.concurrency[0]} CUs reserved"
                                  if runner.concurrency and runner.concurrency[0] else "")}
        cfg["output_digest"] = digest  # P-independent in deterministic mode
        cfg["bits_sources"] = bits_digest()
        if world > 1:
            cfg["bitwise_vs_p1"] = bitwise
            cfg["bitwise_vs_p1_src"] = digest_src
        if ag_choice is not None:
            cfg["all_gather_choice"] = ag_choice
        if diag is not None:
            cfg.update(diag)
        rec = {
            "metric": "edges aggregated/sec, full-graph embed pass, d=128",
            "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic (counter-hash graph seed 11, N(0,1) features, xavier weights)",
            "config": cfg, "roofline": roof, "cpu_baseline": cpu,
        }
        if mb is not None:
            rec["minibatch"] = mb
        print(json.dumps(rec), flush=True)
    hb.stop()
    if world > 1:
        dist.destroy_process_group()


def minibatch_step(dev, warmup: int = 5):
    """A secondary record beside the metric: BASELINE configs[1]'s (C2) training step —
    1M users x 100k items x 50M edges per direction, 2 SAGE layers 'mean' d=64 + NodeEmbedding,
    fanout [10,10], 1024 positive edges x K uniform negatives, cosine head, max-margin loss,
    Adam — timed over 100 (K = 10) / 40 (the reference's K = 2500) steps — sampling,
    forward, backward, optimizer — with the loader's sampling thread (num_workers=2) and
    without (20 steps varied by ±25 % from run to run on one box, 200 by ±7 %)."""
    from gnnrec import nn as gnn
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    from gnnrec.synth import minibatch_graph

    buys = ("user", "buys", "item")
    g = minibatch_graph(64, dev)
    try:  # the §8d rooflines of the minibatch kernels (sampler, cosine, edge MLP)
        roof = minibatch_rooflines(dev, g=g)
    except Exception as exc:  # a secondary measurement never masks the step times
        roof = {"error": repr(exc)}
    out = {"workload": "C2: 1M users x 100k items, 50M edges/dir, 2 SAGE 'mean' d=64, fanout "
                       "[10,10], 1024 pos x K neg, cosine head, Adam (torch fused=True; fp32, synthetic)",
           "rooflines": roof}
    # the three flat keys of the §8d d3/d4 rooflines
    out["sampler_GBs"] = roof.get("sampler", {}).get("GBs")
    out["cosine_frac"] = roof.get("cosine", {}).get("frac")
    out["edge_mlp_mfma_frac"] = roof.get("edge_mlp", {}).get("mfma_frac")
    for K, steps in ((10, 100), (2500, 40)):
        caps = "auto" if K > 100 else "provable"
        # the eager and captured runs consume the SAME batches (same seeds, same warm-up
        # count: the captured loader's learned-capacity batches and the step's own warm-up),
        # so their per-step losses compare step for step
        W = _captured_warmup(warmup, caps)
        eager_losses = None
        for nw in (2, 0):
            torch.manual_seed(0)
            model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True,
                                  0.0, "mean", "cos", "sum", True).to(dev)
            # torch's single-launch Adam (the same update as the reference's default
            # multi-tensor one; C2 K=10 step -0.1..0.3 ms, profiles/r03e_adam_ab.txt);
            # GNNREC_BENCH_ADAM_FUSED=0 keeps the default implementation
            opt = torch.optim.Adam(model.parameters(), lr=0.005,
                                   fused=os.environ.get('GNNREC_BENCH_ADAM_FUSED') != '0')
            el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                                MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                                reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                                negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                                shuffle=True, num_workers=nw)
            it = iter(el)

            def step():
                _, pos_g, neg_g, blocks = next(it)
                _, ps, ns = model(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
                loss = gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])
                opt.zero_grad()
                loss.backward()
                opt.step()
                return loss

            l1 = step().detach()  # batch 1: both runs from the same initial weights
            for _ in range(W - 1):
                step()
            torch.cuda.synchronize()
            losses = []
            t0 = time.perf_counter()
            for _ in range(steps):
                losses.append(step().detach())  # device scalars: no sync in the loop
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            losses = torch.stack([l1] + losses).double().cpu()
            out[f"K{K}_num_workers{nw}"] = {"ms_per_step": round(ms, 3), "steps": steps,
                                            "warmup_batches": W,
                                            "pos_edges_per_s": round(1024 / ms * 1e3),
                                            "loss": float(losses[-1]),
                                            "loss_first": float(losses[1]),
                                            "loss_batch1": float(losses[0])}
            if eager_losses is None:
                eager_losses = losses
            del it, el
        try:
            # K = 2500: the provable capacities pad the first block's 7.3M sampled edges to
            # 11M (every user a potential source); capacities learned from the first batches
            # (static_caps='auto') hold them within 10 % and replay 3.8 -> 3.5 ms per step
            cap = captured_step(g, dev, K, steps, warmup, caps=caps)
            cl = cap.pop("_losses", None)
            if cl is not None and eager_losses is not None:
                el_ = eager_losses[[0, 1, -1]]
                rel = (cl - el_).abs() / el_.abs().clamp_min(1e-30)
                # the same batches, step for step: fp32 rounding apart (the captured step
                # folds the NodeEmbedding and sums over padding rows), which training carries
                # forward — batch 1 (same initial weights) is the tight comparison; at K = 10
                # the eager run does not fold (below FOLD_MIN_SRC_ROWS), so its trajectory
                # drifts from the captured one by Adam-amplified rounding
                cap["loss_rel_diff_vs_eager"] = {"batch1": float(rel[0]), "first": float(rel[1]),
                                                 "last": float(rel[2])}
            out[f"K{K}_num_workers2_captured"] = cap
        except Exception as exc:  # a secondary measurement never masks the others
            out[f"K{K}_num_workers2_captured"] = {"error": repr(exc)}
    return out


def _captured_warmup(warmup: int, caps: str) -> int:
    """Batches a captured run consumes before its timed steps: the step's warm-up and
    capture (at least 3) plus, with learned capacities, the loader's exact learning batches."""
    from gnnrec.sampling import EdgeDataLoader
    return max(warmup, 3) + (EdgeDataLoader.STATIC_LEARN if caps == "auto" else 0)


def captured_step(g, dev, K: int, steps: int, warmup: int, caps: str = "provable"):
    """The same C2 step over EdgeDataLoader(static_shapes=True) batches, recorded once into a
    hipGraph and replayed per batch (gnnrec.capture.CapturedTrainStep): the sampling thread
    builds fixed-shape batches on its own stream, the training thread copies each into the
    captured batch's buffers and launches the graph.  gpu_ms_per_replay: HIP events around
    replays of one batch alone (the replayed step's kernels without the loader's).
    caps: the loader's static_caps ('provable' or 'auto', learned from its first batches)."""
    from gnnrec import nn as gnn
    from gnnrec.capture import CapturedTrainStep
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler

    buys = ("user", "buys", "item")
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=0.005, fused=True)

    def loss_fn(m, batch):
        _, pos_g, neg_g, blocks = batch
        _, ps, ns = m(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        return gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])

    # the host cost of the first-layer fold is gone under capture: fold every first block
    # (no embedding of its source rows, no transposes of it to build in the loader)
    model.train_fold = "1"
    step = CapturedTrainStep(model, opt, loss_fn, warmup=2)
    el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, num_workers=2, static_shapes=True, static_caps=caps)
    el.sampler.first_transposes_below = 0  # what the fold sets: settled before the first batch
    it = iter(el)
    # learned capacities: the first STATIC_LEARN batches come out exact (eager steps), then
    # the step's own warm-up and capture — all before the timed steps
    W = _captured_warmup(warmup, caps)
    l1 = step(next(it)).clone()  # batch 1: from the same initial weights as the eager run
    for _ in range(W - 1):
        loss = step(next(it))
    torch.cuda.synchronize()
    first = None
    t0 = time.perf_counter()
    for k in range(steps):
        loss = step(next(it))
        if k == 0:  # the next replay overwrites the captured loss: keep the first one
            first = loss.clone()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    losses = torch.stack([l1, first, loss.detach()]).double().cpu()
    res = {"ms_per_step": round(ms, 3), "steps": steps, "warmup_batches": W,
           "pos_edges_per_s": round(1024 / ms * 1e3), "loss": float(losses[-1]),
           "loss_first": float(losses[1]), "loss_batch1": float(losses[0]),
           "replays": step.replays, "eager_steps": step.eager_steps,
           "captures": step.captures, "fold": model.train_fold, "static_caps": caps,
           "redone": el.static_redone, "_losses": losses}
    del it, el
    from gnnrec import ops
    res["plan_overflows"] = ops.plan_overflows()  # heavy-row plans past their capacities
    if step.graph is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            step.graph.replay()
        e1.record()
        e1.synchronize()
        # the replayed step's own kernels (the loader's, on the sampling thread's stream,
        # are not in it); the GPU's occupancy of the loop is a kernel-trace measurement
        # (union of kernel intervals, tools/rocpd_timeline.py), not a ratio of these events
        res["gpu_ms_per_replay"] = round(e0.elapsed_time(e1) / 20, 3)
    return res


MFMA_F32_PEAK_TFS = 157.3  # MI355X dense fp32 MFMA, /opt/skills/guides/MI355X_MICROARCH.md
# random-row gathers served by the 256 MB Infinity Cache: 8.6 TB/s chip-wide from a 38 MB table
# (MI355X_MICROARCH.md §Indexed rows: gather into LDS; register gathers read at the same rate)
IC_GATHER_GBS = 8600.0
IC_BYTES = 256 * 2**20


def minibatch_rooflines(dev, reps: int = 50, g=None):
    """SURVEY §8d d3/d4 for the minibatch kernels, at BASELINE configs[1]/[2]'s shapes:
      sampler  (a9 + a10) C2 graph, fanout [10,10], 1024 user + 1024 item seeds: sampled
               edges/s and GB/s of the a9 byte model — per sampled edge 4 B index read +
               4 B write + 8 B relabel mark/scan, per seed 16 B indptr — plus the a10 gathers
               (the block's edge data and input features: read + write); wall time per call
               (the sampler reads sizes back to the host once per layer)
      cosine   (a7) C3 pair graph, 1024 pos x 2500 neg edges, d = 128, the compacted tables
               (1024 user rows, 100k item rows): 1036 B/edge; HIP-event time of the kernel
      edge_mlp (a8) same pair graph through PredictingModule's tail kernel, grouped as the
               cosine (relu(P[u]+Q[v]) -> 128x32 MFMA -> relu . w3 -> sigmoid): executed MFMA
               flops 2*128*32 per edge over the kernel's time against the 157.3 TF fp32 MFMA
               peak, and its gather bytes (512 + 12 B/edge, 528 B/group) against the Infinity
               Cache's gather rate; the per-node P/Q GEMMs beside.
    Kernel times are HIP events on the stream the ops launch on (torch's current stream)."""
    from gnnrec import ops
    from gnnrec.nn import PredictingLayer
    from gnnrec.sampling import MultiLayerNeighborSampler
    from gnnrec.synth import minibatch_graph

    out = {}
    if g is None:
        g = minibatch_graph(64, dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1)
    sampler = MultiLayerNeighborSampler([10, 10])

    def seeds():
        return {"user": torch.randint(0, g.num_nodes("user"), (1024,), device=dev, generator=gen),
                "item": torch.randint(0, g.num_nodes("item"), (1024,), device=dev, generator=gen)}

    for _ in range(20):  # (after the graph build's idle GPU the first calls run slow)
        blocks = sampler.sample_blocks(g, seeds())
    torch.cuda.synchronize()
    t_tot, e_tot, b_tot, span = 0.0, 0, 0, 0.0
    for _ in range(reps):
        sd = seeds()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        blocks = sampler.sample_blocks(g, sd)
        ev1.record()
        torch.cuda.synchronize()
        t_tot += time.perf_counter() - t0
        span += ev0.elapsed_time(ev1)
        for b in blocks:
            for ce in b.canonical_etypes:
                ne = b.num_edges(ce)
                nd = b.number_of_dst_nodes(ce[2])
                e_tot += ne
                b_tot += 16 * ne + 16 * nd  # a9 model
                b_tot += 2 * ne * sum(v.element_size() for k, v in b._edata[ce].items())  # a10
        b0 = blocks[0]
        for nt in b0.ntypes:
            for k, v in b0._src[nt].items():
                if k != "_ID":
                    b_tot += 2 * v.numel() * v.element_size()  # a10 feature gather
    ms = t_tot / reps * 1e3
    fused = sampler._fused_ok(g)
    out["sampler"] = {"ms_per_call": round(ms, 4), "sampled_edges_per_call": e_tot // reps,
                      "gpu_span_ms_per_call": round(span / reps, 4),
                      "sampled_edges_per_s": e_tot / t_tot, "bytes_per_call": b_tot // reps,
                      "GBs": b_tot / t_tot / 1e9, "frac": b_tot / t_tot / 1e9 / HBM_PEAK_GBS,
                      "shape": "C2 graph, fanout [10,10], 1024 user + 1024 item seeds, 2 blocks",
                      "path": ("fused: gnnrec_sample_blocks (begin + pick/scan/finalize per "
                               "block) + one gnnrec_gather_rows_batch, one host size read per "
                               "call") if fused else "per-layer sample_layer",
                      "launches_per_call": (1 + 3 * 2 + 1) if fused else None,
                      "timing": "ms_per_call: wall per sample_blocks call, host included; "
                                "gpu_span: HIP events around the call on its stream"}

    # ---- heads on the C3 pair graph: 1024 positive + 1024 x 2500 negative edges ----------
    d, n_u, n_i, K = 128, 1024, 100_000, 2500
    Hs = torch.randn(n_u, d, device=dev, generator=gen)
    Hd = torch.randn(n_i, d, device=dev, generator=gen)
    src = torch.cat([torch.arange(n_u, device=dev),
                     torch.arange(n_u, device=dev).repeat_interleave(K)])
    dst = torch.randint(0, n_i, (src.numel(),), device=dev, generator=gen)
    E = src.numel()

    def ev_time(fn, n=reps):
        for _ in range(n):  # (the first ~50 launches after other work run up to 10 % slow)
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / n

    # the head as CosinePrediction.pair runs it on the loader's pair graphs: group g = one
    # positive edge (g, pd[g]) and its K negatives (g, nd[g K + j]) — the grouped launch
    ps, pd, nd = src[:n_u], dst[:n_u], dst[n_u:]
    ms = ev_time(lambda: ops.sddmm_cos_grouped(ps, pd, K, nd, Hs, Hd))
    ms_edge = ev_time(lambda: ops.sddmm_cos(src, dst, Hs, Hd))
    # bytes the grouped launch must move: per edge one gathered row + its dst id + the score,
    # per group the source row and its two ids; the gathered table (100k x 128 fp32 = 51 MB)
    # sits in the 256 MB Infinity Cache, so the roof is the cache's random-row gather rate
    b_alg = E * (d * 4 + 8 + 4) + n_u * (d * 4 + 8)
    tbl = n_i * d * 4
    roof = IC_GATHER_GBS if tbl <= IC_BYTES else HBM_PEAK_GBS
    out["cosine"] = {"ms": round(ms, 4), "edges": E, "bytes_per_launch": b_alg,
                     "achieved_GBs": b_alg / ms / 1e6, "peak_GBs": roof,
                     "frac": b_alg / ms / 1e6 / roof,
                     "bound": "infinity-cache gather" if tbl <= IC_BYTES else "hbm",
                     "table_bytes": tbl, "kernel": "sddmm_cos_grouped_kernel",
                     "per_edge_kernel_ms": round(ms_edge, 4),
                     "note": "negatives grouped by their source (negative_sampler.Uniform "
                             "repeats each positive's source K times): one 512-B row + 12 B "
                             "per edge; roof = the Infinity Cache's random-row gather rate "
                             "(MI355X_MICROARCH.md §Indexed rows, 38 MB table) for a "
                             "cache-resident table, else 8 TB/s; per_edge_kernel_ms = "
                             "sddmm_cos_kernel on the expanded lists (two rows per edge)"}

    torch.manual_seed(0)
    pl = PredictingLayer(d).to(dev).eval()
    W1 = pl.hidden_1.weight.detach()
    with torch.no_grad():
        P = ops.gemm(Hs, W1[:, :d], bias=pl.hidden_1.bias)
        Q = ops.gemm(Hd, W1[:, d:])
    w2, b2 = pl.hidden_2.weight.detach(), pl.hidden_2.bias.detach()
    w3, b3 = pl.output.weight.detach().reshape(-1), pl.output.bias.detach()
    # the head as PredictingModule runs it on the loader's pair graphs: the grouped launch
    # (group g = positive (g, pd[g]) + its K negatives, the source's P row read once per 256
    # edges); the per-edge launch over the expanded lists beside it
    ms = ev_time(lambda: ops.edge_mlp_grouped(ps, pd, K, nd, P, Q, w2, b2, w3, b3))
    ms_edge = ev_time(lambda: ops.edge_mlp(src, dst, P, Q, w2, b2, w3, b3))
    ms_pq = ev_time(lambda: (ops.gemm(Hs, W1[:, :d], bias=pl.hidden_1.bias),
                             ops.gemm(Hd, W1[:, d:])))
    fl = E * (2 * 128 * 32)
    # bytes the launch must move: per edge the gathered Q[v] row (512 B from the 51 MB item
    # table: Infinity-Cache resident), its id and the score; per group the P[u] row and two
    # ids — priced, like the cosine head, against the Infinity Cache's random-row rate
    b_alg = E * (128 * 4 + 8 + 4) + n_u * (128 * 4 + 16)
    ref_fl = 2 * E * (2 * d * 128 + 128 * 32 + 32)
    q_tbl = n_i * 128 * 4
    roof_mlp = IC_GATHER_GBS if q_tbl <= IC_BYTES else HBM_PEAK_GBS
    out["edge_mlp"] = {"ms": round(ms, 4), "edges": E, "mfma_flops": fl,
                       "TFs": fl / ms / 1e9, "mfma_frac": fl / ms / 1e9 / MFMA_F32_PEAK_TFS,
                       "bytes_per_launch": b_alg, "achieved_GBs": b_alg / ms / 1e6,
                       "peak_GBs": roof_mlp, "gather_frac": b_alg / ms / 1e6 / roof_mlp,
                       "bound_gather": "infinity-cache gather" if q_tbl <= IC_BYTES else "hbm",
                       "pq_gemms_ms": round(ms_pq, 4),
                       "head_ms": round(ms + ms_pq, 4),
                       "per_edge_kernel_ms": round(ms_edge, 4),
                       "reference_flops": ref_fl,
                       "reference_equivalent_TFs": ref_fl / (ms + ms_pq) / 1e9,
                       "kernel": "edge_mlp_lds_kernel<true> (grouped)",
                       "note": "W1[hu||hv] re-associated into per-node P, Q (two GEMMs): the "
                               "edge kernel runs only the 128x32 layer on the MFMA, over "
                               "LDS-staged tiles of 32 edges (coalesced row loads); "
                               "per_edge_kernel_ms = the same body on the expanded lists; "
                               "reference_equivalent_TFs prices the reference's per-edge "
                               "flops over the whole head"}
    return out


def choose_allgather(args, runner, ex, feats, dev):
    """P > 1: the form of the pass's item all-gathers (Exchange.ag_mode).  'auto' records
    one pass's collectives, replays its all-gathers alone in both forms — RCCL's ring
    all-gather and the all-to-all of the own block that writes every peer over its own
    xGMI link — takes the faster by the max over ranks (every rank must choose the same),
    and runs one more pass in it before the timed region.  Both forms deliver the same
    table, so the output bits do not depend on the choice."""
    from gnnrec.dist import RecordingExchange
    if args.allgather != "auto" or os.environ.get("GNNREC_ALLGATHER"):
        mode = os.environ.get("GNNREC_ALLGATHER") or args.allgather
        ex.ag_mode = mode
        return {"mode": mode, "how": "fixed (--allgather / GNNREC_ALLGATHER)"}
    rec = RecordingExchange(ex)
    runner.ex = rec
    runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    runner.ex = ex
    ags = [c for c in rec.calls if c[0] == "all_gather"]
    if not ags:
        return {"mode": ex.ag_mode, "how": "no all-gather in the timed pass"}
    sub = RecordingExchange(ex)
    sub.calls = ags
    ms = {m: ex.max_scalar(v, dev) for m, v in sub.replay_ms_by_allgather(dev).items()}
    mode = min(ms, key=ms.get)
    ex.ag_mode = mode
    runner.run(feats, replicate_output=False)  # one pass in the chosen form
    torch.cuda.synchronize()
    return {"mode": mode, "how": "auto: the pass's all-gathers replayed alone in both forms, "
                                 "max over ranks, faster kept",
            "replay_ms": {m: round(v, 3) for m, v in ms.items()}, "calls_per_pass": len(ags)}


def multi_gpu_diagnostics(args, runner, ex, feats, model, shard, det, conc, dev, ms_step):
    """Self-diagnosis of a P > 1 run (every rank takes part; rank 0 reports):
      rank_compute_ms  each rank's share of the pass with the same kernels and concurrency
                       but an exchange that moves nothing (gnnrec.dist.ComputeOnlyExchange);
      comm_ms          one pass's collectives issued alone, back to back (RecordingExchange
                       replay), and comm_bytes_per_rank the bytes each rank sends;
      overlap_frac     the share of comm_ms hidden under compute:
                       (max rank_compute + comm − step) / comm, clamped to [0, 1]."""
    from gnnrec.dist import ComputeOnlyExchange, RecordingExchange
    from gnnrec.inference import ShardedFullGraphPass

    world = ex.ws
    rec = RecordingExchange(ex)
    runner.ex = rec
    runner.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    runner.ex = ex
    comm_ms = rec.replay_ms(dev)
    comm_both = rec.replay_ms_by_allgather(dev)
    per_kind = rec.replay_by_kind(dev)
    null = ShardedFullGraphPass(model, shard, ComputeOnlyExchange(world, ex.rk),
                                overlap=not args.no_overlap, deterministic=det, concurrency=conc)
    reps = max(2, min(args.steps, 5))
    null.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        null.run(feats, replicate_output=False)
    torch.cuda.synchronize()
    mine = (time.perf_counter() - t0) / reps * 1e3
    # the same pass with the last layer's item all-gather (every rank ends with the whole
    # item table, as the reference's single-device `y`): what replicate_output costs
    runner.run(feats, replicate_output=True)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(2):
        runner.run(feats, replicate_output=True)
    torch.cuda.synchronize()
    dist.barrier()
    rep_ms = ex.max_scalar((time.perf_counter() - t0) / 2 * 1e3, dev)
    t = torch.tensor([mine, float(shard.local_edge_count())], dtype=torch.float64, device=dev)
    allr = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(allr, t)
    compute = [float(a[0]) for a in allr]
    edges = [int(a[1]) for a in allr]
    overlap = None
    if comm_ms > 0:
        overlap = max(0.0, min(1.0, (max(compute) + comm_ms - ms_step) / comm_ms))
    return {"backend": str(ex.backend), "collective_path": rec.path, "ranks_seen": world,
            "all_gather_mode": getattr(ex, "ag_mode", None),
            "rank_compute_ms": [round(c, 2) for c in compute], "rank_edges": edges,
            "ms_per_step_replicated_output": round(rep_ms, 3),
            "comm_ms": comm_ms, "comm_bytes_per_rank": rec.bytes_sent(),
            # one pass's collectives replayed alone with its all-gathers in each form
            "comm_ms_by_all_gather_mode": {k: round(v, 3) for k, v in comm_both.items()},
            "collectives_per_pass": len(rec.calls), "overlap_frac": overlap,
            # per collective kind, replayed alone: ms per call, bytes each rank sends per
            # call, and bus bandwidth = those bytes / time (nccl-tests' busbw: algbw x
            # (P-1)/P) — against ~153 GB/s per xGMI link, 7 links per GPU
            "comm_by_kind": {k: {"ms": round(v["ms"], 3), "calls_per_pass": v["calls"],
                                 "bytes_sent": v["bytes"],
                                 "busbw_GBs": None if v["busbw_GBs"] is None else round(v["busbw_GBs"], 1)}
                             for k, v in per_kind.items()},
            "rccl": rccl_environment(ex)}


def rccl_environment(ex):
    """What decides RCCL's algorithm for this run: its version and every NCCL_* / RCCL_* /
    HSA_* variable set in the environment (none set = RCCL's defaults)."""
    env = {k: v for k, v in sorted(os.environ.items())
           if k.startswith(("NCCL_", "RCCL_", "HSA_ENABLE_IPC", "HSA_FORCE_FINE"))}
    ver = None
    if ex._rccl:
        try:
            v = torch.cuda.nccl.version()
            ver = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception as exc:  # a diagnostic never fails the bench
            ver = f"unknown ({exc!r})"
    return {"version": ver, "env": env, "defaults": not any(  # (logging does not count)
        k.startswith(("NCCL_", "RCCL_")) and not k.startswith("NCCL_DEBUG") for k in env)}


if __name__ == "__main__":
    main()
