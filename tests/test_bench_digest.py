"""The multi-GPU bench's self-checks, on CPU: the output digest a P > 1 run compares with the
one-GPU run (additive over the ranks' row ranges, so rank digests summed mod 2^64 equal the
one-process digest; one flipped bit on one rank is caught), the committed digest file's
record / lookup, and the progress lines that name a stuck collective."""
import io
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gnnrec.dist import Exchange, ProgressExchange, digest_add, table_digest  # noqa: E402


def _table(n=1000, d=16, seed=0):
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.standard_normal((n, d)).astype(np.float32))


def test_table_digest_is_additive_over_row_ranges():
    t = _table()
    whole = table_digest(t)
    for cuts in ([0, 1000], [0, 1, 999, 1000], [0, 125, 250, 375, 500, 625, 750, 875, 1000],
                 [0, 333, 334, 1000]):
        parts = [table_digest(t[a:b], a) for a, b in zip(cuts, cuts[1:]) if b > a]
        assert digest_add(*parts) == whole, cuts
    # small chunks inside the digest give the same sums as one chunk
    assert table_digest(t, chunk=97) == whole


def test_table_digest_catches_one_bit_and_a_row_swap():
    t = _table()
    whole = table_digest(t)
    f = t.clone()
    f.view(torch.int32).reshape(-1)[12345 % f.numel()] ^= 1
    d = table_digest(f)
    assert d[0] != whole[0] and d[1] != whole[1]
    s = t.clone()
    s[[3, 7]] = s[[7, 3]]
    assert table_digest(s) != whole
    # the same rows at another global offset are another digest
    assert table_digest(t, 1) != whole


def test_p1_digest_record_and_lookup(tmp_path):
    path = str(tmp_path / "p1.json")
    args = bench.parse([])
    ref, why = bench.p1_digest_lookup(path, args)
    assert ref is None and "no digest file" in why
    dg = {"user": "0" * 32, "item": "1" * 32}
    bench.p1_digest_record(path, args, dg, 142.0)
    ref, why = bench.p1_digest_lookup(path, args)
    assert ref is not None and ref["digest"] == dg
    other = bench.parse(["--config", "c5"])
    ref, why = bench.p1_digest_lookup(path, other)
    assert ref is None and "no one-GPU digest of this workload" in why
    bench.p1_digest_record(path, args, {"user": "2" * 32, "item": "3" * 32}, 141.0)  # replaces
    import json
    assert len(json.load(open(path))["entries"]) == 1
    # stale sources: same workload, another bits digest
    data = json.load(open(path))
    data["entries"][0]["sources"] = "deadbeefdeadbeef"
    json.dump(data, open(path, "w"))
    ref, why = bench.p1_digest_lookup(path, args)
    assert ref is None and why.startswith("stale")


def test_bits_digest_is_stable_and_parse_tolerates_unknown_flags():
    assert bench.bits_digest() == bench.bits_digest() and len(bench.bits_digest()) == 16
    # a recorded profile whose flags the parser no longer knows only drops that profile
    a = bench.parse(["--config", "c5", "--flag-from-an-old-round", "3"])
    assert a.config == "c5"


class _Shard:
    def __init__(self, p_lo, p_hi, S):
        self.p_lo, self.p_hi, self.shard_rows = p_lo, p_hi, {"item": S}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest_worker(rank, world, port, perturb, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if perturb is not None:
        os.environ["GNNREC_BENCH_PERTURB_RANK"] = str(perturb)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        users, items = _table(900, 8, 1), _table(100, 8, 2)
        args = bench.parse(["--users", "900", "--items", "100"])
        ub = [0, 400, 900][rank:rank + 2]  # uneven user ranges, as the degree balance makes
        S = 50
        out = {"user": users[ub[0]:ub[1]],
               "item": torch.cat([items[rank * S:(rank + 1) * S], torch.zeros(3, 8)])}
        q.put((rank, bench.output_digest(args, _Shard(ub[0], ub[1], S), out, rank, world,
                                         torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


def _run_digest(perturb):
    ctx = mp.get_context("spawn")
    q, port = ctx.Queue(), _free_port()
    procs = [ctx.Process(target=_digest_worker, args=(r, 2, port, perturb, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_two_rank_digest_equals_one_process_digest_and_catches_a_bad_rank():
    users, items = _table(900, 8, 1), _table(100, 8, 2)
    args = bench.parse(["--users", "900", "--items", "100"])
    one = bench.output_digest(args, _Shard(0, 900, 100), {"user": users, "item": items}, 0, 1,
                              torch.device("cpu"))
    res = _run_digest(None)
    assert res[0] == res[1] == one
    bad = _run_digest(1)
    assert bad[0] == bad[1] and bad[0]["user"] != one["user"] and bad[0]["item"] == one["item"]


def test_progress_exchange_names_every_collective():
    buf = io.StringIO()

    class Runner:
        _layer_idx = 1

    ex = ProgressExchange(Exchange(), Runner(), stream=buf)
    ex.pass_no, ex.checked = 3, True
    ex.layer_start(1)
    full = torch.zeros(8, 4)
    blocks, work = ex.all_to_all_rows(full, async_op=True)
    assert blocks.shape == (1, 8, 4) and work is None
    ex.all_gather_rows(full[:8], torch.zeros(8, 4), async_op=True)
    assert ex.ws == 1 and ex.inner.ag_mode == "rccl"  # everything else is the inner's
    lines = buf.getvalue().splitlines()
    assert lines[0] == "[gnnrec r0] pass 3 layer 1 start"
    assert lines[1] == "[gnnrec r0] pass 3 layer 1 all_to_all (8, 4) issued"
    assert lines[2].startswith("[gnnrec r0] pass 3 layer 1 all_to_all done in ")
    assert lines[3] == "[gnnrec r0] pass 3 layer 1 all_gather (8, 4) issued"
    assert len(lines) == 5
