"""gnnrec_csr_build (the stable LSD radix sort: hist / scan / scatter per pass, then the row
bounds) on random COO edges, HIP events — the sort the loader's transposes and the cosine
backward's item keys run on:
    python tools/micro/radix_one.py [n_edges] [n_dst] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 2_561_024
n_dst = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
g = torch.Generator(device="cuda")
g.manual_seed(0)
src = torch.randint(0, 1 << 20, (E,), device="cuda", generator=g)
dst = torch.randint(0, n_dst, (E,), device="cuda", generator=g)
out = ops.csr_build(src, dst, n_dst)
torch.cuda.synchronize()
ip, ix, eid = out[0], out[1], out[2]
ok = bool(torch.equal(ip[1:] - ip[:-1], torch.bincount(dst, minlength=n_dst)) and
          torch.equal(eid, torch.sort(dst, stable=True).indices) and
          torch.equal(ix.long(), src[eid]))
for _ in range(reps):
    ops.csr_build(src, dst, n_dst)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    ops.csr_build(src, dst, n_dst)
e.record()
e.synchronize()
print(json.dumps({"E": E, "n_dst": n_dst, "matches_torch_stable_sort": ok,
                  "us_per_build": round(s.elapsed_time(e) / reps * 1e3, 1)}), flush=True)
