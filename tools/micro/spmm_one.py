"""One low-degree spmm shape (a minibatch block's relation), timed with HIP events:
    python tools/micro/spmm_one.py n_dst deg n_src d [reps] [reduce] [weighted]
Env knobs of the row kernel apply (GNNREC_ROWQ=0, GNNREC_RQ_CHUNK=<rows per ticket>)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

n_dst, deg, n_src, d = (int(x) for x in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
reduce = sys.argv[6] if len(sys.argv) > 6 else "mean"
weighted = len(sys.argv) > 7 and sys.argv[7] == "1"
g = torch.Generator(device="cuda")
g.manual_seed(0)
indptr = torch.arange(0, (n_dst + 1) * deg, deg, device="cuda", dtype=torch.int64)
indices = torch.randint(0, n_src, (n_dst * deg,), device="cuda", generator=g).int()
X = torch.randn(n_src, d, device="cuda", generator=g)
ew = torch.rand(n_dst * deg, device="cuda", generator=g) if weighted else None


def run():
    return ops.spmm(indptr, indices, X, reduce, edge_weight=ew)


for _ in range(3):
    run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    run()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
gb = n_dst * deg * d * 4 / 1e9
print(f"n_dst={n_dst} deg={deg} n_src={n_src} d={d} {reduce} w={int(weighted)}: {ms * 1e3:.1f} us "
      f"{gb / ms * 1e3 / 1e3:.2f} TB/s gathered", flush=True)
