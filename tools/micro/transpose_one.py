"""Source-major transposes of minibatch-block shapes (gnnrec_csr_transpose: the radix sort
of the block's source ids), HIP-event time per call:  python tools/micro/transpose_one.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
g = torch.Generator(device="cuda")
g.manual_seed(0)
for n_dst, deg, n_src in ((10_000, 10, 100_000), (100_000, 10, 1_000_000), (630_000, 10, 100_000),
                          (1_000_000, 10, 1_000_000), (256_000, 10, 2_560_000)):
    indptr = torch.arange(0, (n_dst + 1) * deg, deg, device="cuda", dtype=torch.int64)
    indices = torch.randint(0, n_src, (n_dst * deg,), device="cuda", generator=g).int()
    for _ in range(3):
        ops.csr_transpose(indptr, indices, n_src, mean=True)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        ops.csr_transpose(indptr, indices, n_src, mean=True)
    e.record()
    torch.cuda.synchronize()
    print(f"E={n_dst * deg:>9d} n_src={n_src:>9d}: {s.elapsed_time(e) * 1e3 / reps:8.1f} us/call",
          flush=True)
