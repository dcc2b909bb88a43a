"""The grouped cosine at C3's shape (1024 positives x K negatives, 100k item rows) in both
forms through the C ABI — gnnrec_sddmm_cos_grouped_f32 (one wave per 64-negative chunk,
item rows from the Infinity Cache) and gnnrec_sddmm_cos_grouped_rows_f32 (the group's
negatives sorted by ~2 MB item slices in LDS, scored slice by slice) — alternating, HIP
events; checks the two are bitwise equal.
    python tools/micro/cos_sliced_ab.py [K] [d] [reps] [n_items]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import _lib  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
d = int(sys.argv[2]) if len(sys.argv) > 2 else 128
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
n_i = int(sys.argv[4]) if len(sys.argv) > 4 else 100000
L = _lib.load()
g = torch.Generator(device="cuda")
g.manual_seed(0)
G, n_u = 1024, 1024
Hs = torch.randn(n_u, d, device="cuda", generator=g)
Hd = torch.randn(n_i, d, device="cuda", generator=g)
ps = torch.randint(0, n_u, (G,), device="cuda", generator=g)
pd = torch.randint(0, n_i, (G,), device="cuda", generator=g)
nd = torch.randint(0, n_i, (G * K,), device="cuda", generator=g)
outs = {}


def run(sliced, of, on):
    st = _lib.stream_ptr()
    P = _lib.ptr
    if sliced:
        rc = L.gnnrec_sddmm_cos_grouped_rows_f32(P(ps), G, P(pd), P(of), K, P(nd), P(on), P(Hs), d,
                                                 P(Hd), d, n_i, d, st)
    else:
        rc = L.gnnrec_sddmm_cos_grouped_f32(P(ps), G, P(pd), P(of), K, P(nd), P(on), P(Hs), d,
                                            P(Hd), d, d, st)
    _lib.check(rc, "cos")


res = {"K": K, "d": d, "n_items": n_i, "table_MB": n_i * d * 4 / 2**20}
for sliced in (False, True):
    of, on = torch.empty(G, device="cuda"), torch.empty(G * K, device="cuda")
    run(sliced, of, on)
    outs[sliced] = (of, on)
torch.cuda.synchronize()
res["bitwise"] = bool(torch.equal(outs[False][0], outs[True][0]) and
                      torch.equal(outs[False][1], outs[True][1]))
times = {False: [], True: []}
for rnd in range(4):
    for sliced in (False, True):
        of, on = outs[sliced]
        for _ in range(3):
            run(sliced, of, on)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            run(sliced, of, on)
        e.record()
        e.synchronize()
        times[sliced].append(s.elapsed_time(e) / reps * 1e3)
b_alg = G * (K + 1) * (d * 4 + 8 + 4) + G * (d * 4 + 8)
for sliced, name in ((False, "grouped_us"), (True, "sliced_us")):
    res[name] = [round(t, 1) for t in times[sliced]]
    res[name.replace("_us", "_TBs")] = round(b_alg / (min(times[sliced]) * 1e-6) / 1e12, 2)
print(json.dumps(res), flush=True)
