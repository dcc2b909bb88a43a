"""The edge MLP tail at C3's shape (1024 positives x K negatives, 100k item rows, P/Q 128
wide) through the C ABI: the register-gather kernel (gnnrec_edge_mlp_regs_f32, not in the
header; round 5's kernel, in builds that have it), the LDS-staged per-edge kernel (gnnrec_edge_mlp_f32) and its grouped form
(gnnrec_edge_mlp_grouped_f32), alternating, HIP events; checks staged per-edge == grouped
bitwise and both against the register kernel.
    python tools/micro/edge_mlp_ab.py [K] [reps] [n_items]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "gnn-recsys_amd"))
import torch  # noqa: E402

from gnnrec import _lib  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
n_i = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
L = _lib.load()
regs = getattr(L, "gnnrec_edge_mlp_regs_f32", None)  # the round-5 kernel, when built
if regs is not None:
    regs.restype = ctypes.c_int
    regs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_void_p] * 8
w3k = getattr(L, "gnnrec_edge_mlp_grouped_glds_f32", None)  # experiment entries, when built
if w3k is not None:
    w3k.restype = ctypes.c_int
    w3k.argtypes = L.gnnrec_edge_mlp_grouped_f32.argtypes
g = torch.Generator(device="cuda")
g.manual_seed(0)
G, n_u = 1024, 1024
P = torch.randn(n_u, 128, device="cuda", generator=g)
Q = torch.randn(n_i, 128, device="cuda", generator=g)
W2 = torch.randn(32, 128, device="cuda", generator=g) * 0.1
b2 = torch.randn(32, device="cuda", generator=g) * 0.1
w3 = torch.randn(32, device="cuda", generator=g) * 0.3
b3 = torch.randn(1, device="cuda", generator=g)
ps = torch.arange(G, device="cuda")
pd = torch.randint(0, n_i, (G,), device="cuda", generator=g)
nd = torch.randint(0, n_i, (G * K,), device="cuda", generator=g)
src = torch.cat([ps.view(-1, 1), ps.view(-1, 1).expand(G, K)], 1).reshape(-1).contiguous()
dst = torch.cat([pd.view(-1, 1), nd.view(G, K)], 1).reshape(-1).contiguous()
E = src.numel()
Pp = _lib.ptr
st = _lib.stream_ptr
outs = {k: torch.empty(E, device="cuda") for k in ("regs", "staged")}
of, on = torch.empty(G, device="cuda"), torch.empty(G * K, device="cuda")
of2, on2 = torch.empty(G, device="cuda"), torch.empty(G * K, device="cuda")
W = (Pp(P), Pp(Q), Pp(W2), Pp(b2), Pp(w3), Pp(b3))


def run(kind):
    if kind == "regs":
        rc = regs(Pp(src), Pp(dst), E, *W, Pp(outs["regs"]), st())
    elif kind == "staged":
        rc = L.gnnrec_edge_mlp_f32(Pp(src), Pp(dst), E, *W, Pp(outs["staged"]), st())
    elif kind == "grouped":
        rc = L.gnnrec_edge_mlp_grouped_f32(Pp(ps), G, Pp(pd), Pp(of), K, Pp(nd), Pp(on), *W, st())
    else:
        rc = w3k(Pp(ps), G, Pp(pd), Pp(of2), K, Pp(nd), Pp(on2), *W, st())
    _lib.check(rc, kind)


kinds = (("regs",) if regs is not None else ()) + ("staged", "grouped") + \
    (("grouped_glds",) if w3k is not None else ())
for k in kinds:
    run(k)
torch.cuda.synchronize()
grouped = torch.cat([of.view(-1, 1), on.view(G, K)], 1).reshape(-1)
res = {"K": K, "edges": E, "n_items": n_i,
       "staged_eq_grouped": bool(torch.equal(outs["staged"], grouped)),
       "max_abs_vs_regs": float((outs["staged"] - outs["regs"]).abs().max())
       if regs is not None else None}
if w3k is not None:
    res["glds_eq_grouped"] = bool(torch.equal(of2, of) and torch.equal(on2, on))
times = {k: [] for k in kinds}
for _ in range(4):
    for k in kinds:
        for _ in range(3):
            run(k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            run(k)
        e.record()
        e.synchronize()
        times[k].append(round(s.elapsed_time(e) / reps * 1e3, 1))
fl = E * 2 * 128 * 32
for k in kinds:
    res[k + "_us"] = times[k]
    res[k + "_mfma_frac"] = round(fl / (min(times[k]) * 1e-6) / 157.3e12, 3)
print(json.dumps(res), flush=True)
