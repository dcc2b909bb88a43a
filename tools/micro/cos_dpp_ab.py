"""The cosine kernels' per-edge reductions as DPP adds (gnnrec_sddmm_cos_f32 /
gnnrec_sddmm_cos_grouped_f32) against the __shfl_xor (ds_bpermute) trees they replace
(experiment entries gnnrec_sddmm_cos_xor_f32 / gnnrec_sddmm_cos_grouped_xor_f32, when built):
C3's shape, d = 128, alternating, HIP events; bitwise checks across all four.
    python tools/micro/cos_dpp_ab.py [K] [reps]"""
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
d, G, n_i = 128, 1024, 100000
L = _lib.load()
V = ctypes.c_void_p
xe = getattr(L, "gnnrec_sddmm_cos_xor_f32", None)
xg = getattr(L, "gnnrec_sddmm_cos_grouped_xor_f32", None)
if xe is not None:
    xe.restype, xe.argtypes = ctypes.c_int, [V, V, ctypes.c_int64, V, V, V, V]
    xg.restype = ctypes.c_int
    xg.argtypes = [V, ctypes.c_int64, V, V, ctypes.c_int64, V, V, V, V, V]
g = torch.Generator(device="cuda")
g.manual_seed(0)
Hs = torch.randn(G, d, device="cuda", generator=g)
Hd = torch.randn(n_i, d, device="cuda", generator=g)
ps = torch.arange(G, device="cuda")
pd = torch.randint(0, n_i, (G,), device="cuda", generator=g)
nd = torch.randint(0, n_i, (G * K,), device="cuda", generator=g)
src = torch.cat([ps, ps.repeat_interleave(K)])
dst = torch.cat([pd, nd])
E = src.numel()
P = _lib.ptr
st = _lib.stream_ptr
bufs = {k: (torch.empty(G, device="cuda"), torch.empty(G * K, device="cuda"), torch.empty(E, device="cuda"))
        for k in ("edge", "grouped", "edge_xor", "grouped_xor")}


def run(kind):
    of, on, oe = bufs[kind]
    if kind == "edge":
        rc = L.gnnrec_sddmm_cos_f32(P(src), P(dst), E, P(Hs), d, P(Hd), d, d, P(oe), st())
    elif kind == "grouped":
        rc = L.gnnrec_sddmm_cos_grouped_f32(P(ps), G, P(pd), P(of), K, P(nd), P(on), P(Hs), d,
                                            P(Hd), d, d, st())
    elif kind == "edge_xor":
        rc = xe(P(src), P(dst), E, P(Hs), P(Hd), P(oe), st())
    else:
        rc = xg(P(ps), G, P(pd), P(of), K, P(nd), P(on), P(Hs), P(Hd), st())
    _lib.check(rc, kind)


kinds = ("edge", "grouped") + (("edge_xor", "grouped_xor") if xe is not None else ())
for k in kinds:
    run(k)
torch.cuda.synchronize()
ref = bufs["edge"][2]
res = {"K": K, "d": d, "edges": E}
for k in kinds:
    of, on, oe = bufs[k]
    got = oe if k.startswith("edge") else torch.cat([of, on])
    res[k + "_bitwise_eq_edge"] = bool(torch.equal(got, ref))
times = {k: [] for k in kinds}
for _ in range(4):
    for k in kinds:
        for _ in range(reps):
            run(k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            run(k)
        e.record()
        e.synchronize()
        times[k].append(round(s.elapsed_time(e) / reps * 1e3, 1))
b_alg = E * (d * 4 + 8 + 4) + G * (d * 4 + 8)
for k in kinds:
    res[k + "_us"] = times[k]
res["grouped_TBs"] = round(b_alg / (min(times["grouped"]) * 1e-6) / 1e12, 2)
print(json.dumps(res), flush=True)
