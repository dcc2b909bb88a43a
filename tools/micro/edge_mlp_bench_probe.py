import json, torch, sys
sys.path.insert(0, "gnn-recsys_amd")
from gnnrec import ops
from gnnrec.nn import PredictingLayer
dev = torch.device("cuda")
gen = torch.Generator(device=dev); gen.manual_seed(1)
d, n_u, n_i, K = 128, 1024, 100_000, 2500
Hs = torch.randn(n_u, d, device=dev, generator=gen)
Hd = torch.randn(n_i, d, device=dev, generator=gen)
src = torch.cat([torch.arange(n_u, device=dev), torch.arange(n_u, device=dev).repeat_interleave(K)])
dst = torch.randint(0, n_i, (src.numel(),), device=dev, generator=gen)
ps, pd, nd = src[:n_u], dst[:n_u], dst[n_u:]
torch.manual_seed(0)
pl = PredictingLayer(d).to(dev).eval()
W1 = pl.hidden_1.weight.detach()
with torch.no_grad():
    P = ops.gemm(Hs, W1[:, :d], bias=pl.hidden_1.bias)
    Q = ops.gemm(Hd, W1[:, d:])
w2, b2 = pl.hidden_2.weight.detach(), pl.hidden_2.bias.detach()
w3, b3 = pl.output.weight.detach().reshape(-1), pl.output.bias.detach()
Pr = torch.randn_like(P); Qr = torch.randn_like(Q)
def t(fn, n=50):
    for _ in range(10): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); e.synchronize()
    return round(s.elapsed_time(e) / n * 1e3, 1)
res = {}
for rnd in range(3):
    for name, fn in (("grouped", lambda: ops.edge_mlp_grouped(ps, pd, K, nd, P, Q, w2, b2, w3, b3)),
                     ("edge", lambda: ops.edge_mlp(src, dst, P, Q, w2, b2, w3, b3)),
                     ("grouped_randPQ", lambda: ops.edge_mlp_grouped(ps, pd, K, nd, Pr, Qr, w2, b2, w3, b3)),
                     ("edge_randPQ", lambda: ops.edge_mlp(src, dst, Pr, Qr, w2, b2, w3, b3))):
        res.setdefault(name, []).append(t(fn))
print(json.dumps(res))
