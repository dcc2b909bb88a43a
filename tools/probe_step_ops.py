"""Which torch ops the C2 training step issues besides the library's own kernels: one eager
static-shape step (the form CapturedTrainStep records) under torch.profiler, the aten ops
grouped by their Python call site (fills, copies, cats, elementwise, reductions, GEMMs).

    python tools/probe_step_ops.py [K]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnn-recsys_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    from gnnrec import nn as gnn
    from gnnrec.capture import CapturedTrainStep
    from gnnrec.sampling import EdgeDataLoader, MultiLayerNeighborSampler, negative_sampler
    from gnnrec.synth import minibatch_graph
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda")
    g = minibatch_graph(64, dev)
    buys = ("user", "buys", "item")
    torch.manual_seed(0)
    model = gnn.ConvModel(g, 3, {"user": 64, "item": 64, "hidden": 64, "out": 64}, True, 0.0,
                          "mean", "cos", "sum", True).to(dev)
    model.train_fold = "1"
    opt = torch.optim.Adam(model.parameters(), lr=0.005, fused=True)

    def loss_fn(m, batch):
        _, pos_g, neg_g, blocks = batch
        _, ps, ns = m(blocks, blocks[0].srcdata["features"], pos_g, neg_g, True)
        return gnn.max_margin_loss(ps, ns, 0.266, K, True, pos_g.edata["recency"])

    el = EdgeDataLoader(g, {buys: torch.arange(g.num_edges(buys))},
                        MultiLayerNeighborSampler([10, 10]), exclude="reverse_types",
                        reverse_etypes={"buys": "bought-by", "bought-by": "buys"},
                        negative_sampler=negative_sampler.Uniform(K), batch_size=1024,
                        shuffle=True, static_shapes=True)
    el.sampler.first_transposes_below = 0
    step = CapturedTrainStep(model, opt, loss_fn, warmup=100)
    it = iter(el)
    for _ in range(4):
        step(next(it))
    batch = next(it)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True,
                 record_shapes=True) as prof:
        step.eager(batch)
        torch.cuda.synchronize()
    skip = ("gnnrec::", "aten::empty", "aten::view", "aten::as_strided", "aten::reshape",
            "aten::detach", "aten::slice", "aten::narrow", "aten::select", "aten::t",
            "aten::transpose", "aten::expand", "aten::unsqueeze", "aten::squeeze", "aten::unbind",
            "aten::resolve", "aten::lift", "aten::alias", "aten::_reshape", "aten::numel",
            "detach", "aten::is_", "aten::result_type", "aten::size", "aten::stride",
            "aten::_has_compatible")
    seen = 0
    for ev in prof.events():
        if ev.name.startswith(skip) or ev.name.startswith("cuda") or \
                ev.name.startswith("hip") or "Optimizer" in ev.name or ev.name.startswith("##"):
            continue
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue  # the outermost aten op only
        stack = [s for s in ev.stack if "gnnrec" in s or "bench" in s or "probe" in s][:3]
        shapes = ev.input_shapes[:3] if ev.input_shapes else []
        print(f"{ev.name:34s} {str(shapes)[:60]:60s} | " + " < ".join(
            s.split("/")[-1] for s in stack))
        seen += 1
    print("outermost non-library ops:", seen)


if __name__ == "__main__":
    main()
