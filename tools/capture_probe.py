"""Which part of the training step breaks a hipGraph capture: capture the forward only, the
forward + backward, or the whole step (+ fused Adam) over one static-shape batch of the
test graph, replay it, and compare with the same part run eagerly.

    python tools/capture_probe.py fwd|bwd|step
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnn-recsys_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tests"))
import torch  # noqa: E402


def main():
    stage = sys.argv[1]
    from test_gpu_capture import _loader, _loss
    from test_gpu_sampling import _graph, _model
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    torch.manual_seed(3)
    it = iter(_loader(g, True, K=4))
    b1, b2 = next(it), next(it)
    m = _model(g, agg="mean").train()
    opt = torch.optim.Adam(m.parameters(), lr=0.01, fused=True, capturable=True)
    f = _loss(4)
    # eager warm-up on the first batch
    loss = f(m, b1)
    opt.zero_grad(set_to_none=True)
    loss.backward()
    opt.step()
    del loss
    torch.cuda.synchronize()
    print("eager warm-up ok", flush=True)
    opt.zero_grad(set_to_none=True)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, capture_error_mode="thread_local"):
        out = f(m, b2)
        if stage in ("bwd", "step"):
            out.backward()
        if stage == "step":
            opt.step()
    print("capture ok", flush=True)
    gr.replay()
    torch.cuda.synchronize()
    print("replay ok", stage, float(out.detach()), flush=True)


if __name__ == "__main__":
    main()
