"""Negative control of test_capture_beside_a_sampling_thread_drawing_negatives: the same
scenario with sampling.RNG_LOCK / capture.RNG_LOCK replaced by no-op locks — does a draw
from the side thread land inside the capture window and raise?
    python tools/probe_rng_race.py [lock: 0 | 1]"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "gnn-recsys_amd"))
import torch  # noqa: E402


class _NoLock:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def main():
    from gnnrec import capture, sampling
    from gnnrec.capture import CapturedTrainStep
    from test_gpu_capture import _loader, _loss
    from test_gpu_sampling import BUYS, DEV, _graph, _model
    lock = len(sys.argv) > 1 and sys.argv[1] == "1"
    if not lock:
        capture.RNG_LOCK = sampling.RNG_LOCK = _NoLock()
    g, _ = _graph(n_u=300, n_i=120, e_b=4000, e_c=3000, min_deg=False)
    batches = [b for b in _loader(g, True)][:3]
    stop, errors, draws = threading.Event(), [], [0]

    def draw():
        neg = sampling.negative_sampler.Uniform(4)
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                while not stop.is_set():
                    neg(g, {BUYS: torch.arange(64, device=DEV)})
                    draws[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e)[:160])

    t = threading.Thread(target=draw, daemon=True)
    t.start()
    main_err = None
    stats = []
    try:
        for _ in range(3):
            m = _model(g, agg="mean").train()
            opt = torch.optim.Adam(m.parameters(), lr=0.01, fused=True)
            step = CapturedTrainStep(m, opt, _loss(4), warmup=1)
            for b in batches:
                step(b)
            stats.append((step.captures, step.replays, step.eager_steps, step.seen))
    except Exception as e:  # noqa: BLE001
        main_err = repr(e)[:160]
    finally:
        stop.set()
        t.join()
    print(json.dumps({"lock": lock, "draws": draws[0], "thread_errors": errors,
                      "capture_error": main_err, "captures_replays_eager_seen": stats}),
          flush=True)


if __name__ == "__main__":
    main()
