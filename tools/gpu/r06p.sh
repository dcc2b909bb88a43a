#!/bin/bash
# round 6 (p): static batches' block data gathered lazily (inside the captured graph) —
# the sampling / capture / C2 tests, then the default bench line
set -o pipefail
O=gpurun_out/${TAG:-r06p}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sampling.py tests/test_gpu_capture.py tests/test_gpu_configs.py -k "not full_size" \
  -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["frac"])
mb = d.get("minibatch", {})
for k, v in mb.items():
    if k.startswith("K"):
        print(k, {kk: v.get(kk) for kk in ("ms_per_step", "loss_rel_diff_vs_eager", "gpu_ms_per_replay", "error")})
r = mb.get("rooflines", {})
print("sampler", r.get("sampler", {}).get("ms_per_call"), "cosine", r.get("cosine", {}).get("ms"), "mlp", r.get("edge_mlp", {}).get("gather_frac"))
PY
