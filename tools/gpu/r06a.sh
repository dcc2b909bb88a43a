#!/bin/bash
# round 6 (a): the new / changed GPU tests (plan overflow, fold on the library GEMMs, grouped
# cosine LPR 64 + stale mark, event-gated emulation, captured C2 steps vs the oracle), then
# the default bench line (C4 + CPU baseline + minibatch with comparable eager/captured losses)
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_capture.py tests/test_gpu_fold.py \
  "tests/test_gpu_parity.py::test_cosine_pair_head_grouped_path_forward_and_gradients" \
  "tests/test_gpu_parity.py::test_cosine_pair_head_ignores_a_stale_grouped_mark" \
  "tests/test_gpu_dist.py::test_async_emulation_lands_late_and_reads_late" \
  -m gpu > $O/tests1.log 2>&1 || { echo "tests1 failed"; tail -40 $O/tests1.log; exit 1; }
tail -1 $O/tests1.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  "tests/test_gpu_configs.py::test_c2_captured_static_steps_match_oracle" \
  -m gpu > $O/tests2.log 2>&1 || { echo "tests2 failed"; tail -40 $O/tests2.log; exit 1; }
grep -E "replay|passed|failed" $O/tests2.log | tail -8
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06a/bench.json").read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["frac"])
mb = d.get("minibatch", {})
for k, v in mb.items():
    if k.startswith("K"):
        print(k, {kk: v.get(kk) for kk in ("ms_per_step", "loss", "loss_first", "loss_rel_diff_vs_eager", "plan_overflows", "error")})
print("sampler", mb.get("rooflines", {}).get("sampler", {}).get("ms_per_call"), "cosine", mb.get("rooflines", {}).get("cosine", {}).get("ms"))
PY
