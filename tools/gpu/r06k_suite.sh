#!/bin/bash
# round 6 (k): the whole GPU suite + smoke on the current sources, then the default bench line
set -o pipefail
O=gpurun_out/${TAG:-r06k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
python - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("frac_spmm_tile"))
mb = d.get("minibatch", {})
for k, v in mb.items():
    if k.startswith("K"):
        print(k, {kk: v.get(kk) for kk in ("ms_per_step", "loss_batch1", "loss_first", "loss", "loss_rel_diff_vs_eager", "gpu_ms_per_replay", "error")})
r = mb.get("rooflines", {})
print("sampler", r.get("sampler", {}).get("ms_per_call"), r.get("sampler", {}).get("gpu_span_ms_per_call"), "cosine", r.get("cosine", {}).get("ms"))
PY
