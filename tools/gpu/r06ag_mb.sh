#!/bin/bash
# round 6 (ag): the bench's minibatch leg alone (eager / captured C2 steps, rooflines)
set -o pipefail
O=gpurun_out/${TAG:-r06ag}
mkdir -p $O
timeout -k 10 600 python -u -c "
import json, torch, bench
print(json.dumps(bench.minibatch_step(torch.device('cuda')), default=str))" > $O/mb.json 2> $O/mb.err || { echo "mb failed"; tail -20 $O/mb.err; exit 1; }
python - $O/mb.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d.items():
    if k.startswith("K"):
        print(k, v.get("ms_per_step"), v.get("gpu_ms_per_replay"))
r = d["rooflines"]
print("sampler", r["sampler"]["ms_per_call"], "cos", r["cosine"]["ms"], "mlp", r["edge_mlp"]["ms"])
PY
