#!/bin/bash
# round 6 (z): the LDS-staged edge MLP — full parity file (goldens with the MLP head
# included), the configs' head tests, and the minibatch rooflines
set -o pipefail
O=gpurun_out/${TAG:-r06z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python -u -c "
import json, torch, bench
print(json.dumps(bench.minibatch_rooflines(torch.device('cuda'))))" > $O/roof.json 2> $O/roof.err || { echo "roof failed"; tail -20 $O/roof.err; exit 1; }
python - $O/roof.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("cosine", "edge_mlp"):
    print(k, {kk: d[k].get(kk) for kk in ("ms", "per_edge_kernel_ms", "frac", "gather_frac", "mfma_frac")})
print("sampler", d["sampler"]["ms_per_call"])
PY
