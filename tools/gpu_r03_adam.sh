#!/bin/bash
# C2/K2500 training steps of bench.py's minibatch field: torch Adam foreach vs fused, alternating
set -o pipefail
for rep in 1 2 3; do
  for f in 0 1; do
    echo -n "ADAM_FUSED=$f "
    GNNREC_BENCH_ADAM_FUSED=$f timeout -k 10 300 python -c "
import sys, json, torch; sys.path.insert(0, '.'); import bench
r = bench.minibatch_step(torch.device('cuda'))
print(json.dumps({k: (v['ms_per_step'], round(v['loss'], 6)) for k, v in r.items() if k != 'workload'}))" 2>/dev/null || exit 1
  done
done
