#!/bin/bash
# C5 pass A/B over env settings, alternating: c5_ab.sh "ENV=a ENV2=b" "ENV=c" ...
set -o pipefail
for rep in 1 2; do
  for e in "$@"; do
    echo -n "[$e] "
    env $e timeout -k 10 300 python bench.py --config c5 --cpu-baseline off --minibatch off --steps 5 --warmup 2 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), {k: round(v,3) for k, v in r.items() if k.startswith('launch_ms') and v})" || exit 1
  done
done
