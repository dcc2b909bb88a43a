#!/bin/bash
# C4 bench A/B over env settings, alternating: c4_env_ab.sh "ENV=a" "ENV=b" ...
set -o pipefail
for rep in 1 2; do
  for e in "$@"; do
    echo -n "[$e] "
    env $e timeout -k 10 300 python bench.py --cpu-baseline off --steps 5 --warmup 2 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), round(r['launch_ms'],3), round(r['frac'],3))" || exit 1
  done
done
