#!/bin/bash
# C4 bench A/B over bench arguments, alternating: c4_args_ab.sh "--segments 8" "--segments 16"
set -o pipefail
for rep in 1 2; do
  for a in "$@"; do
    echo -n "[$a] "
    timeout -k 10 300 python bench.py --cpu-baseline off --steps 5 --warmup 2 $a $EXTRA 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), {k: round(v,3) for k, v in r.items() if k.startswith('launch_ms') and v})" || exit 1
  done
done
