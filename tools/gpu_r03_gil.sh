#!/bin/bash
# C2 step with the sampling thread: GIL switch interval sweep (3 reps each, alternating)
set -o pipefail
for rep in 1 2 3; do
  for si in 0.005 0.001 0.0002; do
    echo "si=$si $(GNNREC_SWITCH_INTERVAL=$si timeout -k 10 120 python -u tools/probe_c2_step.py 10 2 2>/dev/null | tail -1 | python -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(round(d['wall_ms_per_step'],3))")"
  done
done
