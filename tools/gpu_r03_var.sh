#!/bin/bash
# C2 step variance: 200 timed steps per run, 4 runs each of num_workers 2 and 0
set -o pipefail
for rep in 1 2 3 4; do
  for nw in 2 0; do
    echo "nw=$nw $(GNNREC_PROBE_STEPS=200 timeout -k 10 120 python -u tools/probe_c2_step.py 10 $nw 2>/dev/null | tail -1 | python -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(round(d['wall_ms_per_step'],3), {k: round(v,3) for k,v in d['host_phase_ms'].items()})")"
  done
done
