#!/bin/bash
# C2 step: num_workers 0 / 2 and the GIL switch interval
set -o pipefail
for rep in 1 2; do
  for cfg in "0 0.005" "2 0.005" "2 0.0005" "2 0.0001" "1 0.0001"; do
    set -- $cfg
    GNNREC_SWITCH_INTERVAL=$2 timeout -k 10 120 python -u tools/probe_c2_step.py 10 $1 2>/dev/null | tail -1 || exit 1
  done
done
