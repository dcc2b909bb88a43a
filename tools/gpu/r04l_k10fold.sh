#!/bin/bash
# round 4 (l): the first-layer fold at the host-bound K = 10 step (the K = 2500 step gains
# 4.3 -> 3.46 ms): 4 alternations per setting, with and without the sampling thread
set -o pipefail
mkdir -p gpurun_out/r04l
O=gpurun_out/r04l
for nw in 2 0; do
  for f in 1 0 1 0 1 0 1 0; do
    GNNREC_TRAIN_FOLD=$f timeout -k 10 200 python -u tools/probe_c2_step.py 10 $nw > $O/k10_nw${nw}_f$f.log 2>&1 || { echo "probe failed"; tail $O/k10_nw${nw}_f$f.log; exit 1; }
    echo "nw=$nw fold=$f $(tail -1 $O/k10_nw${nw}_f$f.log | grep -o "'wall_ms_per_step': [0-9.]*, 'host_ms_per_step': [0-9.]*")"
  done
done
