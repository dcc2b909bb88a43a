#!/bin/bash
# round 4 (m): GNNREC_TRAIN_FOLD=auto — the first block's source rows at K = 10 / 2500 and the
# C2 step in the default mode at both K (with the sampling thread)
set -o pipefail
mkdir -p gpurun_out/r04m
O=gpurun_out/r04m
timeout -k 10 200 python -u tools/probe_block_sizes.py 10 2500 > $O/block_sizes.log 2>&1 || { echo "sizes failed"; tail $O/block_sizes.log; exit 1; }
grep "^{" $O/block_sizes.log
for K in 10 2500 10 2500; do
  timeout -k 10 200 python -u tools/probe_c2_step.py $K 2 > $O/k${K}.log 2>&1 || { echo "probe failed"; tail $O/k${K}.log; exit 1; }
  echo "K=$K auto $(tail -1 $O/k${K}.log | grep -o "'wall_ms_per_step': [0-9.]*, 'host_ms_per_step': [0-9.]*")"
done
