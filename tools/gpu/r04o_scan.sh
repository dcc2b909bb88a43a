#!/bin/bash
# round 4 (o): the chained scan with its tile staged through LDS (coalesced loads / stores)
# against the previous strided form (tools/_diag/libgnnrec_scan_old.so): exactness, time per
# call at the sampler's sizes; the sampler tests; the C2 step at K = 10 / 2500
set -o pipefail
mkdir -p gpurun_out/r04o
O=gpurun_out/r04o
for v in new old new old; do
  L=""; [ $v = old ] && L="GNNREC_LIB=$PWD/tools/_diag/libgnnrec_scan_old.so"
  echo "== $v"; env $L timeout -k 10 120 python -u tools/micro/scan_one.py 200 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sampling.py \
  tests/test_gpu_parity.py -k "sampl or scan or relabel or block" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for K in 10 2500 10 2500; do
  timeout -k 10 200 python -u tools/probe_c2_step.py $K 2 > $O/k${K}.log 2>&1 || { echo "probe failed"; tail $O/k${K}.log; exit 1; }
  echo "K=$K $(tail -1 $O/k${K}.log | grep -o "'wall_ms_per_step': [0-9.]*, 'host_ms_per_step': [0-9.]*")"
done
