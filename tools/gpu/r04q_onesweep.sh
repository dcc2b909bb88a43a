#!/bin/bash
# round 4 (q): one-sweep radix passes (global digit histogram + one look-back kernel per pass)
# against the three-launch passes (GNNREC_RADIX_ONESWEEP=0): CSR / transpose / sampler
# tests, transpose time per call at block shapes, the C2 step at K = 10 / 2500
set -o pipefail
mkdir -p gpurun_out/r04q
O=gpurun_out/r04q
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_csr.py \
  tests/test_gpu_sampling.py tests/test_gpu_parity.py -k "csr or transpose or sampl or block" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  echo "== onesweep=$v"; GNNREC_RADIX_ONESWEEP=$v timeout -k 10 120 python -u tools/micro/transpose_one.py 100 || exit 1
done
for v in 1 0 1 0; do
  for K in 10 2500; do
    GNNREC_RADIX_ONESWEEP=$v timeout -k 10 200 python -u tools/probe_c2_step.py $K 2 > $O/k${K}_$v.log 2>&1 || { echo "probe failed"; tail $O/k${K}_$v.log; exit 1; }
    echo "onesweep=$v K=$K $(tail -1 $O/k${K}_$v.log | grep -o "'wall_ms_per_step': [0-9.]*, 'host_ms_per_step': [0-9.]*")"
  done
done
