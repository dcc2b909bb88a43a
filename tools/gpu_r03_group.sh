#!/bin/bash
# group-per-row spmm path (d <= 64, mean degree <= 16): bitwise tests, low-degree shapes
# and the C2 step at K = 10 / 2500, GNNREC_SPMM_GROUP=0 (wave per row) vs default
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "spmm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_group_tests.log 2>&1 || { tail -40 gpurun_out/r03_group_tests.log; exit 1; }
tail -1 gpurun_out/r03_group_tests.log
for shape in "1000000 2 1000000 64" "1000000 3 120000 64" "300000 3 1000000 64" "100000 10 1000000 64" "100000 10 100000 32"; do
  for g in 0 16; do
    echo "group=$g $(GNNREC_SPMM_GROUP=$g timeout -k 10 60 python tools/micro/spmm_one.py $shape 20 sum 1 2>/dev/null | tail -1)" || exit 1
  done
done
for K in 10 2500; do
  for g in 0 16 0 16; do
    echo "K=$K group=$g $(GNNREC_SPMM_GROUP=$g timeout -k 10 150 python -u tools/probe_c2_step.py $K 0 2>/dev/null | tail -1)" || exit 1
  done
done
