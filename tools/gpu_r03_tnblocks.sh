#!/bin/bash
# weight-gradient GEMM split-K grid size (GNNREC_TN_BLOCKS): kernel A/B and the C3/C2 steps
set -o pipefail
mkdir -p gpurun_out
GNNREC_TN_BLOCKS=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gemm_tn or lstm_backward or autograd or train or grad" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_tnb_tests.log 2>&1 || { tail -30 gpurun_out/r03_tnb_tests.log; exit 1; }
tail -1 gpurun_out/r03_tnb_tests.log
for rep in 1 2; do
for b in 512 1024 2048; do
  for shape in "1000000 128 128" "200000 128 128" "50000 128 128" "204000 64 64" "10000 64 64"; do
    echo "TN_BLOCKS=$b $(GNNREC_TN_BLOCKS=$b timeout -k 10 60 python tools/micro/gemm_tn_one.py $shape 2>/dev/null | tail -1)"
  done
done
done
for rep in 1 2; do
for b in 512 1024; do
  echo "TN_BLOCKS=$b C3 $(GNNREC_TN_BLOCKS=$b timeout -k 10 200 python -u tools/probe_c2_step.py 2500 0 128 mean_nn 2>/dev/null | tail -1)"
done
done
