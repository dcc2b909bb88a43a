#!/bin/bash
# weight-gradient GEMM: k-major LDS (GNNREC_TN_T=0) vs k-contiguous LDS with b128 reads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "gemm_tn or lstm_backward or autograd or train" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_tn_tests.log 2>&1 || { tail -30 gpurun_out/r03_tn_tests.log; exit 1; }
tail -1 gpurun_out/r03_tn_tests.log
for t in 0 1; do
  for shape in "1000000 128 128" "200000 128 128" "50000 128 128" "100000 128 256" "204000 64 64" "10000 64 64"; do
    echo "TN_T=$t $(GNNREC_TN_T=$t timeout -k 10 60 python tools/micro/gemm_tn_one.py $shape 2>/dev/null | tail -1)"
  done
done
for t in 0 1; do
  echo "TN_T=$t $(GNNREC_TN_T=$t timeout -k 10 200 python -u tools/probe_c2_step.py 2500 0 128 mean_nn 2>/dev/null | tail -1)"
  echo "TN_T=$t $(GNNREC_TN_T=$t timeout -k 10 200 python -u tools/probe_c2_step.py 10 2 2>/dev/null | tail -1)"
done
