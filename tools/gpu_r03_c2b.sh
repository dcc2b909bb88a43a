#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_configs.py -k "not full_size and not c2_csr" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_c2b_tests.log 2>&1 || { tail -40 gpurun_out/r03_c2b_tests.log; exit 1; }
tail -1 gpurun_out/r03_c2b_tests.log
for rep in 1 2 3; do
  for nw in 0 2; do
    timeout -k 10 120 python -u tools/probe_c2_step.py 10 $nw 2>/dev/null | tail -1 || exit 1
  done
done
