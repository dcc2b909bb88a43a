#!/bin/bash
# C2 A/B: the loader's batch head fused (gnnrec::edge_batch_pairs) vs its Python form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampling.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_c2c_tests.log 2>&1 || { tail -40 gpurun_out/r03_c2c_tests.log; exit 1; }
tail -1 gpurun_out/r03_c2c_tests.log
for rep in 1 2 3; do
  for nw in 0 2; do
    for fh in 0 1; do
      GNNREC_FUSED_HEAD=$fh timeout -k 10 120 python -u tools/probe_c2_step.py 10 $nw 2>/dev/null | tail -1 || exit 1
    done
  done
done
