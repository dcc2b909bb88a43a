#!/bin/bash
# Round 3: the 64-row-per-wave GEMM (GNNREC_GEMM_WIDE=<min rows>) and the pair launch's
# side work after its pre-projections (GNNREC_SIDE_AFTER_PRE): parity, GEMM A/B, C5 A/B.
set -o pipefail
mkdir -p gpurun_out
GNNREC_GEMM_WIDE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "gemm or project or golden or sage or train or backward or grad" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_wide_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_wide_tests.log | head; tail -30 gpurun_out/r03_wide_tests.log; exit 1; }
tail -1 gpurun_out/r03_wide_tests.log
for rep in 1 2; do
  for shape in "1000000 256 128 20 one" "1000000 256 128 20 sage" "1000000 128 128 20 one" "200000 128 128 50 one"; do
    for w in 0 1; do
      echo -n "WIDE=$w "; GNNREC_GEMM_WIDE=$w timeout -k 10 60 python3 tools/micro/gemm_one.py $shape || exit 1
    done
  done
done
bash tools/micro/c5_ab.sh "GNNREC_SIDE_AFTER_PRE=0" "GNNREC_SIDE_AFTER_PRE=1" "GNNREC_SIDE_AFTER_PRE=1 GNNREC_GEMM_WIDE=65536" || exit 1
