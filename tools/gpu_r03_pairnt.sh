#!/bin/bash
# pair launch with the low-degree relation's source rows non-temporal: tests, C5 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_configs.py -k "project2 or pair or c5" -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pairnt_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pairnt_tests.log | head; tail -30 gpurun_out/r03_pairnt_tests.log; exit 1; }
tail -1 gpurun_out/r03_pairnt_tests.log
bash tools/micro/c5_ab.sh "GNNREC_SPP2_NT=0" "GNNREC_SPP2_NT=1" || exit 1
