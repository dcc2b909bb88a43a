#!/bin/bash
# LSTM: HIP backward through time and the sharded pass at P = 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_configs.py -k "lstm" -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_lstm_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_lstm_tests.log | head; tail -40 gpurun_out/r03_lstm_tests.log; exit 1; }
tail -12 gpurun_out/r03_lstm_tests.log
