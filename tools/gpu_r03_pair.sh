#!/bin/bash
# Round 3: the pipelined two-relation launch — parity, then a C5 A/B against the old kernel.
set -o pipefail
mkdir -p gpurun_out
LOG=gpurun_out/r03_pair.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "project2 or pair_launch" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $LOG 2>&1 || { echo "parity failed"; tail -30 $LOG; exit 1; }
tail -2 $LOG
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_dist.py -k "pair or side_stream" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider >> $LOG 2>&1 || { echo "async/dist failed"; tail -30 $LOG; exit 1; }
tail -2 $LOG
bash tools/micro/c5_ab.sh "GNNREC_SPP2_PIPE=1" "GNNREC_SPP2_PIPE=0" 2>&1 | tee -a $LOG
