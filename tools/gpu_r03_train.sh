#!/bin/bash
# Round 3: the fused training relation — bitwise test, then the C2 step A/B (fused vs two-node).
set -o pipefail
mkdir -p gpurun_out
LOG=gpurun_out/r03_train.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampling.py -k "fused_training or autograd or training_step" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > $LOG 2>&1 || { echo "tests failed"; tail -40 $LOG; exit 1; }
tail -2 $LOG
for rep in 1 2; do
  for f in 1 0; do
    echo -n "GNNREC_TRAIN_FUSED=$f "; GNNREC_TRAIN_FUSED=$f timeout -k 10 120 python -u tools/probe_c2_step.py 2>/dev/null | tail -1 || exit 1
  done
done
