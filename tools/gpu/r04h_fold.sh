#!/bin/bash
# round 4 (h): NodeEmbedding folded into the first training layer — training tests, then the
# C2 step at K = 10 and the reference's K = 2500 with the fold on / off (GNNREC_TRAIN_FOLD)
set -o pipefail
mkdir -p gpurun_out/r04h
O=gpurun_out/r04h
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sampling.py \
  > $O/tests.log 2>&1 || { echo "sampling tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for K in 2500 10; do
  for f in 1 0 1 0; do
    GNNREC_TRAIN_FOLD=$f timeout -k 10 200 python -u tools/probe_c2_step.py $K 2 > $O/k${K}_f$f.log 2>&1 || { echo "probe failed"; tail $O/k${K}_f$f.log; exit 1; }
    echo "K=$K fold=$f $(tail -1 $O/k${K}_f$f.log | cut -c1-200)"
  done
done
